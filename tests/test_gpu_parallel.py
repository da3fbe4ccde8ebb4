"""Data-parallel product path on the GPU (vaeunet_amd/parallel.py).

* world 2, both ranks on cuda:0, ``gloo`` backend (one card on the test box;
  RCCL refuses two ranks on one device): the REAL fused UNet engine drives
  the buckets through ``Mode.notify`` -> ``grad_ready``; the DP gradients must
  equal the mean over ranks of single-rank gradients, also
  with grad accumulation x2 where the first micro-batch runs under
  ``no_sync`` (train.py:401-411);
* world 1 on the ``nccl`` backend (RCCL): the ReduceOp.AVG branch on the
  engine path.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(i):
    g = torch.Generator().manual_seed(500 + i)
    x = torch.rand(2, 3, 64, 64, generator=g)
    t = (torch.rand(2, 1, 64, 64, generator=g) < 0.05).float()
    return x, t


def _grads(model, x, t):
    from vaeunet_amd.loss import CombinedLoss
    for p in model.parameters():
        p.grad = None
    loss = CombinedLoss()(model(x.cuda().contiguous(memory_format=torch.channels_last)), t.cuda())
    loss.backward()
    return [p.grad.detach().clone() for p in model.parameters()]


def _worker(rank, world, port, backend, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from vaeunet_amd import UNet, parallel
        from vaeunet_amd.init import seeded_init_
        from vaeunet_amd.loss import CombinedLoss
        model = seeded_init_(UNet(3, 1), 0).cuda().to(memory_format=torch.channels_last).train()
        # single-rank gradients of every shard (deterministic kernels: the
        # same on every rank), before the reducer is attached
        single = [_grads(model, *_shard(i)) for i in range(3 * world)]
        red = parallel.attach(model, bucket_bytes=2 * 1024 * 1024)
        launched = []
        orig = red._launch

        def spy(bi):
            launched.append(bi)
            orig(bi)
        red._launch = spy
        res = {}
        # (a) one micro-batch per rank: shard `rank`
        for p in model.parameters():
            p.grad = None
        red.prepare()
        x, t = _shard(rank)
        CombinedLoss()(model(x.cuda().contiguous(memory_format=torch.channels_last)), t.cuda()).backward()
        n_during = len(launched)
        red.finish()
        res["dp"] = [p.grad.detach().cpu().numpy() for p in model.parameters()]
        res["early"] = n_during
        res["nbuckets"] = len(red.buckets)
        # (b) accumulation x2: shards world + 2*rank + {0, 1}; micro-batch 0 under no_sync
        for p in model.parameters():
            p.grad = None
        launched.clear()
        for micro in range(2):
            x, t = _shard(world + 2 * rank + micro) if world > 1 else _shard(micro)
            if micro == 0:
                with red.no_sync():
                    red.prepare()
                    loss = CombinedLoss()(model(x.cuda().contiguous(memory_format=torch.channels_last)), t.cuda())
                    loss.backward()
                    red.finish()
                res["nosync_launches"] = len(launched)
            else:
                red.prepare()
                CombinedLoss()(model(x.cuda().contiguous(memory_format=torch.channels_last)), t.cuda()).backward()
                red.finish()
        res["acc"] = [p.grad.detach().cpu().numpy() for p in model.parameters()]
        # numpy (pickled by value): torch tensors would be shared through file
        # descriptors that die with this process
        res["single"] = [[g.cpu().numpy() for g in s] for s in single]
        torch.cuda.synchronize()
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _run(world, backend):
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join(
        [os.path.dirname(here), here] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _close(a, b):
    a, b = torch.as_tensor(a), torch.as_tensor(b)
    return (a - b).abs().max().item() <= 1e-6 * max(b.abs().max().item(), 1e-12) + 1e-9


def test_dp_world2_gloo_engine_path():
    world = 2
    res = _run(world, "gloo")
    single = res[0]["single"]
    for r in range(world):
        rr = res[r]
        assert rr["nbuckets"] > 1
        assert rr["early"] > 0, "no bucket was all-reduced during the backward"
        assert rr["nosync_launches"] == 0, "collective launched inside no_sync"
        for i, g in enumerate(rr["dp"]):
            want = (single[0][i] + single[1][i]) / 2
            assert _close(g, want), ("dp", r, i)
        for i, g in enumerate(rr["acc"]):
            want = sum(single[world + k][i] for k in range(2 * world)) / world
            assert _close(g, want), ("accumulate", r, i)


def test_dp_world1_nccl_avg_branch():
    res = _run(1, "nccl")[0]
    for i, g in enumerate(res["dp"]):
        assert _close(g, res["single"][0][i])
    for i, g in enumerate(res["acc"]):
        assert _close(g, res["single"][0][i] + res["single"][1][i])


def _graph_worker(rank, world, port, backend, out_q):
    """Eager DP steps vs the same steps captured as one HIP graph with the
    bucketed RCCL all-reduces inside (GraphedTrainStep(reducer=...))."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from vaeunet_amd import UNet, parallel
        from vaeunet_amd.graph import GraphedTrainStep
        from vaeunet_amd.init import seeded_init_
        from vaeunet_amd.loss import CombinedLoss
        from vaeunet_amd.optim import FusedAdamW, clip_grad_norm_
        x, t = _shard(rank)
        x = x.cuda().contiguous(memory_format=torch.channels_last)
        t = t.cuda()
        out = {}
        for mode in ("eager", "graph"):
            model = seeded_init_(UNet(3, 1), 0).cuda().to(memory_format=torch.channels_last).train()
            red = parallel.attach(model, bucket_bytes=2 * 1024 * 1024)
            opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)

            def fb():
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = CombinedLoss()(model(x), t)
                loss.backward()
                return loss
            losses = []
            if mode == "eager":
                for _ in range(4):
                    red.prepare()
                    loss = fb()
                    red.finish()
                    clip_grad_norm_(model.parameters(), 1.0)
                    opt.step()
                    red.zero_grad()
                    losses.append(float(loss.detach()))
                losses = losses[2:]
            else:
                gs = GraphedTrainStep(fb, opt, max_norm=1.0, warmup=2, reducer=red)
                losses = [float(gs.step().detach()) for _ in range(2)]
            torch.cuda.synchronize()
            out[mode] = ([p.detach().cpu().numpy() for p in model.parameters()], losses)
        out_q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_dp_graph_capture_rccl_world1():
    """The captured DP step (RCCL collectives inside the graph) replays to the
    same parameters as the eager DP step.  World size 1: one GPU here (RCCL
    refuses two ranks on one device); gloo collectives are host-side and
    cannot be captured, so the multi-rank path is covered eagerly above."""
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join(
        [os.path.dirname(here), here] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_graph_worker, args=(0, 1, _free_port(), "nccl", q))
    p.start()
    _, res = q.get(timeout=150)
    p.join(timeout=60)
    assert p.exitcode == 0
    pe, le = res["eager"]
    pg, lg = res["graph"]
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(a)), (le, lg)
    for i, (a, b) in enumerate(zip(pg, pe)):
        assert _close(a, b), i


def _unused_worker(rank, world, port, backend, out_q):
    """UNetResNet(latent_injection='none') under the DP reducer: z_initial gets
    no gradient (use_bottleneck False) -- eager DP steps and the captured DP
    step both leave it untouched (.grad None, no AdamW state, no decay)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from vaeunet_amd import UNetResNet, parallel
        from vaeunet_amd.graph import GraphedTrainStep
        from vaeunet_amd.init import seeded_init_
        from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
        from vaeunet_amd.optim import FusedAdamW, clip_grad_norm_
        g = torch.Generator().manual_seed(5)
        x = torch.rand(2, 3, 64, 64, generator=g).cuda().contiguous(memory_format=torch.channels_last)
        t = (torch.rand(2, 1, 64, 64, generator=g) > 0.5).float().cuda()
        res = {}
        for mode in ("eager", "graph"):
            model = seeded_init_(UNetResNet(3, 1, pretrained=False, latent_injection="none"), 0)
            model = model.cuda().to(memory_format=torch.channels_last).train()
            z0 = {n: p.detach().clone() for n, p in model.named_parameters() if n.startswith("z_initial")}
            red = parallel.attach(model, bucket_bytes=2 * 1024 * 1024)
            opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)

            def fb():
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    lg, mu, lv = model(x)
                    loss = CombinedLoss()(lg, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
                loss.backward()
                return loss
            if mode == "eager":
                for _ in range(3):
                    red.prepare()
                    fb()
                    red.finish()
                    clip_grad_norm_([p for p in model.parameters() if p.grad is not None], 1.0)
                    opt.step()
                    red.zero_grad()
            else:
                gs = GraphedTrainStep(fb, opt, max_norm=1.0, warmup=1, reducer=red)
                for _ in range(2):
                    gs.step()
            torch.cuda.synchronize()
            ok = []
            for n, p in model.named_parameters():
                if n.startswith("z_initial"):
                    ok.append((n, p.grad is None, bool(torch.equal(p.detach(), z0[n])), len(opt.state.get(p, {}))))
            moved = sum(1 for n, p in model.named_parameters() if not n.startswith("z_initial") and p.grad is not None)
            res[mode] = (ok, moved)
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_dp_unused_parameter_left_untouched():
    """with the reducer bound, an unused parameter must not pick up a
    zero gradient view, AdamW state or weight decay (torch semantics)."""
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join(
        [os.path.dirname(here), here] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_unused_worker, args=(0, 1, _free_port(), "nccl", q))
    p.start()
    _, res = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    for mode in ("eager", "graph"):
        ok, moved = res[mode]
        assert ok and moved > 0, (mode, ok, moved)
        for name, grad_none, same, nstate in ok:
            assert same and nstate == 0, (mode, name, grad_none, same, nstate)


def _grads_worker(rank, world, port, backend, out_q):
    """Every parameter the single-process backward gives a gradient gets the
    SAME gradient through the DP reducer at world 1 (RCCL AVG over one rank is
    exact), and no other parameter gets one: UNet and UNetResNet in every
    latent-injection mode (the reducer must never drop a gradient
    a backward path forgot to report)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from vaeunet_amd import UNet, UNetResNet, parallel
        from vaeunet_amd.init import seeded_init_
        from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
        g = torch.Generator().manual_seed(9)
        x = torch.rand(2, 3, 64, 64, generator=g).cuda().contiguous(memory_format=torch.channels_last)
        t1 = (torch.rand(2, 1, 64, 64, generator=g) > 0.5).float().cuda()
        t2 = torch.cat([1 - t1, t1], 1)
        cases = [("unet", None)] + [("vae", m) for m in ("all", "none", "first", "last", "bottleneck",
                                                                   "inject_no_bottleneck")]
        res = {}
        for kind, inj in cases:
            grads = []
            for use_red in (False, True):
                if kind == "unet":
                    model = seeded_init_(UNet(3, 2), 0)
                else:
                    model = seeded_init_(UNetResNet(3, 1, pretrained=False, latent_injection=inj), 0)
                model = model.cuda().to(memory_format=torch.channels_last).train()
                if kind == "vae":
                    model.eps_override = torch.randn(2, 32, generator=torch.Generator().manual_seed(3)).cuda()
                red = parallel.attach(model, bucket_bytes=2 * 1024 * 1024) if use_red else None
                if red is not None:
                    red.prepare()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    if kind == "unet":
                        loss = CombinedLoss()(model(x), t2)
                    else:
                        lg, mu, lv = model(x)
                        loss = CombinedLoss()(lg, t1) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
                loss.backward()
                if red is not None:
                    red.finish()
                torch.cuda.synchronize()
                grads.append({n: (p.grad.detach().float().cpu().clone() if p.grad is not None else None)
                              for n, p in model.named_parameters()})
            plain, dp = grads
            bad = [n for n in plain if (plain[n] is None) != (dp[n] is None)
                   or (plain[n] is not None and not torch.equal(plain[n], dp[n]))]
            res[f"{kind}:{inj}"] = (bad, sum(v is None for v in plain.values()), len(plain))
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_dp_reducer_gradients_equal_single_process():
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join(
        [os.path.dirname(here), here] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_grads_worker, args=(0, 1, _free_port(), "nccl", q))
    p.start()
    _, res = q.get(timeout=280)
    p.join(timeout=60)
    assert p.exitcode == 0
    for case, (bad, n_none, n) in res.items():
        assert not bad, (case, bad[:8])
        if case.startswith("unet"):
            assert n_none == 0
