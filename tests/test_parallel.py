"""Data-parallel reducer (vaeunet_amd/parallel.py) on CPU with gloo, world 2.

The fused backward reports finished parameter gradients through
``grad_ready``; buckets must be all-reduced as soon as they are complete (not
at the end), and after ``finish()`` every rank must hold the average of the
per-rank gradients (DDP semantics, SURVEY.md §8e parity check)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(8, 16, 3), nn.BatchNorm2d(16), nn.Conv2d(16, 16, 1),
                         nn.Linear(16, 300), nn.Linear(300, 7))


def _worker(rank, world, port, out_q, bucket_bytes):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vaeunet_amd.parallel import GradBucketReducer
        m = _model()
        # a channels_last weight exercises the layout-preserving grad view
        m[0].weight.data = m[0].weight.data.contiguous(memory_format=torch.channels_last)
        if rank == 1:
            with torch.no_grad():
                for p in m.parameters():
                    p.add_(1.0)  # rank 0's parameters must win the initial broadcast
        red = GradBucketReducer(m.parameters(), bucket_bytes=bucket_bytes)
        params = list(m.parameters())
        results = []
        for step in range(2):
            for q in params:
                q.grad = None  # zero_grad(set_to_none=True) between optimizer steps
            red.prepare()
            launched = []
            # engine order: reverse registration; "accumulate" into the bound views
            for i, p in enumerate(reversed(params)):
                g = torch.full_like(p, float(rank + 1 + step)) * (i + 1)
                p.grad.add_(g)
                red.grad_ready([p])
                launched.append(len(red._handles))
            early = launched[len(params) // 2] > 0
            red.finish()
            results.append(([p.grad.detach().numpy().copy() for p in params], early))
        out_q.put((rank, [p.detach().numpy().copy() for p in params], results,
                   m[0].weight.grad.is_contiguous(memory_format=torch.channels_last)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes", [4096, 1 << 30])
def test_bucketed_allreduce_average_gloo(bucket_bytes):
    world = 2
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join(
        [os.path.dirname(here), here] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, bucket_bytes)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, params, results, cl = q.get(timeout=120)
        res[rank] = (params, results, cl)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = list(_model().parameters())
    for r in range(world):
        params, results, cl = res[r]
        assert cl, "channels_last weight lost its gradient layout"
        for a, b in zip(params, ref):
            assert torch.equal(torch.from_numpy(a), b.detach()), "parameters were not broadcast from rank 0"
        for step, (grads, early) in enumerate(results):
            n = len(grads)
            for i, g in enumerate(grads):
                g = torch.from_numpy(g)
                k = n - i  # position in reverse order (1-based)
                mean = sum(float(rr + 1 + step) for rr in range(world)) / world * k
                assert torch.allclose(g, torch.full_like(g, mean)), (step, i)
            if bucket_bytes == 4096:
                assert early, "buckets were not launched during the backward"


def _accum_worker(rank, world, port, out_q):
    """train.py:401-411 grad-accumulation x2 under DP: the first micro-batch runs
    inside no_sync (no collective, local accumulation), the second reduces the
    sum; the result must be the average over ranks of both micro-batches."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vaeunet_amd.parallel import GradBucketReducer
        m = _model()
        red = GradBucketReducer(m.parameters(), bucket_bytes=4096)
        params = list(m.parameters())
        out = []
        for opt_step in range(2):
            for q in params:
                q.grad = None
            for micro in range(2):
                ctx = red.no_sync() if micro == 0 else _nullctx()
                with ctx:
                    red.prepare()
                    for i, p in enumerate(reversed(params)):
                        p.grad.add_(torch.full_like(p, float(10 * rank + micro + 1 + opt_step)) * (i + 1))
                        red.grad_ready([p])
                    if micro == 0:
                        assert not red._handles, "collective launched inside no_sync"
                    red.finish()
            out.append([p.grad.detach().numpy().copy() for p in params])
        out_q.put((rank, out))
    finally:
        dist.destroy_process_group()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def test_grad_accumulation_no_sync_gloo():
    world = 2
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join(
        [os.path.dirname(here), here] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_accum_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        for opt_step, grads in enumerate(res[r]):
            n = len(grads)
            for i, g in enumerate(grads):
                k = n - i
                # sum over the two micro-batches, averaged over the two ranks
                want = sum(float(10 * rr + mb + 1 + opt_step) for rr in range(world) for mb in range(2)) / world * k
                assert torch.allclose(torch.from_numpy(g), torch.full_like(torch.from_numpy(g), want)), (r, opt_step, i)


def _late_worker(rank, world, port, out_q):
    """A parameter the engine never reports (grad_ready) whose gradient is
    zero on step 0 and non-zero from step 1 on: the reducer must drop it only
    while it is zero (the round-5 reducer cached "unused" from the
    first step and dropped the later gradients for good)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vaeunet_amd.parallel import GradBucketReducer
        m = _model()
        red = GradBucketReducer(m.parameters(), bucket_bytes=4096)
        params = list(m.parameters())
        late = params[2]  # never reported
        out = []
        for step in range(3):
            for q in params:
                q.grad = None
            red.prepare()
            for i, p in enumerate(reversed(params)):
                if p is late:
                    if step >= 1:
                        p.grad.add_(float(rank + 1 + step))
                    continue
                p.grad.add_(torch.full_like(p, float(rank + 1)))
                red.grad_ready([p])
            red.finish()
            out.append(None if late.grad is None else late.grad.detach().numpy().copy())
        out_q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_unreported_parameter_late_gradient_gloo():
    world = 2
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ["PYTHONPATH"] = os.pathsep.join(
        [os.path.dirname(here), here] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_late_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        g0, g1, g2 = res[r]
        assert g0 is None, "a zero, unreported gradient must be reset to None"
        for step, g in ((1, g1), (2, g2)):
            assert g is not None, f"late gradient dropped on step {step}"
            want = sum(float(rr + 1 + step) for rr in range(world)) / world
            assert torch.allclose(torch.from_numpy(g), torch.full_like(torch.from_numpy(g), want)), (r, step)
