"""Benchmark: whole-node images/sec of the VAE-U-Net training step.

Workload (BASELINE.json configs[1], metric quoted on it):
  UNet(n_channels=3, n_classes=2, bilinear=False), synthetic 3x512x512 batches,
  batch 8 per GPU, bf16 (torch.autocast, the train.py:385 path), one step =
  forward + CombinedLoss + backward (+ RCCL gradient all-reduce when N>1) +
  clip_grad_norm_(1.0) + AdamW(lr 1e-4, wd 1e-5) step + zero_grad.
  (train.py:381-411; the optimizer runs every step here, not every 2nd.)

Launch: python bench.py [--gpus N --steps K --warmup W]; for N>1 the driver
uses torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE from the env).
Rank 0 prints ONE JSON line (see README / DESIGN.md §Measurement).  A default
N=1 run (CPU leg on) also runs BASELINE configs[2] -- the UNetResNet VAE step,
same steps / warmup -- as a child process and nests its line under
"secondary.config3_vae"; the headline value is config 2's.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
# algorithmic FLOPs of the 3x3 convolutions per 512x512 image:
# fwd 368.13 + dgrad 367.22 + wgrad 368.13 GFLOP (inc.0 included)
CONV3_GFLOP_PER_IMG = 1103.5
METRIC = "images/sec (whole node) at 3x512x512 bs=8/GPU; Dice parity vs CPU ref"   # BASELINE.json
PMC_TRAFFIC = {"unet": os.path.join(ROOT, "profiles", "pmc_traffic.json"),
               "vae": os.path.join(ROOT, "profiles", "pmc_traffic_vae.json")}


def pmc_traffic(model):
    """HBM bytes per launch of the 3x3 conv kernels from the committed rocprofv3
    PMC passes over this model's bench (tools/gpu_evidence.sh ->
    tools/pmc_traffic.py), or None."""
    try:
        with open(PMC_TRAFFIC[model]) as f:
            v = json.load(f).get("conv3x3_hbm_bytes_per_launch")
        return None if v is None else round(float(v))
    except (OSError, ValueError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 300 timed steps (~4.5 s of graph replay for the UNet, ~2.5 s for the
    # VAE child): long enough for an external GPU-busy sampler polling every
    # few seconds to see the card busy (50 steps were
    # 0.75 s of a ~150 s run), short enough for the default run to stay
    # within minutes
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--classes", type=int, default=2)
    ap.add_argument("--model", choices=("unet", "vae"), default="unet",
                    help="unet = BASELINE configs[1] (the metric); vae = configs[2], UNetResNet + KL")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # 20 rounds ~ 68 us: covers the host enqueue of start event + launch + end
    # event (same box: the 3x3 family read 0.442-0.445 without it, 0.453-0.454
    # with it -- host time had leaked into the brackets; profiles/r6td_timer_delay.txt)
    ap.add_argument("--timer-delay", type=int, default=20,
                    help="roofline leg: GPU sleep rounds (~3.4 us each) queued before every timed launch")
    ap.add_argument("--layer-table", action="store_true",
                    help="print the roofline leg's per-launch GEMM table (shape, kernel, time) to stderr")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the config-3 (VAE) secondary line that a default N=1 UNet run appends "
                         "(--no-cpu-baseline, the A/B and profiling runs, skips it too)")
    ap.add_argument("--cpu-batch", type=int, default=8, help="CPU baseline batch (BASELINE.md §4: 8)")
    ap.add_argument("--cpu-steps", type=int, default=3, help="timed CPU steps per leg after 1 warmup")
    ap.add_argument("--cpu-budget-s", type=float, default=60.0,
                    help="cap on the timed CPU work per leg (fewer steps on a slow host)")
    ap.add_argument("--cpu-no-bf16", action="store_true", help="skip the CPU autocast-bf16 leg")
    ap.add_argument("--torch-optim", action="store_true",
                    help="torch.optim.AdamW + torch clip_grad_norm_ instead of the fused HIP ones")
    ap.add_argument("--engine-flag", action="append", default=[], metavar="NAME=0|1",
                    help="set a vaeunet_amd.engine module switch (A/B runs), e.g. FUSE_BN_BWD_REDUCE=0, or "
                         "MODULE.NAME for another vaeunet_amd module, e.g. vae_engine.LATENT_VECTORS=0")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VAL",
                    help="vu_gemm_set_tuning(KEY, VAL) before the run (library A/B runs; include/vaeunet.h)")
    ap.add_argument("--unsafe-experiment", action="store_true",
                    help="allow --tune experiment modes (VU_TUNE_UNSAFE + *_XM: wrong results by design); "
                         "the JSON line then carries experiment_modes")
    ap.add_argument("--overlap", action="store_true",
                    help="weight gradients on a side stream (engine.OVERLAP_WGRAD; measured slower, A/B only)")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="replay the step as one captured HIP graph (vaeunet_amd.graph); auto = on "
                         "at world size 1 with the fused optimizer; at N > 1 only with 'on' (the captured "
                         "RCCL all-reduces are untested across GPUs: experimental)")
    return ap.parse_args()


def synthetic(B, S, C, rank, dev):
    g = torch.Generator().manual_seed(1000 + rank)
    x = torch.rand(B, 3, S, S, generator=g)
    m = (torch.rand(B, 1, S, S, generator=g) < 0.0085).float()
    t = torch.cat([1 - m, m], 1) if C == 2 else m
    return (x.to(dev).contiguous(memory_format=torch.channels_last),
            t.to(dev).contiguous(memory_format=torch.channels_last))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _cgroup_cpus():
    """CPUs the cgroup CPU quota grants this process (cpu.max / CFS quota), or None."""
    import math
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, math.ceil(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, math.ceil(q / p))
    except (OSError, ValueError):
        pass
    return None


def _cpu_threads():
    """(threads, affinity, quota): the cores this process can actually run on
    -- ``len(os.sched_getaffinity(0))``, capped by the cgroup
    CPU quota when one is set.  On the GPU box the affinity mask lists all 256
    host cores but cpu.max grants 16 CPUs; 256 threads then run a CPU conv 12x
    SLOWER than 16 (profiles/r3_cpu_probe.log), so the quota is the count that
    gives the host its best time."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = _cgroup_cpus()
    return (min(n, quota) if quota else n), n, quota


def _thread_probe(threads, affinity):
    """One CPU 3x3 conv (8x64x256^2) at the chosen thread count and at the full
    affinity count: the evidence for the choice, measured in the same run."""
    import torch.nn.functional as F
    x = torch.randn(8, 64, 256, 256).contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 64, 3, 3).contiguous(memory_format=torch.channels_last)
    out = {}
    for t in sorted({threads, affinity}):
        torch.set_num_threads(t)
        F.conv2d(x, w, padding=1)
        t0 = time.perf_counter()
        F.conv2d(x, w, padding=1)
        out[str(t)] = round((time.perf_counter() - t0) * 1e3, 1)
    return {"what": "ms of one 8x64x256^2 3x3 conv (torch CPU) per thread count", "ms": out}


def _ref_model(args):
    """The oracle model of the benched configuration, same seeded weights as the GPU model."""
    from oracle import cpu_ref as R
    from vaeunet_amd.init import seeded_init_
    if args.model == "vae":
        from vaeunet_amd import UNetResNet
        return R.UNetResNetRef(seeded_init_(UNetResNet(3, 1, pretrained=False), 0).state_dict())
    from vaeunet_amd import UNet
    return R.UNetRef(seeded_init_(UNet(3, args.classes), 0).state_dict())


def _latent_eps(B):
    """A fixed reparameterisation draw (latent 32) shared by the oracle and the
    GPU model in the parity leg (unet_resnet.py:191-194 with eps injected)."""
    return torch.randn(B, 32, generator=torch.Generator().manual_seed(77))


def cpu_baseline(args, dev):
    """The CPU oracle (clean-room restatement of the reference, oracle/cpu_ref.py;
    kind "port") timed on this host: the same synthetic batch
    (B x 3 x S x S, rank-0 seed), 1 warmup + K timed full train steps (fwd,
    loss, bwd, clip, AdamW).  Threads: len(sched_getaffinity) capped by the
    cgroup CPU quota (_cpu_threads; the thread probe measured in the same run
    is reported beside it).  Legs, both on those threads: fp32 (the headline:
    reference semantics) and CPU autocast bf16 (train.py's amp default on
    CPU; --cpu-no-bf16 skips it).  --model vae: UNetResNet with CombinedLoss +
    1e-3 * KL (free bits 1e-3) and a fixed latent draw.

    The first fp32 warmup step's pre-update outputs are also the parity
    reference: the GPU model (fp32 parity mode, same weights, same batch) is
    compared with them (the "Dice parity vs CPU ref" of the metric name)."""
    from oracle import cpu_ref as R
    threads, affinity, quota = _cpu_threads()
    probe = _thread_probe(threads, affinity)
    _progress(f"cpu_baseline thread probe: {probe['ms']}")
    B = args.cpu_batch
    vae = args.model == "vae"
    x, t = synthetic(B, args.size, args.classes, 0, "cpu")
    eps = _latent_eps(B) if vae else None

    def train_step(model, opt):
        if vae:
            return R.vae_train_step(model, opt, x, t, eps)
        return R.train_step(model, opt, x, t)
    plan = [("fp32", "fp32", threads)]
    if not args.cpu_no_bf16:
        plan.append(("bf16", "bf16", threads))
    legs, parity = {}, None
    for name, prec, threads in plan:
        torch.set_num_threads(threads)
        model = _ref_model(args)
        opt = R.AdamW(model.p.values(), lr=1e-4, weight_decay=1e-5)
        ctx = torch.autocast("cpu", dtype=torch.bfloat16) if prec == "bf16" else _Null()
        t0 = time.perf_counter()
        _progress(f"cpu_baseline {name} ({threads} threads): warmup step")
        with ctx, _Heartbeat(f"cpu_baseline {name} warmup"):
            ref_out, ref_loss, _ = train_step(model, opt)  # warmup; pre-update outputs
        warm = time.perf_counter() - t0
        _progress(f"cpu_baseline {name} ({threads} threads) warmup step: {warm:.1f} s")
        if parity is None and prec == "fp32":
            parity = gpu_parity(args, x, t, ref_out, ref_loss, dev, eps)
        # bounded sample: a slow host gets fewer timed steps (stated in "sample")
        n = args.cpu_steps if warm * args.cpu_steps <= args.cpu_budget_s else max(1, int(args.cpu_budget_s // warm))
        t0 = time.perf_counter()
        with ctx, _Heartbeat(f"cpu_baseline {name} timed steps"):
            for i in range(n):
                train_step(model, opt)
                _progress(f"cpu_baseline {name} step {i + 1}/{n}: {time.perf_counter() - t0:.1f} s")
        dt = time.perf_counter() - t0
        legs[name] = {"value": round(B * n / dt, 4), "threads": threads, "steps": n,
                      "s_per_step": round(dt / n, 3)}
    f = legs["fp32"]
    what = ("UNetResNet(3,1) VAE train steps (fwd+CombinedLoss+1e-3*KL+bwd+clip+AdamW)" if vae else
            f"UNet(3,{args.classes}) train steps (fwd+CombinedLoss+bwd+clip+AdamW)")
    out = {"value": f["value"], "unit": "images/sec", "cores": threads, "kind": "port",
           "cpu_model": _cpu_model(), "affinity_cores": affinity, "cgroup_cpu_quota": quota,
           "cores_basis": ("len(sched_getaffinity) capped by the cgroup cpu.max quota" if quota and quota < affinity
                           else "len(sched_getaffinity)"),
           "thread_probe": probe,
           "sample": (f"1 warmup + {f['steps']} timed fp32 {what} on {B}x3x{args.size}x{args.size} "
                      f"(oracle/cpu_ref.py, torch CPU, {threads} threads)"),
           "legs": legs}
    return out, parity


def _progress(msg):
    """Progress of the long CPU legs on stderr (the JSON line stays the only stdout line)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


class _Heartbeat:
    """A stderr line every `every` seconds while a long CPU leg runs (a single
    CPU step can outlast the GPU runner's silence limit)."""

    def __init__(self, what, every=30.0):
        import threading
        self.what, self.every = what, every
        self.stop = threading.Event()
        self.t0 = time.perf_counter()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(self.every):
            _progress(f"{self.what}: {time.perf_counter() - self.t0:.0f} s")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *a):
        self.stop.set()
        return False


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def gpu_parity(args, x, t, ref_out, ref_loss, dev, eps=None):
    """GPU model (fp32 parity mode: no autocast) vs the CPU oracle, same weights,
    same batch (and, for the VAE, the same latent draw): Dice of the class maps
    (argmax for 2 classes, logit > 0 for 1), the reference's own dice_score
    semantics (utils/metrics.py:8-35: both tensors thresholded at 0.5), class
    agreement with the reference margin of EVERY flipped pixel, max |dlogit|,
    |dloss| (and mu / logvar for the VAE)."""
    from vaeunet_amd.init import seeded_init_
    from vaeunet_amd.loss import CombinedLoss, kl_with_free_bits
    from vaeunet_amd.metrics import dice_score
    from oracle import cpu_ref as R
    vae = args.model == "vae"
    if vae:
        from vaeunet_amd import UNetResNet
        model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0)
        model.eps_override = eps
        ref_logits, ref_mu, ref_lv = ref_out
    else:
        from vaeunet_amd import UNet
        model = seeded_init_(UNet(3, args.classes), 0)
        ref_logits = ref_out
    model = model.to(dev).to(memory_format=torch.channels_last).train()
    xg = x.to(dev).contiguous(memory_format=torch.channels_last)
    tg = t.to(dev).contiguous(memory_format=torch.channels_last)
    extra = {}
    with torch.no_grad():
        if vae:
            lg, mu, lv = model(xg)
            loss = CombinedLoss()(lg, tg) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
            for k, a, b in (("mu", mu, ref_mu), ("logvar", lv, ref_lv)):
                extra[f"{k}_max_rel_err"] = float((a.float().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-12))
        else:
            lg = model(xg)
            loss = CombinedLoss()(lg, tg)
        ds_gpu = float(dice_score(lg, ref_logits.float().to(dev).contiguous(memory_format=torch.channels_last)))
    lg = lg.float().cpu()
    ref = ref_logits.float()
    ds_ref = float(R.dice_score(lg.contiguous(), ref.contiguous()))
    if lg.shape[1] == 1:
        fg, fr = lg[:, 0] > 0, ref[:, 0] > 0
        flips = fg != fr
        margins = ref[:, 0].abs()[flips]
    else:
        cg, cr = lg.argmax(1), ref.argmax(1)
        fg, fr = (cg == 1), (cr == 1)
        flips = cg != cr
        margins = (ref[:, 0] - ref[:, 1]).abs()[flips]
    den = int(fg.sum() + fr.sum())
    dice = 1.0 if den == 0 else 2.0 * int((fg & fr).sum()) / den
    out = {"dice_class_map": round(dice, 6), "dice_score_ref_semantics": round(ds_gpu, 7),
           "dice_score_ref_semantics_cpu": round(ds_ref, 7),
           "argmax_agree": round(float((~flips).float().mean()), 8), "argmax_flips": int(flips.sum()),
           "flipped_ref_margins": [float(f"{v:.3e}") for v in margins.tolist()[:32]],
           "max_flipped_ref_margin": float(margins.max()) if margins.numel() else 0.0,
           "max_abs_logit_diff": float((lg - ref).abs().max()),
           "logit_scale": float(ref.abs().max()),
           "loss_abs_diff": abs(float(loss) - float(ref_loss))}
    out.update(extra)
    out["sample"] = (f"{x.shape[0]}x3x{args.size}x{args.size}, fp32 GPU vs oracle/cpu_ref.py fp32, same weights/input"
                     + (", same latent eps; class = logit > 0" if vae else ""))
    return out


def vae_secondary(args):
    """BASELINE configs[2] (UNetResNet VAE train step, same batch / image) as a
    child run of this script -- ``--model vae`` with the same steps / warmup,
    its own 3x3 roofline, no CPU leg -- so the driver's default bench also
    records config 3 (a child process, not an exec: this one has touched the
    GPU).  Its JSON line is nested as-is; the headline value stays config 2."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--model", "vae", "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--batch", str(args.batch), "--size", str(args.size),
           "--no-cpu-baseline", "--graph", args.graph]
    if args.no_roofline:
        cmd.append("--no-roofline")
    _progress("secondary: config-3 VAE run")
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}"}
    lines = r.stdout.strip().splitlines()
    try:
        sec = json.loads(lines[-1])
    except (IndexError, ValueError) as e:   # never lose the measured headline over the secondary
        return {"error": f"unparsable child output: {e!r}"}
    for k in ("metric", "higher_is_better", "vs_baseline", "cpu_baseline", "parity", "data", "n_gpus"):
        sec.pop(k, None)
    return sec


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # nccl = RCCL over xGMI; VU_DIST_BACKEND=gloo rehearses the N>1 path
        # with several ranks sharing one GPU (RCCL refuses duplicate devices)
        backend = os.environ.get("VU_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, init_method="env://")
        if backend == "gloo":
            local = local % torch.cuda.device_count()   # rehearsal: ranks share the card(s)
        elif local >= torch.cuda.device_count():
            raise SystemExit(f"bench: LOCAL_RANK {local} but only {torch.cuda.device_count()} visible GPUs")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from vaeunet_amd import UNet, kernels as K, engine as E
    from vaeunet_amd.init import seeded_init_
    if args.overlap:
        E.OVERLAP_WGRAD = True
    for kv in args.tune:
        from vaeunet_amd import _lib
        key, val = kv.split("=")
        _lib.call("vu_gemm_set_tuning", int(key), int(val))  # raises if the key / value is refused
    for kv in args.engine_flag:
        name, val = kv.split("=")
        mod = E
        if "." in name:   # e.g. vae_engine.LATENT_VECTORS
            import importlib
            modname, name = name.rsplit(".", 1)
            mod = importlib.import_module("vaeunet_amd." + modname)
        if not hasattr(mod, name):
            raise SystemExit(f"bench: no engine switch {name}")
        old = getattr(mod, name)
        # keep the knob's type: a bool switch stays a bool, an integer knob
        # (e.g. kernels.WGRAD_SPLIT_CAP=4) an int, a float knob (e.g.
        # kernels._W3_SLAB_BPS=4.5e12) a float
        if isinstance(old, bool):
            new = bool(int(val))
        elif isinstance(old, int):
            new = int(val)
        elif isinstance(old, float):
            new = float(val)
        else:
            raise SystemExit(f"bench: engine knob {name} has type {type(old).__name__}; bool/int/float only")
        setattr(mod, name, new)
    from vaeunet_amd import _lib as _L
    xm = _L.query("vu_gemm_experiment_modes")
    if xm and not args.unsafe_experiment:
        raise SystemExit(f"bench: experiment modes active (mask {xm}): results are not valid; "
                         "pass --unsafe-experiment for a timing decomposition run")
    from vaeunet_amd.loss import CombinedLoss
    from vaeunet_amd import parallel

    vae = args.model == "vae"
    if vae:
        # BASELINE configs[2]: VAE-U-Net (ResNet34 encoder, latent 32, attention, latent
        # injection "all"), 1 class as train.py's resnet path (train.py:683,693)
        from vaeunet_amd import UNetResNet
        from vaeunet_amd.loss import kl_with_free_bits
        args.classes = 1
        model = seeded_init_(UNetResNet(3, 1, pretrained=False), 0).to(dev).to(memory_format=torch.channels_last)
    else:
        model = seeded_init_(UNet(3, args.classes), 0).to(dev).to(memory_format=torch.channels_last)
    model.train()
    reducer = parallel.attach(model) if world > 1 else None
    if args.torch_optim:
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5, foreach=True)
        clip = lambda ps, m: torch.nn.utils.clip_grad_norm_(ps, m, foreach=True)  # noqa: E731
    else:
        # same math as torch.optim.AdamW / clip_grad_norm_ (tests/test_gpu_optim.py),
        # one multi-tensor launch per phase
        from vaeunet_amd.optim import FusedAdamW, clip_grad_norm_ as clip
        opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    crit = CombinedLoss()
    x, t = synthetic(args.batch, args.size, args.classes, rank, dev)

    def step():
        if reducer is not None:
            reducer.prepare()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if vae:
                logits, mu, lv = model(x)
                loss = crit(logits, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
            else:
                logits = model(x)
                loss = crit(logits, t)
        loss.backward()
        if reducer is not None:
            reducer.finish()
        clip(model.parameters(), 1.0)
        opt.step()
        if reducer is not None:
            reducer.zero_grad()  # one fill per ~25 MB bucket (the .grad views stay bound)
        else:
            opt.zero_grad(set_to_none=True)
        return loss

    graphed = None
    # the step replays as one HIP graph with the fused optimizer at N = 1.  At
    # N > 1 the default is the eager step (the bucketed RCCL all-reduces still
    # overlap the backward): a captured multi-rank step has not been compared
    # with the eager one on a multi-GPU box yet, so it is opt-in ("--graph on",
    # experimental; gloo cannot be captured at all).  The UNet step is
    # GPU-bound, so eager costs it nothing measurable.
    capturable = not args.torch_optim and (world == 1 or dist.get_backend() == "nccl")
    use_graph = args.graph == "on" or (args.graph == "auto" and capturable and world == 1)
    if use_graph:
        if not capturable:
            raise SystemExit("--graph on needs the fused optimizer and (at N > 1) the nccl backend")
        from vaeunet_amd.graph import GraphedTrainStep

        def fwd_bwd():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                if vae:
                    logits, mu, lv = model(x)
                    loss = crit(logits, t) + 1e-3 * kl_with_free_bits(mu, lv, free_bits=1e-3)
                else:
                    loss = crit(model(x), t)
            loss.backward()
            return loss
        # warm-up steps run eagerly inside (weights, optimizer state), then one capture
        graphed = GraphedTrainStep(fwd_bwd, opt, max_norm=1.0, warmup=max(1, args.warmup), reducer=reducer)
    eager_step = step
    if graphed is not None:
        step = graphed.step
    for _ in range(0 if graphed else args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms = dt / args.steps * 1e3
    imgs = args.batch * world * args.steps / dt

    roof = None
    if not args.no_roofline:
        # live per-launch HIP-event timing of the 3x3 implicit-GEMM kernels over
        # 2 further steps (events on the launch stream, one pair per launch)
        K.TIMER = K.LaunchTimer(detail=args.layer_table, delay=args.timer_delay)
        for _ in range(2):
            eager_step()   # the same kernels, launched one by one so each can be bracketed
        if args.layer_table and rank == 0:
            # per-launch table of the second step (stderr): kind, shape, kernel, us, TFLOP/s
            recs = K.TIMER.per_launch()
            for tag, shape, kn, ms, fl in recs[len(recs) // 2:]:
                print(f"LAYER {tag:22s} {shape:40s} {kn:40s} {ms * 1e3:8.1f} us {fl / ms / 1e9:7.0f} TF",
                      file=sys.stderr)
        summ = K.TIMER.summary()
        K.TIMER = None
        fam = {k: v for k, v in summ.items() if k.startswith("conv3x3_") and "image" not in k}
        fl = sum(v[0] for v in fam.values())
        tm = sum(v[1] for v in fam.values())
        n = sum(v[2] for v in fam.values())
        knames = sorted(set().union(*(v[3] for v in fam.values()))) if fam else []
        achieved = fl / (tm * 1e-3) / 1e12 if tm > 0 else 0.0
        roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": pmc_traffic(args.model),
                "traffic_unit": f"HBM bytes per launch ({os.path.relpath(PMC_TRAFFIC[args.model], ROOT)})",
                "kernel": ("3x3 conv fwd/dgrad/wgrad (inc.0 excluded; the weight gradients' vu_slab_reduce "
                           "passes are not in the family): " + ", ".join(knames)),
                "launches_per_step": n // 2,
                "per_kind": {k: {"tflops": round(v[0] / (v[1] * 1e-3) / 1e12, 1),
                                 "ms_per_step": round(v[1] / 2, 3)} for k, v in sorted(summ.items())}}

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(args, dev)
    secondary = None
    if rank == 0 and world == 1 and not vae and not (args.no_secondary or args.no_cpu_baseline):
        secondary = {"config3_vae": vae_secondary(args)}

    if rank == 0:
        line = {"metric": METRIC, "value": round(imgs, 2),
                "unit": "images/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
                "config": {"workload": (f"UNetResNet(3,1) VAE train step (fwd+CombinedLoss+1e-3*KL+bwd"
                                        "+clip+AdamW), random-init weights" if vae else
                                        f"UNet(3,{args.classes}) train step (fwd+CombinedLoss+bwd"
                                        "+clip+AdamW), random-init weights"),
                           "image": f"3x{args.size}x{args.size}", "batch_per_gpu": args.batch,
                           "global_batch": args.batch * world, "parallelism": f"dp{world}",
                           "execution": ("hipgraph-replay" + (" (experimental at N>1)" if world > 1 else ""))
                           if graphed is not None else "eager",
                           "wgrad_side_stream": bool(E.OVERLAP_WGRAD),
                           "bn_bwd_reduce_in_dgrad_epilogue": bool(E.FUSE_BN_BWD_REDUCE)},
                "loss": round(float(loss.item()), 6),
                "roofline": roof, "cpu_baseline": cpu, "parity": parity}
        if secondary is not None:
            line["secondary"] = secondary
        if xm:
            line["experiment_modes"] = xm  # --unsafe-experiment: a timing decomposition, not a result
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
