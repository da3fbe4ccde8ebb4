"""Host-side wrappers: torch tensors (device memory) -> C-ABI calls.

Activations are torch tensors of logical shape [N, C, H, W] in
``channels_last`` memory format, i.e. NHWC in HBM; a channel slice of such a
tensor is still a valid NHWC view with a pixel stride (that is how the
channel concat of unet_parts.py:94 is addressed without a copy).  Every
function launches on the current HIP stream and never synchronises.
"""
import ctypes as C

import torch

from . import _lib
from ._lib import ptr, call, query, stream, VuGather, VuGemmFwd, VuGemmWgrad

CL = torch.channels_last


def dcode(dtype):
    if dtype == torch.bfloat16:
        return _lib.BF16
    if dtype == torch.float32:
        return _lib.F32
    raise TypeError(f"unsupported activation dtype {dtype}")


def empty_act(N, Cc, H, W, dtype, device):
    return torch.empty((N, Cc, H, W), dtype=dtype, device=device, memory_format=CL)


def zeros_act(N, Cc, H, W, dtype, device):
    y = torch.empty((N, Cc, H, W), dtype=dtype, device=device, memory_format=CL)
    zero(y)
    return y


def pstride(t):
    """Pixel stride (elements) of an NHWC view; validates the layout."""
    N, Cc, H, W = t.shape
    s = t.stride()
    if Cc > 1 and s[1] != 1:
        raise ValueError("activation must be channels_last (NHWC)")
    ps = s[3] if W > 1 else (s[2] if H > 1 else (s[0] if N > 1 else Cc))
    if W > 1 and H > 1 and s[2] != W * ps:
        raise ValueError("non-dense NHWC view")
    return ps


def gather(srcs, N, H, W, R=1, S=1, sy=1, sx=1, dy=1, dx=1, oy=0, ox=0, Hs=None, Ws=None):
    g = VuGather()
    if not 1 <= len(srcs) <= 3:
        raise ValueError("1..3 channel sources")
    cend = 0
    for i, t in enumerate(srcs):
        g.src[i] = t.data_ptr()
        g.stride[i] = pstride(t)
        cend += t.shape[1]
        g.cend[i] = cend
    for i in range(len(srcs), 3):
        g.src[i] = None
        g.stride[i] = 0
        g.cend[i] = cend
    g.nsrc, g.C = len(srcs), cend
    g.N, g.H, g.W = N, H, W
    g.Hs = srcs[0].shape[2] if Hs is None else Hs
    g.Ws = srcs[0].shape[3] if Ws is None else Ws
    g.R, g.S, g.sy, g.sx, g.dy, g.dx, g.oy, g.ox = R, S, sy, sx, dy, dx, oy, ox
    # the struct holds raw device pointers: keep the source tensors alive until
    # the launch that consumes this descriptor has been enqueued, otherwise
    # the caching allocator may hand their memory to the next allocation
    g._refs = list(srcs)
    return g


def gather3x3(srcs):
    N, _, H, W = srcs[0].shape
    return gather(srcs, N, H, W, R=3, S=3, oy=-1, ox=-1)


def gather1x1(srcs):
    N, _, H, W = srcs[0].shape
    return gather(srcs, N, H, W)


def gather_convT(du, N, h, w, py=0, px=0):
    """A[m=(n,i,j)][k=(a*2+b)*C + c] = du[n, 2i+a+py, 2j+b+px, c]."""
    return gather([du], N, h, w, R=2, S=2, sy=2, sx=2, oy=py, ox=px)


class LaunchTimer:
    """Optional per-launch HIP-event timing of the GEMM kernels (bench.py's
    roofline leg).  Events are recorded on the current stream — the stream
    the kernels are launched on — so they bracket exactly one launch."""

    def __init__(self, detail=False, delay=0):
        self.recs = []
        # delay > 0: a GPU sleep of ~delay x 3.4 us before each bracketed
        # launch (vu_gpu_delay), so host enqueue time between the start event
        # and the launch is not counted
        self.delay = delay
        self.detail = detail   # keep each launch's problem shape (tools: per-layer tables)
        self.shapes = []

    def per_launch(self):
        """[(tag, shape, kernel, ms, flops)] in launch order (detail=True)."""
        torch.cuda.synchronize()
        return [(r[0], sh, r[4], r[2].elapsed_time(r[3]), r[1]) for r, sh in zip(self.recs, self.shapes)]

    def summary(self):
        """tag -> [flops, ms, launches, {kernel names}]"""
        torch.cuda.synchronize()
        out = {}
        for tag, flops, s, e, kname in self.recs:
            ms = s.elapsed_time(e)
            d = out.setdefault(tag, [0, 0.0, 0, set()])
            d[0] += flops
            d[1] += ms
            d[2] += 1
            if kname:
                d[3].add(kname)
        return out


TIMER = None

# Observation point for the production-size parity tests
# (tests/gemm_audit.py): when set, every GEMM launch goes through
# AUDIT.gemm_fwd / AUDIT.gemm_wgrad, which run the launch and then compare its
# output element by element with the contraction its descriptor defines.  The
# launch itself is the same call either way (same dispatch, same kernel).
AUDIT = None


# kernel ids of vu_gemm_fwd_kernel / vu_gemm_wgrad_tile -> the __global__
# functions the launch runs (the roofline line names what it timed)
FWD_KERNELS = {1: "gemm_fwd_kernel", 2: "gemm_fwd_v2_kernel", 3: "conv3x3_halo_kernel", 4: "conv3x3_pp_kernel",
               5: "gemm_fwd_v5_kernel", 6: "conv3x3_c64_kernel", 7: "conv3x3_sg_kernel", 8: "gemm_stream_kernel",
               9: "conv3x3_image_kernel", 10: "conv_stem_kernel", 12: "gemm_fwd_v2_kernel(small-grid)",
               13: "gemm_fwd_v2_kernel(tail)"}
WGRAD_KERNELS = {1: "gemm_wgrad_kernel", 2: "gemm_wgrad_v2_kernel", 3: "wgrad3x3_halo_kernel"}


def _timed(tag, flops, fn, kname=None, shape=None):
    if TIMER is None:
        return fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    if TIMER.delay:
        call("vu_gpu_delay", TIMER.delay, stream())
    s.record()
    r = fn()
    e.record()
    TIMER.recs.append((tag, flops, s, e, kname() if callable(kname) else kname))
    if TIMER.detail:
        TIMER.shapes.append(shape() if callable(shape) else shape)
    return r


def _gemm_tag(g, kind):
    if g.R == 3 and g.C >= 16:
        return f"conv3x3_{kind}"
    if g.R == 3:
        return f"conv3x3_image_{kind}"
    if g.R == 2:
        return f"convT_{kind}"
    return f"gemm1x1_{kind}"


class Stats:
    """Per-row-tile BatchNorm partials produced by a GEMM epilogue."""

    def __init__(self, psum, pm2, tiles, tile_rows, rows):
        self.psum, self.pm2, self.tiles, self.tile_rows, self.rows = psum, pm2, tiles, tile_rows, rows
        self.minmax = None  # (pmin, pmax) where an fp8 conv epilogue emitted them


class BnbPart:
    """BatchNorm-backward partial sums [nblk][2][C] a GEMM epilogue wrote for
    the BN over ``x`` that its output feeds (VuGemmFwd.bnb_part)."""

    def __init__(self, part, nblk, x):
        self.part, self.nblk, self.x = part, nblk, x


def gemm_fwd(g, wmat, ncol, out, dtype, out_coff=0, bias=None, stats=False, accumulate=False,
             convT=None, kind="fwd", strided=None, bnb=None, flops=None, relu=False, zbias=None):
    """out[m][j] = sum_k A[m][k] wmat[j][k] (+bias).  convT=(oH,oW,opy,opx,cout) selects
    the pixel-shuffle epilogue, strided=(oH,oW,opy,opx) the stride-2 sub-lattice one.
    bnb=(x, coef, relu): also emit the BatchNorm-backward partials of the output
    for the train/eval BN over x (coef = bn_finalize's scale, shift, mean,
    invstd) when the selected kernel can (returns a BnbPart then, else None).
    flops: the algorithmic work the roofline accounting credits this launch
    with (default 2*M*N*K of the GEMM as launched).  relu: epilogue ReLU on
    acc + bias (an eval-mode BatchNorm folded into wmat / bias).  zbias: the
    [N][9][ncol] fp32 per-sample border-class bias table of the latent
    shortcut (VuGemmFwd.zbias, vu_zbias_fwd).  Returns Stats if requested."""
    a = VuGemmFwd()
    a.a = g
    a.b = wmat.data_ptr()
    a.ldb = wmat.shape[-1] if wmat.dim() == 2 else wmat.stride(0)
    a.ncol = ncol
    a.out = out.data_ptr()
    a.out_stride = pstride(out)
    a.out_coff = out_coff
    if convT is not None:
        a.out_mode = 1
        a.oH, a.oW, a.opy, a.opx, a.cout = convT
    elif strided is not None:
        a.out_mode = 2
        a.oH, a.oW, a.opy, a.opx = strided
        a.cout = ncol
    else:
        a.out_mode = 0
    a.bias = bias.data_ptr() if bias is not None else None
    a.zbias = zbias.data_ptr() if zbias is not None else None
    a.accumulate = 1 if accumulate else 0
    a.relu = 1 if relu else 0
    st = None
    if stats:
        rows = g.N * g.H * g.W
        # the row tile depends on whether statistics are requested (kernel
        # choice): query with the statistics pointers set (placeholders)
        a.stat_sum = a.stat_m2 = 1
        bm = query("vu_gemm_fwd_row_tile", C.byref(a), dtype)
        tiles = (rows + bm - 1) // bm
        psum = torch.empty((tiles, ncol), dtype=torch.float32, device=out.device)
        pm2 = torch.empty_like(psum)
        a.stat_sum, a.stat_m2 = psum.data_ptr(), pm2.data_ptr()
        st = Stats(psum, pm2, tiles, bm, rows)
    else:
        a.stat_sum = a.stat_m2 = None
    a.ksplit = 0
    a.workspace = None
    part = None
    if bnb is not None and dtype == _lib.BF16 and not accumulate and out_coff == 0 and bias is None \
            and out.shape[1] == ncol:
        bx, bcoef, brelu = bnb
        a.bnb_xstride = pstride(bx)
        tile = query("vu_gemm_fwd_bnb_tile", C.byref(a), dtype)
        rows = g.N * g.H * g.W
        if tile > 0 and rows % tile == 0:
            nblk = rows // tile
            pbuf = torch.empty((nblk, 2, ncol), dtype=torch.float32, device=out.device)
            a.bnb_x = bx.data_ptr()
            a.bnb_scale, a.bnb_shift = bcoef[0].data_ptr(), bcoef[1].data_ptr()
            a.bnb_mean, a.bnb_invstd = bcoef[2].data_ptr(), bcoef[3].data_ptr()
            a.bnb_part = pbuf.data_ptr()
            a.bnb_relu = 1 if brelu else 0
            part = BnbPart(pbuf, nblk, bx)
    ws = None
    if dtype == _lib.BF16:
        # any bf16 shape may be given split-K by the C-side selector (it returns 0
        # when none is needed), not only the 3x3 ones
        nb = query("vu_gemm_fwd_workspace_bytes", C.byref(a), dtype)
        if nb > 0:
            ws = torch.empty(nb // 4, dtype=torch.float32, device=out.device)
            a.workspace = ws.data_ptr()
    M = g.N * g.H * g.W
    launch = lambda: call("vu_gemm_fwd", C.byref(a), dtype, stream())  # noqa: E731
    if AUDIT is not None:
        AUDIT.gemm_fwd(a, dtype, g, wmat, out, bias, st, launch, zbias=zbias)
    else:
        def kname():
            k = FWD_KERNELS.get(query("vu_gemm_fwd_kernel", C.byref(a), dtype), "?")
            return k + "+splitk_finish_kernel" if ws is not None else k
        _timed(_gemm_tag(g, kind), 2 * M * ncol * g.R * g.S * g.C if flops is None else flops, launch, kname,
               lambda: f"{g.N}x{g.H}x{g.W} C{g.C}->{ncol}" + (" stats" if st is not None else "")
               + (" bnb" if bnb is not None else ""))
    if bnb is not None:
        return part
    return st


SPLIT_PIX = 4096
SPLIT_MAX = 1024
WGRAD_SPLIT_CAP = 0   # A/B runs (tools/enc_bench.py --wsplit): cap on the split-K ways, 0 = none
# Round 5: the halo weight gradient's split count from a time model that
# prices the fp32 slabs (the fill-whole-waves rule gave e.g. the UNetResNet
# 128^2 decoder conv1 256 splits = 377 MB of slabs written and re-read).
WGRAD_SLAB_MODEL = True
_W3_BLOCK_US = 3.0       # per-block fixed cost (first tile latency, slab write issue)
_W3_CU_FLOPS = 4.5e12    # per-block (one CU) weight-gradient rate, measured 4.1-5.2 TFLOP/s
_W3_SLAB_BPS = 5.0e12    # slab write + re-read (8 B per element and split) through L2 / MALL


def _halo_splits(M, ni, nj, tiles, slots, smax, gran):
    """argmin over s of waves(s) * (c0 + 2 (M / s) BI BJ / R) + s ni nj 8 / Bw
    (ties: fewer splits); the per-block term uses the tile's share of ni*nj."""
    per_tile = 2.0 * ni * nj / max(tiles, 1)
    best = None
    for s in range(1, smax + 1):
        waves = -(-tiles * s // slots)
        if waves > 16:
            break
        rows = -(-M // s)
        rows = -(-rows // gran) * gran
        t = waves * (_W3_BLOCK_US * 1e-6 + per_tile * rows / _W3_CU_FLOPS) + s * ni * nj * 8.0 / _W3_SLAB_BPS
        if best is None or t < best[0] - 1e-12:
            best = (t, s)
    return best[1]


def gemm_wgrad(gp, gq, ni, nj, grad, layout, dtype, accumulate, cvalid=None):
    """grad[i*s_i + (j//Cq)*s_tap + (j%Cq)*s_c] (+)= sum_m P[m][i] Q[m][j]."""
    M = gp.N * gp.H * gp.W
    w = VuGemmWgrad()
    w.p, w.q, w.ni, w.nj = gp, gq, ni, nj
    bi, bj = C.c_int(0), C.c_int(0)
    kind = query("vu_gemm_wgrad_tile", C.byref(w), dtype, C.byref(bi), C.byref(bj))
    tiles = ((ni + bi.value - 1) // bi.value) * ((nj + bj.value - 1) // bj.value)
    # split-K over pixels: pick the split count whose block count fills whole
    # waves of resident blocks best (v2/v3: 1 block/CU, v1: 2 blocks/CU); the
    # halo kernel (v3) splits in whole 128-pixel tiles, the others in 64 rows
    slots = 256 if kind >= 2 else 512
    gran = 128 if kind == 3 else 64
    steps = (M + gran - 1) // gran
    smax = max(1, min(256, steps // 4))
    best = (-1.0, 1)
    for s in range(1, smax + 1):
        blocks = tiles * s
        waves = -(-blocks // slots)
        if waves > 8:
            break
        eff = blocks / (waves * slots)
        if eff > best[0] + 1e-9:
            best = (eff, s)
    splits = best[1]
    if kind == 3 and WGRAD_SLAB_MODEL:
        splits = _halo_splits(M, ni, nj, tiles, slots, smax, gran)
    if WGRAD_SPLIT_CAP > 0:
        splits = min(splits, WGRAD_SPLIT_CAP)
    # v2 (1x1 / ConvT): very long pixel ranges per block (> SPLIT_PIX) expose
    # the ring's DMA latency on every step, so a second wave of blocks measured
    # faster (512^2 attention W_x gradient: 256 splits 158 us, 512 splits
    # 112 us); the halo kernel (v3) measured slower with more splits
    while kind == 2 and M // splits > SPLIT_PIX and tiles * splits * 2 <= 8 * slots and splits * 2 <= SPLIT_MAX:
        splits *= 2
    mps = ((-(-M // splits)) + gran - 1) // gran * gran
    splits = -(-M // mps)
    slab = torch.empty((splits, ni, nj), dtype=torch.float32, device=grad.device)
    w.splits, w.m_per_split = splits, mps
    w.out = slab.data_ptr()
    s_i, s_tap, s_c = layout
    cv = gq.C if cvalid is None else cvalid

    def reduce():
        call("vu_slab_reduce", ptr(slab), splits, ni, nj, gq.C, cv, s_i, s_tap, s_c, ptr(grad),
             1 if accumulate else 0, stream())
    if AUDIT is not None:
        def launch():
            call("vu_gemm_wgrad", C.byref(w), dtype, stream())
            reduce()
        AUDIT.gemm_wgrad(w, dtype, kind, gp, gq, ni, nj, grad, layout, accumulate, cv, launch)
        return slab
    _timed(_gemm_tag(gq, "wgrad"), 2 * M * ni * nj,
           lambda: call("vu_gemm_wgrad", C.byref(w), dtype, stream()), WGRAD_KERNELS.get(kind, "?"),
           lambda: f"{gq.N}x{gq.H}x{gq.W} {ni}x{nj} splits {splits}")
    reduce()
    return slab


_PBATCH = None  # job list while a permute_batch() context is open


def permute4(src, base, strides, dims, d3v, dtype, out=None):
    """out[i0][i1][i2][i3] = src[base + sum i*s] (0 for i3 >= d3v), in the
    storage dtype (``out``: a contiguous destination, else a new tensor).
    Inside permute_batch() the launch is deferred and merged."""
    if out is None:
        out = torch.empty(dims, dtype=torch.bfloat16 if dtype == _lib.BF16 else torch.float32,
                          device=src.device)
    if _PBATCH is not None:
        _PBATCH.append((src, base, strides, dims, d3v, out, dtype))
        return out
    call("vu_permute4", ptr(src), base, *strides, *dims, d3v, ptr(out), dtype, stream())
    return out


class permute_batch:
    """Context: every permute4 issued inside becomes one vu_permute4_batch
    launch at exit (the outputs are filled before any later launch on the
    stream reads them)."""

    def __enter__(self):
        global _PBATCH
        self.outer = _PBATCH is not None
        if not self.outer:
            _PBATCH = []
        return self

    def __exit__(self, *exc):
        global _PBATCH
        if self.outer:
            return False
        jobs, _PBATCH = _PBATCH, None
        if not jobs or exc[0] is not None:
            return False
        table, ntap, ctap, crest = job_table(jobs)
        permute_launch(table, len(jobs), ntap, ctap, crest)
        return False


class record_permutes:
    """Context collecting the permute4 jobs issued inside WITHOUT launching
    them (``.jobs``: (src, base, strides, dims, d3v, out, dtype) tuples)."""

    def __enter__(self):
        global _PBATCH
        if _PBATCH is not None:
            raise RuntimeError("record_permutes inside an open permute_batch")
        _PBATCH = self.jobs = []
        return self

    def __exit__(self, *exc):
        global _PBATCH
        _PBATCH = None
        return False


def perm_mode(strides, dims, d3v=None):
    """vu_permute4_batch job mode: 3 = stream (output-fast dim is the
    input-fast one), 5 = the same with the input row-major in the output's
    dim order and no padding (a converting copy: the forward image of a
    channels_last weight), 0-2 = 32x32 tile transpose between that dim and dim 3,
    4 = 3x3 or 2x2 weight image (dims 1, 2 merge into 9 or 4 taps forming one
    contiguous input run with dim 0 or dim 3): 32 x T x 32 tile transpose."""
    # input-fastest dim (among those of extent > 1); a transpose if not dim 3
    cand = [k for k in range(4) if dims[k] > 1] or [3]
    q = min(cand, key=lambda k: (abs(strides[k]), k != cand[-1]))
    if q == cand[-1] or dims[3] == 1:
        # output-fast == input-fast: stream; a plain converting copy when the
        # input is row-major in the output's dim order (no padding)
        if strides[3] == 1 and strides[2] == dims[3] and strides[1] == dims[2] * dims[3] \
                and strides[0] == dims[1] * dims[2] * dims[3] and d3v == dims[3]:
            return 5
        return 3
    T = dims[1] * dims[2]
    if (q in (1, 2) and dims[1] > 1 and dims[2] > 1 and T in (4, 9) and strides[1] == dims[2] * strides[2]
            and abs(strides[2]) == 1 and T * abs(strides[2]) in (abs(strides[0]), abs(strides[3]))):
        return 4
    return q


def job_table(jobs):
    """Device VuPermJob table of permute4 jobs for vu_permute4_batch2 ->
    (table tensor, ntap, tap blocks, other blocks): the 3x3 / 2x2 weight
    images (mode 4) first, each group with its own block prefix."""
    chunk = query("vu_permute4_chunk")
    tt = query("vu_permute4_tile")
    modes = [perm_mode(j[2], j[3], j[4]) for j in jobs]
    order = [i for i in range(len(jobs)) if modes[i] == 4] + [i for i in range(len(jobs)) if modes[i] != 4]
    ntap = sum(1 for m in modes if m == 4)
    arr = (_lib.VuPermJob * len(jobs))()
    c0, ctap = 0, 0
    for k, i in enumerate(order):
        src, base, strides, dims, d3v, out, dtype = jobs[i]
        q = modes[i]
        if k == ntap:
            ctap, c0 = c0, 0          # the other jobs' prefix restarts at 0
        e = arr[k]
        e.inp = src.data_ptr()
        e.base = base
        e.s0, e.s1, e.s2, e.s3 = strides
        e.d0, e.d1, e.d2, e.d3 = dims
        e.d3v, e.dtype = d3v, dtype
        e.out = out.data_ptr()
        e.chunk0 = c0
        e.q = q
        if q in (3, 5):
            c0 += -(-out.numel() // chunk)
        elif q == 4:
            c0 += (-(-dims[0] // 32)) * (-(-dims[3] // 32))
        else:
            a, cc = [k2 for k2 in range(3) if k2 != q]
            c0 += dims[a] * dims[cc] * (-(-dims[q] // tt)) * (-(-dims[3] // tt))
    if ntap == len(jobs):
        ctap, c0 = c0, 0
    dev = jobs[0][5].device
    host = torch.frombuffer(bytearray(arr), dtype=torch.uint8).pin_memory()
    return host.to(dev, non_blocking=True), ntap, ctap, c0


def permute_launch(table, njobs, ntap, ctap, crest):
    call("vu_permute4_batch2", ptr(table), njobs, ntap, ctap, crest, stream())


def bn_finalize(st, C_, gamma, beta, rmean, rvar, nbt, momentum, eps):
    dev = st.psum.device
    coef = torch.empty((4, C_), dtype=torch.float32, device=dev)
    ws = torch.empty(query("vu_bn_finalize_workspace_bytes", st.tiles, C_) // 4 + 1,
                     dtype=torch.float32, device=dev)
    call("vu_bn_finalize", ptr(st.psum), ptr(st.pm2), st.tiles, st.tile_rows, st.rows, C_,
         ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), momentum, eps,
         ptr(coef[0]), ptr(coef[1]), ptr(coef[2]), ptr(coef[3]), ptr(nbt), ptr(ws), stream())
    return coef  # rows: scale, shift, mean, invstd


def bn_forward_fused(st, C_, gamma, beta, rmean, rvar, nbt, momentum, eps, y, out, relu, dtype,
                     res=None, rcoef=None):
    """Train-mode BatchNorm finalize + apply [+ residual] [+ ReLU] as ONE launch
    (vu_bn_fwd_fused) when the tensor is small enough; returns coef (rows:
    scale, shift, mean, invstd), or None when not applicable (the caller then
    runs bn_finalize + the apply)."""
    rs = pstride(res) if res is not None else 0
    if not query("vu_bn_fwd_fused_supported", st.tiles, C_, pstride(y), rs, pstride(out)):
        return None
    coef = torch.empty((4, C_), dtype=torch.float32, device=y.device)
    call("vu_bn_fwd_fused", ptr(st.psum), ptr(st.pm2), st.tiles, st.tile_rows, st.rows, C_,
         ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), ptr(nbt), momentum, eps, ptr(coef),
         ptr(y), pstride(y), ptr(res), rs, ptr(rcoef[0]) if rcoef is not None else None,
         ptr(rcoef[1]) if rcoef is not None else None, ptr(out), pstride(out), 1 if relu else 0, dtype,
         stream())
    return coef


def bn_eval(C_, gamma, beta, rmean, rvar, eps):
    """Eval-mode coefficients; rows: scale, shift, running mean, 1/sqrt(running var + eps)."""
    coef = torch.empty((4, C_), dtype=torch.float32, device=rmean.device)
    call("vu_bn_eval_coeffs", ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), eps, C_,
         ptr(coef[0]), ptr(coef[1]), ptr(coef[2]), ptr(coef[3]), stream())
    return coef


def bn_apply(x, y, coef, relu, dtype):
    N, Cc, H, W = x.shape
    call("vu_bn_apply", ptr(x), pstride(x), ptr(y), pstride(y), N * H * W, Cc,
         ptr(coef[0]), ptr(coef[1]), 1 if relu else 0, dtype, stream())
    return y


class ZbiasRegions:
    """A latent-shortcut conv1's region-partial buffer (vu_zbias_rs_floats
    floats); ``ready`` once the BatchNorm backward apply that wrote conv1's dy
    also wrote the partials (vu_bn_bwd_apply_zrs)."""

    def __init__(self, rs):
        self.rs, self.ready = rs, False


def _apply(dy, x, coef, k, relu, dx, dtype, zrs):
    """The BN backward apply pass; with zrs (a ZbiasRegions) the fused variant
    that also takes the shortcut's region partials of dx, when it serves."""
    N, Cc, H, W = x.shape
    if zrs is not None and query("vu_bn_bwd_apply_zrs_ok", H, W, Cc, pstride(dy), pstride(x), pstride(dx)):
        call("vu_bn_bwd_apply_zrs", ptr(dy), pstride(dy), ptr(x), pstride(x), N, H, W, Cc, ptr(coef[0]),
             ptr(coef[1]), ptr(coef[2]), ptr(k), 1 if relu else 0, ptr(dx), pstride(dx), ptr(zrs.rs), dtype,
             stream())
        zrs.ready = True
        return
    call("vu_bn_bwd_apply", ptr(dy), pstride(dy), ptr(x), pstride(x), N * H * W, Cc, ptr(coef[0]),
         ptr(coef[1]), ptr(coef[2]), ptr(k), 1 if relu else 0, ptr(dx), pstride(dx), dtype,
         stream())


def bn_backward(dy, x, coef, gamma, relu, dgamma, dbeta, acc, dx, dtype, train=True, fused=True, zrs=None):
    """dx = BN(+ReLU) backward; writes/accumulates dgamma, dbeta.  train=False:
    the statistics are constants (eval mode).  fused: small tensors take the
    two-launch path (vu_bn_bwd_fused) instead of reduce + finish + apply.
    zrs: a ZbiasRegions to fill from the apply pass (the reduce + apply path
    only)."""
    N, Cc, H, W = x.shape
    P = N * H * W
    dev = x.device
    ws = torch.empty(query("vu_reduce_workspace_bytes", P, Cc) // 4 + 1, dtype=torch.float32,
                     device=dev)
    # (the small-tensor two-launch path keeps its own, more accurate fp64
    # reduction: a zrs is then left unfilled and the region pass runs)
    if fused and query("vu_bn_bwd_fused_supported", P, Cc, pstride(dy), pstride(x), pstride(dx)):
        call("vu_bn_bwd_fused", ptr(dy), pstride(dy), ptr(x), pstride(x), P, Cc, ptr(coef[0]), ptr(coef[1]),
             ptr(coef[2]), ptr(coef[3]), ptr(gamma), 1 if relu else 0, 1 if train else 0, ptr(dgamma), ptr(dbeta),
             1 if acc else 0, ptr(dx), pstride(dx), ptr(ws), dtype, stream())
        return dx
    k = torch.empty((3, Cc), dtype=torch.float32, device=dev)
    call("vu_bn_bwd_reduce", ptr(dy), pstride(dy), ptr(x), pstride(x), P, Cc, ptr(coef[0]),
         ptr(coef[1]), ptr(coef[2]), ptr(coef[3]), ptr(gamma), 1 if relu else 0,
         1 if train else 0, ptr(dgamma), ptr(dbeta), 1 if acc else 0, ptr(k), ptr(ws), dtype,
         stream())
    _apply(dy, x, coef, k, relu, dx, dtype, zrs)
    return dx


def bn_backward_pool(dp, add, y, coef, gamma, relu, dgamma, dbeta, acc, dx, dtype, train=True):
    """BatchNorm(+ReLU) backward through the 2x2 max-pool that follows it
    (vu_bn_bwd_pool): dp the pooled output's gradient, add the skip gradient
    of the activation (or None); dx = the gradient of y (the BN input)."""
    N, Cc, H, W = y.shape
    P = N * H * W
    ws = workspace_f32(query("vu_reduce_workspace_bytes", P, Cc), y.device)
    k = torch.empty((3, Cc), dtype=torch.float32, device=y.device)
    call("vu_bn_bwd_pool", ptr(y), pstride(y), ptr(dp), pstride(dp), ptr(add), pstride(add) if add is not None else 0,
         N, H, W, Cc, ptr(coef[0]), ptr(coef[1]), ptr(coef[2]), ptr(coef[3]), ptr(gamma), 1 if relu else 0,
         1 if train else 0, ptr(dgamma), ptr(dbeta), 1 if acc else 0, ptr(k), ptr(ws), ptr(dx), pstride(dx),
         dtype, stream())
    return dx


def bn_backward_part(part, dy, x, coef, gamma, relu, dgamma, dbeta, acc, dx, dtype, train=True, zrs=None):
    """bn_backward with the first reduction stage done by the producing GEMM's
    epilogue (a BnbPart): the fp64 finish, then the apply pass (zrs: as
    bn_backward)."""
    N, Cc, H, W = x.shape
    P = N * H * W
    k = torch.empty((3, Cc), dtype=torch.float32, device=x.device)
    nb = query("vu_bn_bwd_finish_workspace_bytes", part.nblk, Cc)
    ws = workspace_f32(nb, x.device) if nb > 0 else None
    call("vu_bn_bwd_finish", ptr(part.part), part.nblk, P, Cc, ptr(gamma), ptr(coef[3]), 1 if train else 0,
         ptr(dgamma), ptr(dbeta), 1 if acc else 0, ptr(k), ptr(ws), stream())
    _apply(dy, x, coef, k, relu, dx, dtype, zrs)
    return dx


def bn_backward_finish(part, x, coef, gamma, dgamma, dbeta, acc, train=True):
    """The fp64 finish of a BnbPart: dgamma / dbeta written (or added) and the
    apply coefficients k (3 x C) returned -- bn_backward_part without its apply."""
    N, Cc, H, W = x.shape
    k = torch.empty((3, Cc), dtype=torch.float32, device=x.device)
    nb = query("vu_bn_bwd_finish_workspace_bytes", part.nblk, Cc)
    ws = workspace_f32(nb, x.device) if nb > 0 else None
    call("vu_bn_bwd_finish", ptr(part.part), part.nblk, N * H * W, Cc, ptr(gamma), ptr(coef[3]), 1 if train else 0,
         ptr(dgamma), ptr(dbeta), 1 if acc else 0, ptr(k), ptr(ws), stream())
    return k


def bn_backward_apply2(dy, x1, coef1, k1, dx1, x2, coef2, k2, dx2, dtype):
    """Backward apply (no ReLU) of two BatchNorms fed by the same dy: dy read
    once (vu_bn_bwd_apply2).  False when the layout is not served."""
    N, Cc, H, W = x1.shape
    if not query("vu_bn_bwd_apply2_ok", Cc, pstride(dy), pstride(x1), pstride(x2), pstride(dx1), pstride(dx2)):
        return False
    call("vu_bn_bwd_apply2", ptr(dy), pstride(dy), ptr(x1), pstride(x1), ptr(x2), pstride(x2), N * H * W, Cc,
         ptr(coef1[2]), ptr(k1), ptr(coef2[2]), ptr(k2), ptr(dx1), pstride(dx1), ptr(dx2), pstride(dx2), dtype,
         stream())
    return True


def chan_sum(x, out, acc, dtype, window=None):
    N, Cc, H, W = x.shape
    y0, x0, Hr, Wr = window if window is not None else (0, 0, H, W)
    ws = torch.empty(query("vu_reduce_workspace_bytes", N * Hr * Wr, Cc) // 4 + 1,
                     dtype=torch.float32, device=x.device)
    call("vu_chan_sum", ptr(x), pstride(x), N, H, W, y0, x0, Hr, Wr, Cc, ptr(out),
         1 if acc else 0, ptr(ws), dtype, stream())


def zero(y):
    """Zero an NHWC tensor or channel slice (HIP fill, no ATen launch)."""
    N, Cc, H, W = y.shape
    call("vu_zero", ptr(y), pstride(y), N * H * W, Cc, dcode(y.dtype), stream())


def copy(x, y, accumulate=False):
    N, Cc, H, W = x.shape
    call("vu_copy", ptr(x), pstride(x), dcode(x.dtype), ptr(y), pstride(y), dcode(y.dtype),
         N * H * W, Cc, 1 if accumulate else 0, stream())


def input_pack(x, Cp, dtype):
    N, Cc, H, W = x.shape
    if x.dtype != torch.float32:
        x = x.float()
    y = empty_act(N, Cp, H, W, torch.bfloat16 if dtype == _lib.BF16 else torch.float32, x.device)
    s = x.stride()
    call("vu_input_pack", ptr(x), s[0], s[1], s[2], s[3], N, Cc, H, W, Cp, ptr(y), dtype, stream())
    return y


def maxpool_fwd(x, dtype):
    N, Cc, H, W = x.shape
    y = empty_act(N, Cc, H // 2, W // 2, x.dtype, x.device)
    call("vu_maxpool2_fwd", ptr(x), pstride(x), N, H, W, Cc, ptr(y), pstride(y), dtype, stream())
    return y


def maxpool_bwd(x, dy, dx, add, dtype):
    N, Cc, H, W = x.shape
    call("vu_maxpool2_bwd", ptr(x), pstride(x), ptr(dy), pstride(dy), N, H, W, Cc, ptr(dx),
         pstride(dx), ptr(add), pstride(add) if add is not None else 0, dtype, stream())
    return dx


def pool_fusable(y):
    """MaxPool2d(2) + BatchNorm fusion applies (vu_bn_apply_maxpool2): even
    H, W; C = 8 * 2^k <= 2048; NHWC strides."""
    N, Cc, H, W = y.shape
    v = Cc // 8
    return (H % 2 == 0 and W % 2 == 0 and Cc % 8 == 0 and 0 < v <= 256 and v & (v - 1) == 0
            and pstride(y) % 8 == 0)


def bn_apply_maxpool(y, a, pool, coef, relu, dtype):
    """a = relu(BN(y)) and pool = maxpool2(a) in one pass."""
    N, Cc, H, W = y.shape
    call("vu_bn_apply_maxpool2", ptr(y), pstride(y), ptr(a), pstride(a), ptr(pool), pstride(pool), N, H, W, Cc,
         ptr(coef[0]), ptr(coef[1]), 1 if relu else 0, dtype, stream())
    return a, pool


def upsample_fwd(x, out, Ho, Wo, py, px, dtype):
    N, Cc, Hi, Wi = x.shape
    Hp, Wp = out.shape[2], out.shape[3]
    call("vu_upsample_fwd", ptr(x), pstride(x), N, Hi, Wi, Cc, ptr(out), pstride(out), Ho, Wo,
         Hp, Wp, py, px, dtype, stream())
    return out


def upsample_bwd(dy, dx, Ho, Wo, py, px, accumulate, dtype):
    N, Cc, Hi, Wi = dx.shape
    Hp, Wp = dy.shape[2], dy.shape[3]
    call("vu_upsample_bwd", ptr(dy), pstride(dy), N, Hi, Wi, Cc, ptr(dx), pstride(dx), Ho, Wo,
         Hp, Wp, py, px, 1 if accumulate else 0, dtype, stream())
    return dx


def workspace_f32(nbytes, device):
    return torch.empty(max(1, nbytes // 4 + 1), dtype=torch.float32, device=device)
