"""Kernel-level parity: each HIP kernel vs a plain PyTorch fp32 CPU reference
of the same op (floating-point kernels, cdna guide: torch fp32 reference).

fp32 storage mode must match to fp32 rounding (MFMA f32 = exact fma chain,
different summation order); bf16 storage mode within bf16 tolerances.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
CL = torch.channels_last


def _k():
    from vaeunet_amd import kernels as K, engine as E
    return K, E


def _dt(mode):
    return torch.float32 if mode == "f32" else torch.bfloat16


def _code(mode):
    return 0 if mode == "f32" else 1


def _tol(mode):
    return (2e-5, 2e-5) if mode == "f32" else (2e-2, 2e-2)


def _act(t, mode):
    return t.to(DEV, _dt(mode)).contiguous(memory_format=CL)


U_STORE = {"f32": 2.0 ** -24, "bf16": 2.0 ** -8}
C_SUM = 1e-5


def _close(got, ref, mode, scale_floor=1e-3, what="", sabs=None, acc=None, u=None):
    """GEMM kernels (``sabs`` given: sum_k |a_k||b_k| of every output element,
    the same reference op on |operands|): PER-ELEMENT bound

      |got - ref| <= u * max(|ref|, |got|)  [+ u * |acc|]  + C_SUM * sabs + 1e-7 * max |ref|

    u = half an ulp of the storage dtype (2^-8 bf16, 2^-24 fp32; ``u``
    overrides it for fp32 weight gradients), acc = the rounded new term of an
    accumulating launch (rounded once more when added), C_SUM the fp32
    summation-order noise of the two sides' accumulations.  Other kernels: a
    max-relative tolerance."""
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    diff = (got - ref).abs()
    if sabs is not None:
        uu = U_STORE[mode] if u is None else u
        g64, r64 = got.double(), ref.double()
        bound = uu * torch.maximum(r64.abs(), g64.abs()) + C_SUM * sabs.detach().double().cpu() \
            + 1e-7 * float(r64.abs().max())
        if acc is not None:
            bound += uu * acc.detach().double().cpu().abs()
        ratio = (g64 - r64).abs() / bound
        i = int(ratio.flatten().argmax())
        assert float(ratio.max()) <= 1.0, (
            f"{what}: per-element bound exceeded at flat index {i} (got {got.flatten()[i].item():.6g}, "
            f"ref {ref.flatten()[i].item():.6g}, bound {bound.flatten()[i].item():.3e}); "
            f"{int((ratio > 1).sum())} elements off")
        return
    err = diff.max().item()
    scale = max(ref.abs().max().item(), scale_floor)
    rtol = 2e-5 if mode == "f32" else 1.5e-2
    i = int(diff.flatten().argmax())
    assert err <= rtol * scale, (f"{what}: max err {err:.3e} vs scale {scale:.3e} at flat index {i} "
                                 f"(got {got.flatten()[i].item():.6g}, ref {ref.flatten()[i].item():.6g}, "
                                 f"{int((diff > rtol * scale).sum())} elements off)")


CONV_CASES = [
    # (N, [cin per source], H, W, cout)
    (2, [64], 16, 16, 64),
    (2, [8], 9, 7, 16),
    (2, [32, 32], 12, 10, 48),
    (1, [128], 32, 32, 128),
    (8, [64], 128, 128, 64),      # BM=128, BN=64 path
    (4, [64, 64], 128, 128, 128),  # BM=128, BN=128 path, two sources
    (2, [24, 8, 16], 6, 6, 40),    # three sources, ragged
    (2, [64, 128], 16, 48, 96),    # bf16 halo kernel: 16x16 tiles, 3 chunks, column tail
    (2, [128], 8, 64, 192),        # bf16 halo wgrad: 128-row co tiles with a 64-row tail
    (8, [256], 32, 32, 256),       # small grid: 64-row co tiles (ResNet34 layer3 shape)
    (4, [512], 16, 16, 512),       # 16-pixel-wide halo wgrad tiles (layer4 shape)
]


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv3x3_fwd_dgrad_wgrad(mode, case):
    K, E = _k()
    N, cins, H, W, co = case
    g = torch.Generator().manual_seed(1)
    xs = [torch.randn(N, c, H, W, generator=g) for c in cins]
    cin = sum(cins)
    w = torch.randn(co, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    # round inputs to the storage dtype so the reference sees the same values
    xs = [x.to(_dt(mode)).float() for x in xs]
    wq = w.to(_dt(mode)).float()
    ref = F.conv2d(torch.cat(xs, 1), wq, padding=1)
    d = _code(mode)
    srcs = [_act(x, mode) for x in xs]
    wdev = w.to(DEV)
    out = K.empty_act(N, co, H, W, _dt(mode), DEV)
    st = K.gemm_fwd(K.gather3x3(srcs), E.w3x3_fwd(wdev, d), co, out, d, stats=True)
    xa = torch.cat(xs, 1).abs()
    _close(out, ref, mode, what="fwd", sabs=F.conv2d(xa, wq.abs(), padding=1))
    # statistics: combine partial (sum, M2) -> mean/var, compare with the stored values
    stored = out.float().cpu()
    n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)],
                     dtype=torch.float64)
    s = st.psum.double().cpu()
    mean = s.sum(0) / n.sum()
    m2 = st.pm2.double().cpu() + n[:, None] * (s / n[:, None] - mean) ** 2
    var = m2.sum(0) / n.sum()
    torch.testing.assert_close(mean.float(), stored.mean((0, 2, 3)), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(var.float(), stored.var((0, 2, 3), unbiased=False), rtol=1e-4, atol=1e-5)
    # input gradient
    dy = torch.randn(N, co, H, W, generator=g).to(_dt(mode)).float()
    dref = torch.nn.grad.conv2d_input((N, cin, H, W), wq, dy, padding=1)
    dx = K.empty_act(N, cin, H, W, _dt(mode), DEV)
    K.gemm_fwd(K.gather3x3([_act(dy, mode)]), E.w3x3_dgrad(wdev, d), cin, dx, d)
    _close(dx, dref, mode, what="dgrad",
           sabs=torch.nn.grad.conv2d_input((N, cin, H, W), wq.abs(), dy.abs(), padding=1))
    # weight gradient, contiguous and channels_last parameter layouts
    wref = torch.nn.grad.conv2d_weight(torch.cat(xs, 1), (co, cin, 3, 3), dy, padding=1)
    wabs = torch.nn.grad.conv2d_weight(xa, (co, cin, 3, 3), dy.abs(), padding=1)
    for fmt in (torch.contiguous_format, CL):
        gw = torch.zeros(co, cin, 3, 3, device=DEV).contiguous(memory_format=fmt)
        K.gemm_wgrad(K.gather1x1([_act(dy, mode)]), K.gather3x3(srcs), co, 9 * cin, gw,
                     E.conv_layout(gw), d, False)
        _close(gw, wref, mode, what=f"wgrad {fmt}", sabs=wabs, u=2.0 ** -23)


V4_CASES = [
    # (N, [cin per source], H, W, cout): ping-pong halo kernel (gemm_fwd4.hip)
    (1, [64], 8, 32, 256),           # 256x256 block tile, 2 chunks
    (2, [96, 64], 16, 64, 256),      # two sources, chunk crosses no source edge, 5 chunks
    (1, [32, 32, 64], 16, 32, 128),  # three sources, 512x128 block tile
    (2, [128], 32, 32, 128),
    (1, [64], 32, 64, 64),           # 1024x64 block tile (32x32 pixels)
    (1, [96, 32], 32, 32, 64),
    (1, [128, 64], 32, 32, 192),    # 1024x64 tiles, three column tiles (padded-concat widths)
]


SPLITK_CASES = [
    # (N, [cin per source], H, W, cout, forced split): split-K ping-pong kernel +
    # splitk_finish_kernel (bias, accumulate, BN partials from the fp32 slabs)
    (1, [64], 8, 32, 256, 2),
    (2, [96, 64], 16, 64, 256, 5),      # two sources, one chunk per split
    (1, [32, 32, 64], 16, 32, 128, 3),  # three sources, uneven chunk ranges
    (1, [128], 32, 64, 64, 2),          # 1024x64 tiles
]

TUNE_V4_MIN_BLOCKS, TUNE_V4_SPLITK = 0, 6
TUNE_DEFAULTS = ((TUNE_V4_MIN_BLOCKS, 256), (TUNE_V4_SPLITK, 1))


def _tune(*kv):
    from vaeunet_amd import _lib
    for k, v in kv:
        _lib.call("vu_gemm_set_tuning", k, v)


def _check_halo_conv(case, row_tiles, kernel=None):
    """forward with BN statistics, bias, accumulate into a channel slice, and
    the flipped-weight input grad, on whatever halo kernel the tuning forces
    (kernel: the vu_gemm_fwd_kernel id the forward must be dispatched to)."""
    K, E = _k()
    N, cins, H, W, co = case[:5]
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(N, c, H, W, generator=g).to(torch.bfloat16).float() for c in cins]
    cin = sum(cins)
    w = torch.randn(co, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    wq = w.to(torch.bfloat16).float()
    b = torch.randn(co, generator=g)
    d = _code("bf16")
    srcs = [_act(x, "bf16") for x in xs]
    out = K.empty_act(N, co, H, W, torch.bfloat16, DEV)
    assert K.query("vu_gemm_fwd_row_tile", *_row_tile_args(K, srcs, E.w3x3_fwd(w.to(DEV), d), co, out)) in row_tiles
    if kernel is not None:
        assert K.query("vu_gemm_fwd_kernel", *_row_tile_args(K, srcs, E.w3x3_fwd(w.to(DEV), d), co, out)) == kernel
    st = K.gemm_fwd(K.gather3x3(srcs), E.w3x3_fwd(w.to(DEV), d), co, out, d, stats=True)
    ref = F.conv2d(torch.cat(xs, 1), wq, padding=1)
    xa = torch.cat(xs, 1).abs()
    _close(out, ref, "bf16", what="fwd", sabs=F.conv2d(xa, wq.abs(), padding=1))
    stored = out.float().cpu()
    n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)],
                     dtype=torch.float64)
    s = st.psum.double().cpu()
    mean = s.sum(0) / n.sum()
    m2 = st.pm2.double().cpu() + n[:, None] * (s / n[:, None] - mean) ** 2
    torch.testing.assert_close(mean.float(), stored.mean((0, 2, 3)), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close((m2.sum(0) / n.sum()).float(), stored.var((0, 2, 3), unbiased=False),
                               rtol=1e-4, atol=1e-5)
    # bias + accumulate into the upper channel slice of a wider tensor
    base = torch.randn(N, co + 64, H, W, generator=g).to(torch.bfloat16).float()
    wide = _act(base, "bf16")
    K.gemm_fwd(K.gather3x3(srcs), E.w3x3_fwd(w.to(DEV), d), co, wide, d, out_coff=64,
               bias=b.to(DEV), accumulate=True)
    exp = base.clone()
    new = ref + b[None, :, None, None]
    exp[:, 64:] += new
    sab = torch.zeros_like(exp)
    sab[:, 64:] = F.conv2d(xa, wq.abs(), b.abs(), padding=1)
    accn = torch.zeros_like(exp)
    accn[:, 64:] = new
    _close(wide, exp, "bf16", what="bias+accumulate", sabs=sab, acc=accn)
    # input gradient (flipped weights) when cin is a tile width
    if cin in (64, 128, 256, 512) and co % 32 == 0:
        dy = torch.randn(N, co, H, W, generator=g).to(torch.bfloat16).float()
        dx = K.empty_act(N, cin, H, W, torch.bfloat16, DEV)
        K.gemm_fwd(K.gather3x3([_act(dy, "bf16")]), E.w3x3_dgrad(w.to(DEV), d), cin, dx, d)
        _close(dx, torch.nn.grad.conv2d_input((N, cin, H, W), wq, dy, padding=1), "bf16", what="dgrad",
               sabs=torch.nn.grad.conv2d_input((N, cin, H, W), wq.abs(), dy.abs(), padding=1))


@pytest.mark.parametrize("case", V4_CASES)
def test_conv3x3_pingpong_kernel(case):
    """bf16 ping-pong halo kernel (gemm_fwd4.hip) forced onto small problems
    (the production dispatcher only picks it for >= 256 blocks)."""
    _tune((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0))
    try:
        _check_halo_conv(case, (128,))
    finally:
        _tune(*TUNE_DEFAULTS)


TUNE_PP_FULL = 27
TUNE_PP_PERSIST = 30


@pytest.mark.parametrize("case", [c for c in V4_CASES if c[4] % 128 == 0])
@pytest.mark.parametrize("grid", [2, 3])
def test_conv3x3_pingpong_persistent(case, grid):
    """The persistent ping-pong walk (VU_TUNE_PP_PERSIST, round 5): a grid of
    2 or 3 blocks walking every tile (the next tile's first halo / weights
    issued during the epilogue) gives the per-element-bounded forward, the
    statistics, bias + accumulate into a channel slice and the input
    gradient, as the one-tile-per-block launch does (grid: blocks walking)."""
    _tune((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0), (TUNE_PP_PERSIST, grid))
    try:
        _check_halo_conv(case, (128,))
    finally:
        _tune(*TUNE_DEFAULTS, (TUNE_PP_PERSIST, 0))


@pytest.mark.parametrize("case", [c for c in V4_CASES if c[4] % 128 == 0])
def test_conv3x3_pingpong_full_phase(case):
    """the one-phase-per-step schedule (VU_TUNE_PP_FULL): the same MFMAs into
    the same accumulators in the same order as the two-phase schedule, so the
    output is bit-identical; plus the full parity check on it."""
    K, E = _k()
    N, cins, H, W, co = case[:5]
    g = torch.Generator().manual_seed(9)
    srcs = [_act(torch.randn(N, c, H, W, generator=g), "bf16") for c in cins]
    w = torch.randn(co, sum(cins), 3, 3, generator=g) / (3 * sum(cins) ** 0.5)
    d = _code("bf16")
    outs = []
    _tune((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0))
    try:
        for full in (0, 1):
            _tune((TUNE_PP_FULL, full))
            out = K.empty_act(N, co, H, W, torch.bfloat16, DEV)
            st = K.gemm_fwd(K.gather3x3(srcs), E.w3x3_fwd(w.to(DEV), d), co, out, d, stats=True)
            torch.cuda.synchronize()
            outs.append((out, st))
        assert torch.equal(outs[0][0], outs[1][0])
        assert torch.equal(outs[0][1].psum, outs[1][1].psum) and torch.equal(outs[0][1].pm2, outs[1][1].pm2)
        _tune((TUNE_PP_FULL, 1))
        _check_halo_conv(case, (128,))
    finally:
        _tune(*TUNE_DEFAULTS, (TUNE_PP_FULL, 1))


@pytest.mark.parametrize("case", SPLITK_CASES)
def test_conv3x3_pingpong_splitk(case):
    """split-K: blocks walk chunk ranges, fp32 slabs, deterministic finish."""
    _tune((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, case[5]))
    try:
        _check_halo_conv(case, (128,))
    finally:
        _tune(*TUNE_DEFAULTS)


SMALL_GRID_CASES = [
    # (N, [cin], H, W, cout): ResNet34 encoder levels on the 128x64 v2 tiles
    (8, [512], 16, 16, 512),   # 16^2 (too narrow for the halo kernels): 4-way split-K
    (8, [256], 32, 32, 256),   # 2-way split-K
    (8, [128], 64, 64, 128),   # no split
]


TUNE_V7 = 16


@pytest.mark.parametrize("case", SMALL_GRID_CASES)
def test_conv3x3_small_grid_v2(case):
    """small grids (gemm_fwd2.hip small-grid mode + split-K finish): bias,
    BN partials per 128 rows, accumulate, input gradient."""
    _tune((TUNE_V7, 0))
    try:
        _check_halo_conv(case, (128,), kernel=12)
    finally:
        _tune((TUNE_V7, 1))


V7_CASES = [
    # (N, [cin], H, W, cout, VU_TUNE_V7 mode): the small-grid two-K-group kernel (gemm_fwd7.hip)
    (8, [512], 16, 16, 512, 1),        # 16-pixel-wide tiles, 2-way split-K + finish
    (4, [512], 16, 16, 512, 1),        # 4-way split-K
    (8, [256], 32, 32, 256, 1),        # 4 x 32 tiles, no split (the ResNet34 layer3 shape)
    (8, [128], 64, 64, 128, 1),        # 512 blocks
    (4, [64, 64], 32, 48, 128, 1),     # two concat sources, 48-wide image -> 8 x 16 tiles
    (2, [512], 32, 32, 1024, 2),       # long K on a 32-wide grid (mode 2; mode 1 leaves it to v4 split-K)
    (8, [1024], 16, 16, 512, 1),       # 32 chunks, 2-way split
]


TUNE_V7_NBW = 17


@pytest.mark.parametrize("nbw", [3, 4])
@pytest.mark.parametrize("case", V7_CASES)
def test_conv3x3_small_grid_v7(case, nbw):
    """small grids on gemm_fwd7.hip (3- and 4-slot weight rings): bias, BN
    partials per 128-pixel tile, accumulate into a channel slice, input
    gradient, split-K slabs."""
    _tune((TUNE_V7, case[5]), (TUNE_V7_NBW, nbw))
    try:
        _check_halo_conv(case, (128,), kernel=7)
    finally:
        _tune((TUNE_V7, 1), (TUNE_V7_NBW, 3))


def test_conv3x3_splitk_auto_32x32_level():
    """the production dispatch of a down4-like layer (512 -> 1024 at 32x32):
    16..255 256x256 tiles -> automatic split-K (default tuning)."""
    _check_halo_conv((2, [512], 32, 32, 1024), (128,))


def test_conv3x3_splitk_auto_832_columns():
    """the production dispatch of the UNetResNet decoder block-1 conv1 input
    gradient (512 -> 832 padded concat channels at 32x32, B=8): 64-column
    ping-pong tiles split over K (the 128/256-column tiles do not divide 832),
    and its forward direction 832 -> 512 on the 256-column split."""
    _check_halo_conv((8, [512], 32, 32, 832), (128,), kernel=4)


IMAGE_CASES = [
    # (N, H, W, cout): the 8-channel (packed 3-channel image) conv kernel (conv_image.hip)
    (2, 16, 64, 64),
    (1, 12, 32, 128),    # two 64-column tiles, image borders on every side
    (3, 8, 48, 64),
]


@pytest.mark.parametrize("case", IMAGE_CASES)
def test_conv3x3_image_kernel(case):
    """inc.0 conv over the channel-padded image: forward with bias and BN
    statistics vs torch fp32 (the padded channels are zero)."""
    K, E = _k()
    N, H, W, co = case
    g = torch.Generator().manual_seed(11)
    x = torch.zeros(N, 8, H, W)
    x[:, :3] = torch.rand(N, 3, H, W, generator=g)
    x = x.to(torch.bfloat16).float()
    w = torch.randn(co, 3, 3, 3, generator=g) / 3
    b = torch.randn(co, generator=g)
    d = _code("bf16")
    xs = _act(x, "bf16")
    wm = E.w3x3_fwd(w.to(DEV), d, 8)
    out = K.empty_act(N, co, H, W, torch.bfloat16, DEV)
    assert K.query("vu_gemm_fwd_row_tile", *_row_tile_args(K, [xs], wm, co, out)) == 64
    st = K.gemm_fwd(K.gather3x3([xs]), wm, co, out, d, bias=b.to(DEV), stats=True)
    ref = F.conv2d(x[:, :3], w.to(torch.bfloat16).float(), b, padding=1)
    _close(out, ref, "bf16", what="image conv",
           sabs=F.conv2d(x[:, :3].abs(), w.to(torch.bfloat16).float().abs(), b.abs(), padding=1))
    stored = out.float().cpu()
    n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)],
                     dtype=torch.float64)
    s = st.psum.double().cpu()
    mean = s.sum(0) / n.sum()
    m2 = st.pm2.double().cpu() + n[:, None] * (s / n[:, None] - mean) ** 2
    torch.testing.assert_close(mean.float(), stored.mean((0, 2, 3)), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close((m2.sum(0) / n.sum()).float(), stored.var((0, 2, 3), unbiased=False),
                               rtol=1e-4, atol=1e-5)


STREAM_CASES = [
    # (K = Cin, N = Cout, accumulate into a channel slice): 1x1 stream kernel (gemm_stream.hip)
    (64, 32, False),
    (128, 64, False),
    (32, 64, True),
    (64, 128, False),   # 8 column fragments per wave tile
    (128, 256, False),  # 16 column fragments, 16-pixel wave tiles
    (64, 128, True),
    (64, 32, True),     # 2 column fragments: the GS < 4 accumulate store pass
    (128, 256, True),   # 16 column fragments, accumulate
]


@pytest.mark.parametrize("case", STREAM_CASES)
def test_gemm_stream_kernel(case):
    """short-K 1x1 GEMM streams (attention W_g/W_x and their input grads at
    256^2/512^2): bias + BN partials, or accumulate into a channel slice."""
    K, E = _k()
    cin, co, acc = case
    N, H, W = 2, 256, 256
    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, cin, H, W, generator=g).to(torch.bfloat16).float()
    w = torch.randn(co, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(co, generator=g)
    d = _code("bf16")
    xs = _act(x, "bf16")
    wm = E.w1x1_fwd(w.to(DEV), d)
    ref = F.conv2d(x, w.to(torch.bfloat16).float(), b)
    sab = F.conv2d(x.abs(), w.to(torch.bfloat16).float().abs(), b.abs())
    if not acc:
        out = K.empty_act(N, co, H, W, torch.bfloat16, DEV)
        assert K.query("vu_gemm_fwd_row_tile", *_row_tile_args(K, [xs], wm, co, out, K.gather1x1)) in (16, 32, 64)
        st = K.gemm_fwd(K.gather1x1([xs]), wm, co, out, d, bias=b.to(DEV), stats=True)
        _close(out, ref, "bf16", what="stream fwd", sabs=sab)
        stored = out.float().cpu()
        n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)],
                         dtype=torch.float64)
        s_ = st.psum.double().cpu()
        mean = s_.sum(0) / n.sum()
        m2 = st.pm2.double().cpu() + n[:, None] * (s_ / n[:, None] - mean) ** 2
        torch.testing.assert_close(mean.float(), stored.mean((0, 2, 3)), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close((m2.sum(0) / n.sum()).float(), stored.var((0, 2, 3), unbiased=False),
                                   rtol=1e-4, atol=1e-4)
    else:
        base = torch.randn(N, co + 32, H, W, generator=g).to(torch.bfloat16).float()
        wide = _act(base, "bf16")
        K.gemm_fwd(K.gather1x1([xs]), wm, co, wide, d, out_coff=32, bias=b.to(DEV), accumulate=True)
        exp = base.clone()
        exp[:, 32:] += ref
        sw, an = torch.zeros_like(exp), torch.zeros_like(exp)
        sw[:, 32:], an[:, 32:] = sab, ref
        _close(wide, exp, "bf16", what="stream accumulate", sabs=sw, acc=an)


@pytest.mark.parametrize("cin,cout", [(128, 64), (64, 32)])
def test_gemm_stream_convT(cin, cout):
    """ConvTranspose2d 2x2/s2 (unet_parts.py:76) on the stream kernel: N = 4*cout
    columns stored through the pixel shuffle, bias per output channel."""
    K, E = _k()
    N, H, W = 2, 128, 128
    g = torch.Generator().manual_seed(17)
    x = torch.randn(N, cin, H, W, generator=g).to(torch.bfloat16).float()
    w = torch.randn(cin, cout, 2, 2, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g)
    d = _code("bf16")
    out = K.empty_act(N, cout, 2 * H, 2 * W, torch.bfloat16, DEV)
    K.gemm_fwd(K.gather1x1([_act(x, "bf16")]), E.wT_fwd(w.to(DEV), d), 4 * cout, out, d, bias=b.to(DEV),
               convT=(2 * H, 2 * W, 0, 0, cout))
    ref = F.conv_transpose2d(x, w.to(torch.bfloat16).float(), b, stride=2)
    _close(out, ref, "bf16", what="stream convT",
           sabs=F.conv_transpose2d(x.abs(), w.to(torch.bfloat16).float().abs(), b.abs(), stride=2))


TUNE_V5 = 10
V5_CASES = [
    # (N, Cin, H, W, Cout, grid cap): persistent short-K GEMM (gemm_fwd5.hip)
    (8, 256, 64, 64, 256, 0),    # 4 K steps, 2 column tiles, one tile per block
    (8, 512, 64, 64, 256, 7),    # 8 K steps, ~37 tiles per block
    (16, 256, 64, 64, 64, 5),    # 64-column tiles
    (8, 1024, 32, 64, 512, 3),   # 16 K steps, 4 column tiles
]


def _stats_check(st, stored):
    n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)],
                     dtype=torch.float64)
    s_ = st.psum.double().cpu()
    mean = s_.sum(0) / n.sum()
    m2 = st.pm2.double().cpu() + n[:, None] * (s_ / n[:, None] - mean) ** 2
    torch.testing.assert_close(mean.float(), stored.mean((0, 2, 3)), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close((m2.sum(0) / n.sum()).float(), stored.var((0, 2, 3), unbiased=False),
                               rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("case", V5_CASES)
def test_gemm_v5_fwd_stats_accumulate(case):
    """1x1 conv with K = 256..1024 on the persistent v5 kernel: bias + BN
    partials (64-row tiles), and the accumulating input gradient into a
    channel slice of a wider tensor; grid caps force several tiles per block
    (the flattened tile / k-step ring crossing tile boundaries)."""
    K, E = _k()
    N, cin, H, W, co, cap = case
    g = torch.Generator().manual_seed(31)
    x = torch.randn(N, cin, H, W, generator=g).to(torch.bfloat16).float()
    w = torch.randn(co, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(co, generator=g)
    wq = w.to(torch.bfloat16).float()
    d = _code("bf16")
    xs = _act(x, "bf16")
    wm = E.w1x1_fwd(w.to(DEV), d)
    _tune((TUNE_V5, cap if cap else 1))
    try:
        out = K.empty_act(N, co, H, W, torch.bfloat16, DEV)
        assert K.query("vu_gemm_fwd_row_tile", *_row_tile_args(K, [xs], wm, co, out, K.gather1x1)) == 64
        st = K.gemm_fwd(K.gather1x1([xs]), wm, co, out, d, bias=b.to(DEV), stats=True)
        _close(out, F.conv2d(x, wq, b), "bf16", what="v5 fwd", sabs=F.conv2d(x.abs(), wq.abs(), b.abs()))
        _stats_check(st, out.float().cpu())
        # input gradient: K = co, N = cin, accumulated into channels [64, 64 + cin)
        du = torch.randn(N, co, H, W, generator=g).to(torch.bfloat16).float()
        base = torch.randn(N, cin + 64, H, W, generator=g).to(torch.bfloat16).float()
        wide = _act(base, "bf16")
        K.gemm_fwd(K.gather1x1([_act(du, "bf16")]), E.w1x1_dgrad(w.to(DEV), d), cin, wide, d, out_coff=64,
                   accumulate=True)
        exp = base.clone()
        new = torch.nn.grad.conv2d_input((N, cin, H, W), wq, du)
        exp[:, 64:] += new
        sw, an = torch.zeros_like(exp), torch.zeros_like(exp)
        sw[:, 64:], an[:, 64:] = torch.nn.grad.conv2d_input((N, cin, H, W), wq.abs(), du.abs()), new
        _close(wide, exp, "bf16", what="v5 dgrad accumulate", sabs=sw, acc=an)
    finally:
        _tune((TUNE_V5, 1))


TUNE_V6 = 11
V6_CASES = [
    # (N, H, W, grid cap): resident-weight 64 -> 64 3x3 kernel (gemm_fwd6.hip),
    # tiles of 16x32 pixels walked persistently (cap < tiles: several per block)
    (1, 16, 32, 2),     # one tile, image border on every side
    (2, 32, 64, 3),     # 8 tiles over 3 blocks (uneven walk)
    (1, 48, 96, 5),     # 9 tiles
    (3, 64, 32, 256),   # 12 tiles, one per block
]


@pytest.mark.parametrize("case", V6_CASES)
def test_conv3x3_c64_resident(case):
    """64 -> 64 3x3 conv forward (bias + BN partials of 64-pixel wave tiles)
    and input gradient on the v6 kernel vs torch fp32 of the bf16-rounded
    operands (unet_parts.py:43 and its backward)."""
    K, E = _k()
    N, H, W, cap = case
    g = torch.Generator().manual_seed(41)
    x = torch.randn(N, 64, H, W, generator=g).to(torch.bfloat16).float()
    w = torch.randn(64, 64, 3, 3, generator=g) / 24.0
    b = torch.randn(64, generator=g)
    wq = w.to(torch.bfloat16).float()
    d = _code("bf16")
    xs = _act(x, "bf16")
    wf = E.w3x3_fwd(w.to(DEV), d)
    _tune((TUNE_V6, cap))
    try:
        out = K.empty_act(N, 64, H, W, torch.bfloat16, DEV)
        assert K.query("vu_gemm_fwd_row_tile", *_row_tile_args(K, [xs], wf, 64, out, K.gather3x3)) == 64
        st = K.gemm_fwd(K.gather3x3([xs]), wf, 64, out, d, bias=b.to(DEV), stats=True)
        _close(out, F.conv2d(x, wq, b, padding=1), "bf16", what="v6 fwd",
               sabs=F.conv2d(x.abs(), wq.abs(), b.abs(), padding=1))
        _stats_check(st, out.float().cpu())
        dy = torch.randn(N, 64, H, W, generator=g).to(torch.bfloat16).float()
        dx = K.empty_act(N, 64, H, W, torch.bfloat16, DEV)
        K.gemm_fwd(K.gather3x3([_act(dy, "bf16")]), E.w3x3_dgrad(w.to(DEV), d), 64, dx, d, kind="dgrad")
        _close(dx, torch.nn.grad.conv2d_input((N, 64, H, W), wq, dy, padding=1), "bf16", what="v6 dgrad",
               sabs=torch.nn.grad.conv2d_input((N, 64, H, W), wq.abs(), dy.abs(), padding=1))
    finally:
        _tune((TUNE_V6, 1))


TUNE_V6_STAG = 34


@pytest.mark.parametrize("cap", [1, 2, 3, 5])
@pytest.mark.parametrize("variant", ["stats_bias", "plain", "relu"])
def test_conv3x3_c64_staggered_bit_identical(variant, cap):
    """The staggered-epilogue resident-weight kernel (conv3x3_c64s_kernel,
    VU_TUNE_V6_STAG = 1, round 6) against the round-5 lock-step kernel on the
    same operands: outputs and BatchNorm partials bit for bit (the same MFMAs
    and additions; only the statistics' store order differs), for 1-9 tiles
    per block (odd and even walks, the last tile's epilogue after the loop)."""
    K, E = _k()
    N, H, W = 2, 48, 96   # 18 tiles
    g = torch.Generator().manual_seed(47)
    x = torch.randn(N, 64, H, W, generator=g).to(torch.bfloat16)
    w = torch.randn(64, 64, 3, 3, generator=g) / 24.0
    b = torch.randn(64, generator=g) if variant == "stats_bias" else None
    d = _code("bf16")
    xs = x.to(DEV).contiguous(memory_format=CL)
    wf = E.w3x3_fwd(w.to(DEV), d)
    res = []
    for stag in (0, 1):
        _tune((TUNE_V6, cap), (TUNE_V6_STAG, stag))
        try:
            out = K.empty_act(N, 64, H, W, torch.bfloat16, DEV)
            out.fill_(7.0)
            st = K.gemm_fwd(K.gather3x3([xs]), wf, 64, out, d, bias=None if b is None else b.to(DEV),
                            stats=variant == "stats_bias", relu=variant == "relu")
            torch.cuda.synchronize()
            res.append((out.clone(), None if st is None else (st.psum.clone(), st.pm2.clone())))
        finally:
            _tune((TUNE_V6, 1), (TUNE_V6_STAG, 1))
    (o0, s0), (o1, s1) = res
    assert torch.equal(o0.view(torch.int16), o1.view(torch.int16))
    if variant == "relu":
        assert float(o1.float().min()) == 0.0
    if s0 is not None:
        assert torch.equal(s0[0], s1[0]) and torch.equal(s0[1], s1[1])


@pytest.mark.parametrize("co", [128, 192])
def test_conv3x3_c64_column_slices(co):
    """64 input channels, 128/192 outputs, no statistics (the input gradient of
    the up4.1 128 -> 64 concat conv): one resident-weight launch per 64-column
    slice, written into channel slices of a wider output (out_coff 64)."""
    K, E = _k()
    N, H, W = 2, 32, 64
    g = torch.Generator().manual_seed(43)
    x = torch.randn(N, 64, H, W, generator=g).to(torch.bfloat16).float()
    w = torch.randn(co, 64, 3, 3, generator=g) / 24.0
    wq = w.to(torch.bfloat16).float()
    d = _code("bf16")
    xs = _act(x, "bf16")
    wf = E.w3x3_fwd(w.to(DEV), d)
    _tune((TUNE_V6, 256))
    try:
        wide = K.empty_act(N, co + 64, H, W, torch.bfloat16, DEV)
        assert K.query("vu_gemm_fwd_kernel", *_row_tile_args(K, [xs], wf, co, wide)) == 6
        K.gemm_fwd(K.gather3x3([xs]), wf, co, wide, d, out_coff=64)
        _close(wide[:, 64:], F.conv2d(x, wq, padding=1), "bf16", what="v6 column slices",
               sabs=F.conv2d(x.abs(), wq.abs(), padding=1))
    finally:
        _tune((TUNE_V6, 1))


@pytest.mark.parametrize("N,H,W", [(2, 64, 64), (1, 96, 160), (64, 13, 13)])
def test_conv_stem_7x7s2(N, H, W):
    """ResNet34 stem (7x7, stride 2, pad 3, 8 packed channels -> 64) on the
    stem kernel (conv_stem.hip): bias + BN partials vs torch fp32 of the
    bf16-rounded operands; odd sizes exercise every border tap."""
    K, E = _k()
    g = torch.Generator().manual_seed(43)
    x = torch.randn(N, 8, H, W, generator=g).to(torch.bfloat16).float()
    w = torch.randn(64, 8, 7, 7, generator=g) / 20.0
    b = torch.randn(64, generator=g)
    wq = w.to(torch.bfloat16).float()
    d = _code("bf16")
    Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    if (N * Ho * Wo) % 64:
        pytest.skip("whole 64-pixel tiles only")
    xs = _act(x, "bf16")
    wf = E.w3x3_fwd(w.to(DEV), d)
    out = K.empty_act(N, 64, Ho, Wo, torch.bfloat16, DEV)
    gth = K.gather([xs], N, Ho, Wo, R=7, S=7, sy=2, sx=2, oy=-3, ox=-3)
    import ctypes as C
    from vaeunet_amd import _lib
    a = _lib.VuGemmFwd()
    a.a, a.b, a.ldb, a.ncol, a.out, a.out_stride, a.out_mode = gth, wf.data_ptr(), wf.shape[-1], 64, out.data_ptr(), K.pstride(out), 0
    assert K.query("vu_gemm_fwd_row_tile", C.byref(a), 1) == 64
    st = K.gemm_fwd(gth, wf, 64, out, d, bias=b.to(DEV), stats=True)
    _close(out, F.conv2d(x, wq, b, stride=2, padding=3), "bf16", what="stem fwd",
           sabs=F.conv2d(x.abs(), wq.abs(), b.abs(), stride=2, padding=3))
    _stats_check(st, out.float().cpu())


@pytest.mark.parametrize("ci,co,h,cap", [(512, 256, 32, 0), (256, 128, 64, 6), (1024, 512, 32, 0)])
def test_gemm_v5_convT(ci, co, h, cap):
    """ConvTranspose2d 2x2/s2 of the deeper decoder levels on v5: forward with
    the pixel-shuffle store (bias per output channel) and the input gradient
    as a 2x2 parity gather (K = 4*co)."""
    K, E = _k()
    N = 8
    g = torch.Generator().manual_seed(37)
    x = torch.randn(N, ci, h, h, generator=g).to(torch.bfloat16).float()
    w = torch.randn(ci, co, 2, 2, generator=g) / ci ** 0.5
    b = torch.randn(co, generator=g)
    wq = w.to(torch.bfloat16).float()
    d = _code("bf16")
    _tune((TUNE_V5, cap if cap else 1))
    try:
        out = K.empty_act(N, co, 2 * h, 2 * h, torch.bfloat16, DEV)
        K.gemm_fwd(K.gather1x1([_act(x, "bf16")]), E.wT_fwd(w.to(DEV), d), 4 * co, out, d, bias=b.to(DEV),
                   convT=(2 * h, 2 * h, 0, 0, co))
        xr = x.clone().requires_grad_(True)
        ref = F.conv_transpose2d(xr, wq, b, stride=2)
        xa = x.abs().requires_grad_(True)
        refa = F.conv_transpose2d(xa, wq.abs(), b.abs(), stride=2)
        _close(out, ref, "bf16", what="v5 convT fwd", sabs=refa)
        du = torch.randn(N, co, 2 * h, 2 * h, generator=g).to(torch.bfloat16).float()
        ref.backward(du)
        refa.backward(du.abs())
        dx = K.empty_act(N, ci, h, h, torch.bfloat16, DEV)
        K.gemm_fwd(K.gather_convT(_act(du, "bf16"), N, h, h), E.wT_dgrad(w.to(DEV), d), ci, dx, d)
        _close(dx, xr.grad, "bf16", what="v5 convT dgrad", sabs=xa.grad)
    finally:
        _tune((TUNE_V5, 1))


def _row_tile_args(K, srcs, wmat, ncol, out, gather=None):
    import ctypes as C
    from vaeunet_amd import _lib
    a = _lib.VuGemmFwd()
    a.a = (gather or K.gather3x3)(srcs)
    a.b = wmat.data_ptr()
    a.ldb = wmat.shape[-1]
    a.ncol = ncol
    a.out = out.data_ptr()
    a.out_stride = K.pstride(out)
    a.out_mode = 0
    return (C.byref(a), 1)


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("case", [(4, 64, 32, 32, 32), (4, 128, 32, 32, 64), (2, 256, 32, 32, 128),
                                  (1, 48, 16, 16, 24),
                                  (16, 64, 64, 64, 32),    # bf16 v2: 1-step K ring, 32-channel K tail
                                  (16, 128, 64, 64, 64),
                                  (2, 64, 8, 256, 32),     # wgrad steps inside 256-wide rows (row wraps)
                                  (2, 256, 4, 128, 128)])  # 128 x 256 wgrad tiles, 64-pixel steps, row wraps
def test_conv1x1_fwd_dgrad_wgrad(mode, case):
    """1x1 conv (attention gate W_g / W_x, unet_parts.py:10-16): forward with
    bias + BN statistics, accumulating input gradient, weight gradient (the
    small-output wgrad tiles: 32x64, 64x128)."""
    K, E = _k()
    N, C_, H, W, F_ = case
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, C_, H, W, generator=g).to(_dt(mode)).float()
    w = (torch.randn(F_, C_, 1, 1, generator=g) / C_ ** 0.5)
    b = torch.randn(F_, generator=g)
    wq = w.to(_dt(mode)).float()
    d = _code(mode)
    u = K.empty_act(N, F_, H, W, _dt(mode), DEV)
    K.gemm_fwd(K.gather1x1([_act(x, mode)]), E.w1x1_fwd(w.to(DEV), d), F_, u, d, bias=b.to(DEV), stats=True)
    _close(u, F.conv2d(x, wq, b), mode, what="fwd", sabs=F.conv2d(x.abs(), wq.abs(), b.abs()))
    du = torch.randn(N, F_, H, W, generator=g).to(_dt(mode)).float()
    base = torch.randn(N, C_, H, W, generator=g).to(_dt(mode)).float()
    dx = _act(base, mode)
    K.gemm_fwd(K.gather1x1([_act(du, mode)]), E.w1x1_dgrad(w.to(DEV), d), C_, dx, d, accumulate=True)
    new = torch.nn.grad.conv2d_input((N, C_, H, W), wq, du)
    _close(dx, base + new, mode, what="dgrad", acc=new,
           sabs=torch.nn.grad.conv2d_input((N, C_, H, W), wq.abs(), du.abs()))
    gw = torch.zeros(F_, C_, 1, 1, device=DEV)
    K.gemm_wgrad(K.gather1x1([_act(du, mode)]), K.gather1x1([_act(x, mode)]), F_, C_, gw,
                 E.conv_layout(gw), d, False)
    _close(gw, torch.nn.grad.conv2d_weight(x, (F_, C_, 1, 1), du), mode, what="wgrad", u=2.0 ** -23,
           sabs=torch.nn.grad.conv2d_weight(x.abs(), (F_, C_, 1, 1), du.abs()))


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("case", [(2, 64, 4, 4, 32, 8, 8), (2, 64, 4, 4, 32, 9, 10),
                                  (8, 128, 64, 64, 64, 128, 128), (8, 128, 64, 64, 64, 130, 129)])
def test_conv_transpose(mode, case):
    """ConvTranspose2d(k2,s2)+bias then F.pad into the skip canvas (unet_parts.py:76,88)."""
    K, E = _k()
    N, ci, h, w, co, H, W = case
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, ci, h, w, generator=g).to(_dt(mode)).float()
    wt = (torch.randn(ci, co, 2, 2, generator=g) / ci ** 0.5)
    b = torch.randn(co, generator=g) * 0.1
    wq = wt.to(_dt(mode)).float()
    dyp, dxp = H - 2 * h, W - 2 * w
    py, px = dyp // 2, dxp // 2
    xr = x.clone().requires_grad_(True)
    wr = wq.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    ref = F.pad(F.conv_transpose2d(xr, wr, br, stride=2), [px, dxp - px, py, dyp - py])
    # the same ops on |operands|: sum_k |a_k||b_k| of every output / gradient element
    xa = x.abs().requires_grad_(True)
    wa = wq.abs().requires_grad_(True)
    ba = b.abs().requires_grad_(True)
    refa = F.pad(F.conv_transpose2d(xa, wa, ba, stride=2), [px, dxp - px, py, dyp - py])
    d = _code(mode)
    u = K.zeros_act(N, co, H, W, _dt(mode), DEV)
    K.gemm_fwd(K.gather1x1([_act(x, mode)]), E.wT_fwd(wt.to(DEV), d), 4 * co, u, d,
               bias=b.to(DEV), convT=(H, W, py, px, co))
    _close(u, ref, mode, what="convT fwd", sabs=refa)
    du = torch.randn(N, co, H, W, generator=g).to(_dt(mode)).float()
    ref.backward(du)
    refa.backward(du.abs())
    dua = _act(du, mode)
    dx = K.empty_act(N, ci, h, w, _dt(mode), DEV)
    K.gemm_fwd(K.gather_convT(dua, N, h, w, py, px), E.wT_dgrad(wt.to(DEV), d), ci, dx, d)
    _close(dx, xr.grad, mode, what="convT dgrad", sabs=xa.grad)
    gw = torch.zeros(ci, co, 2, 2, device=DEV)
    K.gemm_wgrad(K.gather1x1([_act(x, mode)]), K.gather_convT(dua, N, h, w, py, px), ci, 4 * co, gw,
                 E.convT_layout(gw), d, False)
    _close(gw, wr.grad, mode, what="convT wgrad", sabs=wa.grad, u=2.0 ** -23)
    gb = torch.zeros(co, device=DEV)
    K.chan_sum(dua, gb, False, d, window=(py, px, 2 * h, 2 * w))
    _close(gb, br.grad, mode, what="convT bias grad", sabs=ba.grad, u=2.0 ** -23)


TUNE_W2_BIG = 28


@pytest.mark.parametrize("case", [("convT", 4, 512, 16, 16, 256), ("convT", 2, 256, 32, 32, 128),
                                  ("1x1", 8, 512, 16, 16, 256), ("1x1", 2, 384, 24, 20, 320)])
def test_wgrad_v2_big_tiles(case):
    """the 256 x 256-tile, 4-slot-ring variant of the v2 weight gradient
    (VU_TUNE_W2_BIG) on ConvTranspose2d(k2,s2) and 1x1 problems with both
    gradient dimensions >= 256 (partial edge tiles included) vs torch fp32 of
    the bf16 operands; the split count comes from the production heuristic."""
    K, E = _k()
    kind, N, ci, h, w, co = case
    g = torch.Generator().manual_seed(29)
    d = _code("bf16")
    x = torch.randn(N, ci, h, w, generator=g).to(torch.bfloat16).float()
    _tune((TUNE_W2_BIG, 1))
    try:
        if kind == "convT":
            du = torch.randn(N, co, 2 * h, 2 * w, generator=g).to(torch.bfloat16).float()
            gw = torch.zeros(ci, co, 2, 2, device=DEV)
            K.gemm_wgrad(K.gather1x1([_act(x, "bf16")]), K.gather_convT(_act(du, "bf16"), N, h, w, 0, 0), ci, 4 * co,
                         gw, E.convT_layout(gw), d, False)
            xr = x.clone().requires_grad_(True)
            wr = torch.zeros(ci, co, 2, 2, requires_grad=True)
            F.conv_transpose2d(xr, wr, None, stride=2).backward(du)
            xa = x.abs()
            wa = torch.zeros(ci, co, 2, 2, requires_grad=True)
            F.conv_transpose2d(xa, wa, None, stride=2).backward(du.abs())
            _close(gw, wr.grad, "bf16", what="convT wgrad (256x256 tiles)", sabs=wa.grad, u=2.0 ** -23)
        else:
            du = torch.randn(N, co, h, w, generator=g).to(torch.bfloat16).float()
            gw = torch.zeros(co, ci, 1, 1, device=DEV)
            K.gemm_wgrad(K.gather1x1([_act(du, "bf16")]), K.gather1x1([_act(x, "bf16")]), co, ci, gw,
                         E.conv_layout(gw), d, False)
            _close(gw, torch.nn.grad.conv2d_weight(x, (co, ci, 1, 1), du), "bf16", what="1x1 wgrad (256x256 tiles)",
                   u=2.0 ** -23, sabs=torch.nn.grad.conv2d_weight(x.abs(), (co, ci, 1, 1), du.abs()))
    finally:
        _tune((TUNE_W2_BIG, 0))


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("shape", [(2, 16, 8, 8), (2, 8, 11, 9), (2, 3, 5, 7)])
def test_maxpool(mode, shape):
    K, _ = _k()
    g = torch.Generator().manual_seed(3)
    # small integers: plenty of exact ties (first max in scan order wins)
    x = torch.randint(-3, 3, shape, generator=g).float()
    xr = x.clone().requires_grad_(True)
    ref = F.max_pool2d(xr, 2)
    d = _code(mode)
    xa = _act(x, mode)
    y = K.maxpool_fwd(xa, d)
    _close(y, ref, mode, what="pool fwd")
    dy = torch.randn(ref.shape, generator=g).to(_dt(mode)).float()
    ref.backward(dy)
    add = torch.randn(shape, generator=g).to(_dt(mode)).float()
    dx = torch.empty_like(xa)
    K.maxpool_bwd(xa, _act(dy, mode), dx, _act(add, mode), d)
    _close(dx, xr.grad + add, mode, what="pool bwd")


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("shape", [(2, 64, 16, 16), (1, 128, 8, 12), (3, 8, 6, 4), (1, 512, 4, 4)])
def test_bn_maxpool_fusion(mode, shape):
    """Down (unet_parts.py:51-63) with the producing BatchNorm + ReLU fused
    into the max-pool: a and the pooled map equal vu_bn_apply followed by
    vu_maxpool2_fwd bit for bit."""
    K, _ = _k()
    N, C_, H, W = shape
    g = torch.Generator().manual_seed(5)
    d = _code(mode)
    y = _act(torch.randn(shape, generator=g), mode)
    coef = torch.stack([torch.rand(C_, generator=g) + 0.5, torch.randn(C_, generator=g) * 0.3,
                        torch.randn(C_, generator=g) * 0.1, torch.rand(C_, generator=g) + 0.5]).to(DEV)
    assert K.pool_fusable(y)
    a, p = torch.empty_like(y), K.empty_act(N, C_, H // 2, W // 2, y.dtype, DEV)
    K.bn_apply_maxpool(y, a, p, coef, True, d)
    a_ref = torch.empty_like(y)
    K.bn_apply(y, a_ref, coef, True, d)
    assert torch.equal(a, a_ref)
    assert torch.equal(p, K.maxpool_fwd(a_ref, d))


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("case", [(2, 16, 4, 4, 8, 8, 8, 8), (2, 8, 5, 4, 10, 8, 11, 9),
                                  (1, 32, 16, 16, 33, 31, 33, 31), (2, 8, 1, 1, 6, 6, 6, 6)])
def test_upsample_bilinear(mode, case):
    K, _ = _k()
    N, C_, hi, wi, ho, wo, Hp, Wp = case
    g = torch.Generator().manual_seed(4)
    x = torch.randn(N, C_, hi, wi, generator=g).to(_dt(mode)).float()
    xr = x.clone().requires_grad_(True)
    py, px = (Hp - ho) // 2, (Wp - wo) // 2
    up = F.interpolate(xr, size=(ho, wo), mode="bilinear", align_corners=True)
    ref = F.pad(up, [px, Wp - wo - px, py, Hp - ho - py])
    d = _code(mode)
    out = K.empty_act(N, C_, Hp, Wp, _dt(mode), DEV)
    K.upsample_fwd(_act(x, mode), out, ho, wo, py, px, d)
    _close(out, ref, mode, what="upsample fwd")
    dy = torch.randn(N, C_, Hp, Wp, generator=g).to(_dt(mode)).float()
    ref.backward(dy)
    dx = K.empty_act(N, C_, hi, wi, _dt(mode), DEV)
    K.upsample_bwd(_act(dy, mode), dx, ho, wo, py, px, False, d)
    _close(dx, xr.grad, mode, what="upsample bwd")


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("shape", [(4, 64, 16, 16), (2, 24, 5, 7), (8, 128, 64, 64)])
def test_batchnorm_train(mode, relu, shape):
    """BatchNorm2d train mode (+ReLU) fwd/bwd and running stats vs torch."""
    K, E = _k()
    N, C_, H, W = shape
    g = torch.Generator().manual_seed(5)
    y = (torch.randn(shape, generator=g) * 3 + 1).to(_dt(mode)).float()
    bn = torch.nn.BatchNorm2d(C_)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn_dev = torch.nn.BatchNorm2d(C_).to(DEV)
    bn_dev.load_state_dict(bn.state_dict())
    yr = y.clone().requires_grad_(True)
    ref = bn(yr)
    if relu:
        ref = torch.relu(ref)
    d = _code(mode)
    ya = _act(y, mode)
    out = K.empty_act(N, C_, H, W, _dt(mode), DEV)
    # statistics through an identity 1x1 GEMM epilogue
    eye = torch.eye(C_, device=DEV)
    st = K.gemm_fwd(K.gather1x1([ya]), E.w1x1_fwd(eye.view(C_, C_, 1, 1), d), C_, out, d, stats=True)
    coef = E.bn_coef(bn_dev, st, C_)
    a = torch.empty_like(out)
    K.bn_apply(out, a, coef, relu, d)
    _close(a, ref, mode, what="bn fwd")
    torch.testing.assert_close(bn_dev.running_mean.cpu(), bn.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn_dev.running_var.cpu(), bn.running_var, rtol=1e-4, atol=1e-5)
    assert int(bn_dev.num_batches_tracked) == 1
    da = torch.randn(shape, generator=g).to(_dt(mode)).float()
    ref.backward(da)
    dx = E.bn_bwd(_act(da, mode), out, coef, bn_dev, relu, E.Mode(d, torch.device(DEV)))
    got, want = dx.detach().float().cpu(), yr.grad
    if relu:
        # an element whose BN output lies within rounding of zero may take the
        # other side of the ReLU mask (the kernel evaluates y*scale+shift, torch
        # (y-mean)*invstd*w+b): compare everywhere else
        with torch.no_grad():
            pre = torch.nn.functional.batch_norm(y, None, None, bn.weight, bn.bias, True, 0.0, bn.eps)
        keep = pre.abs() > 1e-4 * pre.abs().max()
        got, want = got * keep, want * keep
    _close(got, want, mode, scale_floor=1e-2, what="bn bwd")
    torch.testing.assert_close(bn_dev.weight.grad.cpu(), bn.weight.grad, rtol=2e-3, atol=1e-3)
    torch.testing.assert_close(bn_dev.bias.grad.cpu(), bn.bias.grad, rtol=2e-3, atol=1e-3)


@pytest.mark.parametrize("stats1", [1, 0])
@pytest.mark.parametrize("tiles,tile_rows,C", [(40000, 7, 64), (300, 128, 192), (5, 64, 8), (16385, 4, 16),
                                              (64, 128, 1024)])
def test_bn_finalize_partials(tiles, tile_rows, C, stats1):
    """vu_bn_finalize on synthetic per-tile (sum, M2) partials: several rounds
    per block (tiles > 64 x 256), several blocks and channel groups, a ragged
    last tile, an empty last block (16385 tiles); mean / biased var / running
    stats vs an fp64 combination.  stats1: the one-launch finalize (the last
    block of each channel group combines, VU_TUNE_BN_STATS1 = 1, opt-in) or
    the two-launch path (default)."""
    K, _ = _k()
    from vaeunet_amd import _lib as lib
    lib.call("vu_gemm_set_tuning", 35, stats1)
    try:
        _bn_finalize_partials(K, tiles, tile_rows, C)
    finally:
        lib.call("vu_gemm_set_tuning", 35, 0)


def _bn_finalize_partials(K, tiles, tile_rows, C):
    g = torch.Generator().manual_seed(41)
    rows = tiles * tile_rows - 3
    n = torch.full((tiles,), float(tile_rows), dtype=torch.float64)
    n[-1] = tile_rows - 3
    mu_t = torch.randn(tiles, C, generator=g, dtype=torch.float64) * 0.5 + 2.0
    m2_t = torch.rand(tiles, C, generator=g, dtype=torch.float64) * n[:, None]
    psum = (mu_t * n[:, None]).float()
    pm2 = m2_t.float()
    st = K.Stats(psum.to(DEV), pm2.to(DEV), tiles, tile_rows, rows)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    rm, rv = torch.zeros(C), torch.ones(C)
    nbt = torch.zeros((), dtype=torch.int64)
    rm_d, rv_d, nbt_d = rm.to(DEV), rv.to(DEV), nbt.to(DEV)
    coef = K.bn_finalize(st, C, gamma.to(DEV), beta.to(DEV), rm_d, rv_d, nbt_d, 0.1, 1e-5)
    s64, q64 = psum.double(), pm2.double()
    mean = s64.sum(0) / n.sum()
    M2 = (q64 + n[:, None] * (s64 / n[:, None] - mean) ** 2).sum(0)
    var = M2 / n.sum()
    invstd = 1.0 / torch.sqrt(var + 1e-5)
    c = coef.cpu().double()
    torch.testing.assert_close(c[2], mean, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(c[3], invstd, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(c[0], gamma.double() * invstd, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv_d.cpu().double(), 0.9 + 0.1 * M2 / (n.sum() - 1), rtol=1e-5, atol=1e-6)
    assert int(nbt_d) == 1
    # a second launch reuses the self-resetting arrival counters
    coef2 = K.bn_finalize(st, C, gamma.to(DEV), beta.to(DEV), None, None, None, 0.0, 1e-5)
    assert torch.equal(coef2[:, :].cpu(), coef.cpu())


@pytest.mark.parametrize("shape", [(16, 64, 128, 128), (8, 512, 32, 32), (4, 16, 20, 12)])
def test_chan_sum_fused(shape):
    """per-channel sums (bias gradients) on the fused one-launch reduction:
    256 pixel blocks (the cap), several channel groups, narrow channel
    counts; fixed-order, so two launches agree bitwise."""
    K, _ = _k()
    g = torch.Generator().manual_seed(43)
    x = torch.randn(shape, generator=g).to(torch.bfloat16).float()
    xa = _act(x, "bf16")
    out = torch.zeros(shape[1], device=DEV)
    K.chan_sum(xa, out, False, 1)
    ref = x.double().sum((0, 2, 3))
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-5, atol=1e-3)
    out2 = torch.full((shape[1],), 1.0, device=DEV)
    K.chan_sum(xa, out2, True, 1)
    assert torch.equal(out2.cpu(), out.cpu() + 1.0)


def test_loss_kernels_vs_oracle():
    from vaeunet_amd.loss import CombinedLoss, dice_loss, kl_with_free_bits
    from oracle import cpu_ref as R
    g = torch.Generator().manual_seed(6)
    for shape, p in [((2, 1, 64, 64), 0.02), ((3, 2, 16, 16), 0.3), ((2, 1, 8, 8), 0.0)]:
        x = torch.randn(shape, generator=g) * 3
        t = (torch.rand(shape, generator=g) < p).float()
        xr = x.clone().requires_grad_(True)
        ref = R.combined_loss(xr, t)
        ref.backward()
        xd = x.to(DEV).requires_grad_(True)
        out = CombinedLoss()(xd, t.to(DEV))
        out.backward()
        assert abs(out.item() - ref.item()) < 1e-5
        torch.testing.assert_close(xd.grad.cpu(), xr.grad, rtol=1e-4, atol=1e-8)
        assert abs(dice_loss(x.to(DEV), t.to(DEV)).item() - R.dice_loss(x, t).item()) < 1e-6
    mu = torch.randn(8, 32, generator=g)
    lv = torch.randn(8, 32, generator=g)
    mu[0, 0] = 0.0
    lv[0, 0] = 0.0
    for fb in (1e-3, 0.0, 0.5):
        m, v = mu.clone().requires_grad_(True), lv.clone().requires_grad_(True)
        ref = R.kl_with_free_bits(m, v, fb)
        ref.backward()
        md, vd = mu.to(DEV).requires_grad_(True), lv.to(DEV).requires_grad_(True)
        out = kl_with_free_bits(md, vd, free_bits=fb)
        (2.0 * out).backward()
        assert abs(out.item() - ref.item()) < 1e-5 * max(1.0, abs(ref.item()))
        torch.testing.assert_close(md.grad.cpu(), 2 * m.grad, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(vd.grad.cpu(), 2 * v.grad, rtol=1e-5, atol=1e-7)


def test_permute_batch_matches_single_launches():
    """engine.refresh_weights: all stale derived weight images rebuilt in one
    vu_permute4_batch launch equal the one-launch-per-image builds."""
    K, E = _k()
    g = torch.Generator().manual_seed(9)
    ws = [torch.randn(64, 32, 3, 3, generator=g).to(DEV), torch.randn(16, 8, 1, 1, generator=g).to(DEV),
          torch.randn(32, 16, 2, 2, generator=g).to(DEV),
          torch.randn(64, 3, 3, 3, generator=g).to(DEV).contiguous(memory_format=CL),
          torch.randn(72, 40, 3, 3, generator=g).to(DEV),   # ragged 32-tiles of the tap-merged transpose
          torch.randn(40, 24, 3, 3, generator=g).to(DEV).contiguous(memory_format=CL),  # converting copy
          torch.randn(136, 72, 3, 3, generator=g).to(DEV).contiguous(memory_format=CL)]  # ragged 64-tile transposes
    for d in (0, 1):
        single = [E.w3x3_fwd(ws[0], d), E.w3x3_dgrad(ws[0], d), E.w1x1_fwd(ws[1], d), E.w1x1_dgrad(ws[1], d),
                  E.wT_fwd(ws[2], d), E.wT_dgrad(ws[2], d), E.w3x3_fwd(ws[3], d, 8),
                  E.w3x3_fwd(ws[4], d, 48), E.w3x3_dgrad(ws[4], d, 64), E.w3x3_fwd(ws[5], d), E.w3x3_dgrad(ws[5], d),
                  E.w3x3_fwd(ws[6], d), E.w3x3_dgrad(ws[6], d)]
        single = [t.clone() for t in single]
        for w in ws:
            w.mul_(1.0)  # bump the version: every image is stale
        E.refresh_weights(ws)
        batched = [E.w3x3_fwd(ws[0], d), E.w3x3_dgrad(ws[0], d), E.w1x1_fwd(ws[1], d), E.w1x1_dgrad(ws[1], d),
                   E.wT_fwd(ws[2], d), E.wT_dgrad(ws[2], d), E.w3x3_fwd(ws[3], d, 8),
                   E.w3x3_fwd(ws[4], d, 48), E.w3x3_dgrad(ws[4], d, 64), E.w3x3_fwd(ws[5], d), E.w3x3_dgrad(ws[5], d),
                  E.w3x3_fwd(ws[6], d), E.w3x3_dgrad(ws[6], d)]
        for a, b in zip(single, batched):
            assert torch.equal(a, b)
    # the round-4 tap-merged path is the one taken for the 3x3 images (and the ConvT input-gradient image)
    jobs = []
    with K.record_permutes() as rec:
        for w in ws:
            w.mul_(1.0)
        E.refresh_weights(ws)
        jobs = rec.jobs
    modes = [K.perm_mode(j[2], j[3], j[4]) for j in jobs]
    assert modes.count(4) >= 5, modes   # w3x3 fwd / dgrad of ws[0], ws[4] and the wT dgrad image
    assert modes.count(5) >= 1, modes   # the channels_last weight's forward image without padding
    assert modes.count(0) >= 2, modes   # the channels_last weights' input-gradient images: 64 x 64 transposes


@pytest.mark.parametrize("shape", [(8, 3, 64, 96), (3, 3, 17, 29), (2, 1, 5, 7), (1, 8, 16, 16)])
@pytest.mark.parametrize("cl", [True, False])
@pytest.mark.parametrize("d", [0, 1])
def test_input_pack_8_channels(shape, cl, d):
    """vu_input_pack to 8 channels (the image packing of inc.0 / the ResNet
    stem, one pixel per thread since round 4): the zero-padded NHWC copy,
    bit-exact (bf16 by round-to-nearest-even as torch's .to(bfloat16))."""
    K, _ = _k()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(*shape, generator=g).to(DEV)
    if cl:
        x = x.contiguous(memory_format=CL)
    y = K.input_pack(x, 8, d)
    N, C, H, W = shape
    ref = torch.zeros(N, 8, H, W, device=DEV)
    ref[:, :C] = x
    ref = ref.to(torch.bfloat16 if d == 1 else torch.float32)
    assert torch.equal(y.permute(0, 2, 3, 1).contiguous(), ref.permute(0, 2, 3, 1).contiguous())


@pytest.mark.parametrize("case", [
    # (N, cin, cout, k, H) of a stride-2 conv (ResNet34 downsampling convs and their 1x1 shortcuts)
    (8, 128, 256, 3, 64), (8, 256, 512, 3, 32), (8, 64, 128, 1, 128), (8, 256, 512, 1, 32), (2, 64, 128, 3, 30),
    (2, 64, 128, 3, 31)])
@pytest.mark.parametrize("zi", [True, False])
@pytest.mark.parametrize("acc", [False, True])
def test_conv_stride2_input_grad_parity_classes(case, zi, acc):
    """stride-2 input gradient, bf16 storage, vs torch's conv2d_input: 3x3 as
    one stride-1 conv over the zero-inserted dy (zi, vu_zero_insert2 + the
    halo kernels; the default) or as four parity-class GEMMs scattered onto
    the sub-lattices (out_mode 2; gemm_fwd2.hip small-grid mode incl. split-K
    finish, or the generic kernel) -- 1x1 shortcuts always the latter;
    overwrite and accumulate."""
    from vaeunet_amd import _lib, vae_engine as V, engine as E
    N, ci, co, k, H = case
    g = torch.Generator().manual_seed(3)
    conv = torch.nn.Conv2d(ci, co, k, stride=2, padding=k // 2, bias=False)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(co, ci, k, k, generator=g) / (k * ci ** 0.5))
    conv = conv.to(DEV)
    Ho = (H + 2 * (k // 2) - k) // 2 + 1
    dy = torch.randn(N, co, Ho, Ho, generator=g).to(torch.bfloat16).float()

    class _M:
        d = _lib.BF16

        @staticmethod
        def act(n, c, h, w):
            return K.empty_act(n, c, h, w, torch.bfloat16, DEV)

    K, _ = _k()
    base = torch.randn(N, ci, H, H, generator=g).to(torch.bfloat16).float()
    dx = _act(base, "bf16") if acc else torch.empty(N, ci, H, H, dtype=torch.bfloat16, device=DEV).contiguous(
        memory_format=CL)
    old = E.S2_ZERO_INSERT_DGRAD
    E.S2_ZERO_INSERT_DGRAD = zi
    try:
        V.conv_dgrad(_M, _act(dy, "bf16"), conv, dx, acc)
        torch.cuda.synchronize()
    finally:
        E.S2_ZERO_INSERT_DGRAD = old
    wq = conv.weight.detach().cpu().to(torch.bfloat16).float()
    ref = torch.nn.grad.conv2d_input((N, ci, H, H), wq, dy, stride=2, padding=k // 2)
    sab = torch.nn.grad.conv2d_input((N, ci, H, H), wq.abs(), dy.abs(), stride=2, padding=k // 2)
    _close(dx, ref + base if acc else ref, "bf16", what="stride-2 dgrad", sabs=sab, acc=ref if acc else None)


@pytest.mark.parametrize("shape", [(2, 64, 17, 23, 2), (1, 128, 9, 9, 1), (3, 64, 64, 64, 3), (1, 32, 5, 3, 4)])
@pytest.mark.parametrize("d", [0, 1])
def test_outconv_pointwise_fwd(shape, d):
    """OutConv's 1x1 -> J <= 4 logits (vu_pointwise_fwd, unet_parts.py:97-103),
    ragged pixel tails included (the round-4 clamped, unguarded row loads):
    vs torch fp32 conv2d of the same (bf16-rounded) input, per element within
    fp32 summation-order error."""
    import types
    import torch.nn.functional as F
    from vaeunet_amd import engine as E
    N, C, H, W, J = shape
    g = torch.Generator().manual_seed(11)
    conv = torch.nn.Conv2d(C, J, 1).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(J, C, 1, 1, generator=g) / C ** 0.5)
        conv.bias.copy_(torch.randn(J, generator=g))
    x = torch.randn(N, C, H, W, generator=g).to(DEV, torch.bfloat16 if d == 1 else torch.float32)
    x = x.contiguous(memory_format=CL)
    y, _ = E.outconv_fwd(types.SimpleNamespace(d=d), conv, x)
    with torch.no_grad():
        ref = F.conv2d(x.float(), conv.weight, conv.bias)
        mag = F.conv2d(x.float().abs(), conv.weight.abs()) + conv.bias.abs()[None, :, None, None]
    assert y.shape == ref.shape
    assert ((y - ref).abs() <= 1e-5 * mag + 1e-6).all(), float((y - ref).abs().max())
