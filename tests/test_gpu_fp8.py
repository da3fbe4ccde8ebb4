"""fp8 (OCP e4m3fn) 3x3 conv path (BASELINE.json configs[4], csrc/conv_fp8.hip).

* the quantisers are bit-exact against torch.float8_e4m3fn (same fp32 scale,
  same clamp, round-to-nearest-even);
* the conv equals fp32 convolution of the DEQUANTISED operands (e4m3 products
  are exact in fp32; only the summation order and the bf16 output rounding
  differ), with BN partial statistics, bias, channel-slice output, 1-3
  concat sources and blocks that walk several tiles (grid cap);
* the error against the unquantised fp32 conv is only reported (the
  reference has no fp8 path) and loosely bounded here.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
CL = torch.channels_last
TUNE_FP8_GRID = 4


def _act(t, dtype=torch.bfloat16):
    return t.to(DEV, dtype).contiguous(memory_format=CL)


def _bytes(q):
    return q.cpu().contiguous().view(torch.uint8)


def test_quantize_bit_exact():
    from vaeunet_amd import fp8
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 64, 8, 16, generator=g) * 3
    x[0, :4, 0, 0] = torch.tensor([0.0, -0.0, 1e-3, -7.5])   # zeros, an e4m3-subnormal value
    for dtype in (torch.bfloat16, torch.float32):
        xd = _act(x, dtype)
        am = fp8.amax([xd])
        assert am.item() == xd.float().abs().max().item()
        q, dq = fp8.quantize(xd, am)
        s = torch.tensor(448.0, dtype=torch.float32) / am.cpu()
        qr = (xd.float().cpu() * s).clamp(-448, 448).to(torch.float8_e4m3fn)
        assert torch.equal(_bytes(q), _bytes(qr))
        assert dq.item() == (1.0 / s).item()


def test_quantize_rows_bit_exact():
    from vaeunet_amd import fp8
    g = torch.Generator().manual_seed(1)
    m = torch.randn(48, 576, generator=g)
    m[3] = 0.0                                                 # all-zero row: scale 1
    q, dq = fp8.quantize_rows(m.to(DEV))
    s = torch.tensor(448.0) / m.abs().amax(1)
    s[3] = 1.0
    qr = (m * s[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(_bytes(q), _bytes(qr))
    assert torch.equal(dq.cpu(), 1.0 / s)


FP8_CASES = [
    # (N, [cin per source], H, W, cout, grid cap)
    (1, [64], 8, 32, 256, 0),           # 256x256 tiles, one tile
    (2, [64], 16, 64, 256, 3),          # 8 tiles over 3 blocks
    (1, [64, 64], 16, 32, 384, 2),      # two sources, 512x128 tiles, 3 column tiles
    (2, [128], 32, 32, 128, 3),
    (2, [64], 32, 64, 64, 3),           # 1024x64 tiles
    (3, [64, 64, 64], 32, 32, 64, 2),   # three sources, odd chunk count
    (1, [64], 1024, 1024, 64, 0),       # config 5 layer shape: 64->64 at 1x64x1024x1024
    # small grids (tiles < CUs): split-K over chunk ranges + the deterministic finish
    (2, [1024], 32, 64, 256, 0),        # 16 tiles -> 2 splits (capped: >= 8 chunks per split)
    (1, [512, 512], 32, 32, 256, 0),    # two sources, the splits meet at the source boundary
    (1, [512, 1024], 32, 32, 256, 0),   # 24 chunks over 3 splits, one inside the second source
]


@pytest.mark.parametrize("case", FP8_CASES)
def test_conv3x3_fp8(case):
    from vaeunet_amd import _lib, fp8
    N, cins, H, W, co, cap = case
    g = torch.Generator().manual_seed(7)
    xs = [torch.randn(N, c, H, W, generator=g) for c in cins]
    cin = sum(cins)
    w = torch.randn(co, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    b = torch.randn(co, generator=g)
    _lib.call("vu_gemm_set_tuning", TUNE_FP8_GRID, cap)
    try:
        srcs = [_act(x) for x in xs]
        am = fp8.amax(srcs)
        qs, dq = [], None
        for t in srcs:
            q, dq = fp8.quantize(t, am)
            qs.append(q)
        wq, ws = fp8.quantize_weight(w.to(DEV))
        out, st = fp8.conv3x3(qs, dq, wq, ws, co, bias=b.to(DEV), stats=True)
        # fp32 conv of the dequantised operands
        xd = torch.cat([q.cpu().float() for q in qs], 1) * dq.item()
        wd = (wq.cpu().float() * ws.cpu()[:, None]).view(co, 3, 3, cin).permute(0, 3, 1, 2)
        ref = F.conv2d(xd, wd, b, padding=1)
        got = out.float().cpu()
        err = (got - ref).abs()
        # bf16 output rounding (half an ulp of the stored value's binade) plus
        # fp32 summation-order noise of the K-term dot products
        # (|err_sum| <~ sqrt(K) * 2^-24 * sum_k |x_k w_k|, bounded by 1e-5 * that sum)
        s_abs = F.conv2d(xd.abs(), wd.abs(), b.abs(), padding=1)
        bound = 2.0 ** -8 * torch.maximum(ref.abs(), got.abs()) + 1e-5 * s_abs + 1e-6 * ref.abs().max()
        assert (err <= bound).all(), (f"max err {err.max().item():.3e}, "
                                      f"{int((err > bound).sum())} elements off")
        # BN partials of the stored bf16 values
        n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)],
                         dtype=torch.float64)
        s = st.psum.double().cpu()
        mean = s.sum(0) / n.sum()
        m2 = st.pm2.double().cpu() + n[:, None] * (s / n[:, None] - mean) ** 2
        torch.testing.assert_close(mean.float(), got.mean((0, 2, 3)), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close((m2.sum(0) / n.sum()).float(), got.var((0, 2, 3), unbiased=False),
                                   rtol=1e-4, atol=1e-5)
        # channel-slice output of a wider tensor
        wide = torch.zeros(N, co + 64, H, W, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
        fp8.conv3x3(qs, dq, wq, ws, co, out=wide, out_coff=64, bias=b.to(DEV))
        assert torch.equal(wide[:, 64:].float().cpu(), got)
        assert not wide[:, :64].any()
        # reported: error vs the unquantised conv (loose bound only)
        full = F.conv2d(torch.cat([x.bfloat16().float() for x in xs], 1), w, b, padding=1)
        rel = ((got - full).abs().max() / full.abs().max()).item()
        assert rel < 0.1, rel
    finally:
        _lib.call("vu_gemm_set_tuning", TUNE_FP8_GRID, 0)


def test_fp8_rejects_unserved_shapes():
    from vaeunet_amd import fp8
    x = _act(torch.randn(1, 32, 8, 32))          # 32 channels: not a whole 64-channel chunk
    w = torch.randn(64, 32, 3, 3, device=DEV)
    with pytest.raises(ValueError):
        fp8.conv3x3_q([x], w)


def test_double_conv_fp8_close_to_bf16_path():
    """DoubleConv forward with fp8 convs vs the bf16 path (train-mode BN)."""
    from vaeunet_amd import DoubleConv, fp8
    torch.manual_seed(3)
    mod = DoubleConv(64, 64).to(DEV)
    x = _act(torch.randn(2, 64, 32, 64))
    y8 = fp8.double_conv_forward(mod, x).float()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        yb = mod(x).float()
    rel = ((y8 - yb).abs().max() / yb.abs().max()).item()
    assert rel < 0.15, rel


TUNE_FP8_C64 = 23


@pytest.mark.parametrize("shape", [(1, 1024, 1024), (2, 256, 512), (3, 256, 384), (2, 256, 512, 2), (1, 512, 512, 1)])
def test_conv3x3_fp8_c64_matches_step_loop(shape):
    """64 -> 64 fp8 conv on the resident-weight tile-stream kernel (default for
    these shapes; LDS-staged (2) and direct (1) output stores) vs the
    step-loop kernel (0): the same taps in the same order on
    the same 32x32x64 MFMA fragments, so the bf16 outputs are bit-identical;
    the BN partials (64- vs 128-pixel tiles) combine to the same moments."""
    from vaeunet_amd import _lib, fp8
    # (N, H, W[, k]): k = 2 -> 128 input channels as two 64-channel sources,
    # k = 1 -> one 128-channel source (the two-chunk resident-weight variant)
    N, H, W = shape[:3]
    cins = [64] if len(shape) == 3 else ([64, 64] if shape[3] == 2 else [128])
    g = torch.Generator().manual_seed(11)
    xs = [torch.randn(N, c, H, W, generator=g) for c in cins]
    w = torch.randn(64, sum(cins), 3, 3, generator=g) / (3 * sum(cins) ** 0.5)
    b = torch.randn(64, generator=g)
    xa = [_act(x) for x in xs]
    am = fp8.amax(xa)
    qs = []
    for t in xa:
        q, dq = fp8.quantize(t, am)
        qs.append(q)
    wq, ws = fp8.quantize_weight(w.to(DEV))
    res = {}
    for c64 in (2, 1, 0):
        _lib.call("vu_gemm_set_tuning", TUNE_FP8_C64, c64)
        try:
            out, st = fp8.conv3x3(qs, dq, wq, ws, 64, bias=b.to(DEV), stats=True)
            torch.cuda.synchronize()
            res[c64] = (out, st)
        finally:
            _lib.call("vu_gemm_set_tuning", TUNE_FP8_C64, 2)
    (o2, s2), (o1, s1), (o0, s0) = res[2], res[1], res[0]
    assert s2.tile_rows == 64 and s1.tile_rows == 64 and s0.tile_rows == 128
    assert torch.equal(o1, o0)
    assert torch.equal(o2, o0)
    assert torch.equal(s2.psum, s1.psum) and torch.equal(s2.pm2, s1.pm2)

    def moments(st):
        n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)],
                         dtype=torch.float64)
        s = st.psum.double().cpu()
        mean = s.sum(0) / n.sum()
        m2 = st.pm2.double().cpu() + n[:, None] * (s / n[:, None] - mean) ** 2
        return mean, m2.sum(0) / n.sum()
    m1, v1 = moments(s1)
    m0, v0 = moments(s0)
    torch.testing.assert_close(m1, m0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(v1, v0, rtol=1e-5, atol=1e-6)


TUNE_FP8_SPLIT = 24


def test_conv3x3_fp8_split_matches_unsplit():
    """split-K (default for small grids) vs one block per tile: same MACs,
    partial tiles scaled before the fp32 slab sum -> equal to fp32 rounding of
    the accumulation, i.e. bf16 outputs within one rounding step."""
    from vaeunet_amd import _lib, fp8
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 1024, 64, 64, generator=g)
    w = torch.randn(512, 1024, 3, 3, generator=g) / (3 * 1024 ** 0.5)
    xa = _act(x)
    am = fp8.amax([xa])
    q, dq = fp8.quantize(xa, am)
    wq, ws = fp8.quantize_weight(w.to(DEV))
    outs = []
    for sp in (1, 0):
        _lib.call("vu_gemm_set_tuning", TUNE_FP8_SPLIT, sp)
        try:
            from vaeunet_amd._lib import VuConvFp8  # noqa: F401
            out, st = fp8.conv3x3([q], dq, wq, ws, 512, stats=True)
            torch.cuda.synchronize()
            outs.append((out.float().cpu(), st))
        finally:
            _lib.call("vu_gemm_set_tuning", TUNE_FP8_SPLIT, 1)
    (a, sa), (b, sb) = outs
    torch.testing.assert_close(a, b, rtol=8e-3, atol=1e-3)
    # (the finish's statistics tiles are 128 consecutive pixels, the kernel's
    # its wave tiles: compare the combined moments)
    for st, ref in ((sa, a), (sb, b)):
        mean = st.psum.double().sum(0).cpu() / st.rows
        torch.testing.assert_close(mean.float(), ref.mean((0, 2, 3)), rtol=1e-4, atol=1e-5)


def _q8_ref(x, sc, sh, relu, am_prev):
    """CPU restatement of vu_bn_apply_fp8: z = x*sc + sh (two fp32 roundings),
    relu, q = e4m3(clamp(z * 448/am_prev, +-448))."""
    xf = x.float().cpu()
    z = xf if sc is None else xf * sc.cpu()[None, :, None, None] + sh.cpu()[None, :, None, None]
    if relu:
        z = z.clamp_min(0.0)
    s = torch.tensor(448.0) / torch.tensor(am_prev) if am_prev > 0 else torch.tensor(1.0)
    return z, (z * s).clamp(-448, 448).to(torch.float8_e4m3fn), s


@pytest.mark.parametrize("C_,dtype,slot", [(64, torch.bfloat16, 0), (128, torch.bfloat16, 2),
                                            (512, torch.float32, 1), (8, torch.bfloat16, 1)])
def test_bn_apply_fp8_bit_exact(C_, dtype, slot):
    """Fused BN apply + ReLU + e4m3 quantise with the delayed scale: bytes equal
    the unfused restatement; the next slot receives max |z| exactly, the one
    after is cleared, dq = 1/s; values above the stale amax saturate."""
    from vaeunet_amd import fp8
    g = torch.Generator().manual_seed(C_)
    x = torch.randn(2, C_, 9, 23, generator=g) * 2
    sc = torch.randn(C_, generator=g)
    sh = torch.randn(C_, generator=g) * 0.3
    xd = _act(x, dtype)
    ds = fp8.DelayedScale(DEV)
    ds.t = slot
    for relu, am_prev in ((True, 1.75), (False, 40.0)):     # 1.75: far below max|z| -> saturation
        ring = torch.tensor([5.0, 5.0, 5.0])
        ring[slot] = am_prev
        ds.ring.copy_(ring)
        q, dq = fp8.bn_apply_quant(xd, (sc.to(DEV), sh.to(DEV)), relu, ds)
        z, qr, s = _q8_ref(xd, sc, sh, relu, am_prev)
        assert torch.equal(_bytes(q), _bytes(qr))
        assert dq.item() == (1.0 / s).item()
        r = ds.ring.cpu()
        assert r[slot].item() == am_prev
        assert r[(slot + 1) % 3].item() == max(5.0, z.abs().max().item())   # max-accumulated
        assert r[(slot + 2) % 3].item() == 0.0
    # calibration: max|z| into the read slot only, nothing stored
    ds.ring.zero_()
    fp8.calibrate(xd, None, False, ds)
    assert ds.ring.cpu()[slot].item() == xd.float().abs().max().item()
    assert ds.ring.cpu().count_nonzero().item() == 1


def test_bn_apply_fp8_rejects_unserved_channels():
    from vaeunet_amd import _lib, fp8
    xd = _act(torch.randn(1, 24, 4, 4))                       # 24 / 8 = 3: not a power of two
    with pytest.raises(Exception):
        fp8.bn_apply_quant(xd, None, True, fp8.DelayedScale(DEV))
    assert _lib is not None


@pytest.mark.parametrize("up", [False, True])
def test_double_conv_fp8_delayed_scaling(up):
    """Delayed-scaling fp8 DoubleConv over three steps of the same batch
    (train-mode BN: same batch statistics, so the recorded amax is the one
    the just-in-time path computes): close to the just-in-time fp8 path and
    to the bf16 path every step; the rings carry amax(x) and max BN1 output."""
    from vaeunet_amd import DoubleConv, fp8
    torch.manual_seed(4)
    cins = [64, 64] if up else [64]
    mod = DoubleConv(sum(cins), 128).to(DEV)
    xs = [_act(torch.randn(2, c, 32, 64).relu()) for c in cins]
    yj = fp8.double_conv_forward(mod, xs, delayed=False).float()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        yb = mod(torch.cat(xs, 1)).float()
    for step in range(3):
        yd = fp8.double_conv_forward(mod, xs, delayed=True).float()
        assert ((yd - yj).abs().max() / yj.abs().max()).item() < 0.03, step
        assert ((yd - yb).abs().max() / yb.abs().max()).item() < 0.15, step
        ds_in, ds_mid, _ = mod._vu_fp8_scales
        assert ds_in.t == step + 1
        assert ds_in.ring[ds_in.slot].item() == max(float(t.float().abs().max()) for t in xs)
        assert ds_mid.ring[ds_mid.slot].item() > 0


def test_double_conv_fp8_default_is_self_contained():
    """the default forward scales just in time, so a second call on
    a 4x-larger input is not clipped by the first call's amax; a delayed call
    after reset_scales calibrates again (equal to just-in-time on its first
    call); chained arguments on the just-in-time path are refused only on the
    round-5 two-pass form (JIT_MINMAX False)."""
    from vaeunet_amd import DoubleConv, fp8
    torch.manual_seed(8)
    mod = DoubleConv(64, 64).to(DEV)
    x = _act(torch.randn(2, 64, 32, 64).relu())
    x4 = _act(4.0 * torch.randn(2, 64, 32, 64).relu())
    fp8.double_conv_forward(mod, x)
    y_default = fp8.double_conv_forward(mod, x4).float()
    fresh = DoubleConv(64, 64).to(DEV)
    fresh.load_state_dict(mod.state_dict())
    y_fresh = fp8.double_conv_forward(fresh, x4).float()
    assert torch.equal(y_default, y_fresh)
    fp8.double_conv_forward(mod, x, delayed=True)     # history at x's range
    fp8.reset_scales(mod)
    y_cal = fp8.double_conv_forward(mod, x4, delayed=True).float()   # calibrates on x4
    assert ((y_cal - y_fresh).abs().max() / y_fresh.abs().max()).item() < 0.03
    old = fp8.JIT_MINMAX
    try:
        fp8.JIT_MINMAX = False
        with pytest.raises(ValueError):
            fp8.double_conv_forward(mod, None, x_q=([x], torch.ones(1, device=DEV)))
    finally:
        fp8.JIT_MINMAX = old


@pytest.mark.parametrize("up", [False, True])
def test_double_conv_fp8_jit_chained(up):
    """Chained just-in-time blocks (round 6): an e4m3 input quantised just in
    time by the producer gives the bf16-input block's output bit for bit (the
    same exact amax, the same quantiser); the e4m3 output's scale is the exact
    max of relu(BN2(y2)) from conv2's min / max epilogue (the largest code is
    448) and its dequantised values are the bf16-output block's up to one
    e4m3 rounding."""
    from vaeunet_amd import DoubleConv, fp8
    torch.manual_seed(9)
    cins = [64, 64] if up else [64]
    mod = DoubleConv(sum(cins), 64 if up else 128).to(DEV)
    xs = [_act(torch.randn(2, c, 64, 128).relu()) for c in cins]
    ref = fp8.double_conv_forward(mod, xs)                   # bf16 in, bf16 out
    ds = fp8.DelayedScale(DEV)
    for t in xs:
        fp8.calibrate(t, None, False, ds)
    qs = []
    for t in xs:
        q, xdq = fp8.bn_apply_quant(t, None, False, ds)
        qs.append(q)
    y = fp8.double_conv_forward(mod, None, x_q=(qs, xdq))     # e4m3 in, bf16 out
    assert torch.equal(y, ref)
    q, dq = fp8.double_conv_forward(mod, None, x_q=(qs, xdq), out_fp8=True)
    assert q.dtype == fp8.E4M3
    assert q.float().abs().max().item() == 448.0
    got, r = q.float() * dq, ref.float()
    err = (got - r).abs()
    assert (err <= 2.0 ** -3 * r.abs() + 1e-3 * r.abs().max()).all()


def test_double_conv_fp8_chained():
    """Chained fp8 blocks: an e4m3 input from the producer (x_q) and an e4m3
    output (BN2 apply fused with the quantise, its own delayed scale): the
    dequantised output is the bf16-output block's result up to one e4m3
    rounding (relative step 2^-3 below 448, saturation above the stale amax),
    every step."""
    from vaeunet_amd import DoubleConv, fp8
    torch.manual_seed(6)
    mod = DoubleConv(64, 64).to(DEV)
    x = _act(torch.randn(2, 64, 32, 64).relu())
    ds = fp8.DelayedScale(DEV)
    fp8.calibrate(x, None, False, ds)
    xq, xdq = fp8.bn_apply_quant(x, None, False, ds)
    for step in range(3):
        ref = fp8.double_conv_forward(mod, None, delayed=True, x_q=([xq], xdq))   # same input, bf16 output
        q, dq = fp8.double_conv_forward(mod, None, delayed=True, x_q=([xq], xdq), out_fp8=True)
        got = q.float() * dq
        err = (got - ref.float()).abs()
        assert (err <= 2.0 ** -3 * ref.float().abs() + 1e-3 * ref.float().abs().max()).all(), step


# (N, [cin per source], H, W, cout): the step-loop kernel (256 / 128 / 64
# column tiles) and the two resident-weight 64-channel kernels (one and two
# 64-channel chunks)
MINMAX_CASES = [
    (2, [64], 16, 64, 256),
    (2, [128], 32, 32, 128),
    (2, [64], 32, 64, 64),
    (2, [64], 256, 512, 64),        # resident weights, one chunk (512 tiles)
    (2, [64, 64], 256, 512, 64),    # resident weights, two chunks
]


@pytest.mark.parametrize("case", MINMAX_CASES)
def test_conv3x3_fp8_minmax_partials(case):
    """VuConvFp8.stat_min / stat_max (round 6): per statistics tile and
    channel, the min / max of the stored bf16 output -- combined over the
    tiles they equal the output's per-channel min / max exactly; and
    vu_fp8_relu_amax on them equals, bit for bit, the max |relu(y*s + t)|
    that vu_bn_apply_fp8's calibration pass measures over every element."""
    from vaeunet_amd import fp8
    N, cins, H, W, co = case
    g = torch.Generator().manual_seed(19)
    xs = [_act(torch.randn(N, c, H, W, generator=g).relu()) for c in cins]
    w = torch.randn(co, sum(cins), 3, 3, generator=g) / (3 * sum(cins) ** 0.5)
    am = fp8.amax(xs)
    qs = []
    for t in xs:
        q, dq = fp8.quantize(t, am)
        qs.append(q)
    wq, ws = fp8.quantize_weight(w.to(DEV))
    y, st = fp8.conv3x3(qs, dq, wq, ws, co, stats=True, minmax=True)
    assert st.minmax is not None
    pmin, pmax = st.minmax
    yf = y.float()
    torch.testing.assert_close(pmin.min(0).values, yf.amin((0, 2, 3)), rtol=0, atol=0)
    torch.testing.assert_close(pmax.max(0).values, yf.amax((0, 2, 3)), rtol=0, atol=0)
    assert bool((pmin <= pmax).all())
    sc = (torch.rand(co, generator=g) * 2 - 0.5).to(DEV)    # some negative scales
    sh = (torch.randn(co, generator=g) * 0.3).to(DEV)
    for relu in (True, False):
        ds = fp8.relu_amax_scale(st.minmax, (sc, sh), relu, DEV)
        cal = fp8.DelayedScale(DEV)
        fp8.calibrate(y, (sc, sh), relu, cal)
        assert ds.ring[0].item() == cal.ring[0].item(), (relu, ds.ring[0].item(), cal.ring[0].item())
        assert ds.ring[1].item() == 0.0 and ds.ring[2].item() == 0.0


@pytest.mark.parametrize("up", [False, True])
def test_double_conv_fp8_jit_minmax_matches_two_pass(up):
    """Just-in-time DoubleConv (default, round 6: conv2's input scale from
    conv1's min / max epilogue, BN1 + ReLU fused with the quantise) against
    the round-5 form (BN1 apply to bf16, then amax + quantise passes): the
    same scale up to the bf16 rounding of the activation, so the outputs
    agree to the e4m3 quantisation step; and both stay close to bf16."""
    from vaeunet_amd import DoubleConv, fp8
    torch.manual_seed(6)
    cins = [64, 64] if up else [64]
    mod = DoubleConv(sum(cins), 64 if up else 128).to(DEV)
    xs = [_act(torch.randn(2, c, 256, 512).relu()) for c in cins]
    old = fp8.JIT_MINMAX
    try:
        fp8.JIT_MINMAX = True
        yn = fp8.double_conv_forward(mod, xs).float()
        fp8.JIT_MINMAX = False
        yo = fp8.double_conv_forward(mod, xs).float()
    finally:
        fp8.JIT_MINMAX = old
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        yb = mod(torch.cat(xs, 1)).float()
    assert ((yn - yo).abs().max() / yo.abs().max()).item() < 0.03
    assert ((yn - yb).abs().max() / yb.abs().max()).item() < 0.15
