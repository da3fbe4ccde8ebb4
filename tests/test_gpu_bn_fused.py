"""Single-launch small-tensor BatchNorm forward (vu_bn_fwd_fused, bn.hip) vs the
two-launch finalize + apply path (vu_bn_finalize + vu_bn_apply /
vu_bn_add_relu) and vs torch's batch statistics (unet_parts.py:41-45,
unet_resnet.py BasicBlock tail)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _k():
    from vaeunet_amd import kernels as K
    return K


def _stats(y, tile):
    """per-tile (sum, centered M2) partials of an NHWC tensor, as the GEMM epilogues emit them"""
    K = _k()
    N, C, H, W = y.shape
    flat = y.permute(0, 2, 3, 1).reshape(-1, C).double().cpu()
    P = flat.shape[0]
    tiles = (P + tile - 1) // tile
    ps = torch.zeros(tiles, C, dtype=torch.float64)
    pm = torch.zeros(tiles, C, dtype=torch.float64)
    for t in range(tiles):
        blk = flat[t * tile:(t + 1) * tile]
        ps[t] = blk.sum(0)
        pm[t] = ((blk - blk.mean(0)) ** 2).sum(0)
    return K.Stats(ps.float().to(DEV), pm.float().to(DEV), tiles, tile, P)


CASES = [
    # (N, C, H, W, residual: None | "plain" | "bn")
    (8, 256, 32, 32, None),     # 64 tiles (ResNet34 layer3)
    (8, 512, 16, 16, "plain"),  # 16 tiles, identity residual (layer4 BasicBlock tail)
    (8, 128, 64, 64, "bn"),     # 256 tiles, downsample residual with its own BN
    (2, 96, 10, 12, None),      # ragged pixel count (tile tail), 3 channel groups
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", CASES)
def test_bn_fwd_fused_matches_two_launch_path(case, dt):
    K = _k()
    from vaeunet_amd import _lib
    N, C, H, W, resk = case
    d = _lib.BF16 if dt == torch.bfloat16 else _lib.F32
    g = torch.Generator().manual_seed(7)
    y = (torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(dt).to(DEV).contiguous(memory_format=torch.channels_last)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    st = _stats(y, 128)
    res = rcoef = None
    if resk is not None:
        res = torch.randn(N, C, H, W, generator=g).to(dt).to(DEV).contiguous(memory_format=torch.channels_last)
        if resk == "bn":
            rcoef = torch.stack([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)]).to(DEV)
    out = torch.empty_like(y)
    rm, rv, nbt = torch.zeros(C, device=DEV), torch.ones(C, device=DEV), torch.zeros((), dtype=torch.int64, device=DEV)
    assert K.query("vu_bn_fwd_fused_supported", st.tiles, C, K.pstride(y), K.pstride(y), K.pstride(out))
    coef = K.bn_forward_fused(st, C, gamma, beta, rm, rv, nbt, 0.1, 1e-5, y, out, True, d, res=res, rcoef=rcoef)
    assert coef is not None
    # reference: the two-launch path on the same partials
    rm2, rv2, nbt2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV), torch.zeros((), dtype=torch.int64,
                                                                                        device=DEV)
    coef2 = K.bn_finalize(st, C, gamma, beta, rm2, rv2, nbt2, 0.1, 1e-5)
    out2 = torch.empty_like(y)
    if res is None:
        K.bn_apply(y, out2, coef2, True, d)
    else:
        K.call("vu_bn_add_relu", K.ptr(y), K.pstride(y), K.ptr(coef2[0]), K.ptr(coef2[1]), K.ptr(res), K.pstride(res),
               K.ptr(rcoef[0]) if rcoef is not None else None, K.ptr(rcoef[1]) if rcoef is not None else None,
               N * H * W, C, K.ptr(out2), K.pstride(out2), d, K.stream())
    torch.cuda.synchronize()
    # same fp64 combine up to summation order: coefficients to a few fp32 ulps
    torch.testing.assert_close(coef, coef2, rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(rm, rm2, rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(rv, rv2, rtol=2e-6, atol=1e-7)
    assert int(nbt) == int(nbt2) == 1
    tol = dict(rtol=1e-2, atol=1e-2) if dt == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out.float(), out2.float(), **tol)
    # and against torch's batch statistics
    yf = y.float()
    mean, var = yf.mean((0, 2, 3)), yf.var((0, 2, 3), unbiased=False)
    torch.testing.assert_close(coef[2], mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(coef[3], 1.0 / torch.sqrt(var + 1e-5), rtol=1e-4, atol=1e-5)
    z = (yf - mean[None, :, None, None]) / torch.sqrt(var + 1e-5)[None, :, None, None] * gamma[None, :, None, None] \
        + beta[None, :, None, None]
    if res is not None:
        r = res.float()
        if rcoef is not None:
            r = r * rcoef[0][None, :, None, None] + rcoef[1][None, :, None, None]
        z = z + r
    torch.testing.assert_close(out.float(), torch.relu(z), **(dict(rtol=2e-2, atol=3e-2) if dt == torch.bfloat16
                                                            else dict(rtol=1e-4, atol=1e-4)))


BWD_CASES = [
    # (N, C, H, W, relu, train)
    (8, 256, 32, 32, True, True),
    (8, 512, 16, 16, False, True),
    (8, 128, 64, 64, True, True),    # 128 partial blocks: the largest the fused path takes
    (2, 64, 10, 12, True, False),    # eval-mode statistics (constants), ragged pixel count
    (3, 128, 7, 9, True, True),      # bf16 one-launch path (P <= 8192): P not a multiple of its 512 lanes
    (2, 64, 64, 64, True, True),     # P = 8192: the largest the bf16 one-launch path takes
]


@pytest.mark.parametrize("onepass", [0, 1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", BWD_CASES)
def test_bn_bwd_fused_matches_three_launch_path(case, dt, onepass):
    """vu_bn_bwd_fused (partial pass + fp64 finish folded into the apply; bf16
    tensors of <= 8192 pixels: the one-launch kernel) vs vu_bn_bwd_reduce +
    vu_bn_bwd_apply, and vs torch autograd of BN(+ReLU)."""
    K = _k()
    from vaeunet_amd import _lib
    N, C, H, W, relu, train = case
    d = _lib.BF16 if dt == torch.bfloat16 else _lib.F32
    g = torch.Generator().manual_seed(11)
    cl = torch.channels_last
    x = (torch.randn(N, C, H, W, generator=g) + 0.3).to(dt).to(DEV).contiguous(memory_format=cl)
    dy = torch.randn(N, C, H, W, generator=g).to(dt).to(DEV).contiguous(memory_format=cl)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    xf = x.float()
    mean, var = xf.mean((0, 2, 3)), xf.var((0, 2, 3), unbiased=False)
    invstd = 1.0 / torch.sqrt(var + 1e-5)
    coef = torch.stack([gamma * invstd, beta - mean * gamma * invstd, mean, invstd]).contiguous()
    assert K.query("vu_bn_bwd_fused_supported", N * H * W, C, K.pstride(dy), K.pstride(x), K.pstride(x))
    outs = []
    _lib.call("vu_gemm_set_tuning", 31, onepass)   # VU_TUNE_BN_ONEPASS (bf16, P <= 8192; off by default)
    try:
        for fused in (True, False):
            dx = torch.empty_like(x)
            dg, db = torch.full((C,), 0.25, device=DEV), torch.full((C,), -0.5, device=DEV)
            K.bn_backward(dy, x, coef, gamma, relu, dg, db, True, dx, d, train=train, fused=fused)
            outs.append((dx, dg, db))
        torch.cuda.synchronize()
    finally:
        _lib.call("vu_gemm_set_tuning", 31, 0)
    (dx1, dg1, db1), (dx2, dg2, db2) = outs
    torch.testing.assert_close(dg1, dg2, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db1, db2, rtol=1e-5, atol=1e-4)
    tol = dict(rtol=1e-2, atol=1e-2) if dt == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dx1.float(), dx2.float(), **tol)
    # torch autograd reference (fp32, the same stored inputs; accumulate onto 0.25 / -0.5)
    xr = xf.detach().clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    if train:
        z = torch.nn.functional.batch_norm(xr, None, None, gr, br, training=True, eps=1e-5)
    else:
        z = torch.nn.functional.batch_norm(xr, mean, var, gr, br, training=False, eps=1e-5)
    if relu:
        z = torch.relu(z)
    z.backward(dy.float())
    torch.testing.assert_close(dg1, gr.grad + 0.25, rtol=1e-3, atol=2e-2)
    torch.testing.assert_close(db1, br.grad - 0.5, rtol=1e-3, atol=2e-2)
    torch.testing.assert_close(dx1.float(), xr.grad, **(dict(rtol=3e-2, atol=3e-2) if dt == torch.bfloat16
                                                       else dict(rtol=1e-3, atol=1e-4)))


POOL_CASES = [
    # (N, C, H, W, relu, train, skip gradient)
    (2, 64, 32, 48, True, True, True),
    (2, 128, 16, 16, True, True, False),
    (1, 64, 8, 12, False, True, True),     # no ReLU between the BN and the pool
    (2, 64, 6, 8, True, False, True),      # eval-mode statistics
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", POOL_CASES)
def test_bn_bwd_through_maxpool(case, dt):
    """vu_bn_bwd_pool (the BN(+ReLU) backward read through the following 2x2
    max-pool: activation, argmax and pool-input gradient recomputed per window)
    vs the materialised path: vu_bn_apply_maxpool2's activation, vu_maxpool2_bwd
    (+ skip gradient) and the BN backward -- the BN sees bit-identical dz, so
    dgamma / dbeta agree to the summation order and dx to one rounding."""
    K = _k()
    from vaeunet_amd import _lib
    N, C, H, W, relu, train, skip = case
    d = _lib.BF16 if dt == torch.bfloat16 else _lib.F32
    g = torch.Generator().manual_seed(17)
    cl = torch.channels_last
    y = (torch.randn(N, C, H, W, generator=g) + 0.2).to(dt).to(DEV).contiguous(memory_format=cl)
    # ties in the pooled windows: repeat some values
    y[:, :, 1::4, :] = y[:, :, 0::4, :]
    dp = torch.randn(N, C, H // 2, W // 2, generator=g).to(dt).to(DEV).contiguous(memory_format=cl)
    add = torch.randn(N, C, H, W, generator=g).to(dt).to(DEV).contiguous(memory_format=cl) if skip else None
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    yf = y.float()
    mean, var = yf.mean((0, 2, 3)), yf.var((0, 2, 3), unbiased=False)
    invstd = 1.0 / torch.sqrt(var + 1e-5)
    coef = torch.stack([gamma * invstd, beta - mean * gamma * invstd, mean, invstd]).contiguous()
    # the forward: activation + pool in one pass, as the engine runs it
    act = torch.empty_like(y)
    pooled = torch.empty_like(dp)
    K.bn_apply_maxpool(y, act, pooled, coef, relu, d)
    ws8 = K.pstride(add) if add is not None else 8
    assert K.query("vu_bn_bwd_pool_supported", H, W, C, K.pstride(y), K.pstride(dp), ws8, K.pstride(y))
    dg1, db1 = torch.full((C,), 0.25, device=DEV), torch.full((C,), -0.5, device=DEV)
    dx1 = torch.empty_like(y)
    K.bn_backward_pool(dp, add, y, coef, gamma, relu, dg1, db1, True, dx1, d, train=train)
    da = torch.empty_like(y)
    K.maxpool_bwd(act, dp, da, add, d)
    dg2, db2 = torch.full((C,), 0.25, device=DEV), torch.full((C,), -0.5, device=DEV)
    dx2 = torch.empty_like(y)
    K.bn_backward(da, y, coef, gamma, relu, dg2, db2, True, dx2, d, train=train, fused=False)
    torch.cuda.synchronize()
    torch.testing.assert_close(dg1, dg2, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db1, db2, rtol=1e-5, atol=1e-4)
    scale = float(dx2.float().abs().max())
    err = float((dx1.float() - dx2.float()).abs().max())
    assert err <= (2.0 ** -7 if dt == torch.bfloat16 else 1e-5) * scale, (err, scale)
