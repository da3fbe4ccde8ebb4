"""BatchNorm-backward partial sums emitted by the input-gradient GEMM epilogue
(VuGemmFwd.bnb_part: the ping-pong kernel and its split-K finish) against torch on the stored output: per
channel sum dz and sum dz * xhat, dz = output masked by the forward ReLU --
the first stage of vu_bn_bwd_reduce (unet_parts.py:41-45 in train mode,
backward).  Finished by vu_bn_bwd_finish into dgamma / dbeta."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
TUNE_V4_MIN_BLOCKS, TUNE_V4_SPLITK, TUNE_V6 = 0, 6, 11


def _tune(*kv):
    from vaeunet_amd import _lib
    for k, v in kv:
        _lib.call("vu_gemm_set_tuning", k, v)


def _act(t):
    return t.to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)


CASES = [
    # (name, N, cout (dy channels), cin (dx / BN channels), H, W, tuning, expected tile)
    ("pp128", 2, 128, 128, 16, 32, ((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0)), 128),
    ("pp256", 2, 64, 256, 8, 64, ((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0)), 128),
    ("pp64", 1, 128, 64, 32, 32, ((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0)), 128),
    ("splitk_finish", 2, 128, 128, 16, 32, ((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 2)), 128),
]
DEFAULTS = ((TUNE_V4_MIN_BLOCKS, 256), (TUNE_V4_SPLITK, 1), (TUNE_V6, 1))


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("relu", [True, False])
def test_dgrad_epilogue_bn_backward_partials(case, relu):
    from vaeunet_amd import kernels as K, engine as E, _lib
    name, N, co, ci, H, W, tune, tile = case
    g = torch.Generator().manual_seed(17)
    w = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    dy = torch.randn(N, co, H, W, generator=g)
    x = torch.randn(N, ci, H, W, generator=g)           # the BN input (pre-normalisation)
    scale = torch.randn(ci, generator=g)
    shift = torch.randn(ci, generator=g)
    mean = torch.randn(ci, generator=g) * 0.1
    invstd = torch.rand(ci, generator=g) + 0.5
    coef = [t.to(DEV) for t in (scale, shift, mean, invstd)]
    d = _lib.BF16
    xs = _act(x)
    _tune(*tune)
    try:
        dx = K.empty_act(N, ci, H, W, torch.bfloat16, DEV)
        part = K.gemm_fwd(K.gather3x3([_act(dy)]), E.w3x3_dgrad(w.to(DEV), d), ci, dx, d, kind="dgrad",
                          bnb=(xs, coef, relu))
        assert part is not None and part.nblk * tile == N * H * W, name
        gamma = torch.rand(ci, generator=g).to(DEV)
        dgamma = torch.empty(ci, device=DEV)
        dbeta = torch.empty(ci, device=DEV)
        k = torch.empty(3, ci, device=DEV)
        ws = torch.empty(max(1, _lib.query("vu_bn_bwd_finish_workspace_bytes", part.nblk, ci) // 4), device=DEV)
        _lib.call("vu_bn_bwd_finish", K.ptr(part.part), part.nblk, N * H * W, ci, K.ptr(gamma), K.ptr(coef[3]), 1,
                  K.ptr(dgamma), K.ptr(dbeta), 0, K.ptr(k), K.ptr(ws), K.stream())
        # the same sums from the stored output, fp64 on the host
        dz = dx.double().cpu()
        xq = xs.double().cpu()
        if relu:
            keep = (xs.float().cpu() * scale[None, :, None, None] + shift[None, :, None, None]) > 0
            dz = dz * keep
        xhat = (xq - mean.double()[None, :, None, None]) * invstd.double()[None, :, None, None]
        s0 = dz.sum((0, 2, 3))
        s1 = (dz * xhat).sum((0, 2, 3))
        sc0 = dz.abs().sum((0, 2, 3)).max()
        sc1 = (dz * xhat).abs().sum((0, 2, 3)).max()
        torch.testing.assert_close(dbeta.double().cpu(), s0, rtol=0, atol=2e-6 * float(sc0))
        torch.testing.assert_close(dgamma.double().cpu(), s1, rtol=0, atol=2e-6 * float(sc1))
        # and the output itself is unchanged by the extra epilogue work
        ref = torch.nn.grad.conv2d_input((N, ci, H, W), w.to(torch.bfloat16).float(),
                                         dy.to(torch.bfloat16).float(), padding=1)
        err = (dx.float().cpu() - ref).abs().max() / ref.abs().max()
        assert err < 1e-2, err
    finally:
        _tune(*DEFAULTS)


@pytest.mark.parametrize("shape", [(1, 32, 24, 8, 8), (2, 64, 64, 32, 64)], ids=["generic", "v6"])
def test_unsupported_shapes_fall_back(shape):
    """A kernel without the epilogue (generic; the resident-weight 64 -> 64
    kernel, where it measured slower) reports tile 0 and gemm_fwd returns
    None: the engine then runs the separate vu_bn_bwd_reduce."""
    from vaeunet_amd import kernels as K, engine as E, _lib
    g = torch.Generator().manual_seed(3)
    N, co, ci, H, W = shape
    _tune((TUNE_V6, 3))
    w = torch.randn(co, ci, 3, 3, generator=g)
    dy = _act(torch.randn(N, co, H, W, generator=g))
    xs = _act(torch.randn(N, ci, H, W, generator=g))
    coef = [torch.ones(ci, device=DEV) for _ in range(4)]
    dx = K.empty_act(N, ci, H, W, torch.bfloat16, DEV)
    try:
        part = K.gemm_fwd(K.gather3x3([dy]), E.w3x3_dgrad(w.to(DEV), _lib.BF16), ci, dx, _lib.BF16, kind="dgrad",
                          bnb=(xs, coef, True))
    finally:
        _tune(*DEFAULTS)
    assert part is None
