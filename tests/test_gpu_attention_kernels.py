"""Attention-gate memory-bound kernels (attention.hip; AttentionGate,
unet_parts.py:7-30): the batched kernels (VU_TUNE_ATTN = 1, default) against
the one-row kernels (VU_TUNE_ATTN = 0) -- same pixel -> lane assignment and
summation order, so equal up to the compiler's fma contraction -- and the forward pair against
a torch fp32 restatement of psi / gate."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
TUNE_ATTN = 22


def _k():
    from vaeunet_amd import kernels as K
    return K


def _set(v):
    _k().call("vu_gemm_set_tuning", TUNE_ATTN, v)


def _run(dt, P, F, C, seed):
    K = _k()
    from vaeunet_amd import _lib
    d = _lib.BF16 if dt == torch.bfloat16 else _lib.F32
    g = torch.Generator().manual_seed(seed)
    ug = torch.randn(P, F, generator=g).to(dt).to(DEV)
    ux = torch.randn(P, F, generator=g).to(dt).to(DEV)
    co = [(torch.rand(F, generator=g) + 0.5).to(DEV), (torch.randn(F, generator=g) * 0.3).to(DEV),
          (torch.rand(F, generator=g) + 0.5).to(DEV), (torch.randn(F, generator=g) * 0.3).to(DEV)]
    wpsi = (torch.randn(F, generator=g) / F ** 0.5).to(DEV)
    bpsi = torch.randn(1, generator=g).to(DEV)
    x = torch.randn(P, C, generator=g).to(dt).to(DEV)
    dout = torch.randn(P, C, generator=g).to(dt).to(DEV)
    cq = torch.tensor([1.3, -0.2], device=DEV)
    dq = torch.randn(P, generator=g).to(DEV)
    tile = K.query("vu_attn_tile_rows")
    tiles = (P + tile - 1) // tile
    outs = {}
    for mode in (1, 0):
        _set(mode)
        try:
            q = torch.empty(P, device=DEV)
            psum, pm2 = torch.empty(tiles, device=DEV), torch.empty(tiles, device=DEV)
            K.call("vu_attn_psi_fwd", K.ptr(ug), K.ptr(ux), P, F, K.ptr(co[0]), K.ptr(co[1]), K.ptr(co[2]),
                   K.ptr(co[3]), K.ptr(wpsi), K.ptr(bpsi), K.ptr(q), K.ptr(psum), K.ptr(pm2), tile, d, K.stream())
            pmap = torch.empty(P, device=DEV)
            out = torch.empty_like(x)
            K.call("vu_attn_gate_fwd", K.ptr(q), K.ptr(cq), K.ptr(x), C, P, C, K.ptr(pmap), K.ptr(out), C, d,
                   K.stream())
            dx = torch.empty_like(x)
            dbnq = torch.empty(P, device=DEV)
            K.call("vu_attn_gate_bwd", K.ptr(dout), C, K.ptr(x), C, K.ptr(pmap), P, C, K.ptr(dx), C, K.ptr(dbnq),
                   d, K.stream())
            ds = torch.empty_like(ug)
            dw, db = torch.zeros(F, device=DEV), torch.zeros(1, device=DEV)
            ws = K.workspace_f32(K.query("vu_attn_psi_bwd_workspace_bytes", P, F), DEV)
            K.call("vu_attn_psi_bwd", K.ptr(ug), K.ptr(ux), P, F, K.ptr(co[0]), K.ptr(co[1]), K.ptr(co[2]),
                   K.ptr(co[3]), K.ptr(wpsi), K.ptr(dq), K.ptr(ds), K.ptr(dw), K.ptr(db), 0, K.ptr(ws), d,
                   K.stream())
            torch.cuda.synchronize()
            outs[mode] = dict(q=q, psum=psum, pm2=pm2, pmap=pmap, out=out, dx=dx, dbnq=dbnq, ds=ds, dw=dw, db=db)
        finally:
            _set(1)
    return outs, (ug, ux, co, wpsi, bpsi, x, cq)


CASES = [
    # (P, F_int, C): the UNet levels' gate shapes, and ragged pixel counts
    (4096, 32, 64),
    (2048 + 77, 64, 128),
    (1024 + 5, 128, 256),
    (512 + 200, 256, 512),
    (300, 512, 512),
    (999, 8, 1024),     # F_int = 8 (one lane per pixel); C > 512: one-row gate backward
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", CASES)
def test_attention_batched_kernels_match_one_row(case, dt):
    P, F, C = case
    outs, _ = _run(dt, P, F, C, seed=P + F)
    a, b = outs[1], outs[0]
    # same lanes and summation order, but the compiler may contract the
    # per-lane sums differently (fma vs mul + add): fp32 rounding, and one
    # bf16 rounding step on the stored activations
    for k in a:
        if a[k].dtype == torch.bfloat16:
            torch.testing.assert_close(a[k].float(), b[k].float(), rtol=8e-3, atol=1e-5, msg=k)
        else:
            torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-5, msg=k)


@pytest.mark.parametrize("case", [(2048 + 77, 64, 128), (300, 512, 512)])
def test_attention_forward_vs_torch(case):
    P, F, C = case
    outs, (ug, ux, co, wpsi, bpsi, x, cq) = _run(torch.float32, P, F, C, seed=5)
    o = outs[1]
    s = torch.relu(ug * co[0] + co[1] + ux * co[2] + co[3])
    q = s @ wpsi + bpsi
    torch.testing.assert_close(o["q"], q, rtol=1e-5, atol=1e-5)
    p = torch.sigmoid(q * cq[0] + cq[1])
    torch.testing.assert_close(o["pmap"], p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(o["out"], x * p[:, None], rtol=1e-5, atol=1e-6)
    tile = 256
    for t in range(o["psum"].numel()):
        blk = q[t * tile:(t + 1) * tile].double()
        assert abs(float(o["psum"][t]) - float(blk.sum())) < 1e-3
        assert abs(float(o["pm2"][t]) - float(((blk - blk.mean()) ** 2).sum())) < 1e-3 * (1 + float(o["pm2"][t]))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", CASES[:5])
def test_psi_bwd_emits_both_batchnorm_partials(dt, case):
    """Round 6: vu_attn_psi_bwd_bnb writes the same ds bits as vu_attn_psi_bwd
    (dwpsi / dbpsi to fp32 rounding), and its per-block (sum ds, sum ds*xhat) partials for the
    W_g and W_x BatchNorms, finished by vu_bn_bwd_finish, equal the fp64 sums
    over the stored ds (what the separate vu_bn_bwd_reduce passes computed)."""
    K = _k()
    from vaeunet_amd import _lib
    P, F, _ = case
    d = _lib.BF16 if dt == torch.bfloat16 else _lib.F32
    g = torch.Generator().manual_seed(41)
    ug = torch.randn(P, F, generator=g).to(dt).to(DEV)
    ux = torch.randn(P, F, generator=g).to(dt).to(DEV)
    co = [(torch.rand(F, generator=g) + 0.5).to(DEV), (torch.randn(F, generator=g) * 0.3).to(DEV),
          (torch.rand(F, generator=g) + 0.5).to(DEV), (torch.randn(F, generator=g) * 0.3).to(DEV)]
    mg, ig = (torch.randn(F, generator=g) * 0.2).to(DEV), (torch.rand(F, generator=g) + 0.5).to(DEV)
    mx, ix = (torch.randn(F, generator=g) * 0.2).to(DEV), (torch.rand(F, generator=g) + 0.5).to(DEV)
    wpsi = (torch.randn(F, generator=g) / F ** 0.5).to(DEV)
    dq = torch.randn(P, generator=g).to(DEV)
    assert K.query("vu_attn_psi_bwd_bnb_ok", F)
    res = {}
    for fused in (False, True):
        ds = torch.empty_like(ug)
        dw, db = torch.zeros(F, device=DEV), torch.zeros(1, device=DEV)
        ws = K.workspace_f32(K.query("vu_attn_psi_bwd_workspace_bytes", P, F), DEV)
        args = [K.ptr(ug), K.ptr(ux), P, F, K.ptr(co[0]), K.ptr(co[1]), K.ptr(co[2]), K.ptr(co[3]), K.ptr(wpsi),
                K.ptr(dq), K.ptr(ds), K.ptr(dw), K.ptr(db), 0, K.ptr(ws)]
        if fused:
            nb = K.query("vu_attn_psi_bwd_blocks", P)
            bg = torch.full((nb, 2, F), float("nan"), device=DEV)
            bx = torch.full((nb, 2, F), float("nan"), device=DEV)
            K.call("vu_attn_psi_bwd_bnb", *args, K.ptr(mg), K.ptr(ig), K.ptr(mx), K.ptr(ix), K.ptr(bg), K.ptr(bx),
                   d, K.stream())
        else:
            K.call("vu_attn_psi_bwd", *args, d, K.stream())
        torch.cuda.synchronize()
        res[fused] = (ds.clone(), dw.clone(), db.clone())
    # ds bit-identical; the psi weight / bias gradients equal up to the
    # compiler's fma contraction in the two instantiations
    assert torch.equal(res[False][0], res[True][0])
    for a, b in zip(res[False][1:], res[True][1:]):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6 * float(a.abs().max()))
    ds = res[True][0].double().cpu()
    for part, u, m, i in ((bg, ug, mg, ig), (bx, ux, mx, ix)):
        assert not bool(torch.isnan(part).any())
        gamma = torch.ones(F, device=DEV)
        dgamma, dbeta, k = torch.empty(F, device=DEV), torch.empty(F, device=DEV), torch.empty(3, F, device=DEV)
        wsf = torch.empty(max(1, _lib.query("vu_bn_bwd_finish_workspace_bytes", nb, F) // 4), device=DEV)
        _lib.call("vu_bn_bwd_finish", K.ptr(part), nb, P, F, K.ptr(gamma), K.ptr(i), 1, K.ptr(dgamma), K.ptr(dbeta),
                  0, K.ptr(k), K.ptr(wsf), K.stream())
        xhat = (u.double().cpu() - m.double().cpu()) * i.double().cpu()
        s0, s1 = ds.sum(0), (ds * xhat).sum(0)
        torch.testing.assert_close(dbeta.double().cpu(), s0, rtol=0, atol=2e-6 * float(ds.abs().sum(0).max()))
        torch.testing.assert_close(dgamma.double().cpu(), s1, rtol=0,
                                   atol=2e-6 * float((ds * xhat).abs().sum(0).max()))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("P,F", [(4096, 32), (2048 + 77, 64), (777, 256), (300, 512)])
def test_paired_bn_backward_apply_bit_identical(dt, P, F):
    """Round 6: vu_bn_bwd_apply2 (the attention gate's two BatchNorms from one
    read of ds) writes the bits of two vu_bn_bwd_apply calls (no ReLU)."""
    K = _k()
    from vaeunet_amd import _lib
    d = _lib.BF16 if dt == torch.bfloat16 else _lib.F32
    g = torch.Generator().manual_seed(43)
    ds, x1, x2 = (torch.randn(P, F, generator=g).to(dt).to(DEV) for _ in range(3))
    c1 = [(torch.rand(F, generator=g) + 0.5).to(DEV) for _ in range(4)]
    c2 = [(torch.rand(F, generator=g) + 0.5).to(DEV) for _ in range(4)]
    k1, k2 = torch.randn(3, F, generator=g).to(DEV), torch.randn(3, F, generator=g).to(DEV)
    ref = []
    for x, c, k in ((x1, c1, k1), (x2, c2, k2)):
        o = torch.empty_like(x)
        K.call("vu_bn_bwd_apply", K.ptr(ds), F, K.ptr(x), F, P, F, K.ptr(c[0]), K.ptr(c[1]), K.ptr(c[2]), K.ptr(k), 0,
               K.ptr(o), F, d, K.stream())
        ref.append(o)
    o1, o2 = torch.full_like(x1, float("nan")), torch.full_like(x2, float("nan"))
    assert K.query("vu_bn_bwd_apply2_ok", F, F, F, F, F, F)
    K.call("vu_bn_bwd_apply2", K.ptr(ds), F, K.ptr(x1), F, K.ptr(x2), F, P, F, K.ptr(c1[2]), K.ptr(k1), K.ptr(c2[2]),
           K.ptr(k2), K.ptr(o1), F, K.ptr(o2), F, d, K.stream())
    torch.cuda.synchronize()
    assert torch.equal(o1, ref[0]) and torch.equal(o2, ref[1])
