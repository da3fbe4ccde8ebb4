"""The latent-broadcast shortcut of a DecoderBlock's conv1 (round 5,
csrc/zbias.hip + the VuGemmFwd.zbias epilogue; unet/unet_resnet.py:37-41,
92-99): against the convolution of the concat with the per-sample constant
z map it replaces -- the forward GEMM on every kernel that serves it (the
ping-pong kernel, its split-K finish, the generic kernel, bf16 and fp32), and
the backward's weight-gradient z columns and pixel-summed map gradient."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last
TUNE_V4_MIN_BLOCKS, TUNE_V4_SPLITK, TUNE_GEN = 0, 6, 12
TUNE_DEFAULTS = ((TUNE_V4_MIN_BLOCKS, 256), (TUNE_V4_SPLITK, 1), (TUNE_GEN, 4))


def _tune(*kv):
    from vaeunet_amd import _lib
    for k, v in kv:
        _lib.call("vu_gemm_set_tuning", k, v)


def _job(w, cz0, L, H, W, act, table=None):
    from vaeunet_amd import _lib
    j = _lib.VuZbJob()
    j.w = w.data_ptr()
    j.ws_co, j.ws_ci, j.ws_ky, j.ws_kx = w.stride()
    j.cz0, j.L, j.co, j.H, j.W = cz0, L, w.shape[0], H, W
    j.act = act.data_ptr()
    j.table = table.data_ptr() if table is not None else None
    return j


def _table(w, cz0, L, H, W, act):
    from vaeunet_amd import kernels as K
    N, co = act.shape[0], w.shape[0]
    table = torch.empty((N, 9, co), dtype=torch.float32, device=DEV)
    arr = (type(_job(w, cz0, L, H, W, act)) * 1)()
    arr[0] = _job(w, cz0, L, H, W, act, table)
    K.call("vu_zbias_fwd", arr, 1, N, K.stream())
    return table


# (N, [cin per non-z source], L, H, W, cout, mode, tuning, kernel id)
FWD_CASES = [
    (2, [64, 64], 32, 32, 32, 64, "bf16", ((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0)), 4),    # pp<64>
    (2, [64, 64], 32, 16, 64, 128, "bf16", ((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0)), 4),   # pp<128>
    (1, [128, 64], 32, 8, 32, 256, "bf16", ((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 0)), 4),   # pp<256>
    (2, [128, 64], 32, 16, 32, 256, "bf16", ((TUNE_V4_MIN_BLOCKS, 0), (TUNE_V4_SPLITK, 2)), 4),  # split-K finish
    (2, [64, 64], 32, 12, 20, 64, "bf16", ((TUNE_GEN, 1),), 1),                                  # generic bf16
    (2, [32, 24], 32, 9, 13, 48, "f32", (), 1),                                                  # generic fp32
]


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("case", FWD_CASES)
def test_zbias_forward_matches_concat_conv(case, relu):
    """conv over [sources] + zbias == conv over [sources, broadcast z map]
    (the map holds the storage-rounded vectors), per element within the
    GEMM bound, with the BatchNorm statistics of the stored output.  relu:
    the folded eval-BN inference form (VuGemmFwd.relu with the table, ADVICE
    r5: the ping-pong kernel's ZB instantiation ignored p.relu)."""
    from vaeunet_amd import kernels as K, engine as E
    N, cins, L, H, W, co, mode, tune, kern = case
    dt = torch.bfloat16 if mode == "bf16" else torch.float32
    d = 1 if mode == "bf16" else 0
    g = torch.Generator().manual_seed(21)
    xs = [torch.randn(N, c, H, W, generator=g).to(dt).float() for c in cins]
    lead = sum(cins)
    w = (torch.randn(co, lead + L, 3, 3, generator=g) / (3 * (lead + L) ** 0.5)).to(DEV)
    act = torch.rand(N, L, generator=g).to(dt).float().to(DEV)   # ReLU'd vectors, storage-rounded
    table = _table(w, lead, L, H, W, act)
    # the table from a channels_last copy of the weight (the model's layout) is the same
    table_cl = _table(w.contiguous(memory_format=CL), lead, L, H, W, act)
    torch.testing.assert_close(table_cl, table, rtol=1e-6, atol=1e-7)
    w_odd = torch.empty(co, lead + L + 1, 3, 3, device=DEV)[:, 1:]   # unaligned rows: the scalar staging path
    w_odd.copy_(w)
    torch.testing.assert_close(_table(w_odd, lead, L, H, W, act), table, rtol=1e-6, atol=1e-7)
    srcs = [x.to(DEV, dt).contiguous(memory_format=CL) for x in xs]
    out = K.empty_act(N, co, H, W, dt, DEV)
    _tune(*tune)
    try:
        wm = E.w3x3_fwd(w, d, cin_use=lead)
        from vaeunet_amd import _lib
        a = _lib.VuGemmFwd()
        a.a = K.gather3x3(srcs)
        a.b, a.ldb, a.ncol = wm.data_ptr(), wm.shape[-1], co
        a.out, a.out_stride, a.out_mode = out.data_ptr(), K.pstride(out), 0
        a.zbias = table.data_ptr()
        a.relu = 1 if relu else 0
        assert K.query("vu_gemm_fwd_kernel", C.byref(a), d) == kern
        st = K.gemm_fwd(K.gather3x3(srcs), wm, co, out, d, stats=True, zbias=table, relu=relu)
    finally:
        _tune(*TUNE_DEFAULTS)
    zmap = act.cpu()[:, :, None, None].expand(N, L, H, W)
    wq = w.cpu().to(dt).float() if mode == "bf16" else w.cpu()
    xcat = torch.cat(xs + [zmap], 1)
    # the shortcut keeps the fp32 weights for the z part (the map path rounds them to bf16)
    wz = torch.cat([wq[:, :lead], w.cpu()[:, lead:]], 1)
    ref = F.conv2d(xcat.double(), wz.double(), padding=1)
    sab = F.conv2d(xcat.abs().double(), wz.abs().double(), padding=1)
    if relu:
        assert float(ref.min()) < 0  # the case exercises the clamp
        ref = ref.clamp_min(0)
    got = out.double().cpu()
    u = 2.0 ** -8 if mode == "bf16" else 2.0 ** -24
    bound = u * torch.maximum(ref.abs(), got.abs()) + 1e-5 * sab + 1e-7 * float(ref.abs().max())
    err = (got - ref).abs()
    assert bool((err <= bound).all()), float((err / bound).max())
    stored = out.double().cpu()
    n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)], dtype=torch.float64)
    s = st.psum.double().cpu()
    mean = s.sum(0) / n.sum()
    m2 = st.pm2.double().cpu() + n[:, None] * (s / n[:, None] - mean) ** 2
    torch.testing.assert_close(mean, stored.mean((0, 2, 3)), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m2.sum(0) / n.sum(), stored.var((0, 2, 3), unbiased=False), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("mode", ["bf16", "f32"])
@pytest.mark.parametrize("shape", [(8, 32, 16, 16, 64), (2, 32, 7, 12, 512), (3, 16, 2, 5, 96), (2, 16, 48, 72, 64),
                                   (2, 16, 9, 40, 1024)])
@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("cl", [False, True])
def test_zbias_backward_matches_map_gradient(mode, shape, acc, cl):
    """From conv1's pre-BN gradient dy: the weight gradient's z columns
    (written / accumulated; the other columns untouched) and the pixel sums
    of the z map's gradient (the split partials the latent backward sums)
    equal conv2d_weight / conv2d_input of the broadcast map, in fp64."""
    from vaeunet_amd import kernels as K
    N, L, H, W, co = shape
    lead = 64
    dt = torch.bfloat16 if mode == "bf16" else torch.float32
    g = torch.Generator().manual_seed(23)
    fmt = CL if cl else torch.contiguous_format   # the model's weights are channels_last after .to(CL)
    w = (torch.randn(co, lead + L, 3, 3, generator=g) / 10).to(DEV).contiguous(memory_format=fmt)
    act = torch.rand(N, L, generator=g).to(DEV)
    dy = torch.randn(N, co, H, W, generator=g).to(dt)
    dyd = dy.to(DEV).contiguous(memory_format=CL)
    dw = torch.randn(co, lead + L, 3, 3, generator=g).to(DEV).contiguous(memory_format=fmt)
    dw0 = dw.clone()
    part = torch.full((N * 32 * L,), float("nan"), dtype=torch.float32, device=DEV)
    rs = torch.empty(K.query("vu_zbias_rs_floats", N, co, H, W), dtype=torch.float32, device=DEV)
    arr = (type(_job(w, lead, L, H, W, act)) * 1)()
    j = _job(w, lead, L, H, W, act)
    j.dy, j.dy_stride = dyd.data_ptr(), K.pstride(dyd)
    j.rs, j.part, j.dw, j.grad_acc = rs.data_ptr(), part.data_ptr(), dw.data_ptr(), 1 if acc else 0
    arr[0] = j
    K.call("vu_zbias_bwd", arr, 1, N, 1 if mode == "bf16" else 0, K.stream())
    torch.cuda.synchronize()
    zmap = act.cpu().double()[:, :, None, None].expand(N, L, H, W)
    dy64 = dy.double()
    gw = torch.nn.grad.conv2d_weight(zmap, (co, L, 3, 3), dy64, padding=1)
    gwa = torch.nn.grad.conv2d_weight(zmap.abs(), (co, L, 3, 3), dy64.abs(), padding=1)
    exp_w = gw + (dw0.cpu().double()[:, lead:] if acc else 0)
    got_w = dw.cpu().double()[:, lead:]
    assert bool(((got_w - exp_w).abs() <= 1e-5 * gwa + 2.0 ** -24 * exp_w.abs() + 1e-12).all())
    assert torch.equal(dw[:, :lead], dw0[:, :lead])
    dmap = torch.nn.grad.conv2d_input((N, L, H, W), w.cpu().double()[:, lead:], dy64, padding=1)
    dmapa = torch.nn.grad.conv2d_input((N, L, H, W), w.cpu().double()[:, lead:].abs(), dy64.abs(), padding=1)
    dc = dmap.sum((2, 3))
    got_dc = part.view(N, 32, L).double().cpu().sum(1)
    assert bool(((got_dc - dc).abs() <= 1e-5 * dmapa.sum((2, 3)) + 1e-12).all())
    assert not bool(torch.isnan(part).any())   # every split written (unused ones zero)


@pytest.mark.parametrize("mode", ["bf16", "f32"])
@pytest.mark.parametrize("shape", [(8, 32, 16, 16, 64), (2, 32, 7, 12, 512), (3, 16, 2, 5, 96), (2, 16, 48, 72, 64),
                                   (2, 16, 9, 40, 1024), (2, 16, 64, 64, 128)])
@pytest.mark.parametrize("relu", [False, True])
def test_fused_region_partials_bit_identical(mode, shape, relu):
    """Round 6: conv1's BatchNorm backward apply with the shortcut's region
    partials (vu_bn_bwd_apply_zrs) against vu_bn_bwd_apply followed by
    vu_zbias_bwd's own region pass -- dy, every rs float and the outputs of
    the remaining launches (z columns of dW, dc partials) bit-identical."""
    from vaeunet_amd import kernels as K
    N, L, H, W, co = shape
    lead = 64
    dt = torch.bfloat16 if mode == "bf16" else torch.float32
    dcode = 1 if mode == "bf16" else 0
    g = torch.Generator().manual_seed(31)
    w = (torch.randn(co, lead + L, 3, 3, generator=g) / 10).to(DEV).contiguous(memory_format=CL)
    act = torch.rand(N, L, generator=g).to(DEV)
    da = torch.randn(N, co, H, W, generator=g).to(dt).to(DEV).contiguous(memory_format=CL)
    x = torch.randn(N, co, H, W, generator=g).to(dt).to(DEV).contiguous(memory_format=CL)
    scale = (torch.rand(co, generator=g) + 0.5).to(DEV)
    shift = (torch.randn(co, generator=g) * 0.3).to(DEV)
    mean = (torch.randn(co, generator=g) * 0.2).to(DEV)
    k = torch.randn(3, co, generator=g).to(DEV).contiguous()
    out = []
    for fused in (False, True):
        dy = torch.full_like(da, float("nan"))
        rs = torch.full((K.query("vu_zbias_rs_floats", N, co, H, W),), float("nan"), dtype=torch.float32, device=DEV)
        part = torch.full((N * 32 * L,), float("nan"), dtype=torch.float32, device=DEV)
        dw = torch.zeros(co, lead + L, 3, 3, device=DEV).contiguous(memory_format=CL)
        if fused:
            assert K.query("vu_bn_bwd_apply_zrs_ok", H, W, co, K.pstride(da), K.pstride(x), K.pstride(dy))
            K.call("vu_bn_bwd_apply_zrs", da.data_ptr(), K.pstride(da), x.data_ptr(), K.pstride(x), N, H, W, co,
                   scale.data_ptr(), shift.data_ptr(), mean.data_ptr(), k.data_ptr(), 1 if relu else 0,
                   dy.data_ptr(), K.pstride(dy), rs.data_ptr(), dcode, K.stream())
        else:
            K.call("vu_bn_bwd_apply", da.data_ptr(), K.pstride(da), x.data_ptr(), K.pstride(x), N * H * W, co,
                   scale.data_ptr(), shift.data_ptr(), mean.data_ptr(), k.data_ptr(), 1 if relu else 0,
                   dy.data_ptr(), K.pstride(dy), dcode, K.stream())
        arr = (type(_job(w, lead, L, H, W, act)) * 1)()
        j = _job(w, lead, L, H, W, act)
        j.dy, j.dy_stride = dy.data_ptr(), K.pstride(dy)
        j.rs, j.part, j.dw, j.grad_acc = rs.data_ptr(), part.data_ptr(), dw.data_ptr(), 0
        j.rs_ready = 1 if fused else 0
        arr[0] = j
        K.call("vu_zbias_bwd", arr, 1, N, dcode, K.stream())
        torch.cuda.synchronize()
        out.append((dy.clone(), rs.clone(), part.clone(), dw.clone()))
    (dy0, rs0, p0, w0), (dy1, rs1, p1, w1) = out
    assert not bool(torch.isnan(dy1.float()).any()) and not bool(torch.isnan(rs1).any())
    assert torch.equal(dy0, dy1)
    assert torch.equal(rs0, rs1)
    assert torch.equal(p0, p1)
    assert torch.equal(w0, w1)


def test_region_pass_skips_only_ready_jobs():
    """Two shortcut jobs in one vu_zbias_bwd, only the first with its
    partials from the fused apply (rs_ready): both jobs' outputs equal the
    all-unfused run bit for bit (the second job's region pass still runs)."""
    from vaeunet_amd import kernels as K
    N, L, dcode = 2, 16, 1
    g = torch.Generator().manual_seed(5)
    shapes = [(16, 20, 64), (8, 12, 128)]
    jobs = []
    for H, W, co in shapes:
        w = (torch.randn(co, 64 + L, 3, 3, generator=g) / 10).to(DEV).contiguous(memory_format=CL)
        act = torch.rand(N, L, generator=g).to(DEV)
        da = torch.randn(N, co, H, W, generator=g).to(torch.bfloat16).to(DEV).contiguous(memory_format=CL)
        x = torch.randn(N, co, H, W, generator=g).to(torch.bfloat16).to(DEV).contiguous(memory_format=CL)
        bn = [(torch.rand(co, generator=g) + 0.5).to(DEV), (torch.randn(co, generator=g) * 0.3).to(DEV),
              (torch.randn(co, generator=g) * 0.2).to(DEV), torch.randn(3, co, generator=g).to(DEV).contiguous()]
        jobs.append((H, W, co, w, act, da, x, bn))
    res = []
    for fuse_first in (False, True):
        arr = (type(_job(jobs[0][3], 64, L, 4, 4, jobs[0][4])) * 2)()
        outs = []
        for i, (H, W, co, w, act, da, x, bn) in enumerate(jobs):
            dy = torch.empty_like(da)
            rs = torch.full((K.query("vu_zbias_rs_floats", N, co, H, W),), float("nan"), device=DEV)
            part = torch.full((N * 32 * L,), float("nan"), device=DEV)
            dw = torch.zeros(co, 64 + L, 3, 3, device=DEV).contiguous(memory_format=CL)
            args = (bn[0].data_ptr(), bn[1].data_ptr(), bn[2].data_ptr(), bn[3].data_ptr(), 1)
            if fuse_first and i == 0:
                K.call("vu_bn_bwd_apply_zrs", da.data_ptr(), K.pstride(da), x.data_ptr(), K.pstride(x), N, H, W, co,
                       *args, dy.data_ptr(), K.pstride(dy), rs.data_ptr(), dcode, K.stream())
            else:
                K.call("vu_bn_bwd_apply", da.data_ptr(), K.pstride(da), x.data_ptr(), K.pstride(x), N * H * W, co,
                       *args, dy.data_ptr(), K.pstride(dy), dcode, K.stream())
            j = _job(w, 64, L, H, W, act)
            j.dy, j.dy_stride = dy.data_ptr(), K.pstride(dy)
            j.rs, j.part, j.dw, j.grad_acc = rs.data_ptr(), part.data_ptr(), dw.data_ptr(), 0
            j.rs_ready = 1 if (fuse_first and i == 0) else 0
            arr[i] = j
            outs.append((dy, rs, part, dw))
        K.call("vu_zbias_bwd", arr, 2, N, dcode, K.stream())
        torch.cuda.synchronize()
        res.append([tuple(t.clone() for t in o) for o in outs])
    for a, b in zip(res[0], res[1]):
        for ta, tb in zip(a, b):
            assert torch.equal(ta, tb)
