"""Per-element audit of GEMM launches (test infrastructure).

Installed as ``vaeunet_amd.kernels.AUDIT`` it receives every implicit-GEMM
launch the engine makes -- forward / input-gradient (``vu_gemm_fwd``) and
weight-gradient (``vu_gemm_wgrad`` + ``vu_slab_reduce``) -- runs it exactly as
the product path would (same descriptor, same dispatcher, so the same kernel:
v4 ping-pong, v6 resident weights, v7 small-grid, split-K, stream, image,
stem, ...), and then evaluates the contraction the descriptor DEFINES
(include/vaeunet.h: ``VuGather`` / ``VuGemmFwd`` / ``VuGemmWgrad``) in fp64 on
the device from the very same operands:

  fwd    out[m][j] = relu?(sum_k A[m][k] B[j][k] + zbias[n][cls(h, w)][j] + bias)  (+ old out)
         A = im2col of the (1-3) NHWC channel sources, zero padding;
         B = the derived weight image the kernel read;
  wgrad  grad[i, tap, c] = sum_m P[m][i] Q[m][tap*C + c]  (+ old grad).

The fp64 evaluation is F.conv2d / conv2d_input / conv2d_weight of those
operands written as an explicit tap sum (unfold), i.e. a convolution of the
bf16-rounded operands with no rounding of its own worth counting.

Each output element must satisfy the per-element bound

  |got - exp| <= u * max(|exp|, |got|)  (+ u * |new term| when accumulating)
                 + c * sum_k |A[m][k]| |B[j][k]|  +  1e-7 * max |exp|

u = 2^-8 for bf16 storage (round to nearest: half an ulp of the binade),
2^-24 for fp32; c = 1e-5 (fwd, K <= 9216) / 2e-5 (wgrad, K = pixels, split
into fp32 slabs) covers the fp32 summation-order noise of the MFMA
accumulation (|err| ~ sqrt(steps) * 2^-24 * sum |a b|).  Every element the
launch must NOT write (other channel slices, the other sub-lattices) is
checked to be bit-unchanged, and the BatchNorm partial statistics the
epilogue emitted are checked against the stored output.
"""
import ctypes as C

import torch
import torch.nn.functional as F

U = {0: 2.0 ** -24, 1: 2.0 ** -8}
C_FWD = 1e-5
C_WGRAD = 2e-5
FLOOR = 1e-7


def _bits(t):
    """bit pattern of a tensor (NaN-safe equality of untouched memory)."""
    if t.dtype in (torch.bfloat16, torch.float16):
        return t.view(torch.int16)
    if t.dtype == torch.float32:
        return t.view(torch.int32)
    return t


def _sync(t):
    if t.is_cuda:
        torch.cuda.synchronize()


def _storage_view(t):
    """the whole storage of ``t`` as a flat tensor of its dtype."""
    n = t.untyped_storage().nbytes() // t.element_size()
    return torch.as_strided(t, (n,), (1,), 0)


class _Im2col:
    """A[m][k] of a VuGather, per image chunk, in fp64 (and |A|)."""

    def __init__(self, g):
        self.g = g
        self.R, self.S = g.R, g.S
        self.pt = max(0, -g.oy)
        self.pl = max(0, -g.ox)
        self.pb = max(0, (g.H - 1) * g.sy + (g.R - 1) * g.dy + g.oy - (g.Hs - 1))
        self.pr = max(0, (g.W - 1) * g.sx + (g.S - 1) * g.dx + g.ox - (g.Ws - 1))

    def taps(self, n0, n1):
        """yields (tap, A_tap [n*H*W, C] fp64)."""
        g = self.g
        xs = [t[n0:n1, :, :g.Hs, :g.Ws] for t in g._refs]
        cs = sum(t.shape[1] for t in xs)
        if cs != g.C:
            raise AssertionError(f"gather channels {g.C} != sources {cs}")
        x = (torch.cat(xs, 1) if len(xs) > 1 else xs[0]).double()
        if x.shape[2] < g.Hs or x.shape[3] < g.Ws:
            raise AssertionError("gather image larger than its source tensor")
        xp = F.pad(x, [self.pl, self.pr, self.pt, self.pb])
        for r in range(self.R):
            for s in range(self.S):
                h0 = r * g.dy + g.oy + self.pt
                w0 = s * g.dx + g.ox + self.pl
                v = xp[:, :, h0:h0 + (g.H - 1) * g.sy + 1:g.sy, w0:w0 + (g.W - 1) * g.sx + 1:g.sx]
                assert v.shape[2] == g.H and v.shape[3] == g.W, (v.shape, g.H, g.W)
                yield r * self.S + s, v.permute(0, 2, 3, 1).reshape(-1, g.C)


class GemmAudit:
    """Collects one record per launch: (op, kernel, shape, worst err/bound,
    elements off).  ``strict``: raise at the first failing launch."""

    def __init__(self, strict=True, chunk_pixels=1 << 19):
        self.records = []
        self.strict = strict
        self.chunk_pixels = chunk_pixels

    # ---------------------------------------------------------------- forward
    def gemm_fwd(self, a, dtype, g, wmat, out, bias, st, launch, zbias=None):
        kern = self.kernel_of(a, dtype)
        pre = out.clone()
        launch()
        _sync(out)
        ncol, K = a.ncol, g.R * g.S * g.C
        B = torch.as_strided(wmat, (ncol, K), (a.ldb, 1), wmat.storage_offset()).double()
        Babs = B.abs()
        bvec = None
        if bias is not None:
            bvec = bias.double()
            if a.out_mode == 1:
                bvec = bvec[torch.arange(ncol, device=out.device) % a.cout]
        u = U[dtype]
        worst, off, nel = 0.0, 0, 0
        written = torch.zeros(out.shape, dtype=torch.bool, device=out.device)
        col = _Im2col(g)
        HW = g.H * g.W
        zcls = None
        if zbias is not None:   # VuGemmFwd.zbias: row m = (n, h, w) adds zbias[n][cls(h, w)]
            rc = lambda v, L: torch.where(v == 0, 0, torch.where(v == L - 1, 2, 1))  # noqa: E731
            hh = torch.arange(g.H, device=out.device)[:, None].expand(g.H, g.W)
            ww = torch.arange(g.W, device=out.device)[None, :].expand(g.H, g.W)
            zcls = (3 * rc(hh, g.H) + rc(ww, g.W)).reshape(-1)
            zb64 = zbias.double()
        step = max(1, self.chunk_pixels // HW)
        emax = 0.0
        pieces = []
        for n0 in range(0, g.N, step):
            n1 = min(g.N, n0 + step)
            res = torch.zeros((n1 - n0) * HW, ncol, dtype=torch.float64, device=out.device)
            sab = torch.zeros_like(res)
            for tap, A in col.taps(n0, n1):
                Bt = B[:, tap * g.C:(tap + 1) * g.C]
                res.addmm_(A, Bt.t())
                sab.addmm_(A.abs(), Babs[:, tap * g.C:(tap + 1) * g.C].t())
            if zcls is not None:
                zt = zb64[n0:n1][:, zcls, :].reshape(-1, ncol)
                res += zt
                sab += zt.abs()
            if bvec is not None:
                res += bvec
                sab += bvec.abs()
            if a.relu:
                res.clamp_(min=0)
            for view_got, view_pre, view_w, cols in self._regions(a, g, out, pre, written, n0, n1):
                got = view_got.permute(0, 2, 3, 1).reshape(-1, view_got.shape[1]).double()
                new = res[:, cols]
                exp = new.clone()
                bound = C_FWD * sab[:, cols]
                if a.accumulate:
                    exp += view_pre.permute(0, 2, 3, 1).reshape(-1, view_got.shape[1]).double()
                    bound += u * new.abs()
                view_w.fill_(True)
                pieces.append((got, exp, bound))
                emax = max(emax, float(exp.abs().max()))
            # evaluate this chunk's pieces now (memory), with the global floor later
            for got, exp, bound in pieces:
                err = (got - exp).abs()
                bnd = bound + u * torch.maximum(exp.abs(), got.abs())
                ratio = err / (bnd + FLOOR * max(emax, 1e-30))
                worst = max(worst, float(ratio.max()))
                off += int((ratio > 1).sum())
                nel += err.numel()
            pieces = []
        untouched = bool(torch.equal(_bits(out)[~written], _bits(pre)[~written]))
        if st is not None:
            self._check_stats(a, g, out, st)
        rec = dict(op="fwd", kernel=int(kern), M=g.N * g.H * g.W, N=ncol, K=K, R=g.R, C=g.C, H=g.H,
                   mode=int(a.out_mode), acc=int(a.accumulate), worst=worst, off=off, n=nel,
                   untouched=untouched, stats=st is not None)
        self._finish(rec)

    def _regions(self, a, g, out, pre, written, n0, n1):
        """(got view, pre view, written-mask view, result columns) per written
        region of the launch's output for images n0..n1-1."""
        c0 = a.out_coff
        if a.out_mode == 0:
            sl = (slice(n0, n1), slice(c0, c0 + a.ncol))
            yield out[sl], pre[sl], written[sl], slice(0, a.ncol)
        elif a.out_mode == 1:
            co = a.cout
            for ab in range(4):
                y0, x0 = (ab >> 1) + a.opy, (ab & 1) + a.opx
                sl = (slice(n0, n1), slice(c0, c0 + co), slice(y0, y0 + 2 * g.H - 1, 2),
                      slice(x0, x0 + 2 * g.W - 1, 2))
                yield out[sl], pre[sl], written[sl], slice(ab * co, (ab + 1) * co)
        else:
            sl = (slice(n0, n1), slice(c0, c0 + a.ncol), slice(a.opy, a.opy + 2 * g.H - 1, 2),
                  slice(a.opx, a.opx + 2 * g.W - 1, 2))
            yield out[sl], pre[sl], written[sl], slice(0, a.ncol)

    def _check_stats(self, a, g, out, st):
        assert a.out_mode == 0 and not a.accumulate
        y = out[:, a.out_coff:a.out_coff + a.ncol].double()
        n = torch.tensor([min(st.tile_rows, st.rows - t * st.tile_rows) for t in range(st.tiles)],
                         dtype=torch.float64, device=out.device)
        s = st.psum.double()
        mean = s.sum(0) / n.sum()
        m2 = st.pm2.double() + n[:, None] * (s / n[:, None] - mean) ** 2
        var = m2.sum(0) / n.sum()
        rmean = y.mean((0, 2, 3))
        rvar = y.var((0, 2, 3), unbiased=False)
        scale = float(y.abs().max()) + 1e-30
        dm = float((mean - rmean).abs().max())
        dv = float(((var - rvar).abs() / (rvar + 1e-6 * scale * scale)).max())
        assert dm <= 1e-5 * scale, f"BN partial mean off by {dm:.3e} (scale {scale:.3e})"
        assert dv <= 1e-4, f"BN partial variance off by {dv:.3e} (relative)"

    # --------------------------------------------------------- weight gradient
    def gemm_wgrad(self, w, dtype, kind, gp, gq, ni, nj, grad, layout, accumulate, cvalid, launch):
        store = _storage_view(grad)
        pre = store.clone()
        launch()
        _sync(grad)
        HW = gp.H * gp.W
        step = max(1, self.chunk_pixels // HW)
        res = torch.zeros(ni, nj, dtype=torch.float64, device=grad.device)
        sab = torch.zeros_like(res)
        cp, cq = _Im2col(gp), _Im2col(gq)
        for n0 in range(0, gp.N, step):
            n1 = min(gp.N, n0 + step)
            P = torch.cat([A for _, A in cp.taps(n0, n1)], 1)[:, :ni]
            Pabs = P.abs()
            for tap, Q in cq.taps(n0, n1):
                lo, hi = tap * gq.C, min(nj, (tap + 1) * gq.C)
                if lo >= nj:
                    break
                res[:, lo:hi] += P.t() @ Q[:, :hi - lo]
                sab[:, lo:hi] += Pabs.t() @ Q[:, :hi - lo].abs()
        taps = nj // gq.C
        s_i, s_tap, s_c = layout
        shape, strides = (ni, taps, cvalid), (s_i, s_tap, s_c)
        off0 = grad.storage_offset()
        G = torch.as_strided(store, shape, strides, off0).double()
        Gp = torch.as_strided(pre, shape, strides, off0).double()
        new = res.view(ni, taps, gq.C)[:, :, :cvalid]
        exp = new + Gp if accumulate else new
        u = U[0]
        err = (G - exp).abs()
        bound = 2 * u * torch.maximum(exp.abs(), G.abs()) + C_WGRAD * sab.view(ni, taps, gq.C)[:, :, :cvalid] \
            + FLOOR * float(exp.abs().max())
        ratio = err / (bound + 1e-300)
        # every element of grad outside the written (i, tap, c < cvalid) set,
        # and everything else in its storage, must be bit-unchanged
        idx = torch.arange(store.numel(), device=grad.device)
        keep = torch.ones(store.numel(), dtype=torch.bool, device=grad.device)
        keep[torch.as_strided(idx, shape, strides, off0).reshape(-1)] = False
        untouched = bool(torch.equal(_bits(store)[keep], _bits(pre)[keep]))
        rec = dict(op="wgrad", kernel=int(kind), M=gp.N * HW, N=nj, K=gp.N * HW, R=gq.R, C=gq.C, H=gq.H,
                   mode=0, acc=int(accumulate), ni=ni, worst=float(ratio.max()), off=int((ratio > 1).sum()),
                   n=err.numel(), untouched=untouched, stats=False)
        self._finish(rec)

    @staticmethod
    def kernel_of(a, dtype):
        from vaeunet_amd import _lib
        return _lib.query("vu_gemm_fwd_kernel", C.byref(a), dtype)

    # ------------------------------------------------------------------ common
    def _finish(self, rec):
        self.records.append(rec)
        if self.strict:
            assert rec["off"] == 0, f"per-element bound exceeded: {rec}"
            assert rec["untouched"], f"launch wrote outside its output region: {rec}"

    def summary(self):
        lines = []
        for r in self.records:
            lines.append(f"{r['op']:5s} k{r['kernel']:<2d} R{r['R']} M={r['M']:>8d} N={r['N']:>5d} "
                         f"C={r['C']:>5d} H={r['H']:>4d} mode{r['mode']} acc{r['acc']} "
                         f"worst {r['worst']:.3f} off {r['off']}/{r['n']}")
        return "\n".join(lines)
