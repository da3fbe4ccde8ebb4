// Weight-gradient GEMM: slab[s][i][j] = sum_{m in split s} P[m][i] * Q[m][j].
//
// Both operands are "m-major" (the reduction index m = pixel is the strided
// one): P is the output gradient dY [pixels][Cout] and Q the im2col gather of
// the layer input (3x3 taps, 1x1, or the ConvTranspose sub-pixel gather).
// This covers dW of every conv in unet_parts.py (3x3 :40,43; 1x1 :11,15,100;
// ConvT 2x2 :76) — the "wgrad" third of the 1,103.5 GFLOP/img 3x3 budget.
//
// Tiling: 256 threads = 4 waves (2x2), output tile BI x BJ, 64 pixels per
// step, LDS double buffer [m][col] staged through registers.  bf16: the MFMA
// operands are read k(=m)-contiguous straight out of the [m][col] image with
// the gfx950 transposing LDS read ds_read_b64_tr_b16 (cdna_hip_programming
// T10), on a 32-byte-block XOR swizzle that makes both the 16-byte writes and
// the transposed reads bank-conflict free.  fp32: MFMA 16x16x4 f32, one
// ds_read_b32 per operand (lanes on consecutive columns, rows padded).
// Split-K over m writes fp32 slabs, reduced in a fixed order (deterministic).
#include <stdlib.h>
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int BMR = 64;  // pixels per step

// Column decode of one 16-byte chunk of a gather operand (fixed per thread).
struct ColDec {
  int r, s;      // tap
  int t;         // source
  int64_t coff;  // channel offset inside source t
  bool ok;
};

VU_DEV ColDec col_decode(const VuGather& g, int col, int ncols) {
  ColDec d;
  d.ok = col < ncols;
  int cc = d.ok ? col : 0;
  int tap = cc / g.C, ch = cc - tap * g.C;
  d.r = tap / g.S;
  d.s = tap - d.r * g.S;
  d.t = (ch >= g.cend[0]) + (g.nsrc > 2 && ch >= g.cend[1]);
  int c0 = d.t == 0 ? 0 : g.cend[d.t - 1];
  d.coff = ch - c0;
  return d;
}

template <typename T>
VU_DEV u32x4 gather_t(const VuGather& g, const ColDec& d, int n, int h, int w, bool mok) {
  u32x4 z = {0, 0, 0, 0};
  if (!mok || !d.ok) return z;
  int hs = h * g.sy + d.r * g.dy + g.oy;
  int ws = w * g.sx + d.s * g.dx + g.ox;
  if ((unsigned)hs >= (unsigned)g.Hs || (unsigned)ws >= (unsigned)g.Ws) return z;
  const T* base = reinterpret_cast<const T*>(g.src[d.t]);
  int64_t pix = ((int64_t)n * g.Hs + hs) * g.Ws + ws;
  return *reinterpret_cast<const u32x4*>(base + pix * g.stride[d.t] + d.coff);
}

// ---- LDS image addressing ----
// bf16: rows of RB bytes (= 2*BI), 32-byte blocks XOR-swizzled by f(m).
template <int RB> VU_DEV int tr_off(int m, int col) {
  int blk = col >> 4;
  int f;
  if (RB == 256) f = (m & 3) | ((m >> 1) & 4);
  else f = ((m >> 1) & 1) | ((m >> 2) & 2);
  return m * RB + ((blk ^ f) << 5) + ((col & 15) << 1);
}

template <typename T, int BI> struct Img;
template <int BI> struct Img<bf16_t, BI> {
  static constexpr int RB = BI * 2;
  static constexpr int BYTES = BMR * RB;
  // byte offset of the 16-byte chunk holding columns [col, col+8) of row m
  static VU_DEV int chunk_off(int m, int col) { return tr_off<RB>(m, col); }
};
template <int BI> struct Img<float, BI> {
  static constexpr int RB = BI * 4 + 64;  // pad: rows m, m+1 16 banks apart
  static constexpr int BYTES = BMR * RB;
  static VU_DEV int chunk_off(int m, int col) { return m * RB + col * 4; }
};

template <typename T, int BI, int BJ>
__global__ __launch_bounds__(256, 2) void gemm_wgrad_kernel(VuGemmWgrad p) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int CPI = BI / EPC, CPJ = BJ / EPC;  // chunks per row
  constexpr int LI = BMR * CPI / 256, LJ = BMR * CPJ / 256;  // loads per thread
  constexpr int TI = BI / 32, TJ = BJ / 32;
  using IP = Img<T, BI>;
  using IQ = Img<T, BJ>;
  constexpr int BUF = IP::BYTES + IQ::BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const VuGather& gp = p.p;
  const VuGather& gq = p.q;
  const int64_t M = (int64_t)gp.N * gp.H * gp.W;
  const int itiles = (p.ni + BI - 1) / BI, jtiles = (p.nj + BJ - 1) / BJ;
  const int ntile = itiles * jtiles;
  const int nblk = ntile * p.splits;
  const int bid = xcd_remap(blockIdx.x, nblk);
  const int split = bid / ntile;
  const int tile = bid - split * ntile;
  const int it = tile / jtiles, jt = tile - it * jtiles;
  const int i0 = it * BI, j0 = jt * BJ;
  const int64_t mbeg = (int64_t)split * p.m_per_split;
  const int64_t mend = (mbeg + p.m_per_split < M) ? mbeg + p.m_per_split : M;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wi = wid >> 1, wj = wid & 1;

  // Each thread loads chunk columns (tid % CP) of rows (tid / CP) + k*(256/CP).
  const int pcol = (tid % CPI) * EPC, prow = tid / CPI;
  const int qcol = (tid % CPJ) * EPC, qrow = tid / CPJ;
  constexpr int PSTEP = 256 / CPI, QSTEP = 256 / CPJ;
  const ColDec dp = col_decode(gp, i0 + pcol, p.ni);
  const ColDec dq = col_decode(gq, j0 + qcol, p.nj);

  // Row (pixel) state for each loaded row, advanced incrementally by BMR.
  int pn[LI], ph[LI], pw[LI];
  int qn[LJ], qh[LJ], qw[LJ];
  auto decode = [&](int64_t m, int& n, int& h, int& w) {
    int hw = gp.H * gp.W;
    int64_t mm = m < M ? m : 0;
    n = (int)(mm / hw);
    int rem = (int)(mm - (int64_t)n * hw);
    h = rem / gp.W;
    w = rem - h * gp.W;
  };
  auto advance = [&](int& n, int& h, int& w) {
    w += BMR;
    while (w >= gp.W) { w -= gp.W; if (++h == gp.H) { h = 0; ++n; } }
  };
#pragma unroll
  for (int k = 0; k < LI; ++k) decode(mbeg + prow + k * PSTEP, pn[k], ph[k], pw[k]);
#pragma unroll
  for (int k = 0; k < LJ; ++k) decode(mbeg + qrow + k * QSTEP, qn[k], qh[k], qw[k]);

  u32x4 rp[LI], rq[LJ];
  auto load = [&](int64_t mb) {
#pragma unroll
    for (int k = 0; k < LI; ++k) {
      int64_t m = mb + prow + k * PSTEP;
      rp[k] = gather_t<T>(gp, dp, pn[k], ph[k], pw[k], m < mend);
    }
#pragma unroll
    for (int k = 0; k < LJ; ++k) {
      int64_t m = mb + qrow + k * QSTEP;
      rq[k] = gather_t<T>(gq, dq, qn[k], qh[k], qw[k], m < mend);
    }
  };
  auto adv_all = [&]() {
#pragma unroll
    for (int k = 0; k < LI; ++k) advance(pn[k], ph[k], pw[k]);
#pragma unroll
    for (int k = 0; k < LJ; ++k) advance(qn[k], qh[k], qw[k]);
  };
  auto store_lds = [&](int buf) {
    char* Pb = smem + buf * BUF;
    char* Qb = Pb + IP::BYTES;
#pragma unroll
    for (int k = 0; k < LI; ++k)
      *reinterpret_cast<u32x4*>(Pb + IP::chunk_off(prow + k * PSTEP, pcol)) = rp[k];
#pragma unroll
    for (int k = 0; k < LJ; ++k)
      *reinterpret_cast<u32x4*>(Qb + IQ::chunk_off(qrow + k * QSTEP, qcol)) = rq[k];
  };

  constexpr bool CMP = sizeof(T) == 4;  // fp32: compensated sum of per-step partials
  f32x4 acc[TI][TJ], cmp[CMP ? TI : 1][CMP ? TJ : 1];
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int b = 0; b < TJ; ++b) acc[a][b] = f32x4{0, 0, 0, 0};
  if constexpr (CMP)
#pragma unroll
    for (int a = 0; a < TI; ++a)
#pragma unroll
      for (int b = 0; b < TJ; ++b) cmp[a][b] = f32x4{0, 0, 0, 0};

  const int nsteps = mend > mbeg ? (int)((mend - mbeg + BMR - 1) / BMR) : 0;
  if (nsteps > 0) {
    load(mbeg);
    adv_all();
    store_lds(0);
  }
  __syncthreads();
  const int g4 = lane >> 4, li = lane & 15;
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
    if (st + 1 < nsteps) { load(mbeg + (int64_t)(st + 1) * BMR); adv_all(); }
    const char* Pb = smem + cur * BUF;
    const char* Qb = Pb + IP::BYTES;
    if constexpr (sizeof(T) == 2) {
      typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
      const int q = li >> 2, pp = li & 3;
#pragma unroll
      for (int ks = 0; ks < BMR / 32; ++ks) {
        u32x4 af[TI], bf[TJ];
#pragma unroll
        for (int a = 0; a < TI; ++a) {
          int col = wi * (BI / 2) + a * 16 + 4 * pp;
          int m = ks * 32 + 8 * g4 + q;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(Pb + tr_off<IP::RB>(m, col) - 0));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_s16x4*)(Pb + tr_off<IP::RB>(m + 4, col)));
          u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
          af[a] = u32x4{l2[0], l2[1], h2[0], h2[1]};
        }
#pragma unroll
        for (int b = 0; b < TJ; ++b) {
          int col = wj * (BJ / 2) + b * 16 + 4 * pp;
          int m = ks * 32 + 8 * g4 + q;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Qb + tr_off<IQ::RB>(m, col)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Qb + tr_off<IQ::RB>(m + 4, col)));
          u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
          bf[b] = u32x4{l2[0], l2[1], h2[0], h2[1]};
        }
#pragma unroll
        for (int a = 0; a < TI; ++a)
#pragma unroll
          for (int b = 0; b < TJ; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, af[a]), __builtin_bit_cast(bf16x8, bf[b]), acc[a][b], 0, 0, 0);
      }
    } else {
      // fp32 (parity mode): the step's 64 pixels summed by their own MFMA
      // chain, then added to the running sum with Kahan compensation (the
      // split's chain otherwise grows with m_per_split; gemm_fwd.hip)
      f32x4 part[TI][TJ];
#pragma unroll
      for (int a = 0; a < TI; ++a)
#pragma unroll
        for (int b = 0; b < TJ; ++b) part[a][b] = f32x4{0, 0, 0, 0};
#pragma unroll 4
      for (int ks = 0; ks < BMR / 4; ++ks) {
        float af[TI], bf[TJ];
        int m = ks * 4 + g4;
#pragma unroll
        for (int a = 0; a < TI; ++a)
          af[a] = *reinterpret_cast<const float*>(Pb + IP::chunk_off(m, wi * (BI / 2) + a * 16 + li));
#pragma unroll
        for (int b = 0; b < TJ; ++b)
          bf[b] = *reinterpret_cast<const float*>(Qb + IQ::chunk_off(m, wj * (BJ / 2) + b * 16 + li));
#pragma unroll
        for (int a = 0; a < TI; ++a)
#pragma unroll
          for (int b = 0; b < TJ; ++b)
            part[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a], bf[b], part[a][b], 0, 0, 0);
      }
#pragma unroll
      for (int a = 0; a < TI; ++a)
#pragma unroll
        for (int b = 0; b < TJ; ++b) kahan_add(acc[a][b], cmp[a][b], part[a][b]);
    }
    if (st + 1 < nsteps) store_lds(cur ^ 1);
    __syncthreads();
  }

  if constexpr (CMP)
#pragma unroll
    for (int a = 0; a < TI; ++a)
#pragma unroll
      for (int b = 0; b < TJ; ++b) acc[a][b] -= cmp[a][b];
  // ---- store fp32 partial tile: lane holds C[4*g4 + r][li] ----
  float* out = p.out + (int64_t)split * p.ni * p.nj;
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int b = 0; b < TJ; ++b) {
      int j = j0 + wj * (BJ / 2) + b * 16 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int i = i0 + wi * (BI / 2) + a * 16 + 4 * g4 + r;
        if (i < p.ni && j < p.nj) out[(int64_t)i * p.nj + j] = acc[a][b][r];
      }
    }
}

template <typename T, int BI, int BJ>
int launch_wg(const VuGemmWgrad& p, hipStream_t st) {
  int itiles = (p.ni + BI - 1) / BI, jtiles = (p.nj + BJ - 1) / BJ;
  int64_t nblk = (int64_t)itiles * jtiles * p.splits;
  if (nblk <= 0) return 0;
  hipLaunchKernelGGL((gemm_wgrad_kernel<T, BI, BJ>), dim3((unsigned)nblk), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

template <typename T>
int dispatch_wg(const VuGemmWgrad& p, hipStream_t st) {
  if (p.ni <= 64) return launch_wg<T, 64, 128>(p, st);
  return launch_wg<T, 128, 128>(p, st);
}

// slab reduce + permute into the parameter-gradient layout
// Sum of the split-K slabs in a fixed order.  A 256-thread block covers 64
// consecutive outputs x 4 split lanes; each lane keeps 4 independent
// accumulators so its slab loads overlap (with many splits the serial chain,
// not bandwidth, was the limit), then the 4 lanes fold in LDS.
__global__ void slab_reduce_kernel(const float* slab, int splits, int ni, int nj, int C, int cvalid,
                                   int64_t s_i, int64_t s_tap, int64_t s_c, float* out, int accumulate) {
  __shared__ float sh[4][64];
  const int l = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t tot = (int64_t)ni * nj;
  const int64_t idx = (int64_t)blockIdx.x * 64 + l;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (idx < tot) {
    int k = q;
    for (; k + 12 < splits; k += 16)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += slab[(int64_t)(k + 4 * u) * tot + idx];
    for (; k < splits; k += 4) a[0] += slab[(int64_t)k * tot + idx];
  }
  sh[q][l] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (q != 0 || idx >= tot) return;
  float s = (sh[0][l] + sh[1][l]) + (sh[2][l] + sh[3][l]);
  int i = (int)(idx / nj), j = (int)(idx - (int64_t)i * nj);
  int tap = j / C, c = j - tap * C;
  if (c >= cvalid) return;
  float* o = out + i * s_i + tap * s_tap + c * s_c;
  *o = accumulate ? *o + s : s;
}

// Vectorised form (tot % 4 == 0): a thread owns 4 consecutive outputs
// (16-byte slab loads), SL split lanes per output group, 4 independent
// accumulators per lane.  The slabs were just written by the weight-gradient
// kernel and sit in the L2s / Infinity Cache, so the reduce is bound by the
// bytes it keeps in flight, not by HBM: 16-byte loads x 4 accumulators x
// up to 16 split lanes keep ~8x more in flight than one float per lane.
template <int SL>
__global__ void __launch_bounds__(256) slab_reduce4_kernel(const float* slab, int splits, int ni, int nj, int C,
                                                          int cvalid, int64_t s_i, int64_t s_tap, int64_t s_c,
                                                          float* out, int accumulate) {
  constexpr int L = 256 / SL;  // float4 output groups per block
  __shared__ f32x4 sh[SL][L];
  const int l = threadIdx.x % L, q = threadIdx.x / L;
  const int64_t tot4 = (int64_t)ni * nj / 4;
  const int64_t idx4 = (int64_t)blockIdx.x * L + l;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab);
  f32x4 a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (idx4 < tot4) {
    int k = q;
    for (; k + 3 * SL < splits; k += 4 * SL)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += s4[(int64_t)(k + u * SL) * tot4 + idx4];
    // (the < 4 remaining splits of a lane: clamped loads issued together
    // measured slower here -- the duplicate loads cost more than the round
    // trips, profiles/r4al_ab_epilogue_latency.log)
    for (; k < splits; k += SL) a[0] += s4[(int64_t)k * tot4 + idx4];
  }
  sh[q][l] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (q != 0 || idx4 >= tot4) return;
  f32x4 s = sh[0][l];
#pragma unroll
  for (int w = 1; w < SL; ++w) s += sh[w][l];
  // the 4 destinations, then (accumulate) their old values loaded together
  // before the first store (loaded behind the stores they were 4 round trips)
  float* o[4];
  float old[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t idx = idx4 * 4 + e;
    const int i = (int)(idx / nj), j = (int)(idx - (int64_t)i * nj);
    const int tap = j / C, c = j - tap * C;
    o[e] = c < cvalid ? out + i * s_i + tap * s_tap + c * s_c : nullptr;
  }
  if (accumulate) {
#pragma unroll
    for (int e = 0; e < 4; ++e) old[e] = o[e] ? *o[e] : 0.f;
  }
  // the values formed (one wait for the loads) before the guarded stores:
  // sunk into the branches, each store waited vmcnt(0) -- for the previous
  // store too
  float val[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    val[e] = accumulate ? old[e] + s[e] : s[e];
    asm volatile("" : "+v"(val[e]));
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (o[e]) *o[e] = val[e];
}

template <int SL>
void launch_slab4(const float* slab, int splits, int ni, int nj, int C, int cvalid, int64_t s_i, int64_t s_tap,
                  int64_t s_c, float* out, int accumulate, hipStream_t st) {
  constexpr int L = 256 / SL;
  const int64_t tot4 = (int64_t)ni * nj / 4;
  hipLaunchKernelGGL(slab_reduce4_kernel<SL>, dim3((unsigned)((tot4 + L - 1) / L)), dim3(256), 0, st, slab, splits,
                     ni, nj, C, cvalid, s_i, s_tap, s_c, out, accumulate);
}

}  // namespace

int gemm_wgrad_v2_tile(const VuGemmWgrad& p, int dtype, int* bi, int* bj);
int gemm_wgrad_v2_launch(const VuGemmWgrad& p, hipStream_t st);
int gemm_wgrad_v3_tile(const VuGemmWgrad& p, int dtype, int* bi, int* bj);
int gemm_wgrad_v3_launch(const VuGemmWgrad& p, hipStream_t st);

extern int g_tune_gen;  // gemm_fwd.hip (VU_TUNE_GEN)
static bool use_v2w(int dtype) { return g_tune_gen >= 2 && dtype == VU_BF16; }
static bool use_v3w(int dtype) { return g_tune_gen >= 3 && use_v2w(dtype); }

// Output tile the dispatcher will use (host split-K heuristic).  Returns the
// kernel generation: 3 = halo kernel (splits must be whole 128-pixel tiles),
// 2 = large-tile LDS-DMA kernel, 1 = register-staged kernel.
extern "C" int vu_gemm_wgrad_tile(const VuGemmWgrad* args, int dtype, int* bi, int* bj) {
  if (use_v3w(dtype) && gemm_wgrad_v3_tile(*args, dtype, bi, bj)) return 3;
  if (use_v2w(dtype) && gemm_wgrad_v2_tile(*args, dtype, bi, bj)) return 2;
  *bi = args->ni <= 64 ? 64 : 128;
  *bj = 128;
  return 1;
}

extern "C" int vu_gemm_wgrad(const VuGemmWgrad* args, int dtype, void* stream) {
  int epc = dtype == VU_BF16 ? 8 : 4;
  const VuGather* gs[2] = {&args->p, &args->q};
  for (auto g : gs) {
    if (g->C % epc != 0 || g->nsrc < 1 || g->nsrc > 3) return (int)hipErrorInvalidValue;
    for (int t = 0; t < g->nsrc; ++t)
      if (g->cend[t] % epc != 0 || g->stride[t] % epc != 0) return (int)hipErrorInvalidValue;
  }
  if (args->p.N != args->q.N || args->p.H != args->q.H || args->p.W != args->q.W)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  int bi, bj;
  if (use_v3w(dtype) && args->m_per_split % 128 == 0 && gemm_wgrad_v3_tile(*args, dtype, &bi, &bj))
    return gemm_wgrad_v3_launch(*args, st);
  if (use_v2w(dtype) && gemm_wgrad_v2_tile(*args, dtype, &bi, &bj)) return gemm_wgrad_v2_launch(*args, st);
  return dtype == VU_BF16 ? dispatch_wg<bf16_t>(*args, st) : dispatch_wg<float>(*args, st);
}

int g_tune_slab4 = 1;  // VU_TUNE_SLAB4 = 0: the scalar slab reduce (A/B runs)
static bool slab4_on() { return g_tune_slab4 != 0; }

extern "C" int vu_slab_reduce(const float* slab, int splits, int ni, int nj, int C, int cvalid, int64_t s_i,
                              int64_t s_tap, int64_t s_c, float* out, int accumulate, void* stream) {
  int64_t tot = (int64_t)ni * nj;
  if (tot == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (tot % 4 == 0 && reinterpret_cast<uintptr_t>(slab) % 16 == 0 && slab4_on()) {
    // split lanes: about 4 slab loads per lane, at most 16 lanes
    if (splits >= 64) launch_slab4<16>(slab, splits, ni, nj, C, cvalid, s_i, s_tap, s_c, out, accumulate, st);
    else if (splits >= 32) launch_slab4<8>(slab, splits, ni, nj, C, cvalid, s_i, s_tap, s_c, out, accumulate, st);
    else if (splits >= 16) launch_slab4<4>(slab, splits, ni, nj, C, cvalid, s_i, s_tap, s_c, out, accumulate, st);
    else if (splits >= 8) launch_slab4<2>(slab, splits, ni, nj, C, cvalid, s_i, s_tap, s_c, out, accumulate, st);
    else launch_slab4<1>(slab, splits, ni, nj, C, cvalid, s_i, s_tap, s_c, out, accumulate, st);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)((tot + 63) / 64)), dim3(256), 0,
                     (hipStream_t)stream, slab, splits, ni, nj, C, cvalid, s_i, s_tap, s_c, out, accumulate);
  return (int)hipGetLastError();
}
