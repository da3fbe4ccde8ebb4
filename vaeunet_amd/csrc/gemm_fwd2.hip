// Implicit-GEMM forward-type kernel, large-tile bf16 variant ("v2").
//
// Same contract as gemm_fwd.hip (out[m][j] = sum_k A[m][k] B[j][k], A an
// im2col gather of up to three NHWC sources), used for the bf16 GEMMs the
// halo kernel (gemm_fwd3.hip) does not take: 1x1 convs (attention gates,
// ConvTranspose2d as a GEMM with a pixel-shuffle store, input gradients of
// 1x1 convs) and strided / parity-class gathers:
//   * 8 waves (512 threads), block tile 256 x 128 (waves 4x2, 64x64 each) or
//     256 x 64 (waves 8x1, 32x64 each) for narrow outputs;
//   * operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per
//     lane, no VGPR staging, no ds_write): each lane computes its own gather
//     address — zero padding, K / M / N tails point the lane at a 16-byte
//     zero page — and the XOR swizzle is applied on the SOURCE chunk so the
//     LDS image stays lane-linear (cdna_hip_programming §5.4 rule 21);
//   * an NS-slot LDS ring (NS = min(3, K steps): short-K 1x1 GEMMs keep the
//     footprint small so several blocks share a CU and hide each other's
//     load latency), counted vmcnt + raw s_barrier, 16x16x32 bf16 MFMA,
//     conflict-free ds_read_b128 fragment reads;
//   * epilogue: the bf16-rounded tile staged in LDS (half the footprint of
//     fp32), BatchNorm partial statistics on exactly those values, 16-byte
//     coalesced stores; out_mode 1 scatters the ConvTranspose2d(k=2, s=2)
//     pixel shuffle, out_mode 2 a stride-2 parity lattice.
#include "common.h"
#include "../../include/vaeunet.h"
#include <stdlib.h>

static __device__ __attribute__((aligned(16))) uint32_t vu_zero_page[16];  // 16 B of zeros: padding lanes DMA from here

namespace {

constexpr int KB = 128;  // bytes of K per LDS row per step (64 bf16)
typedef __attribute__((address_space(3))) void lds_void;

VU_DEV int swz(int row, int chunk) { return row * KB + ((chunk ^ (row & 7)) << 4); }


template <int BM, int BN, int WM, int WN, int NS, bool SPLIT = false, int OCC = 1>
__global__ __launch_bounds__(WM * WN * 64, OCC) void gemm_fwd_v2_kernel(VuGemmFwd p) {
  constexpr int NT = WM * WN * 64;
  constexpr int EPC = 8;                  // bf16 per 16-byte chunk
  constexpr int BKE = 64;                 // K elements per step
  constexpr int LA = BM * 8 / NT;         // A glds per thread per step
  constexpr int LB = BN * 8 / NT;         // B glds per thread per step
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int ES = BN + 8;              // bf16 epilogue row stride (16-byte aligned rows)
  constexpr int STAGE = (BM + BN) * KB;
  constexpr int NSTAGE = NS;              // LDS ring: DMA runs NS-1 K steps ahead
  constexpr int MAIN = NSTAGE * STAGE;
  constexpr int EPI = BM * ES * 2;
  constexpr int RED = (NT / BN) * BN * 4;
  constexpr int LDS_BYTES = (MAIN > EPI ? MAIN : EPI) + RED;
  static_assert(LA >= 1 && LB >= 1, "tile too small for the thread count");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const VuGather& g = p.a;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  const int K = g.R * g.S * g.C;
  const int mtiles = (int)((M + BM - 1) / BM);
  const int ntiles = (p.ncol + BN - 1) / BN;
  // SPLIT: the block index also picks a contiguous range of K steps (kidx)
  const int ksplit = SPLIT ? p.ksplit : 1;
  const int bid0 = xcd_remap(blockIdx.x, mtiles * ntiles * ksplit);
  const int kidx = SPLIT ? bid0 / (mtiles * ntiles) : 0;
  const int bid = SPLIT ? bid0 - kidx * (mtiles * ntiles) : bid0;
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int pchunk = lane & 7;  // physical chunk this lane writes

  // rows this thread loads: row = (i*NT + tid) / 8; its 16-byte chunk of a
  // row is the same for every row (row & 7 == (tid >> 3) & 7).  Per row the
  // pixel index and the strided base coordinates are resolved once; a step
  // then only adds the tap's (uniform) offset -- the per-step gather decode
  // otherwise costs more VALU time than the step's MFMAs.
  const int lchunk_a = pchunk ^ ((tid >> 3) & 7);
  int64_t rpix[LA];   // pixel index of (n, h*sy, w*sx) in the source image
  int rh[LA], rw[LA]; // h*sy, w*sx (-1 << 20 for rows beyond M: never in bounds)
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    int row = (i * NT + tid) >> 3;
    int64_t m = m0 + row;
    const bool ok = m < M;
    int64_t mm = ok ? m : 0;
    int hw = g.H * g.W;
    const int n = (int)(mm / hw);
    int rem = (int)(mm - (int64_t)n * hw);
    const int h = rem / g.W;
    const int w = rem - h * g.W;
    rh[i] = ok ? h * g.sy : -(1 << 20);
    rw[i] = w * g.sx;
    rpix[i] = ((int64_t)n * g.Hs + h * g.sy) * g.Ws + w * g.sx;
  }
  const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
  const void* zp = (const void*)vu_zero_page;
  const bf16_t* brow[LB];
  int lchunk_b[LB];
  bool bok[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    int row = (i * NT + tid) >> 3;
    lchunk_b[i] = pchunk ^ (row & 7);
    bok[i] = n0 + row < p.ncol;
    brow[i] = bmat + (int64_t)(bok[i] ? n0 + row : 0) * p.ldb + lchunk_b[i] * EPC;
  }

  auto stage = [&](int kt, int buf) {
    const int k0 = kt * BKE;
    const int tap = k0 / g.C;
    const int r = tap / g.S, s = tap - (tap / g.S) * g.S;
    const int cbase = k0 - tap * g.C;
    const int t = (cbase >= g.cend[0]) + (g.nsrc > 2 && cbase >= g.cend[1]);
    const int c0 = t == 0 ? 0 : g.cend[t - 1];
    const bf16_t* src = reinterpret_cast<const bf16_t*>(g.src[t]) + (cbase - c0) + lchunk_a * EPC;
    const int64_t st = g.stride[t];
    const int dh = r * g.dy + g.oy, dw = s * g.dx + g.ox;
    const int64_t dpix = (int64_t)dh * g.Ws + dw;
    const bool cin = cbase + lchunk_a * EPC < g.cend[t];
    char* A = smem + buf * STAGE;
    char* B = A + BM * KB;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const void* gp = zp;
      if (cin && (unsigned)(rh[i] + dh) < (unsigned)g.Hs && (unsigned)(rw[i] + dw) < (unsigned)g.Ws)
        gp = src + (rpix[i] + dpix) * st;
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(A + (i * NT + wid * 64) * 16), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const void* gp = (bok[i] && k0 + lchunk_b[i] * EPC < K) ? (const void*)(brow[i] + k0) : zp;
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(B + (i * NT + wid * 64) * 16), 16, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  const int nkt = (K + BKE - 1) / BKE;
  const int kb = SPLIT ? kidx * nkt / ksplit : 0;
  const int nk = (SPLIT ? (kidx + 1) * nkt / ksplit : nkt) - kb;
  // Pipeline: stage kt+2 is issued right after the barrier of step kt, into
  // the ring slot step kt-1 just finished reading.  Each thread's own DMA is
  // retired by a COUNTED vmcnt (the NL loads of the newest stage may stay in
  // flight), then the raw s_barrier makes every thread's landed bytes
  // visible; no __syncthreads() (it would drain vmcnt to 0) in the loop.
  constexpr int NL = LA + LB;
  stage(kb, 0);
  if (NSTAGE >= 3 && nk > 1) stage(kb + 1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (NSTAGE >= 3 && kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (NSTAGE >= 3 && kt + 2 < nk) stage(kb + kt + 2, (kt + 2) % NSTAGE);
    else if (NSTAGE == 2 && kt + 1 < nk) stage(kb + kt + 1, (kt + 1) % NSTAGE);
    const int cur = kt % NSTAGE;
    const char* A = smem + cur * STAGE;
    const char* B = A + BM * KB;
    // the second k-half's fragments are read while the first half's MFMAs issue
    u32x4 af[2][TM], bf[2][TN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[kk][i] = *reinterpret_cast<const u32x4*>(A + swz(wm * (BM / WM) + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[kk][j] = *reinterpret_cast<const u32x4*>(B + swz(wn * (BN / WN) + j * 16 + (lane & 15), ch));
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[kk][i]),
                                                              __builtin_bit_cast(bf16x8, bf[kk][j]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  if (SPLIT) {
    // raw fp32 partial tile -> slab kidx (rows m0 + ..., all valid: M % BM == 0)
    float* slab = p.workspace + (int64_t)kidx * M * p.ncol;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * (BN / WN) + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = m0 + wm * (BM / WM) + i * 16 + 4 * (lane >> 4) + r;
          slab[row * p.ncol + col] = acc[i][j][r];
        }
      }
    return;
  }
  __syncthreads();  // every wave is done with the ring before the epilogue reuses it

  // ---- epilogue: bf16-rounded tile in LDS, BN statistics, 16-byte stores ----
  bf16_t* E = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int col = wn * (BN / WN) + j * 16 + (lane & 15);
      int gj = n0 + col;
      float bv = 0.f;
      if (p.bias && gj < p.ncol) bv = p.bias[p.out_mode == 1 ? gj % p.cout : gj];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = wm * (BM / WM) + i * 16 + 4 * (lane >> 4) + r;
        E[row * ES + col] = (bf16_t)f2bf(epi_act(acc[i][j][r] + bv, p.relu));
      }
    }
  __syncthreads();

  const int rows_valid = (int)((M - m0) < BM ? (M - m0) : BM);
  if (p.stat_sum) {
    float* red = reinterpret_cast<float*>(smem + LDS_BYTES - RED);
    constexpr int PARTS = NT / BN;
    constexpr int RPP = BM / PARTS;
    static_assert(RPP % 16 == 0, "statistics rows per thread: whole batches of 16");
    const int col = tid % BN, part = tid / BN;
    const int r0 = part * RPP, nv = rows_valid - r0;   // rows of this part that are valid (may be <= 0)
    // Round 6: 16 LDS reads in flight per batch (a loop-carried read per row
    // was one LDS round trip per row, twice: ~3 us of a 12 us short-K launch);
    // same sums in the same order
    float s = 0.f;
    for (int rb = 0; rb < RPP; rb += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = bf2f(E[(r0 + rb + u) * ES + col]);
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (rb + u < nv) s += v[u];
    }
    red[part * BN + col] = s;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int q = 0; q < PARTS; ++q) tot += red[q * BN + col];
    const float mean = tot / (float)rows_valid;
    float m2 = 0.f;
    for (int rb = 0; rb < RPP; rb += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = bf2f(E[(r0 + rb + u) * ES + col]);
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (rb + u < nv) { float d = v[u] - mean; m2 += d * d; }
    }
    __syncthreads();
    red[part * BN + col] = m2;
    __syncthreads();
    if (part == 0 && n0 + col < p.ncol) {
      float tm2 = 0.f;
#pragma unroll
      for (int q = 0; q < PARTS; ++q) tm2 += red[q * BN + col];
      p.stat_sum[(int64_t)mt * p.ncol + n0 + col] = tot;
      p.stat_m2[(int64_t)mt * p.ncol + n0 + col] = tm2;
    }
  }

  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
  constexpr int CPR = BN / 8;
  constexpr int NIT = BM * CPR / NT;
  static_assert(BM * CPR % NT == 0, "whole store iterations");
  // Round 6: the destinations (and, accumulating, the old values) of every
  // iteration first, then the adds and stores: a load -> store per iteration
  // was one memory round trip each
  bf16_t* dsts[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = it * NT + tid;
    int row = e / CPR, cc = (e - row * CPR) * 8;
    dsts[it] = nullptr;
    if (row >= rows_valid) continue;
    int gj = n0 + cc;
    if (gj >= p.ncol) continue;
    int64_t m = m0 + row;
    bf16_t* dst;
    if (p.out_mode == 0) {
      dst = out + m * p.out_stride + p.out_coff + gj;
    } else {
      int hw = g.H * g.W;
      int n = (int)(m / hw);
      int rem = (int)(m - (int64_t)n * hw);
      int h = rem / g.W, w = rem - (rem / g.W) * g.W;
      if (p.out_mode == 2) {
        dst = out + (((int64_t)n * p.oH + 2 * h + p.opy) * p.oW + 2 * w + p.opx) * p.out_stride + p.out_coff + gj;
      } else {
        // ConvTranspose2d(k=2, s=2): column gj = (2a+b)*cout + co -> pixel (2h+a, 2w+b)
        int ab = gj / p.cout, co = gj - ab * p.cout;
        int oy = 2 * h + (ab >> 1) + p.opy, ox = 2 * w + (ab & 1) + p.opx;
        dst = out + (((int64_t)n * p.oH + oy) * p.oW + ox) * p.out_stride + p.out_coff + co;
      }
    }
    dsts[it] = dst;
  }
  Vec8<bf16_t> old[NIT];
  if (p.accumulate) {
#pragma unroll
    for (int it = 0; it < NIT; ++it)
      if (dsts[it]) old[it].load(dsts[it]);
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    if (!dsts[it]) continue;
    const int e = it * NT + tid;
    const int row = e / CPR, cc = (e - row * CPR) * 8;
    Vec8<bf16_t> v;
    v.v = *reinterpret_cast<const u32x4*>(E + row * ES + cc);
    if (p.accumulate) {
#pragma unroll
      for (int q = 0; q < 8; ++q) old[it].set(q, old[it].get(q) + v.get(q));
      old[it].store(dsts[it]);
    } else {
      v.store(dsts[it]);
    }
  }
}

template <int BM, int BN, int WM, int WN, int NS, int OCC = 1>
int launch(const VuGemmFwd& p, hipStream_t st) {
  int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  int64_t nblk = ((M + BM - 1) / BM) * ((p.ncol + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_fwd_v2_kernel<BM, BN, WM, WN, NS, false, OCC>), dim3((unsigned)nblk), dim3(WM * WN * 64), 0,
                     st, p);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN>
int launch_ns(const VuGemmFwd& p, hipStream_t st) {
  const int nk = (p.a.R * p.a.S * p.a.C + 63) / 64;
  if (nk == 1) return launch<BM, BN, WM, WN, 1>(p, st);
  if (nk == 2) return launch<BM, BN, WM, WN, 2>(p, st);
  return launch<BM, BN, WM, WN, 3>(p, st);
}

// Tile configuration for short-K problems (<= 2 K steps of 64), where a
// block's life is dominated by its load latency and epilogue: 0 = 256-row
// tiles, 1 = 128-row tiles (8 waves), 2 = 128-row tiles (4 waves).
}  // namespace
int g_v2_cfg = 0;  // VU_TUNE_V2_CFG (A/B runs): the configuration short-K problems get
namespace {
int v2_cfg(const VuGemmFwd& p) {
  const int nk = (p.a.R * p.a.S * p.a.C + 63) / 64;
  return nk <= 2 ? g_v2_cfg : 0;
}

}  // namespace

// Row tile of the v2 kernel for this problem, or 0 when v2 does not apply
// (fp32, channel groups not 64-aligned — a single 1x1 source may end on a
// 32-channel boundary —, ragged column counts, or too few tiles to fill the
// chip).
static bool v2_shape_ok(const VuGemmFwd& p, int dtype) {
  const VuGather& g = p.a;
  if (dtype != VU_BF16) return false;
  const bool one = g.R == 1 && g.S == 1;
  for (int t = 0; t < g.nsrc; ++t) {
    const bool last = t == g.nsrc - 1;
    if (g.stride[t] % 8 != 0) return false;
    if (g.cend[t] % 64 != 0 && !(one && last && g.cend[t] % 32 == 0)) return false;
  }
  if (p.ncol % 8 != 0 || p.ldb % 8 != 0) return false;
  if (p.out_mode == 1) {
    if (p.cout % 8 != 0 || p.out_stride % 8 != 0 || p.out_coff % 8 != 0) return false;
  } else if (p.out_stride % 8 != 0 || p.out_coff % 8 != 0) {
    return false;
  }
  return (int64_t)g.N * g.H * g.W > 0;
}

int gemm_fwd_v2_bm(const VuGemmFwd& p, int dtype) {
  const VuGather& g = p.a;
  if (!v2_shape_ok(p, dtype)) return 0;
  int64_t M = (int64_t)g.N * g.H * g.W;
  int bn = p.ncol <= 64 ? 64 : 128;
  int64_t tiles = ((M + 255) / 256) * ((p.ncol + bn - 1) / bn);
  if (tiles < 256) return 0;
  const int cfg = v2_cfg(p);
  return cfg == 0 || cfg == 4 ? 256 : 128;
}

// Small grids (the ResNet34 encoder's 64^2 / 32^2 / 16^2 levels: too few
// 256-row tiles to fill the chip, 16^2 images too narrow for the 3x3 halo
// kernels' 32-pixel rows): 128 x 64 tiles of 4 waves, two blocks per CU,
// split-K to >= 2 blocks per CU when the tiles alone do not reach it (fp32
// slabs + the deterministic finish of gemm_fwd4.hip).  Returns the split
// (>= 1) when served, else 0.
bool g_small = true;  // VU_TUNE_V2_SMALL

// (The stride-2 parity-class input gradients -- out_mode 2 -- measured 0.3 %
// slower end to end on these tiles than on the generic kernel, VAE same-box
// A/B profiles/r3_ab_parity_v2small.log; they stay there.  splitk_finish_kernel
// handles out_mode 2 all the same.)
int gemm_fwd_v2_small(const VuGemmFwd& p, int dtype) {
  if (!g_small || dtype != VU_BF16 || p.out_mode != 0) return 0;
  const VuGather& g = p.a;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.stride[t] % 8 != 0 || g.cend[t] % 64 != 0) return 0;
  if (p.ncol % 64 != 0 || p.ldb % 8 != 0 || p.out_stride % 8 != 0 || p.out_coff % 8 != 0) return 0;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  if (M % 128 != 0) return 0;
  const int64_t big = ((M + 255) / 256) * ((p.ncol + 127) / 128);
  const int64_t tiles = (M / 128) * (p.ncol / 64);
  const int nk = (g.R * g.S * g.C + 63) / 64;
  if (big >= 256 || tiles < 64 || nk < 8) return 0;
  int ks = (int)((512 + tiles - 1) / tiles);
  if (ks > nk / 8) ks = nk / 8;
  return ks < 1 ? 1 : ks;
}

int64_t gemm_fwd_v2_small_workspace(const VuGemmFwd& p, int dtype) {
  const int ks = gemm_fwd_v2_small(p, dtype);
  return ks > 1 ? (int64_t)ks * p.a.N * p.a.H * p.a.W * p.ncol * (int64_t)sizeof(float) : 0;
}

int splitk_finish_launch(const VuGemmFwd& p, hipStream_t st);  // gemm_fwd4.hip

int gemm_fwd_v2_small_launch(const VuGemmFwd& p, hipStream_t st) {
  const int ks = gemm_fwd_v2_small(p, VU_BF16);
  if (ks <= 1) return launch_ns<128, 64, 2, 2>(p, st);
  if (!p.workspace) return (int)hipErrorInvalidValue;
  VuGemmFwd q = p;
  q.ksplit = ks;
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  const int64_t nblk = (M / 128) * (p.ncol / 64) * ks;
  hipLaunchKernelGGL((gemm_fwd_v2_kernel<128, 64, 2, 2, 3, true>), dim3((unsigned)nblk), dim3(256), 0, st, q);
  return splitk_finish_launch(q, st);
}

// Every other bf16 GEMM the v2 gather serves -- the ones no tile-count rule
// above admits: the ResNet34 decoder's attention-gate 1x1 convs (F_int = 32
// columns) and the downsample shortcuts' stride-2 input gradients at the 64^2
// .. 16^2 levels (out_mode 2), K of one or a few 64-steps.  One 128 x 64
// tile per block (4 waves), no split: these are latency-bound launches of a
// few microseconds, and the generic register-staged kernel they fell to took
// ~11 us each (round-3 config-3 profile).  VU_TUNE_V2_SMALL = 0 turns it off.
int gemm_fwd_v2_tail(const VuGemmFwd& p, int dtype) {
  return g_small && v2_shape_ok(p, dtype) ? 128 : 0;
}

int gemm_fwd_v2_tail_launch(const VuGemmFwd& p, hipStream_t st) { return launch_ns<128, 64, 2, 2>(p, st); }

int gemm_fwd_v2_tune(int key, int value) {
  if (key == VU_TUNE_V2_SMALL) {
    g_small = value != 0;
    return 0;
  }
  return -1;
}

int gemm_fwd_v2_launch(const VuGemmFwd& p, hipStream_t st) {
  switch (v2_cfg(p)) {
    case 1:
      if (p.ncol <= 64) return launch_ns<128, 64, 4, 2>(p, st);
      return launch_ns<128, 128, 2, 4>(p, st);
    case 2:
      if (p.ncol <= 64) return launch_ns<128, 64, 2, 2>(p, st);
      return launch_ns<128, 128, 2, 2>(p, st);
    case 3:
      if (p.ncol <= 64) return launch<128, 64, 2, 2, 2, 2>(p, st);
      return launch<128, 128, 2, 2, 2, 2>(p, st);
    case 4:
      if (p.ncol <= 64) return launch<256, 64, 8, 1, 2>(p, st);
      return launch<256, 128, 4, 2, 2>(p, st);
    case 5:
      if (p.ncol <= 128) return launch<128, 128, 2, 4, 2>(p, st);
      return launch<128, 256, 2, 4, 2>(p, st);
    default:
      if (p.ncol <= 64) return launch_ns<256, 64, 8, 1>(p, st);
      return launch_ns<256, 128, 4, 2>(p, st);
  }
}
