// Persistent short-K GEMM ("v5", bf16): out[m][j] = sum_k A[m][k] B[j][k]
// for the 1x1-type problems of gemm_fwd2.hip whose K is a few 64-wide steps
// (K = 128..2048: attention-gate convs and their input gradients below the
// 256^2 level, ConvTranspose2d forward with the pixel-shuffle store, the
// ConvTranspose2d input gradient as a 2x2 parity gather).
//
// With 4-16 K steps per 256-row tile, a block that loads, computes and then
// stages its tile through LDS for the stores spends most of its life in the
// pipeline fill and the epilogue (gemm_fwd2.hip measured 270-450 TFLOP/s
// here).  This kernel keeps one block per CU alive over a strided walk of
// tiles and flattens (tile, k-step) into ONE stream of steps, so the LDS-DMA
// ring never drains: the first stages of tile t+1 are in flight while tile t
// finishes and stores.
//
//   * MFMA(B-fragment, A-fragment): the accumulator rows are output COLUMNS,
//     so a lane owns 4*GS consecutive output columns of one pixel (B rows are
//     read in a permuted order, as in gemm_stream.hip) and stores 16/32-byte
//     pieces straight from registers -- no LDS staging, no barrier;
//   * the B tile's LDS swizzle takes bit 3/4 of the row instead of bit 2 so
//     the permuted fragment reads stay conflict-free;
//   * BatchNorm partial statistics per wave (64 rows) by DPP row sums;
//   * accumulate (input gradients): the old output values are loaded at the
//     start of the tile's last step, before the next stage's DMA, so waiting
//     for them does not drain the ring.
#include "common.h"
#include "../../include/vaeunet.h"

static __device__ __attribute__((aligned(16))) uint32_t v5_zero_page[16];

namespace {

constexpr int KB = 128;  // bytes of K per LDS row per step (64 bf16)
constexpr int BM = 256, WM = 4, WN = 2, NT = WM * WN * 64, NS = 3;
typedef __attribute__((address_space(3))) void lds_void;

VU_DEV int swz_a(int row, int chunk) { return row * KB + ((chunk ^ (row & 7)) << 4); }
template <int GS>
VU_DEV int fb(int row) { return (row & 3) | (((row >> (GS == 4 ? 4 : 3)) & 1) << 2); }
template <int GS>
VU_DEV int swz_b(int row, int chunk) { return row * KB + ((chunk ^ fb<GS>(row)) << 4); }

// 256-column tiles (round 6, VU_TUNE_V5_WIDE): 32-wide K steps, 64-byte LDS
// rows.  ds_read_b128 serves 16-lane groups {0-3,12-15,20-27}, ...; a lane
// reads row r16 = lane & 15 (+ a fragment base) at chunk lane >> 4, so the
// physical chunk is the logical one XOR 2 * bit 2 of the row for A and XOR
// 2 * bit 5 for B (whose fragment rows step by 32 every 4 lanes): every
// group then hits 16 distinct 16-byte slots of a 256-byte bank window.
VU_DEV int swz_aw(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4); }
VU_DEV int swz_bw(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 5) & 1) << 1)) << 4); }

template <int N>
VU_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int R>
VU_DEV float ror_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false));
}
VU_DEV float row16_sum(float v) { return ror_add<1>(ror_add<2>(ror_add<4>(ror_add<8>(v)))); }
VU_DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
VU_DEV float lo_f(uint32_t w) { return __uint_as_float(w << 16); }
VU_DEV float hi_f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

struct Pix { int n, h, w; bool ok; };

// Tile t of the walk -> (row tile, column tile).  grp (VU_TUNE_V5_GRP, round
// 6): consecutive runs of 32 tiles -- the tiles one XCD's 32 CUs hold at a
// time -- cover a 4 x 8 block of the tile grid instead of 2 x 16, when the
// grid divides that way (per XCD: A of 4 row tiles + B of 8 column tiles
// instead of 2 + 16, 4 instead of 5 MB at K = 1024).
VU_DEV void v5_tile(int t, int ntiles, int grp, int& mt, int& nt) {
  if (grp) {
    const int g = t >> 5, i = t & 31, ngc = ntiles >> 3;
    const int gr = g / ngc;
    mt = gr * 4 + (i >> 3);
    nt = (g - gr * ngc) * 8 + (i & 7);
  } else {
    mt = t / ntiles;
    nt = t - mt * ntiles;
  }
}

template <int BN, bool STATS, bool ACC, bool RELU = false>  // RELU: epilogue ReLU (VuGemmFwd.relu)
__global__ __launch_bounds__(NT, 1) void gemm_fwd_v5_kernel(VuGemmFwd p, int grp) {
  constexpr bool WD = BN == 256;        // round 6: 256 x 256 tiles on 32-wide K steps
  static_assert(!(WD && ACC), "the wide tiles have no accumulate variant (registers)");
  constexpr int KBY = WD ? 64 : KB;     // bytes of K per LDS row per step
  constexpr int KST = KBY / 2;          // K elements per step
  constexpr int CH = KBY / 16;          // 16-byte chunks per row
  constexpr int RS = WD ? 2 : 3;        // log2(CH)
  constexpr int NSW = WD ? 4 : NS;      // ring slots: NSW - 1 steps in flight (96 KB either way)
  constexpr int KK = KST / 32;          // MFMA k-slabs per step
  constexpr int WNC = BN / WN;          // columns per wave: 128, 64 or 32
  constexpr int TM = BM / WM / 16;      // 4 pixel fragments per wave
  constexpr int TN = WNC / 16;          // 8, 4 or 2 column fragments per wave
  constexpr int GS = TN;                // a lane owns 4*GS consecutive columns
  constexpr int CPL = GS / 2;           // 16-byte pieces per lane and pixel
  constexpr int LA = BM * CH / NT, LB = BN * CH / NT, NL = LA + LB;
  constexpr int NST = TM * CPL + (STATS ? 2 * TN : 0);  // vector stores per epilogue
  constexpr int STAGE = (BM + BN) * KBY;
  __shared__ __attribute__((aligned(16))) char smem[NSW * STAGE];

  const VuGather& g = p.a;
  const int M = g.N * g.H * g.W;  // < 2^31 (host check)
  const int HW = g.H * g.W;
  const int K = g.R * g.S * g.C;
  const int nk = (K + KST - 1) / KST;
  const int ntiles = p.ncol / BN;
  const int T = (M / BM) * ntiles;
  const int G = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, G);
  const int mine = (T - lb + G - 1) / G;
  const int S = mine * nk;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int gq = lane >> 4, r16 = lane & 15;
  const int pchunk = lane & (CH - 1);
  // pixel -> (n, h, w) and ConvT column -> (tap, channel) decodes: once per
  // tile per row, by multiply-shift (runtime integer divisions were ~1/3 of
  // the kernel's VALU instructions)
  const FastDiv div_hw((uint32_t)HW), div_w((uint32_t)g.W), div_co((uint32_t)(p.cout > 0 ? p.cout : 1));
  const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
  const void* zp = (const void*)v5_zero_page;

  // ---- staging state: the tile / k-step the next stage() call loads ----
  // A lane's rows and chunks are fixed; per (tile, tap, source) SEGMENT of
  // k-steps its row pointers are resolved once and then advance by 64
  // channels per step (the per-step gather decode cost more VALU time than
  // the MFMAs of the step).
  // row & 7 (row bit 2 for the wide tiles) is the same for all LA rows
  const int lch_a = WD ? pchunk ^ (((tid >> 4) & 1) << 1) : pchunk ^ ((tid >> 3) & 7);
  int sg_t = lb, sg_kt = 0, seg_step = 0, seg_rem = 0;
  const bf16_t* ap[LA];
  const bf16_t* bp[LB];
  int lch_b[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i)
    lch_b[i] = WD ? pchunk ^ ((((i * NT + tid) >> 7) & 1) << 1) : pchunk ^ fb<GS>((i * NT + tid) >> 3);
  Pix pa[LA];
  auto stage = [&](int slot) {
    const int k0 = sg_kt * KST;
    const int tap = k0 / g.C;
    const int cbase = k0 - tap * g.C;
    if (sg_kt == 0) {
      int mt, ntl;
      v5_tile(sg_t, ntiles, grp, mt, ntl);
      const int n0 = ntl * BN;
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        const int m = mt * BM + ((i * NT + tid) >> RS);
        pa[i].n = (int)div_hw.div((uint32_t)m);
        const int rem = m - pa[i].n * HW;
        pa[i].h = (int)div_w.div((uint32_t)rem);
        pa[i].w = rem - pa[i].h * g.W;
      }
#pragma unroll
      for (int i = 0; i < LB; ++i)
        bp[i] = bmat + (int64_t)(n0 + ((i * NT + tid) >> RS)) * p.ldb + lch_b[i] * 8;
    }
    if (sg_kt == 0 || cbase == 0 || cbase == g.cend[0] || (g.nsrc > 2 && cbase == g.cend[1])) {
      const int r = tap / g.S, s = tap - (tap / g.S) * g.S;
      const int t = (cbase >= g.cend[0]) + (g.nsrc > 2 && cbase >= g.cend[1]);
      const int c0 = t == 0 ? 0 : g.cend[t - 1];
      const bf16_t* src = reinterpret_cast<const bf16_t*>(g.src[t]);
      const int64_t st = g.stride[t];
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        const int hs = pa[i].h * g.sy + r * g.dy + g.oy;
        const int ws = pa[i].w * g.sx + s * g.dx + g.ox;
        ap[i] = nullptr;
        if ((unsigned)hs < (unsigned)g.Hs && (unsigned)ws < (unsigned)g.Ws)
          ap[i] = src + (((int64_t)pa[i].n * g.Hs + hs) * g.Ws + ws) * st + (cbase - c0) + lch_a * 8;
      }
      seg_step = 0;
      seg_rem = g.cend[t] - cbase;
    }
    char* A = smem + slot * STAGE;
    char* B = A + BM * KBY;
    const int off = seg_step * KST;
    const bool cin = lch_a * 8 < seg_rem - off;  // channel tail of the source
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const void* gp = (ap[i] != nullptr && cin) ? (const void*)(ap[i] + off) : zp;
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(A + (i * NT + wid * 64) * 16), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const void* gp = k0 + lch_b[i] * 8 < K ? (const void*)(bp[i] + k0) : zp;
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(B + (i * NT + wid * 64) * 16), 16, 0, 0);
    }
    ++seg_step;
    if (++sg_kt == nk) {
      sg_kt = 0;
      sg_t += G;
    }
  };

  // B row (output column, wave-local) read by fragment j, lane row rr
  auto wrow = [&](int j, int rr) { return 4 * GS * (rr >> 2) + 4 * j + (rr & 3); };
  // destination of this lane's columns [col0, col0 + 4*GS) of pixel m
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
  auto dst_of = [&](int m, int col0) -> bf16_t* {
    if (p.out_mode == 0) return out + (int64_t)m * p.out_stride + p.out_coff + col0;
    const int n = (int)div_hw.div((uint32_t)m);
    const int rem = m - n * HW;
    const int h = (int)div_w.div((uint32_t)rem), w = rem - h * g.W;
    if (p.out_mode == 2)
      return out + ((int64_t)(n * p.oH + 2 * h + p.opy) * p.oW + 2 * w + p.opx) * p.out_stride + p.out_coff + col0;
    const int ab = (int)div_co.div((uint32_t)col0), co = col0 - ab * p.cout;
    const int oy = 2 * h + (ab >> 1) + p.opy, ox = 2 * w + (ab & 1) + p.opx;
    return out + ((int64_t)(n * p.oH + oy) * p.oW + ox) * p.out_stride + p.out_coff + co;
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  u32x4 old[TM][CPL];
  bf16_t* dst[TM];

  int ct = lb, ckt = 0;  // tile / k-step being computed
  stage(0);
#pragma unroll
  for (int q = 1; q < NSW - 1; ++q)
    if (S > q) stage(q);
  for (int s = 0; s < S; ++s) {
    const bool after_epi = s > 0 && ckt == 0;
    // steps issued after s that may stay in flight (and the last epilogue's stores)
    if (NSW == 4 && s + 2 < S) {
      if (after_epi) wait_vm<2 * NL + NST>(); else wait_vm<2 * NL>();
    } else if (s + 1 < S) {
      if (after_epi) wait_vm<NL + NST>(); else wait_vm<NL>();
    } else {
      if (after_epi) wait_vm<NST>(); else wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool last = ckt == nk - 1;
    int mt, ntl;
    v5_tile(ct, ntiles, grp, mt, ntl);
    const int m0 = mt * BM, n0 = ntl * BN;
    const int col0 = n0 + wn * WNC + 4 * GS * gq;
    if (last) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        dst[i] = dst_of(m0 + wm * 64 + 16 * i + r16, col0);
        if (ACC) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) old[i][c] = *reinterpret_cast<const u32x4*>(dst[i] + 8 * c);
        }
      }
    }
    if (s + NSW - 1 < S) stage((s + NSW - 1) % NSW);
    const char* A = smem + (s % NSW) * STAGE;
    const char* B = A + BM * KBY;
    u32x4 af[KK][TM], bf[KK][TN];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int ch = kk * 4 + gq;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[kk][i] = *reinterpret_cast<const u32x4*>(A + (WD ? swz_aw(wm * 64 + 16 * i + r16, ch)
                                                             : swz_a(wm * 64 + 16 * i + r16, ch)));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[kk][j] = *reinterpret_cast<const u32x4*>(B + (WD ? swz_bw(wn * WNC + wrow(j, r16), ch)
                                                             : swz_b<GS>(wn * WNC + wrow(j, r16), ch)));
    }
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[kk][j]),
                                                              __builtin_bit_cast(bf16x8, af[kk][i]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (!last) {
      ++ckt;
      continue;
    }
    // ---- epilogue from registers: acc[i][j][r] = pixel m0 + wm*64 + 16i + r16,
    //      column col0 + 4j + r ----
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      f32x4 bv = f32x4{0, 0, 0, 0};
      if (p.bias) {
        const int c = col0 + 4 * j;
        bv = *reinterpret_cast<const f32x4*>(p.bias + (p.out_mode == 1 ? c % p.cout : c));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = rnd<bf16_t>(acc[i][j][r] + bv[r]);
    }
    if constexpr (RELU)
#pragma unroll
      for (int i = 0; i < TM; ++i) epi_relu(acc[i]);
    // the old values were loaded before stage(s + NSW - 1): only that stage may stay in flight
    if (ACC) {
      if (s + NSW - 1 < S) wait_vm<NL>(); else wait_vm<0>();
    }
    if (STATS) {
      const int srow = (m0 >> 6) + wm;  // 64-row statistics tile
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 sm, m2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sv = 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i) sv += acc[i][j][r];
          sv = row16_sum(sv);
          const float mean = sv * (1.f / 64.f);
          float v = 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const float d = acc[i][j][r] - mean;
            v += d * d;
          }
          sm[r] = sv;
          m2[r] = row16_sum(v);
        }
        if (r16 == 0) {
          *reinterpret_cast<f32x4*>(p.stat_sum + (int64_t)srow * p.ncol + col0 + 4 * j) = sm;
          *reinterpret_cast<f32x4*>(p.stat_m2 + (int64_t)srow * p.ncol + col0 + 4 * j) = m2;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const f32x4 a = acc[i][2 * c], b = acc[i][2 * c + 1];
        u32x4 v;
        if (ACC) {
          const u32x4 o = old[i][c];
          v = u32x4{pack2(lo_f(o[0]) + a[0], hi_f(o[0]) + a[1]), pack2(lo_f(o[1]) + a[2], hi_f(o[1]) + a[3]),
                    pack2(lo_f(o[2]) + b[0], hi_f(o[2]) + b[1]), pack2(lo_f(o[3]) + b[2], hi_f(o[3]) + b[3])};
        } else {
          v = u32x4{pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(b[0], b[1]), pack2(b[2], b[3])};
        }
        *reinterpret_cast<u32x4*>(dst[i] + 8 * c) = v;
      }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    ckt = 0;
    ct += G;
  }
}

int cu_count5() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

int g_v5 = 1;  // VU_TUNE_V5: 0 off, 1 on, k >= 2 on with the grid capped at k (tests)
int g_v5_grp = 0;  // VU_TUNE_V5_GRP

template <int BN, bool STATS, bool ACC>
int launch5(const VuGemmFwd& p, hipStream_t st) {
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  const int64_t mtiles = M / BM, ntiles = p.ncol / BN;
  const int64_t T = mtiles * ntiles;
  int64_t grid = T < cu_count5() ? T : cu_count5();
  if (g_v5 >= 2 && grid > g_v5) grid = g_v5;
  const int grp = g_v5_grp && ntiles >= 8 && ntiles % 8 == 0 && mtiles % 4 == 0 && T % 32 == 0 ? 1 : 0;
  if (p.relu)
    hipLaunchKernelGGL((gemm_fwd_v5_kernel<BN, STATS, ACC, true>), dim3((unsigned)grid), dim3(NT), 0, st, p, grp);
  else
    hipLaunchKernelGGL((gemm_fwd_v5_kernel<BN, STATS, ACC>), dim3((unsigned)grid), dim3(NT), 0, st, p, grp);
  return (int)hipGetLastError();
}

template <int BN>
int launch_bn(const VuGemmFwd& p, hipStream_t st) {
  const bool stats = p.stat_sum != nullptr, acc = p.accumulate != 0;
  if constexpr (BN == 256) {
    if (acc) return (int)hipErrorInvalidValue;
    return stats ? launch5<BN, true, false>(p, st) : launch5<BN, false, false>(p, st);
  } else {
    if (stats) return acc ? launch5<BN, true, true>(p, st) : launch5<BN, true, false>(p, st);
    return acc ? launch5<BN, false, true>(p, st) : launch5<BN, false, false>(p, st);
  }
}

int g_v5_wide = 0;  // VU_TUNE_V5_WIDE

// the 256 x 256 tiles: a whole round of tiles (one per CU), no accumulate,
// ConvTranspose outputs in 32-channel runs, at least two 32-wide K steps
bool wide_ok(const VuGemmFwd& p) {
  if (!g_v5_wide || p.accumulate || p.ncol % 256 != 0) return false;
  if (p.out_mode == 1 && p.cout % 32 != 0) return false;
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  const int K = p.a.R * p.a.S * p.a.C;
  if (K < 64) return false;
  return (M / BM) * (p.ncol / 256) >= cu_count5();
}

}  // namespace

int gemm_fwd_v2_bm(const VuGemmFwd& p, int dtype);  // gemm_fwd2.hip (shared eligibility)

// Statistics row tile (64) when v5 serves this problem, else 0: every v2
// problem with whole 256-row tiles, 64 / 128-multiple column counts, a
// 32-bit pixel count and at least 2 K steps.
int gemm_fwd_v5_bm(const VuGemmFwd& p, int dtype) {
  if (g_v5 == 0 || gemm_fwd_v2_bm(p, dtype) == 0) return 0;
  const VuGather& g = p.a;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  if (M % BM != 0 || M >= ((int64_t)1 << 31)) return 0;
  if (p.ncol != 64 && p.ncol % 128 != 0) return 0;
  if (p.out_mode == 1 && p.cout % 16 != 0) return 0;
  if (p.out_mode != 0 && p.out_mode != 1 && p.out_mode != 2) return 0;
  if (p.ldb < 0 || (p.out_stride % 8) != 0 || (p.out_coff % 8) != 0) return 0;
  const int nk = (g.R * g.S * g.C + 63) / 64;
  if (nk < 2) return 0;
  return 64;
}

int gemm_fwd_v5_launch(const VuGemmFwd& p, hipStream_t st) {
  if (p.ncol == 64) return launch_bn<64>(p, st);
  if (wide_ok(p)) return launch_bn<256>(p, st);
  return launch_bn<128>(p, st);
}

int gemm_fwd_v5_tune(int key, int value) {
  if (key == VU_TUNE_V5) {
    g_v5 = value < 0 ? 0 : value;
    return 0;
  }
  if (key == VU_TUNE_V5_WIDE) {
    g_v5_wide = value ? 1 : 0;
    return 0;
  }
  if (key == VU_TUNE_V5_GRP) {
    g_v5_grp = value ? 1 : 0;
    return 0;
  }
  return -1;
}
