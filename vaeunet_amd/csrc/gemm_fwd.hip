// Implicit-GEMM "forward-type" kernel: out[m][j] = sum_k A[m][k] * B[j][k].
//
// One kernel family covers every dense contraction on the forward and
// input-gradient paths of the reference model:
//   * 3x3 conv, pad 1, no bias      (DoubleConv, unet_parts.py:40,43)
//   * 3x3 conv input gradient      (same gather over dY, flipped weights)
//   * 1x1 conv + bias               (AttentionGate W_g / W_x, unet_parts.py:11,15)
//   * ConvTranspose2d(k=2, s=2)     (unet_parts.py:76) as a GEMM whose
//                                    epilogue performs the pixel shuffle,
//     and its input gradient (gather of the 2x2 sub-pixels).
// A is gathered from NHWC sources on the fly (im2col is never stored; the
// channel concat of unet_parts.py:94 is a per-k-tile source select), B is a
// dense [ncol][K] weight matrix prepared once per step (vu_permute4).
//
// Tiling (CDNA4): 256 threads = 4 waves (2x2), block tile BM x BN, K-step of
// 128 bytes per row (64 bf16 / 32 fp32), LDS double buffer staged through
// registers (the gather + zero padding is done on the way in), XOR-swizzled
// 16-byte chunks (conflict-free ds_read_b128), MFMA 16x16x32 bf16 (speed
// mode) or 16x16x4 f32 (parity mode; exact fp32 fma chain).  The epilogue
// stages the fp32 tile through LDS, computes per-tile BatchNorm partial
// statistics (sum, centered M2) on the dtype-rounded values and writes
// 16-byte coalesced rows.
#include <stdlib.h>
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int KB = 128;  // bytes of K per LDS row per k-step

VU_DEV int swz(int row, int chunk) { return row * KB + ((chunk ^ (row & 7)) << 4); }

template <typename T> struct Mma;
template <> struct Mma<bf16_t> {
  static VU_DEV f32x4 run(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  // Lane group g holds k = 4g..4g+3 of a 16-wide k chunk; MFMA i consumes
  // element i of every lane, so the four MFMAs together cover all 16 k.
  static VU_DEV f32x4 run(u32x4 a, u32x4 b, f32x4 c) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[i]), __uint_as_float(b[i]), c, 0, 0, 0);
    return c;
  }
};

struct RowPix { int n, h, w; bool ok; };

// VuGemmFwd.zbias of output row m (pixel (n, h, w)), column j
VU_DEV float zbias_at(const VuGemmFwd& p, int64_t m, int j) {
  const int hw = p.a.H * p.a.W;
  const int n = (int)(m / hw), rem = (int)(m - (int64_t)n * hw);
  const int h = rem / p.a.W, w = rem - (rem / p.a.W) * p.a.W;
  const int cls = 3 * zb_class(h, p.a.H) + zb_class(w, p.a.W);
  return p.zbias[((int64_t)n * 9 + cls) * p.ncol + j];
}

template <typename T>
VU_DEV u32x4 gather_chunk(const VuGather& g, const RowPix& rp, int tap, int ch) {
  // ch: channel of the first element of this 16-byte chunk (all in one source)
  u32x4 z = {0, 0, 0, 0};
  if (!rp.ok) return z;
  int r = tap / g.S, s = tap - r * g.S;
  int hs = rp.h * g.sy + r * g.dy + g.oy;
  int ws = rp.w * g.sx + s * g.dx + g.ox;
  if ((unsigned)hs >= (unsigned)g.Hs || (unsigned)ws >= (unsigned)g.Ws) return z;
  int t = (ch >= g.cend[0]) + (g.nsrc > 2 && ch >= g.cend[1]);
  int c0 = t == 0 ? 0 : g.cend[t - 1];
  const T* base = reinterpret_cast<const T*>(g.src[t]);
  int64_t pix = ((int64_t)rp.n * g.Hs + hs) * g.Ws + ws;
  return *reinterpret_cast<const u32x4*>(base + pix * g.stride[t] + (ch - c0));
}

template <typename T, int BM, int BN, bool ALIGNED>
__global__ __launch_bounds__(256, 2) void gemm_fwd_kernel(VuGemmFwd p) {
  constexpr int EPC = 16 / sizeof(T);      // elements per 16-byte chunk
  constexpr int BKE = KB / sizeof(T);      // elements of K per step
  constexpr int RA = BM / 32, RB = BN / 32;  // rows per thread (A, B)
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 tiles per wave
  constexpr int ES = BN + 4;                 // epilogue row stride (floats)
  constexpr int MAIN_BYTES = 2 * (BM + BN) * KB;
  constexpr int EPI_BYTES = BM * ES * 4;
  constexpr int LDS_BYTES = (MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES) + 4 * BN * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const VuGather& g = p.a;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  const int K = g.R * g.S * g.C;
  const int mtiles = (int)((M + BM - 1) / BM);
  const int ntiles = (p.ncol + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int chunk = tid & 7;

  RowPix rp[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    int64_t m = m0 + (tid >> 3) + 32 * i;
    rp[i].ok = m < M;
    int64_t mm = rp[i].ok ? m : 0;
    int hw = g.H * g.W;
    rp[i].n = (int)(mm / hw);
    int rem = (int)(mm - (int64_t)rp[i].n * hw);
    rp[i].h = rem / g.W;
    rp[i].w = rem - rp[i].h * g.W;
  }
  const T* bmat = reinterpret_cast<const T*>(p.b);

  u32x4 ra[RA], rb[RB];
  auto load = [&](int kt) {
    int k0 = kt * BKE;
    if (ALIGNED) {
      int tap = k0 / g.C;
      int ch = k0 - tap * g.C + chunk * EPC;
#pragma unroll
      for (int i = 0; i < RA; ++i) ra[i] = gather_chunk<T>(g, rp[i], tap, ch);
    } else {
      int kk = k0 + chunk * EPC;
      int tap = kk / g.C;
      int ch = kk - tap * g.C;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        if (kk < K) ra[i] = gather_chunk<T>(g, rp[i], tap, ch);
        else ra[i] = u32x4{0, 0, 0, 0};
      }
    }
    int kk = k0 + chunk * EPC;
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      int j = n0 + (tid >> 3) + 32 * i;
      if (j < p.ncol && kk < K)
        rb[i] = *reinterpret_cast<const u32x4*>(bmat + (int64_t)j * p.ldb + kk);
      else
        rb[i] = u32x4{0, 0, 0, 0};
    }
  };
  auto store_lds = [&](int buf) {
    char* A = smem + buf * (BM + BN) * KB;
    char* B = A + BM * KB;
#pragma unroll
    for (int i = 0; i < RA; ++i)
      *reinterpret_cast<u32x4*>(A + swz((tid >> 3) + 32 * i, chunk)) = ra[i];
#pragma unroll
    for (int i = 0; i < RB; ++i)
      *reinterpret_cast<u32x4*>(B + swz((tid >> 3) + 32 * i, chunk)) = rb[i];
  };

  // fp32 (parity mode): two-level accumulation.  Each 32-element K-step is
  // summed by its own MFMA chain into a fresh tile, which is then added to the
  // running sum with Kahan compensation: the rounding error no longer grows
  // with K (a single MFMA chain over K = 9*Cin = 576-9216 carried 1.4-4.4x the
  // error of the blocked CPU GEMMs the fp32 oracle runs on, VERDICT r5 item 1,
  // tools/fp32_err_probe.py).  bf16 (speed mode) keeps the single chain.
  constexpr bool CMP = sizeof(T) == 4;
  f32x4 acc[TM][TN], cmp[CMP ? TM : 1][CMP ? TN : 1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  if constexpr (CMP)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) cmp[i][j] = f32x4{0, 0, 0, 0};

  const int nk = (K + BKE - 1) / BKE;
  load(0);
  store_lds(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load(kt + 1);
    const char* A = smem + cur * (BM + BN) * KB;
    const char* B = A + BM * KB;
    f32x4 part[CMP ? TM : 1][CMP ? TN : 1];
    if constexpr (CMP)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) part[i][j] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 af[TM], bf[TN];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const u32x4*>(A + swz(wm * (BM / 2) + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[j] = *reinterpret_cast<const u32x4*>(B + swz(wn * (BN / 2) + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (CMP) part[i][j] = Mma<T>::run(af[i], bf[j], part[i][j]);
          else acc[i][j] = Mma<T>::run(af[i], bf[j], acc[i][j]);
        }
    }
    if constexpr (CMP)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) kahan_add(acc[i][j], cmp[i][j], part[i][j]);
    if (kt + 1 < nk) store_lds(cur ^ 1);
    __syncthreads();
  }
  if constexpr (CMP)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] -= cmp[i][j];

  // ---- epilogue: stage fp32 tile (+bias, rounded to T) in LDS ----
  float* E = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int col = wn * (BN / 2) + j * 16 + (lane & 15);
      int gj = n0 + col;
      float bv = 0.f;
      if (p.bias && gj < p.ncol) bv = p.bias[p.out_mode == 1 ? gj % p.cout : gj];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + r;
        float a = acc[i][j][r];
        if (p.zbias && gj < p.ncol && m0 + row < M) a += zbias_at(p, m0 + row, gj);
        E[row * ES + col] = rnd<T>(epi_act(a + bv, p.relu));
      }
    }
  __syncthreads();

  const int rows_valid = (int)((M - m0) < BM ? (M - m0) : BM);
  if (p.stat_sum) {
    float* red = reinterpret_cast<float*>(smem + LDS_BYTES - 4 * BN * 4);
    constexpr int PARTS = 256 / BN;
    constexpr int RPP = BM / PARTS;
    const int col = tid % BN, part = tid / BN;
    float s = 0.f;
    for (int r = part * RPP; r < (part + 1) * RPP; ++r)
      if (r < rows_valid) s += E[r * ES + col];
    red[part * BN + col] = s;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int q = 0; q < PARTS; ++q) tot += red[q * BN + col];
    const float mean = tot / (float)rows_valid;
    float m2 = 0.f;
    for (int r = part * RPP; r < (part + 1) * RPP; ++r)
      if (r < rows_valid) { float d = E[r * ES + col] - mean; m2 += d * d; }
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

  // ---- coalesced store: 8 consecutive columns per thread-iteration ----
  T* out = reinterpret_cast<T*>(p.out);
  const bool vec_ok = (p.ncol % 8) == 0 && (p.out_mode == 1 ? (p.cout % 8) == 0 : ((p.out_stride % 8) == 0 && (p.out_coff % 8) == 0));
  constexpr int CPR = BN / 8;  // chunks per row
  for (int e = tid; e < BM * CPR; e += 256) {
    int row = e / CPR, cc = (e - row * CPR) * 8;
    if (row >= rows_valid) continue;
    int gj = n0 + cc;
    if (gj >= p.ncol) continue;
    int64_t m = m0 + row;
    T* dst;
    if (p.out_mode == 0) {
      dst = out + m * p.out_stride + p.out_coff + gj;
    } else if (p.out_mode == 2) {
      // stride-2 sub-lattice (input gradient of a stride-2 conv, one parity)
      int hw = g.H * g.W;
      int n = (int)(m / hw);
      int rem = (int)(m - (int64_t)n * hw);
      int h = rem / g.W, w = rem - (rem / g.W) * g.W;
      dst = out + (((int64_t)n * p.oH + 2 * h + p.opy) * p.oW + 2 * w + p.opx) * p.out_stride + p.out_coff + gj;
    } else {
      int hw = g.H * g.W;
      int n = (int)(m / hw);
      int rem = (int)(m - (int64_t)n * hw);
      int h = rem / g.W, w = rem - (rem / g.W) * g.W;
      int ab = gj / p.cout, co = gj - ab * p.cout;
      int oy = 2 * h + (ab >> 1) + p.opy, ox = 2 * w + (ab & 1) + p.opx;
      dst = out + (((int64_t)n * p.oH + oy) * p.oW + ox) * p.out_stride + p.out_coff + co;
    }
    const float* src = E + row * ES + cc;
    if (vec_ok && gj + 8 <= p.ncol) {
      Vec8<T> v;
      if (p.accumulate) {
        v.load(dst);
#pragma unroll
        for (int q = 0; q < 8; ++q) v.set(q, v.get(q) + src[q]);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v.set(q, src[q]);
      }
      v.store(dst);
    } else {
      for (int q = 0; q < 8 && gj + q < p.ncol; ++q) {
        if (p.out_mode != 1) st1<T>(dst + q, p.accumulate ? ld1<T>(dst + q) + src[q] : src[q]);
        else {
          // scalar scatter (ragged cout)
          int jj = gj + q, ab = jj / p.cout, co = jj - ab * p.cout;
          int hw = g.H * g.W;
          int n = (int)(m / hw);
          int rem = (int)(m - (int64_t)n * hw);
          int h = rem / g.W, w = rem - (rem / g.W) * g.W;
          int oy = 2 * h + (ab >> 1) + p.opy, ox = 2 * w + (ab & 1) + p.opx;
          st1<T>(out + (((int64_t)n * p.oH + oy) * p.oW + ox) * p.out_stride + p.out_coff + co, src[q]);
        }
      }
    }
  }
}

template <typename T, int BM, int BN>
int launch_fwd(const VuGemmFwd& p, hipStream_t st) {
  constexpr int BKE = KB / sizeof(T);
  const VuGather& g = p.a;
  bool aligned = (g.C % BKE) == 0;
  for (int t = 0; t < g.nsrc; ++t) aligned = aligned && (g.cend[t] % BKE) == 0;
  int64_t M = (int64_t)g.N * g.H * g.W;
  int64_t nblk = ((M + BM - 1) / BM) * ((p.ncol + BN - 1) / BN);
  if (nblk <= 0) return 0;
  if (aligned)
    hipLaunchKernelGGL((gemm_fwd_kernel<T, BM, BN, true>), dim3((unsigned)nblk), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_fwd_kernel<T, BM, BN, false>), dim3((unsigned)nblk), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

int pick_bm(const VuGemmFwd& p) {
  int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  int64_t t128 = ((M + 127) / 128) * ((p.ncol + 127) / 128);
  return t128 >= 512 ? 128 : 64;
}

template <typename T>
int dispatch_fwd(const VuGemmFwd& p, hipStream_t st) {
  int bm = pick_bm(p);
  if (bm == 128) {
    // fp32: 128 x 64 tiles only (the compensated accumulators of a 128 x 128
    // tile spill)
    if (sizeof(T) == 4 || p.ncol <= 64) return launch_fwd<T, 128, 64>(p, st);
    if constexpr (sizeof(T) == 2) return launch_fwd<T, 128, 128>(p, st);
  }
  return launch_fwd<T, 64, 64>(p, st);
}

}  // namespace

// large-tile LDS-DMA variant (gemm_fwd2.hip)
int gemm_fwd_v2_bm(const VuGemmFwd& p, int dtype);
int gemm_fwd_v2_launch(const VuGemmFwd& p, hipStream_t st);
int gemm_fwd_v2_small(const VuGemmFwd& p, int dtype);
int gemm_fwd_v2_small_launch(const VuGemmFwd& p, hipStream_t st);
int gemm_fwd_v2_tail(const VuGemmFwd& p, int dtype);
int gemm_fwd_v2_tail_launch(const VuGemmFwd& p, hipStream_t st);
int64_t gemm_fwd_v2_small_workspace(const VuGemmFwd& p, int dtype);
int gemm_fwd_v3_bm(const VuGemmFwd& p, int dtype);
int gemm_fwd_v3_launch(const VuGemmFwd& p, hipStream_t st);
int gemm_fwd_v4_bm(const VuGemmFwd& p, int dtype);
int gemm_fwd_v4_launch(const VuGemmFwd& p, hipStream_t st);
int64_t gemm_fwd_v4_workspace(const VuGemmFwd& p, int dtype);
int conv_image_bm(const VuGemmFwd& p, int dtype);      // conv_image.hip (3-channel image conv)
int conv_stem_bm(const VuGemmFwd& p, int dtype);       // conv_stem.hip (ResNet34 7x7/s2 stem)
int conv_stem_launch(const VuGemmFwd& p, hipStream_t st);
int conv_image_launch(const VuGemmFwd& p, hipStream_t st);
int gemm_stream_bm(const VuGemmFwd& p, int dtype);     // gemm_stream.hip (short-K 1x1 streams)
int gemm_stream_launch(const VuGemmFwd& p, hipStream_t st);
int gemm_fwd_v5_bm(const VuGemmFwd& p, int dtype);     // gemm_fwd5.hip (persistent short-K GEMM)
int gemm_fwd_v5_launch(const VuGemmFwd& p, hipStream_t st);
int gemm_fwd_v6_bm(const VuGemmFwd& p, int dtype);     // gemm_fwd6.hip (64 -> 64 3x3, resident weights)
int gemm_fwd_v6_launch(const VuGemmFwd& p, hipStream_t st);
int gemm_fwd_v6_bnb_tile(const VuGemmFwd& p, int dtype);
int gemm_fwd_v4_bnb_tile(const VuGemmFwd& p, int dtype);
int gemm_fwd_v7_bm(const VuGemmFwd& p, int dtype);     // gemm_fwd7.hip (small-grid 3x3, two K groups)
int gemm_fwd_v7_launch(const VuGemmFwd& p, hipStream_t st);
int64_t gemm_fwd_v7_workspace(const VuGemmFwd& p, int dtype);

// Highest kernel generation the dispatchers may pick (vu_gemm_set_tuning
// VU_TUNE_GEN; tests and A/B runs only -- no environment lookups in the
// library): 1 = generic kernels only, 2 = + LDS-DMA tiles / 1x1 streams,
// 3 = + halo kernels, 4 (default) = + ping-pong / resident-weight kernels.
int g_tune_gen = 4;

static bool use_v2(int dtype) { return g_tune_gen >= 2 && dtype == VU_BF16; }
static bool use_v3(int dtype) { return g_tune_gen >= 3 && use_v2(dtype); }
static bool use_v4(int dtype) { return g_tune_gen >= 4 && use_v3(dtype); }

// VuGemmFwd.zbias problems run on the ping-pong kernel (incl. its split-K
// finish) when it serves them, else on the generic kernel: the only two
// epilogues that add the per-sample border-class bias
static bool zb_v4(const VuGemmFwd* a, int dtype) { return use_v4(dtype) && gemm_fwd_v4_bm(*a, dtype); }
static bool zb_ok(const VuGemmFwd* a) {
  return a->out_mode == 0 && a->a.H >= 2 && a->a.W >= 2 && !a->bnb_part;
}

extern "C" int64_t vu_gemm_fwd_row_tile(const VuGemmFwd* args, int dtype) {
  if (args->zbias) return zb_v4(args, dtype) ? 128 : pick_bm(*args);
  if (use_v2(dtype)) {
    int bm = conv_image_bm(*args, dtype);
    if (bm) return bm;
    bm = conv_stem_bm(*args, dtype);
    if (bm) return bm;
    bm = gemm_stream_bm(*args, dtype);
    if (bm) return bm;
  }
  if (use_v4(dtype)) {
    int bm = gemm_fwd_v6_bm(*args, dtype);
    if (bm) return bm;
    bm = gemm_fwd_v4_bm(*args, dtype);
    if (bm) return bm;
    bm = gemm_fwd_v7_bm(*args, dtype);
    if (bm) return bm;
  }
  if (use_v2(dtype) && gemm_fwd_v2_small(*args, dtype)) return 128;
  if (use_v3(dtype) && gemm_fwd_v3_bm(*args, dtype)) return 256;
  if (use_v2(dtype)) {
    int bm = gemm_fwd_v5_bm(*args, dtype);
    if (bm) return bm;
    bm = gemm_fwd_v2_bm(*args, dtype);
    if (bm) return bm;
    bm = gemm_fwd_v2_tail(*args, dtype);
    if (bm) return bm;
  }
  return pick_bm(*args);
}

extern "C" int64_t vu_gemm_fwd_workspace_bytes(const VuGemmFwd* args, int dtype) {
  if (args->zbias) return zb_v4(args, dtype) ? gemm_fwd_v4_workspace(*args, dtype) : 0;
  if (use_v2(dtype) && (conv_image_bm(*args, dtype) || conv_stem_bm(*args, dtype) || gemm_stream_bm(*args, dtype)))
    return 0;
  if (use_v4(dtype) && gemm_fwd_v6_bm(*args, dtype)) return 0;
  if (use_v4(dtype) && gemm_fwd_v4_bm(*args, dtype)) return gemm_fwd_v4_workspace(*args, dtype);
  if (use_v4(dtype) && gemm_fwd_v7_bm(*args, dtype)) return gemm_fwd_v7_workspace(*args, dtype);
  if (use_v2(dtype) && gemm_fwd_v2_small(*args, dtype)) return gemm_fwd_v2_small_workspace(*args, dtype);
  return 0;
}

// The BatchNorm-backward partial tile of the kernel the dispatcher below picks
// (it must mirror the dispatch order), 0 when that kernel cannot emit them.
extern "C" int64_t vu_gemm_fwd_bnb_tile(const VuGemmFwd* args, int dtype) {
  if (args->zbias) return 0;
  if (use_v2(dtype) && (conv_image_bm(*args, dtype) || conv_stem_bm(*args, dtype) || gemm_stream_bm(*args, dtype)))
    return 0;
  if (use_v4(dtype) && gemm_fwd_v6_bm(*args, dtype)) return gemm_fwd_v6_bnb_tile(*args, dtype);
  if (use_v4(dtype) && gemm_fwd_v4_bm(*args, dtype)) return gemm_fwd_v4_bnb_tile(*args, dtype);
  return 0;
}

// Which kernel the dispatcher below picks (mirrors its order; tests assert the
// path they mean to cover): 1 generic, 2 v2 LDS-DMA tiles, 3 v3 halo, 4 v4
// ping-pong, 5 v5 persistent short-K, 6 v6 resident weights, 7 v7 small-grid,
// 8 1x1 stream, 9 image conv, 10 7x7 stem, 12 v2 small-grid mode, 13 v2
// tail (small grids nothing else admits).
extern "C" int vu_gemm_fwd_kernel(const VuGemmFwd* args, int dtype) {
  if (args->zbias) return zb_v4(args, dtype) ? 4 : 1;
  if (use_v2(dtype) && conv_image_bm(*args, dtype)) return 9;
  if (use_v2(dtype) && conv_stem_bm(*args, dtype)) return 10;
  if (use_v2(dtype) && gemm_stream_bm(*args, dtype)) return 8;
  if (use_v4(dtype) && gemm_fwd_v6_bm(*args, dtype)) return 6;
  if (use_v4(dtype) && gemm_fwd_v4_bm(*args, dtype)) return 4;
  if (use_v4(dtype) && gemm_fwd_v7_bm(*args, dtype)) return 7;
  if (use_v2(dtype) && gemm_fwd_v2_small(*args, dtype)) return 12;
  if (use_v3(dtype) && gemm_fwd_v3_bm(*args, dtype)) return 3;
  if (use_v2(dtype) && gemm_fwd_v5_bm(*args, dtype)) return 5;
  if (use_v2(dtype) && gemm_fwd_v2_bm(*args, dtype)) return 2;
  if (use_v2(dtype) && gemm_fwd_v2_tail(*args, dtype)) return 13;
  return 1;
}

extern "C" int vu_gemm_fwd(const VuGemmFwd* args, int dtype, void* stream) {
  const VuGather& g = args->a;
  if (args->bnb_part && vu_gemm_fwd_bnb_tile(args, dtype) == 0) return (int)hipErrorInvalidValue;
  if (args->bnb_part && args->relu) return (int)hipErrorInvalidValue;  // (an inference-only epilogue)
  int epc = dtype == VU_BF16 ? 8 : 4;
  if (g.C % epc != 0 || g.nsrc < 1 || g.nsrc > 3) return (int)hipErrorInvalidValue;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.cend[t] % epc != 0 || g.stride[t] % epc != 0) return (int)hipErrorInvalidValue;
  if ((args->ldb % epc) != 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (args->zbias) {
    if (!zb_ok(args)) return (int)hipErrorInvalidValue;
    if (zb_v4(args, dtype)) return gemm_fwd_v4_launch(*args, st);
    return dtype == VU_BF16 ? dispatch_fwd<bf16_t>(*args, st) : dispatch_fwd<float>(*args, st);
  }
  if (use_v2(dtype) && conv_image_bm(*args, dtype)) return conv_image_launch(*args, st);
  if (use_v2(dtype) && conv_stem_bm(*args, dtype)) return conv_stem_launch(*args, st);
  if (use_v2(dtype) && gemm_stream_bm(*args, dtype)) return gemm_stream_launch(*args, st);
  if (use_v4(dtype) && gemm_fwd_v6_bm(*args, dtype)) return gemm_fwd_v6_launch(*args, st);
  if (use_v4(dtype) && gemm_fwd_v4_bm(*args, dtype)) return gemm_fwd_v4_launch(*args, st);
  if (use_v4(dtype) && gemm_fwd_v7_bm(*args, dtype)) return gemm_fwd_v7_launch(*args, st);
  if (use_v2(dtype) && gemm_fwd_v2_small(*args, dtype)) return gemm_fwd_v2_small_launch(*args, st);
  if (use_v3(dtype) && gemm_fwd_v3_bm(*args, dtype)) return gemm_fwd_v3_launch(*args, st);
  if (use_v2(dtype) && gemm_fwd_v5_bm(*args, dtype)) return gemm_fwd_v5_launch(*args, st);
  if (use_v2(dtype) && gemm_fwd_v2_bm(*args, dtype)) return gemm_fwd_v2_launch(*args, st);
  if (use_v2(dtype) && gemm_fwd_v2_tail(*args, dtype)) return gemm_fwd_v2_tail_launch(*args, st);
  return dtype == VU_BF16 ? dispatch_fwd<bf16_t>(*args, st) : dispatch_fwd<float>(*args, st);
}

extern "C" void vu_abi_struct_sizes(int64_t* out) {
  out[0] = sizeof(VuGather);
  out[1] = sizeof(VuGemmFwd);
  out[2] = sizeof(VuGemmWgrad);
  out[3] = sizeof(VuConvFp8);
  out[4] = sizeof(VuPermJob);
  out[5] = sizeof(VuMtEntry);
  out[6] = sizeof(VuLatentJob);
  out[7] = sizeof(VuLatentHeads);
  out[8] = sizeof(VuZbJob);
}
