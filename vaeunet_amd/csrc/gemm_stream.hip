// Short-K 1x1 GEMMs as HBM streams ("stream" kernel, bf16):
// out[m][j] = sum_k A[m][k] B[j][k] (+bias) with K = 32, 64 or 128 and
// N <= 256 -- the AttentionGate W_g / W_x convolutions of the 256^2 / 512^2
// levels (unet_parts.py:11,15), their input gradients (accumulated into the
// skip / gate gradients) and the 256^2 -> 512^2 ConvTranspose2d
// (unet_parts.py:76, pixel-shuffle store).  These move 2-3 bytes per flop: at
// 256-row LDS tiles (gemm_fwd2.hip) a block's life is its load latency and
// epilogue, so they ran at 1.5-4 TB/s.  Here:
//
//   * the weight matrix (<= 64 KB) and bias are copied into LDS ONCE per
//     block and the blocks are persistent (one pass over the pixel tiles);
//     an opaque per-tile LDS offset keeps the compiler from hoisting the
//     weight fragments out of the tile loop (KS x NJ fragments would not fit
//     the register file at N = 256);
//   * each wave streams its own 16*NF-pixel tiles straight from global: all
//     K of a tile (16 bytes = 8 channels per lane and k-step) is in flight
//     before the first MFMA;
//   * MFMA(weights, pixels), weight rows read in a permuted order so a lane
//     owns 4*GS consecutive output columns of one pixel (16/32-byte stores,
//     the ConvT pixel shuffle keeps them contiguous), BN partials per wave
//     tile by DPP row sums, optional accumulate (input gradients).
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

template <bool B> struct BoolTag { static constexpr bool value = B; };

typedef __attribute__((address_space(3))) void lds_void;

template <int R>
VU_DEV float ror_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false));
}
VU_DEV float row16_sum(float v) { return ror_add<1>(ror_add<2>(ror_add<4>(ror_add<8>(v)))); }

VU_DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

constexpr int NT = 256;  // 4 waves

// KS: k-steps of 32 (K = 32*KS); NJ: 16-column fragments (N = 16*NJ);
// NF: 16-pixel fragments per wave tile; PD: tiles of loads in flight per wave
// beyond the one being computed (1, or 2 = VU_TUNE_STREAM_PD: with 8 waves per
// CU one tile of loads in flight is ~32 KB per CU, which by Little's law at
// ~2 us of loaded HBM latency caps the kernel near 4 TB/s).
template <int KS, int NJ, int NF, bool RELU = false, int PD = 1>  // RELU: epilogue ReLU (VuGemmFwd.relu)
__global__ __launch_bounds__(NT, 2) void gemm_stream_kernel(VuGemmFwd p) {
  constexpr int K = 32 * KS, N = 16 * NJ, PX = 16 * NF;
  constexpr int GS = NJ < 4 ? NJ : 4;   // fragments per column group (4*GS consecutive columns per lane)
  __shared__ __attribute__((aligned(16))) char wsm[N * K * 2];
  __shared__ __attribute__((aligned(16))) float bsm[N];  // bias per output column (ConvT: per cout, expanded)

  const VuGather& g = p.a;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  const int ntiles = (int)(M / PX);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gq = lane >> 4, r16 = lane & 15;

  // A-row r of fragment j -> weight row (output column) of the permuted order
  auto wrow = [&](int j, int r) { return (j / GS) * 16 * GS + 4 * GS * (r >> 2) + 4 * (j % GS) + (r & 3); };
  // weights -> LDS in FRAGMENT order: the 64 lanes' 16-byte pieces of
  // fragment (j, ks) are one contiguous KiB, so every fragment read is a
  // conflict-free ds_read_b128 (row-major rows of 128/256 bytes put the 16
  // rows a read touches on the same banks: 16-way conflicts)
  {
    const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
    constexpr int PIECES = NJ * KS * 64;
    for (int e = threadIdx.x; e < PIECES; e += NT) {
      const int l = e & 63, jk = e >> 6, j = jk / KS, ks = jk - j * KS;
      *reinterpret_cast<u32x4*>(wsm + e * 16) =
          *reinterpret_cast<const u32x4*>(bmat + (int64_t)wrow(j, l & 15) * p.ldb + 32 * ks + 8 * (l >> 4));
    }
    for (int c = threadIdx.x; c < N; c += NT) bsm[c] = p.bias ? p.bias[p.out_mode == 1 ? c % p.cout : c] : 0.f;
    __syncthreads();
  }

  const bf16_t* src = reinterpret_cast<const bf16_t*>(g.src[0]);
  const int64_t st = g.stride[0];
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
  const int HW = g.H * g.W;
  const FastDiv div_hw((uint32_t)HW), div_w((uint32_t)g.W), div_co((uint32_t)(p.cout > 0 ? p.cout : 1));

  // the next tile's operands are loaded before this tile's MFMAs and stores:
  // one tile of loads always in flight per wave (latency, not bandwidth,
  // bounded a wave that loaded, computed and stored in turn)
  const int tstride = gridDim.x * (NT / 64);
  auto load = [&](int tile, u32x4 (&dst)[NF][KS]) {
    const int64_t pb = (int64_t)tile * PX;
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        dst[f][ks] = *reinterpret_cast<const u32x4*>(src + (pb + 16 * f + r16) * st + 32 * ks + 8 * gq);
  };
  u32x4 pn[NF][KS], pn2[NF][KS];
  int tile = blockIdx.x * (NT / 64) + wid;
  if (tile < ntiles) load(tile, pn);
  if (PD == 2 && tile + tstride < ntiles) load(tile + tstride, pn2);
  for (; tile < ntiles; tile += tstride) {
    const int64_t pb = (int64_t)tile * PX;
    // opaque LDS offset: the weight fragments and bias are re-read per tile
    // instead of being hoisted out of the tile loop (KS x NJ fragments would
    // not fit the register file at N = 256)
    int lo = 0;
    asm volatile("" : "+v"(lo));
    u32x4 pf[NF][KS];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) pf[f][ks] = pn[f][ks];
    if constexpr (PD == 2) {
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) pn[f][ks] = pn2[f][ks];
      if (tile + 2 * tstride < ntiles) load(tile + 2 * tstride, pn2);
    } else {
      if (tile + tstride < ntiles) load(tile + tstride, pn);
    }
    f32x4 acc[NF][NJ];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[f][j] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const u32x4 wf = *reinterpret_cast<const u32x4*>(wsm + lo + ((j * KS + ks) * 64 + lane) * 16);
#pragma unroll
        for (int f = 0; f < NF; ++f)
          acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf),
                                                              __builtin_bit_cast(bf16x8, pf[f][ks]), acc[f][j], 0, 0, 0);
      }
    // acc[f][j][r]: pixel pb + 16f + r16, column (j/GS)*16*GS + 4*GS*gq + 4*(j%GS) + r
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(
          reinterpret_cast<const char*>(bsm) + lo + ((j / GS) * 16 * GS + 4 * GS * gq + 4 * (j % GS)) * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[f][j][r] = rnd<bf16_t>(acc[f][j][r] + bv[r]);
    }
    if constexpr (RELU)
#pragma unroll
      for (int f = 0; f < NF; ++f) epi_relu(acc[f]);
    if (p.stat_sum) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        f32x4 sm, m2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sv = 0.f;
#pragma unroll
          for (int f = 0; f < NF; ++f) sv += acc[f][j][r];
          sv = row16_sum(sv);
          const float mean = sv * (1.f / PX);
          float v = 0.f;
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            const float d = acc[f][j][r] - mean;
            v += d * d;
          }
          sm[r] = sv;
          m2[r] = row16_sum(v);
        }
        if (r16 == 0) {
          const int col = (j / GS) * 16 * GS + 4 * GS * gq + 4 * (j % GS);
          *reinterpret_cast<f32x4*>(p.stat_sum + (int64_t)tile * p.ncol + col) = sm;
          *reinterpret_cast<f32x4*>(p.stat_m2 + (int64_t)tile * p.ncol + col) = m2;
        }
      }
    }
    // stores.  GS = 4: a lane holds 16 consecutive columns (two 16-byte
    // chunks) of one pixel per 64-column group; two lane-row swaps
    // (permlane16 + permlane32) regroup them so that each store instruction
    // writes 64 contiguous bytes per pixel (lane row q: columns 32h + 8q ..
    // +7 of the group) instead of 16-byte pieces at a 32-byte stride.
    // ConvT pixel shuffle: the (n, h, w) decode of a pixel and the (tap,
    // channel) split of a column by multiply-shift (runtime divisions here
    // were ~20 VALU each, three per 16-byte store)
    auto dst_of = [&](int64_t m, int col0) -> bf16_t* {
      if (p.out_mode == 1) {
        const int n = (int)div_hw.div((uint32_t)m);
        const int rem = (int)m - n * HW;
        const int h = (int)div_w.div((uint32_t)rem), w = rem - h * g.W;
        const int ab = (int)div_co.div((uint32_t)col0), co = col0 - ab * p.cout;
        const int oy = 2 * h + (ab >> 1) + p.opy, ox = 2 * w + (ab & 1) + p.opx;
        return out + ((int64_t)(n * p.oH + oy) * p.oW + ox) * p.out_stride + p.out_coff + co;
      }
      return out + m * p.out_stride + p.out_coff + col0;
    };
    auto add_old = [&](u32x4& v, const u32x4 o) {
#pragma unroll
      for (int w = 0; w < 4; ++w)
        v[w] = pack2(__uint_as_float(o[w] << 16) + __uint_as_float(v[w] << 16),
                     __uint_as_float(o[w] & 0xffff0000u) + __uint_as_float(v[w] & 0xffff0000u));
    };
    // Two instantiations of the store pass behind ONE uniform branch: with
    // `if (accumulate) load` inside the loop, the vmcnt(0) the compiler puts
    // after that branch ran for plain stores too -- every store waited for
    // the previous one (and for the next tile's prefetch), which is where
    // most of this kernel's wave cycles were spent waiting.  Accumulate: the
    // old values of a pixel fragment's stores are loaded together first.
    auto store_pass = [&](auto acc_tag) {
      constexpr bool ACC = decltype(acc_tag)::value;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int64_t m = pb + 16 * f + r16;
        if constexpr (GS == 4) {
          u32x4 c[NJ / GS][2];
          bf16_t* dst[NJ / GS][2];
#pragma unroll
          for (int grp = 0; grp < NJ / GS; ++grp) {
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              const f32x4 a = acc[f][grp * 4 + 2 * h2], b = acc[f][grp * 4 + 2 * h2 + 1];
              c[grp][h2] = u32x4{pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(b[0], b[1]), pack2(b[2], b[3])};
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              const auto r1 = __builtin_amdgcn_permlane16_swap(c[grp][0][w], c[grp][1][w], false, false);
              const auto r2 = __builtin_amdgcn_permlane32_swap(r1[0], r1[1], false, false);
              c[grp][0][w] = r2[0];
              c[grp][1][w] = r2[1];
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) dst[grp][h] = dst_of(m, grp * 64 + 32 * h + 8 * gq);
          }
          if constexpr (ACC) {
            u32x4 o[NJ / GS][2];
#pragma unroll
            for (int grp = 0; grp < NJ / GS; ++grp)
#pragma unroll
              for (int h = 0; h < 2; ++h) o[grp][h] = *reinterpret_cast<const u32x4*>(dst[grp][h]);
#pragma unroll
            for (int grp = 0; grp < NJ / GS; ++grp)
#pragma unroll
              for (int h = 0; h < 2; ++h) add_old(c[grp][h], o[grp][h]);
          }
#pragma unroll
          for (int grp = 0; grp < NJ / GS; ++grp)
#pragma unroll
            for (int h = 0; h < 2; ++h) *reinterpret_cast<u32x4*>(dst[grp][h]) = c[grp][h];
        } else {
          bf16_t* dst = dst_of(m, 4 * GS * gq);   // NJ == GS: one column group
          u32x4 v[GS / 2];
#pragma unroll
          for (int h2 = 0; h2 < GS / 2; ++h2) {
            const f32x4 a = acc[f][2 * h2], b = acc[f][2 * h2 + 1];
            v[h2] = u32x4{pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(b[0], b[1]), pack2(b[2], b[3])};
          }
          if constexpr (ACC) {
            // out += result: unpack the stored pairs and round the sums once
            u32x4 o[GS / 2];
#pragma unroll
            for (int h2 = 0; h2 < GS / 2; ++h2) o[h2] = *reinterpret_cast<const u32x4*>(dst + 8 * h2);
#pragma unroll
            for (int h2 = 0; h2 < GS / 2; ++h2) {
              const f32x4 a = acc[f][2 * h2], b = acc[f][2 * h2 + 1];
              v[h2] = u32x4{pack2(__uint_as_float(o[h2][0] << 16) + a[0], __uint_as_float(o[h2][0] & 0xffff0000u) + a[1]),
                            pack2(__uint_as_float(o[h2][1] << 16) + a[2], __uint_as_float(o[h2][1] & 0xffff0000u) + a[3]),
                            pack2(__uint_as_float(o[h2][2] << 16) + b[0], __uint_as_float(o[h2][2] & 0xffff0000u) + b[1]),
                            pack2(__uint_as_float(o[h2][3] << 16) + b[2], __uint_as_float(o[h2][3] & 0xffff0000u) + b[3])};
            }
          }
#pragma unroll
          for (int h2 = 0; h2 < GS / 2; ++h2) *reinterpret_cast<u32x4*>(dst + 8 * h2) = v[h2];
        }
      }
    };
    if (p.accumulate) store_pass(BoolTag<true>{});
    else store_pass(BoolTag<false>{});
  }
}

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// pixel fragments per wave tile: NF*NJ <= 16 accumulator fragments, NF*KS <= 8 operand registers sets
constexpr int nf_of(int ks, int nj) {
  return (16 / nj < 4 ? 16 / nj : 4) < (8 / ks) ? (16 / nj < 4 ? 16 / nj : 4) : 8 / ks;
}

int g_pd = 1;  // VU_TUNE_STREAM_PD

template <int KS, int NJ>
int launch_nj(const VuGemmFwd& p, hipStream_t st) {
  constexpr int NF = nf_of(KS, NJ);
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  const int64_t tiles = M / (16 * NF);
  int64_t nblk = (tiles + 3) / 4;
  const int64_t cap = 2 * (int64_t)cu_count();
  if (nblk > cap) nblk = cap;
  if (p.relu)
    hipLaunchKernelGGL((gemm_stream_kernel<KS, NJ, NF, true>), dim3((unsigned)nblk), dim3(NT), 0, st, p);
  else if (g_pd == 2)
    hipLaunchKernelGGL((gemm_stream_kernel<KS, NJ, NF, false, 2>), dim3((unsigned)nblk), dim3(NT), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_stream_kernel<KS, NJ, NF>), dim3((unsigned)nblk), dim3(NT), 0, st, p);
  return (int)hipGetLastError();
}

template <int KS>
int launch_ks(const VuGemmFwd& p, hipStream_t st) {
  switch (p.ncol / 16) {
    case 2: return launch_nj<KS, 2>(p, st);
    case 4: return launch_nj<KS, 4>(p, st);
    case 8: return launch_nj<KS, 8>(p, st);
    case 16: return launch_nj<KS, 16>(p, st);
    default: return (int)hipErrorInvalidValue;
  }
}

bool g_enabled = true;  // VU_TUNE_STREAM

}  // namespace

// Row tile (16*NF pixels) when the stream kernel serves this problem, else 0:
// bf16 1x1 gather of ONE NHWC source with K = C in {32, 64, 128}, N in {32,
// 64, 128, 256}, plain (mode 0, optional accumulate) or ConvT pixel-shuffle
// (mode 1, no statistics) output, whole tiles, enough tiles to fill the chip.
int gemm_stream_bm(const VuGemmFwd& p, int dtype) {
  const VuGather& g = p.a;
  if (!g_enabled || dtype != VU_BF16) return 0;
  if (g.R != 1 || g.S != 1 || g.sy != 1 || g.sx != 1 || g.oy != 0 || g.ox != 0 || g.Hs != g.H ||
      g.Ws != g.W || g.nsrc != 1)
    return 0;
  if (g.C != 32 && g.C != 64 && g.C != 128) return 0;
  const int nj = p.ncol / 16;
  if (p.ncol % 16 != 0 || (nj != 2 && nj != 4 && nj != 8 && nj != 16)) return 0;
  if (g.stride[0] % 8 != 0 || p.ldb % 8 != 0 || p.ldb < g.C || p.out_stride % 8 != 0 || p.out_coff % 8 != 0)
    return 0;
  if (p.out_mode == 1) {
    if (p.stat_sum || p.cout % 16 != 0 || p.ncol != 4 * p.cout) return 0;
  } else if (p.out_mode != 0) {
    return 0;
  }
  const int ks = g.C / 32;
  const int px = 16 * nf_of(ks, nj);
  const int64_t M = (int64_t)g.N * g.H * g.W;
  if (M % px != 0 || M >= ((int64_t)1 << 31) || M / px < 4 * 2 * (int64_t)cu_count()) return 0;
  return px;
}

int gemm_stream_launch(const VuGemmFwd& p, hipStream_t st) {
  switch (p.a.C) {
    case 32: return launch_ks<1>(p, st);
    case 64: return launch_ks<2>(p, st);
    case 128: return launch_ks<4>(p, st);
    default: return (int)hipErrorInvalidValue;
  }
}

int gemm_stream_tune(int key, int value) {
  if (key == VU_TUNE_STREAM) {
    g_enabled = value != 0;
    return 0;
  }
  if (key == VU_TUNE_STREAM_PD) {
    if (value != 1 && value != 2) return (int)hipErrorInvalidValue;
    g_pd = value;
    return 0;
  }
  return -1;
}
