// The ResNet34 stem of UNetResNet's encoder (conv1: 7x7, stride 2, pad 3,
// 3 -> 64 channels; unet_resnet.py:131-137 via timm resnet34), bf16, input
// packed to 8 channels (vu_input_pack).  K = 49 taps x 8 channels = 392 per
// output pixel: too short and too oddly shaped (8 channels per tap, stride 2)
// for the halo or LDS-DMA GEMM tiles, so it ran on the generic v1 kernel at
// ~200 TFLOP/s.  Like the 3x3 image conv (conv_image.hip) this treats it as
// an output stream with a little MFMA work per pixel:
//
//   * K-step = 4 taps x 8 channels: lane group g of the 16x16x32 operand is
//     tap 4*ks + g, i.e. ONE 16-byte load (8 channels of one input pixel)
//     per lane and step, straight from global / L1 (the 7x7 windows of
//     neighbouring output pixels overlap 3.5x: L1/L2 serve the re-reads);
//   * the weights (64 x 13 steps, 52 KiB) live in LDS in fragment order,
//     loaded once per persistent block; each B fragment read (1 KiB,
//     lane-linear, conflict-free) feeds the 4 pixel fragments of the wave
//     tile, and the pixel loads run 2 steps ahead of the MFMAs;
//   * MFMA(weights, pixels) with permuted weight rows (a lane owns 16
//     consecutive output channels of one pixel), bias, bf16 rounding,
//     BatchNorm partials per 64-pixel wave tile (DPP row sums) and
//     permlane-regrouped stores of 64 contiguous bytes per pixel.
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

template <int R>
VU_DEV float ror_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false));
}
VU_DEV float row16_sum(float v) { return ror_add<1>(ror_add<2>(ror_add<4>(ror_add<8>(v)))); }
VU_DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

constexpr int KR = 7, TAPS = KR * KR;   // 49
constexpr int KS = (TAPS + 3) / 4;      // 13 K-steps of 4 taps
constexpr int NT = 256;                 // 4 waves
constexpr int TP = 64;                  // pixels per wave tile (also the BN statistics row tile)
constexpr int NF = TP / 16;             // pixel fragments per wave tile
constexpr int WLDS = KS * 4 * 64 * 16;  // 53,248 B: [ks][j][lane] 16-byte fragment pieces

template <bool RELU>  // epilogue ReLU (VuGemmFwd.relu) as its own instantiation
__global__ __launch_bounds__(NT, 2) void conv_stem_kernel(VuGemmFwd p) {
  __shared__ __attribute__((aligned(16))) char wl[WLDS];
  const VuGather& g = p.a;
  const int Ho = g.H, Wo = g.W, HWo = Ho * Wo;
  const int Hs = g.Hs, Ws = g.Ws;
  const int M = g.N * HWo;
  const int ntiles = M / TP;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gq = lane >> 4, r16 = lane & 15;
  const bf16_t* src = reinterpret_cast<const bf16_t*>(g.src[0]);
  const int64_t st = g.stride[0];
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);

  // ---- weights -> LDS in fragment order: piece (ks, j, lane) = row
  //      16*(r16>>2) + 4j + (r16&3) (permuted), tap 4*ks + gq, 8 channels ----
  {
    const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
    for (int q = threadIdx.x; q < KS * 4 * 64; q += NT) {
      const int ks = q >> 8, j = (q >> 6) & 3, l = q & 63;
      const int n = 16 * ((l & 15) >> 2) + 4 * j + (l & 3);
      const int tap = 4 * ks + (l >> 4);
      u32x4 v = u32x4{0, 0, 0, 0};
      if (tap < TAPS) v = *reinterpret_cast<const u32x4*>(bmat + (int64_t)n * p.ldb + tap * 8);
      *reinterpret_cast<u32x4*>(wl + q * 16) = v;
    }
  }
  __syncthreads();

  for (int tile = blockIdx.x * (NT / 64) + wid; tile < ntiles; tile += gridDim.x * (NT / 64)) {
    const int pb = tile * TP;
    // input window origin (tap 0) of this lane's pixel in each fragment; a
    // tap adds a lane offset that depends on the K-step only (32-bit)
    const bf16_t* wb[NF];
    int oy[NF], ox[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int m = pb + 16 * i + r16;
      const int n = m / HWo, rem = m - (m / HWo) * HWo;
      const int h = rem / Wo, w = rem - (rem / Wo) * Wo;
      oy[i] = h * g.sy + g.oy;
      ox[i] = w * g.sx + g.ox;
      wb[i] = src + (((int64_t)n * Hs + oy[i]) * Ws + ox[i]) * st;
    }
    const int sti = (int)st;
    auto load = [&](int ks, u32x4 (&a)[NF]) {
      const int tap = 4 * ks + gq;
      const int ry = tap / KR, rx = tap - (tap / KR) * KR;
      const int off = (ry * Ws + rx) * sti;
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const bool ok = tap < TAPS && (unsigned)(oy[i] + ry) < (unsigned)Hs && (unsigned)(ox[i] + rx) < (unsigned)Ws;
        a[i] = ok ? *reinterpret_cast<const u32x4*>(wb[i] + off) : u32x4{0, 0, 0, 0};
      }
    };
    f32x4 acc[NF][4];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    // pixel fragments of steps ks, ks+1, ks+2 (rotated by register moves, so
    // no array is indexed by the loop counter)
    u32x4 a0[NF], a1[NF], a2[NF];
    load(0, a0);
    load(1, a1);
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 2 < KS) load(ks + 2, a2);
      u32x4 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const u32x4*>(wl + ((ks * 4 + j) * 64 + lane) * 16);
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                              __builtin_bit_cast(bf16x8, a0[i]), acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        a0[i] = a1[i];
        a1[i] = a2[i];
      }
      // keep the scheduler from hoisting later steps' loads (register blow-up)
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- epilogue: acc[i][j][r] = pixel pb + 16i + r16, channel 16gq + 4j + r ----
    f32x4 bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bv[j] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + 16 * gq + 4 * j) : f32x4{0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = rnd<bf16_t>(acc[i][j][r] + bv[j][r]);
    if constexpr (RELU)
#pragma unroll
      for (int i = 0; i < NF; ++i) epi_relu(acc[i]);
    if (p.stat_sum) {
      // lane (gq, r16) keeps channel 16gq + r16 = lane of the wave tile
      float ms = 0.f, mq = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sv = 0.f;
#pragma unroll
          for (int i = 0; i < NF; ++i) sv += acc[i][j][r];
          sv = row16_sum(sv);
          const float mean = sv * (1.f / TP);
          float q = 0.f;
#pragma unroll
          for (int i = 0; i < NF; ++i) {
            const float d = acc[i][j][r] - mean;
            q += d * d;
          }
          q = row16_sum(q);
          if (r16 == 4 * j + r) {
            ms = sv;
            mq = q;
          }
        }
      p.stat_sum[(int64_t)tile * p.ncol + lane] = ms;
      p.stat_m2[(int64_t)tile * p.ncol + lane] = mq;
    }
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      u32x4 cv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = acc[i][2 * h], e = acc[i][2 * h + 1];
        cv[h] = u32x4{pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(e[0], e[1]), pack2(e[2], e[3])};
      }
      // regroup: store h of lane gq writes channels 32h + 8gq .. +7
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const auto r1 = __builtin_amdgcn_permlane16_swap(cv[0][w], cv[1][w], false, false);
        const auto r2 = __builtin_amdgcn_permlane32_swap(r1[0], r1[1], false, false);
        cv[0][w] = r2[0];
        cv[1][w] = r2[1];
      }
      bf16_t* dst = out + (int64_t)(pb + 16 * i + r16) * p.out_stride + p.out_coff + 8 * gq;
#pragma unroll
      for (int h = 0; h < 2; ++h) *reinterpret_cast<u32x4*>(dst + 32 * h) = cv[h];
    }
  }
}

int cu_count_stem() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

}  // namespace

// Row tile (64) when this kernel serves the problem, else 0: bf16 7x7
// stride-2 pad-3 conv over ONE 8-channel NHWC source into 64 output
// channels, plain store, whole 64-pixel tiles.
int conv_stem_bm(const VuGemmFwd& p, int dtype) {
  const VuGather& g = p.a;
  if (dtype != VU_BF16 || p.out_mode != 0 || p.accumulate) return 0;
  if (g.R != KR || g.S != KR || g.sy != 2 || g.sx != 2 || g.dy != 1 || g.dx != 1 || g.oy != -3 || g.ox != -3 ||
      g.nsrc != 1 || g.C != 8)
    return 0;
  if (g.stride[0] % 8 != 0 || p.ncol != 64 || p.ldb % 8 != 0 || p.ldb < TAPS * 8) return 0;
  if (p.out_stride % 8 != 0 || p.out_coff % 8 != 0) return 0;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  if (M % TP != 0 || (int64_t)g.N * g.Hs * g.Ws * g.stride[0] >= ((int64_t)1 << 31)) return 0;
  return TP;
}

int conv_stem_launch(const VuGemmFwd& p, hipStream_t st) {
  const int64_t tiles = (int64_t)p.a.N * p.a.H * p.a.W / TP;
  int64_t nblk = (tiles + 3) / 4;
  const int64_t cap = 2 * (int64_t)cu_count_stem();  // persistent: 2 blocks (8 waves) per CU
  if (nblk > cap) nblk = cap;
  if (p.relu)
    hipLaunchKernelGGL(conv_stem_kernel<true>, dim3((unsigned)nblk), dim3(NT), 0, st, p);
  else
    hipLaunchKernelGGL(conv_stem_kernel<false>, dim3((unsigned)nblk), dim3(NT), 0, st, p);
  return (int)hipGetLastError();
}
