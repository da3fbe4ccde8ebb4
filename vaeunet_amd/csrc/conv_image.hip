// The 3-channel image convolution (inc.0 = the first conv of
// DoubleConv(n_channels, 64), unet_parts.py:40 via unet_model.py:21), bf16,
// input packed to 8 channels (vu_input_pack).  K = 9 taps x 8 channels = 72
// is far too short for the halo kernels (18-36 K-steps amortise their
// pipelines) and the generic tiled kernel spent 250 us on what is a 268 MB
// output stream; this kernel treats it as what it is, an HBM-bound stream
// with a little MFMA work per pixel:
//
//   * no LDS: each wave owns 64 consecutive pixels x 64 output channels;
//     the weights (64 x 72) live in registers for the whole launch, the input
//     taps come straight from global/L1 (16 bytes = 8 channels of one pixel
//     per lane, the next fragment's taps prefetched behind the MFMAs);
//   * K-step = 4 taps x 8 channels (3 steps, taps 9-11 zero): lane group g of
//     the 16x16x32 MFMA operand is tap 4*ks + g;
//   * MFMA(weights, pixels) with the weight rows read in a permuted order
//     (as gemm_fwd5.hip) so a lane holds 16 consecutive output channels of one
//     pixel: two 16-byte NHWC stores per fragment, BatchNorm partials per
//     64-pixel wave tile by DPP row sums.
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

template <int R>
VU_DEV float ror_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false));
}
VU_DEV float row16_sum(float v) { return ror_add<1>(ror_add<2>(ror_add<4>(ror_add<8>(v)))); }

VU_DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

constexpr int NT = 256;  // 4 waves
constexpr int TP = 64;   // pixels per wave tile (4 fragments; also the BN statistics row tile)
constexpr int NF = TP / 16;

template <bool RELU>  // epilogue ReLU (VuGemmFwd.relu) as its own instantiation
__global__ __launch_bounds__(NT, 2) void conv3x3_image_kernel(VuGemmFwd p) {
  const VuGather& g = p.a;
  const int H = g.H, W = g.W, HW = g.H * g.W;
  const int M = g.N * HW;
  const int nct = p.ncol / 64;
  const int ntiles = (M / TP) * nct;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gq = lane >> 4;           // k group: tap 4*ks + gq
  const int r16 = lane & 15;
  const bf16_t* src = reinterpret_cast<const bf16_t*>(g.src[0]);
  const int64_t st = g.stride[0];
  const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
  // permuted weight row of A-row r16 in fragment j: 16*(r16>>2) + 4*j + (r16&3)
  const int wr = 16 * (r16 >> 2) + (r16 & 3);
  const int cb16 = 16 * gq;           // acc[i][j][r]: channel n0 + cb16 + 4*j + r

  u32x4 wf[4][3];
  int cur_nt = -1;
  const FastDiv div_hw((uint32_t)HW), div_w((uint32_t)W);  // (n, h, w) decode by multiply-shift

  // taps of the 16 pixels of fragment i of tile base pb (one 16-byte load per k-step)
  auto load_px = [&](int m, u32x4* pf) {
    const int n = (int)div_hw.div((uint32_t)m);
    const int rem = m - n * HW;
    const int h = (int)div_w.div((uint32_t)rem), w = rem - h * W;
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int tap = 4 * ks + gq;
      const int y = h + tap / 3 - 1, x = w + (tap - (tap / 3) * 3) - 1;
      pf[ks] = u32x4{0, 0, 0, 0};
      if (tap < 9 && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
        pf[ks] = *reinterpret_cast<const u32x4*>(src + ((int64_t)(n * H + y) * W + x) * st);
    }
  };

  // (a cross-tile prefetch of the next tile's first fragment measured slower:
  // its registers cost the third wave per SIMD, 88 -> 102 us)
  for (int tile = blockIdx.x * (NT / 64) + wid; tile < ntiles; tile += gridDim.x * (NT / 64)) {
    const int mt = tile / nct, nt = tile - mt * nct;
    const int pb = mt * TP, n0 = nt * 64;
    if (nt != cur_nt) {
      cur_nt = nt;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
          const int tap = 4 * ks + gq;
          wf[j][ks] = u32x4{0, 0, 0, 0};
          if (tap < 9) wf[j][ks] = *reinterpret_cast<const u32x4*>(bmat + (int64_t)(n0 + wr + 4 * j) * p.ldb + tap * 8);
        }
    }
    f32x4 acc[NF][4];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    u32x4 pf[3], pn[3];
    load_px(pb + r16, pf);
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      if (i + 1 < NF) load_px(pb + (i + 1) * 16 + r16, pn);
#pragma unroll
      for (int ks = 0; ks < 3; ++ks)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[j][ks]),
                                                              __builtin_bit_cast(bf16x8, pf[ks]), acc[i][j], 0, 0, 0);
      if (i + 1 < NF) {
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) pf[ks] = pn[ks];
      }
    }
    // ---- epilogue: bias, bf16 rounding, BN partials, 16-byte stores
    const int c0 = n0 + cb16;
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float bv = p.bias[c0 + 4 * j + r];
#pragma unroll
          for (int i = 0; i < NF; ++i) acc[i][j][r] += bv;
        }
    }
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = rnd<bf16_t>(acc[i][j][r]);
    if constexpr (RELU)
#pragma unroll
      for (int i = 0; i < NF; ++i) epi_relu(acc[i]);
    if (p.stat_sum) {
      float* ss = p.stat_sum + (int64_t)mt * p.ncol + c0;
      float* sq = p.stat_m2 + (int64_t)mt * p.ncol + c0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 sm, m2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float sv = 0.f;
#pragma unroll
          for (int i = 0; i < NF; ++i) sv += acc[i][j][r];
          sv = row16_sum(sv);
          const float mean = sv * (1.f / TP);
          float v = 0.f;
#pragma unroll
          for (int i = 0; i < NF; ++i) {
            const float d = acc[i][j][r] - mean;
            v += d * d;
          }
          sm[r] = sv;
          m2[r] = row16_sum(v);
        }
        if (r16 == 0) {
          *reinterpret_cast<f32x4*>(ss + 4 * j) = sm;
          *reinterpret_cast<f32x4*>(sq + 4 * j) = m2;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int64_t m = pb + i * 16 + r16;
      bf16_t* dst = out + m * p.out_stride + p.out_coff + c0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u32x4 pk;
        pk[0] = pack2(acc[i][2 * h][0], acc[i][2 * h][1]);
        pk[1] = pack2(acc[i][2 * h][2], acc[i][2 * h][3]);
        pk[2] = pack2(acc[i][2 * h + 1][0], acc[i][2 * h + 1][1]);
        pk[3] = pack2(acc[i][2 * h + 1][2], acc[i][2 * h + 1][3]);
        *reinterpret_cast<u32x4*>(dst + 8 * h) = pk;
      }
    }
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

}  // namespace

// Row tile (64) when this kernel serves the problem, else 0: bf16 3x3
// stride-1 pad-1 conv over ONE 8-channel NHWC source, 64-column output tiles,
// plain store (no accumulate), whole 64-pixel tiles.
int conv_image_bm(const VuGemmFwd& p, int dtype) {
  const VuGather& g = p.a;
  if (dtype != VU_BF16 || p.out_mode != 0 || p.accumulate) return 0;
  if (g.R != 3 || g.S != 3 || g.sy != 1 || g.sx != 1 || g.dy != 1 || g.dx != 1 || g.oy != -1 ||
      g.ox != -1 || g.Hs != g.H || g.Ws != g.W || g.nsrc != 1 || g.C != 8)
    return 0;
  if (g.stride[0] % 8 != 0 || p.ncol % 64 != 0 || p.ldb % 8 != 0 || p.ldb < 72) return 0;
  if (p.out_stride % 8 != 0 || p.out_coff % 8 != 0) return 0;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  if (M % TP != 0 || M >= ((int64_t)1 << 31)) return 0;
  return TP;
}

int conv_image_launch(const VuGemmFwd& p, hipStream_t st) {
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  const int64_t tiles = (M / TP) * (p.ncol / 64);
  int64_t nblk = (tiles + 3) / 4;
  const int64_t cap = 8 * (int64_t)cu_count();  // 2 blocks (8 waves) per CU, 4 rounds
  if (nblk > cap) nblk = cap;
  if (p.relu)
    hipLaunchKernelGGL(conv3x3_image_kernel<true>, dim3((unsigned)nblk), dim3(NT), 0, st, p);
  else
    hipLaunchKernelGGL(conv3x3_image_kernel<false>, dim3((unsigned)nblk), dim3(NT), 0, st, p);
  return (int)hipGetLastError();
}
