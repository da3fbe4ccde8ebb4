// 3x3 / stride-1 / pad-1 convolution as an implicit GEMM over a HALO tile
// ("v3", bf16).  Serves the U-Net's DoubleConv forward convs
// (unet_parts.py:40,43) and their stride-1 data-gradient convs (flipped
// weights), i.e. every 3x3 conv of the hot path but the image conv.
//
// Why a halo: the v2 kernel gathers every 3x3 tap of a 256-pixel row tile
// separately, so each input pixel crosses L2 -> LDS nine times and every lane
// recomputes a gather address per tap.  Here a block owns a TH x TW pixel
// tile of one image; per 64-channel chunk it DMA-loads the (TH+2) x (TW+2)
// halo ONCE (340 pixels for 8x32 instead of 9 x 256) and the nine taps read
// it in place from LDS with a shifted row index.  Only the weights stream per
// tap.
//
//   * 8 waves, output tile 256 pixels x BN (128: waves 4x2, 64x64 each; 64:
//     waves 8x1, 32x64 each), 16x16x32 bf16 MFMA;
//   * halo and weight tiles land by LDS-DMA (global_load_lds_dwordx4) with
//     the XOR chunk swizzle applied on the source address (lane-linear LDS
//     image, conflict-free ds_read_b128 fragment reads); padding pixels are
//     DMA'd from a zero page;
//   * weights: 3-slot ring, two taps ahead; halo: double-buffered, the next
//     chunk's halo is DMA'd one piece per tap during the current chunk; every
//     wait is a COUNTED vmcnt followed by a raw s_barrier;
//   * epilogue identical to v1/v2: fp32 tile in LDS, BatchNorm per-tile
//     (sum, centered M2) on the bf16-rounded values, 16-byte stores.
#include "common.h"
#include "../../include/vaeunet.h"

static __device__ __attribute__((aligned(16))) uint32_t vu_zero_page3[16];

namespace {

constexpr int KB = 128;  // bytes per LDS row (64 bf16 channels)
typedef __attribute__((address_space(3))) void lds_void;

VU_DEV int swz(int row, int chunk) { return row * KB + ((chunk ^ (row & 7)) << 4); }

template <int TW>
struct Geo {
  static constexpr int TH = 256 / TW;
  static constexpr int HW = TW + 2;               // halo row length
  static constexpr int HP = (TH + 2) * HW;        // halo pixels
};

template <int BN, int WM, int WN, int TW, int NHB>
__global__ __launch_bounds__(512, 1) void conv3x3_halo_kernel(VuGemmFwd p) {
  constexpr int NT = 512;
  constexpr int BM = 256;
  constexpr int TH = Geo<TW>::TH, HW = Geo<TW>::HW, HP = Geo<TW>::HP;
  constexpr int NH = (HP * 8 + NT - 1) / NT;      // halo DMA instrs per thread
  constexpr int HALO = NH * NT * 16;              // bytes per halo buffer (padded)
  constexpr int LB = BN * 8 / NT;                 // weight DMA instrs per thread per tap
  constexpr int BSTG = BN * KB;
  constexpr int NBS = 3;
  constexpr int MAIN = NHB * HALO + NBS * BSTG;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int ES = BN + 4;
  constexpr int EPI = BM * ES * 4;
  constexpr int RED = (NT / BN) * BN * 4;
  constexpr int LDS_BYTES = (MAIN > EPI ? MAIN : EPI) + RED;
  static_assert(NH <= 7, "next-chunk halo pieces must be issued >= 2 taps before use");
  static_assert(LB >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const VuGather& g = p.a;
  const int H = g.H, W = g.W;
  const int tx_n = W / TW, ty_n = H / TH;
  const int mtiles = g.N * ty_n * tx_n;
  const int ntiles = (p.ncol + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, mtiles * ntiles);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int img = mt / (ty_n * tx_n);
  const int trem = mt - img * (ty_n * tx_n);
  const int y0 = (trem / tx_n) * TH, x0 = (trem - (trem / tx_n) * tx_n) * TW;
  const int n0 = nt * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int pchunk = lane & 7;
  const int nchunk = g.C / 64;
  const int nk = nchunk * 9;

  // halo slots of this thread: pixel index in the image (or -1 = padding)
  int hpix[NH];
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    int hp = (i * NT + tid) >> 3;
    int hy = hp / HW, hx = hp - (hp / HW) * HW;
    int y = y0 - 1 + hy, x = x0 - 1 + hx;
    bool ok = hp < HP && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    hpix[i] = ok ? (img * H + y) * W + x : -1;
  }
  const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
  const void* zp = (const void*)vu_zero_page3;
  char* const hbuf = smem;
  char* const bbuf = smem + NHB * HALO;

  auto chunk_src = [&](int c, const bf16_t*& src, int64_t& st) {
    const int cb = c * 64;
    const int t = (cb >= g.cend[0]) + (g.nsrc > 2 && cb >= g.cend[1]);
    const int c0 = t == 0 ? 0 : g.cend[t - 1];
    src = reinterpret_cast<const bf16_t*>(g.src[t]) + (cb - c0);
    st = g.stride[t];
  };
  auto halo_piece = [&](int c, int i) {
    const bf16_t* src;
    int64_t st;
    chunk_src(c, src, st);
    const int hp = (i * NT + tid) >> 3;
    const int lchunk = pchunk ^ (hp & 7);
    const void* gp = hpix[i] >= 0 ? (const void*)(src + (int64_t)hpix[i] * st + lchunk * 8) : zp;
    char* dst = hbuf + (c % NHB) * HALO + (i * NT + wid * 64) * 16;
    __builtin_amdgcn_global_load_lds(gp, (lds_void*)dst, 16, 0, 0);
  };
  auto wstage = [&](int s) {
    const int c = s / 9, t = s - (s / 9) * 9;
    const int k0 = t * g.C + c * 64;
    char* B = bbuf + (s % NBS) * BSTG;
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      int row = (i * NT + tid) >> 3;
      int lchunk = pchunk ^ (row & 7);
      int j = n0 + row;
      const void* gp = zp;
      if (j < p.ncol) gp = bmat + (int64_t)j * p.ldb + k0 + lchunk * 8;
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(B + (i * NT + wid * 64) * 16), 16, 0, 0);
    }
  };
  // DMA instrs issued in loop step u (for the counted waits below)
  auto hp_at = [&](int u) -> int {
    if (u < 0) return 0;
    const int c = u / 9, t = u - (u / 9) * 9;
    return (NHB > 1 && t < NH && c + 1 < nchunk) ? 1 : 0;
  };

  // fragment row bases: local output pixel of row (lane & 15) of each i-tile
  int hrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int m = wm * (BM / WM) + i * 16 + (lane & 15);
    int ty = m / TW, tx = m - (m / TW) * TW;
    hrow[i] = ty * HW + tx;
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  // prologue: halo of chunk 0, weights of steps 0 and 1
#pragma unroll
  for (int i = 0; i < NH; ++i) halo_piece(0, i);
  wstage(0);
  if (nk > 1) wstage(1);

  for (int s = 0; s < nk; ++s) {
    const int c = s / 9, t = s - (s / 9) * 9;
    // wait for weights(s) [and, at t == 0, the halo of chunk c, issued earlier]:
    // what may stay in flight is everything issued after weights(s)
    int younger = (s >= 1 ? (LB * (s + 1 < nk ? 1 : 0) + hp_at(s - 1)) : LB * (nk > 1 ? 1 : 0)) + hp_at(s - 2);
    if (NHB == 1 && t == 0 && c > 0) younger = 0;
    switch (younger) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (NHB == 1 && t == 0 && c > 0) {
      // single halo buffer: reload it in place (only when a chunk follows)
#pragma unroll
      for (int i = 0; i < NH; ++i) halo_piece(c, i);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (s + 2 < nk) wstage(s + 2);
    if (NHB > 1 && t < NH && c + 1 < nchunk) {
#pragma unroll
      for (int i = 0; i < NH; ++i)
        if (i == t) halo_piece(c + 1, i);
    }
    const char* A = hbuf + (c % NHB) * HALO;
    const char* B = bbuf + (s % NBS) * BSTG;
    const int toff = (t / 3) * HW + (t - (t / 3) * 3);
    // both k-halves' fragments are read up front: the second half's reads
    // complete under the first half's MFMAs
    u32x4 af[2][TM], bf[2][TN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) af[kk][i] = *reinterpret_cast<const u32x4*>(A + swz(hrow[i] + toff, ch));
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
  __syncthreads();

  // ---- epilogue ----
  float* E = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int col = wn * (BN / WN) + j * 16 + (lane & 15);
      int gj = n0 + col;
      float bv = 0.f;
      if (p.bias && gj < p.ncol) bv = p.bias[gj];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = wm * (BM / WM) + i * 16 + 4 * (lane >> 4) + r;
        E[row * ES + col] = rnd<bf16_t>(epi_act(acc[i][j][r] + bv, p.relu));
      }
    }
  __syncthreads();

  if (p.stat_sum) {
    float* red = reinterpret_cast<float*>(smem + LDS_BYTES - RED);
    constexpr int PARTS = NT / BN;
    constexpr int RPP = BM / PARTS;
    const int col = tid % BN, part = tid / BN;
    float s = 0.f;
#pragma unroll 8
    for (int r = part * RPP; r < (part + 1) * RPP; ++r) s += E[r * ES + col];
    red[part * BN + col] = s;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int q = 0; q < PARTS; ++q) tot += red[q * BN + col];
    const float mean = tot * (1.f / BM);
    float m2 = 0.f;
#pragma unroll 8
    for (int r = part * RPP; r < (part + 1) * RPP; ++r) { float d = E[r * ES + col] - mean; m2 += d * d; }
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
  for (int e = tid; e < BM * CPR; e += NT) {
    int row = e / CPR, cc = (e - row * CPR) * 8;
    int gj = n0 + cc;
    if (gj >= p.ncol) continue;
    int ty = row / TW, tx = row - (row / TW) * TW;
    int64_t m = ((int64_t)img * H + y0 + ty) * W + x0 + tx;
    bf16_t* dst = out + m * p.out_stride + p.out_coff + gj;
    const float* src = E + row * ES + cc;
    Vec8<bf16_t> v;
    if (p.accumulate) {
      v.load(dst);
#pragma unroll
      for (int q = 0; q < 8; ++q) v.set(q, v.get(q) + src[q]);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) v.set(q, src[q]);
    }
    v.store(dst);
  }
}

template <int BN, int WM, int WN, int TW, int NHB>
int launch(const VuGemmFwd& p, hipStream_t st) {
  const VuGather& g = p.a;
  int64_t mt = (int64_t)g.N * (g.H / Geo<TW>::TH) * (g.W / TW);
  int64_t nblk = mt * ((p.ncol + BN - 1) / BN);
  hipLaunchKernelGGL((conv3x3_halo_kernel<BN, WM, WN, TW, NHB>), dim3((unsigned)nblk), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

int pick_tw(const VuGather& g) {
  if (g.W % 32 == 0 && g.H % 8 == 0) return 32;
  if (g.W % 16 == 0 && g.H % 16 == 0) return 16;
  return 0;
}

}  // namespace

// Row tile (256) when the halo kernel serves this problem, else 0: bf16, a
// 3x3 stride-1 pad-1 gather over same-size sources, 64-channel aligned
// source groups, plain NHWC output, and an image that tiles by 8x32 / 16x16.
int gemm_fwd_v3_bm(const VuGemmFwd& p, int dtype) {
  const VuGather& g = p.a;
  if (dtype != VU_BF16 || p.out_mode != 0) return 0;
  if (g.R != 3 || g.S != 3 || g.sy != 1 || g.sx != 1 || g.dy != 1 || g.dx != 1 || g.oy != -1 ||
      g.ox != -1 || g.Hs != g.H || g.Ws != g.W)
    return 0;
  if (g.C % 64 != 0) return 0;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.cend[t] % 64 != 0 || g.stride[t] % 8 != 0) return 0;
  if (p.ncol % 8 != 0 || p.out_stride % 8 != 0 || p.out_coff % 8 != 0 || p.ldb % 8 != 0) return 0;
  if (!pick_tw(g)) return 0;
  if ((int64_t)g.N * g.H * g.W >= (int64_t)1 << 31) return 0;
  return 256;
}

int gemm_fwd_v3_launch(const VuGemmFwd& p, hipStream_t st) {
  const int tw = pick_tw(p.a);
  const bool one = p.a.C == 64;
  if (p.ncol <= 64) {
    if (tw == 32) return one ? launch<64, 8, 1, 32, 1>(p, st) : launch<64, 8, 1, 32, 2>(p, st);
    return one ? launch<64, 8, 1, 16, 1>(p, st) : launch<64, 8, 1, 16, 2>(p, st);
  }
  if (tw == 32) return launch<128, 4, 2, 32, 2>(p, st);
  return launch<128, 4, 2, 16, 2>(p, st);
}
