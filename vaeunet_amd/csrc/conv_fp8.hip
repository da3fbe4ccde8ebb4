// fp8 (OCP e4m3fn) 3x3 convolution forward -- BASELINE.json configs[4]
// ("fp8 NHWC implicit-GEMM 3x3 conv path on CDNA4 fp8 MFMA, 3x1024x1024"):
// the DoubleConv convolutions (unet_parts.py:40,43) with e4m3 activations
// (one scale per tensor) and e4m3 weights (one scale per output channel),
// fp32 accumulation, bf16 output and BatchNorm partials from the epilogue.
// The reference has no fp8 path; SURVEY.md asks for the error vs fp32 to be
// reported.  The kernel itself is checked against fp32 convolution of the
// DEQUANTISED operands (tests/test_gpu_fp8.py).
//
// The kernel is the persistent ping-pong halo kernel of gemm_fwd5.hip with
// the bytes reinterpreted: one K-step is one tap x 64 input channels, so the
// 64-byte halo rows, 64-byte weight rows and the whole DMA schedule carry
// over, and the MFMA is v_mfma_f32_32x32x64_f8f6f4 (e4m3 x e4m3, unit block
// scales): 64 k per instruction at twice the bf16 rate, so a K-step does
// twice the work of a bf16 K-step in the same MFMA cycles.
//
//   * wave tile 128 pixels x 64 channels = 4 (pixel) x 2 (channel) 32x32
//     fragments (128 accumulator registers, as in v4/v5);
//   * A = weights: lane l reads row chperm(l&31) of the fragment's 32 rows,
//     bytes 32*(l>>5).. (32 consecutive k); chperm makes accumulator register
//     r of lane l hold output channel 16*(l>>5) + r, so a lane owns 16
//     consecutive channels of one pixel (two 16-byte bf16 stores);
//   * B = pixels: lane l reads the halo row of pixel l&31, bytes 32*(l>>5)..;
//   * a lane's 32 bytes are two 16-byte pieces of a 64-byte row.  With the
//     32-lane fragments every ds_read_b128 lane group would hit each bank
//     quad 4 times, so the DMA stores piece c of row r at piece c ^ ((r>>2)&3)
//     (source-side swizzle, LDS-DMA stays lane-linear) and the reads undo it:
//     conflict-free for any row offset (taps shift the halo rows);
//   * epilogue (registers, the next tile's data is in flight in LDS):
//     acc * x_scale * w_scale[co] (+ bias), bf16 rounding, per-wave (sum,
//     centered M2) over its 128 pixels, 16-byte NHWC stores.
#include "common.h"
#include "../../include/vaeunet.h"

#include <cstring>

static __device__ __attribute__((aligned(16))) uint32_t vu_zero_page8[16];

int splitk_finish_launch(const VuGemmFwd& p, hipStream_t st);  // gemm_fwd4.hip

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int BN> struct PP;
template <> struct PP<256> { static constexpr int WM = 2, WN = 4, TH = 8, TW = 32; };
template <> struct PP<128> { static constexpr int WM = 4, WN = 2, TH = 16, TW = 32; };
template <> struct PP<64> { static constexpr int WM = 8, WN = 1, TH = 32, TW = 32; };

VU_DEV void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
  }
}

VU_DEV void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int R>
VU_DEV float ror_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false));
}
// sum over the 32 lanes of a half-wave (every lane receives the total): DPP
// row sums, then v_permlane16_swap pairs rows 0/1 and 2/3 (a VALU exchange;
// a __shfl_xor across rows is an LDS ds_bpermute round trip)
VU_DEV float half32_sum(float v) {
  v = ror_add<1>(ror_add<2>(ror_add<4>(ror_add<8>(v))));
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

VU_DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

// min / max over the 32 lanes of a half-wave (VuConvFp8.stat_min / stat_max):
// the half32_sum network with fminf / fmaxf
template <int R>
VU_DEV float ror_max(float v) {
  return fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false)));
}
template <int R>
VU_DEV float ror_min(float v) {
  return fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false)));
}
VU_DEV float half32_max(float v) {
  v = ror_max<1>(ror_max<2>(ror_max<4>(ror_max<8>(v))));
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
VU_DEV float half32_min(float v) {
  v = ror_min<1>(ror_min<2>(ror_min<4>(ror_min<8>(v))));
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fminf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// ---- butterfly transpose-reduce over the 32 lanes of a half-wave ----------
// v[k] (32 slots per lane) -> lane m of the half holds sum over the half's
// lanes of slot m: each step pairs lanes across one lane bit and halves the
// array (31 exchanges in all instead of 32 five-step row reductions).  Lane
// bit 4 by v_permlane16_swap, 3 by row_ror:8, 2 by row_half_mirror +
// quad reversal, 1 and 0 by quad permutations (all VALU: no LDS crossbar).
template <int CTRL>
VU_DEV float dmov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
VU_DEV float lx1(float v) { return dmov<0xB1>(v); }             // lane ^ 1
VU_DEV float lx2(float v) { return dmov<0x4E>(v); }             // lane ^ 2
VU_DEV float lx4(float v) { return dmov<0x1B>(dmov<0x141>(v)); }  // lane ^ 4
VU_DEV float lx8(float v) { return dmov<0x128>(v); }            // lane ^ 8 (row_ror:8)

VU_DEV float bfly32_reduce(const float (&v)[32], int lane) {
  const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
  float w[16], x[8], y[4], z[2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[k]), __float_as_uint(v[k + 16]), false, false);
    w[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // even rows: slot k, odd rows: slot k + 16
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = (b3 ? w[k + 8] : w[k]) + lx8(b3 ? w[k] : w[k + 8]);
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = (b2 ? x[k + 4] : x[k]) + lx4(b2 ? x[k] : x[k + 4]);
#pragma unroll
  for (int k = 0; k < 2; ++k) z[k] = (b1 ? y[k + 2] : y[k]) + lx2(b1 ? y[k] : y[k + 2]);
  return (b0 ? z[1] : z[0]) + lx1(b0 ? z[0] : z[1]);
}

// 16-slot transpose-reduce over the 16 lanes of a DPP row with min or max:
// lane m of the row receives slot m's min / max over the row (OP 0 / 1)
template <int OP>
VU_DEV float bfly16_op(const float (&v)[16], int lane) {
  auto f = [](float a, float b) { return OP ? fmaxf(a, b) : fminf(a, b); };
  const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
  float x[8], y[4], z[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = f(b3 ? v[k + 8] : v[k], lx8(b3 ? v[k] : v[k + 8]));
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = f(b2 ? x[k + 4] : x[k], lx4(b2 ? x[k] : x[k + 4]));
#pragma unroll
  for (int k = 0; k < 2; ++k) z[k] = f(b1 ? y[k + 2] : y[k], lx2(b1 ? y[k] : y[k + 2]));
  return f(b0 ? z[1] : z[0], lx1(b0 ? z[0] : z[1]));
}

// the same transpose-reduce with min or max (OP 0 = min, 1 = max)
template <int OP>
VU_DEV float bfly32_op(const float (&v)[32], int lane) {
  auto f = [](float a, float b) { return OP ? fmaxf(a, b) : fminf(a, b); };
  const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
  float w[16], x[8], y[4], z[2];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[k]), __float_as_uint(v[k + 16]), false, false);
    w[k] = f(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = f(b3 ? w[k + 8] : w[k], lx8(b3 ? w[k] : w[k + 8]));
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = f(b2 ? x[k + 4] : x[k], lx4(b2 ? x[k] : x[k + 4]));
#pragma unroll
  for (int k = 0; k < 2; ++k) z[k] = f(b1 ? y[k + 2] : y[k], lx2(b1 ? y[k] : y[k + 2]));
  return f(b0 ? z[1] : z[0], lx1(b0 ? z[0] : z[1]));
}

// inverse: lane m of a half holds the value of slot m -> every lane gets all 32
VU_DEV void bfly32_bcast(float m, int lane, float (&out)[32]) {
  const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
  float z[2], y[4], x[8], w[16];
  {
    const float q = lx1(m);
    z[0] = b0 ? q : m;
    z[1] = b0 ? m : q;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float q = lx2(z[k]);
    y[k] = b1 ? q : z[k];
    y[k + 2] = b1 ? z[k] : q;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float q = lx4(y[k]);
    x[k] = b2 ? q : y[k];
    x[k + 4] = b2 ? y[k] : q;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float q = lx8(x[k]);
    w[k] = b3 ? q : x[k];
    w[k + 8] = b3 ? x[k] : q;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[k]), __float_as_uint(w[k]), false, false);
    out[k] = __uint_as_float(r[0]);       // slot k (bit 4 clear): the even row's value
    out[k + 16] = __uint_as_float(r[1]);  // slot k + 16: the odd row's
  }
}

// piece swizzle of a 64-byte row (see header)
VU_DEV int pswz(int row, int piece) { return (piece ^ ((row >> 2) & 3)) << 4; }

// 32-byte operand of a 32x32x64 fp8 fragment: logical pieces 2h, 2h+1 of row r
VU_DEV i32x8 frag32(const char* base, int row, int h) {
  const char* rp = base + row * 64;
  const u32x4 a = *reinterpret_cast<const u32x4*>(rp + pswz(row, 2 * h));
  const u32x4 b = *reinterpret_cast<const u32x4*>(rp + pswz(row, 2 * h + 1));
  return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
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

int g_grid = 0;  // VU_TUNE_FP8_GRID: grid cap (tests); 0 = CU count
int g_xm = 0;    // VU_TUNE_FP8_XM: experiment mode (A/B timing only)

// XM: experiment modes (A/B timing only, results wrong): 1 = no MFMAs, 2 = no DMA in the loop
template <int BN, int XM = 0>
__global__ __launch_bounds__(512, 1) void conv3x3_fp8_kernel(VuConvFp8 p) {
  constexpr int WM = PP<BN>::WM, WN = PP<BN>::WN, TH = PP<BN>::TH, TW = PP<BN>::TW;
  constexpr int BM = TH * TW;
  static_assert(BM == WM * 128 && BN == WN * 64 && WM * WN == 8, "wave grid");
  constexpr int HW = TW + 2, HP = (TH + 2) * HW;
  constexpr int HPIECES = HP * 4;                 // 16-byte pieces per chunk halo
  constexpr int NHP1 = (HPIECES + 255) / 256;     // halo DMA slots per half-1 thread
  constexpr int HALO = HP * 64;
  constexpr int WPIECES = BN * 4;
  constexpr int LB0 = WPIECES / 256;              // weight DMA slots per half-0 thread
  constexpr int LB0A = (LB0 + 1) / 2;
  constexpr int WSLOT = BN * 64;
  constexpr int NBW = 3;
  constexpr int PPS1 = (NHP1 + 7) / 8;
  constexpr int LDS_BYTES = 2 * HALO + NBW * WSLOT;
  static_assert(LDS_BYTES <= 163840, "LDS");
  static_assert(NHP1 <= 8 * PPS1 && LB0 >= 1, "DMA schedule");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const VuGather& g = p.a;
  const int H = g.H, W = g.W;
  const int tx_n = W / TW, ty_n = H / TH;
  const int mtiles = g.N * ty_n * tx_n;
  const int ntiles = p.ncol / BN;
  const int T = mtiles * ntiles;
  const int G = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, G);
  const int ntl = (T - lb + G - 1) / G;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int grp = wid >> 2;
  const int nchunk = g.C / 64;                    // 64 e4m3 channels = one 64-byte row
  const int nk = nchunk * 9;
  const int S = ntl * nk;

  struct Tile { int img, y0, x0, n0, mt; };
  auto tile_of = [&](int i) -> Tile {
    const int tile = lb + i * G;
    Tile q;
    q.mt = tile / ntiles;
    q.n0 = (tile - q.mt * ntiles) * BN;
    q.img = q.mt / (ty_n * tx_n);
    const int trem = q.mt - q.img * (ty_n * tx_n);
    q.y0 = (trem / tx_n) * TH;
    q.x0 = (trem - (trem / tx_n) * tx_n) * TW;
    return q;
  };

  const int gt = tid & 255;
  const int gw = wid & 3;
  const uint8_t* bmat = reinterpret_cast<const uint8_t*>(p.w);
  const void* zp = (const void*)vu_zero_page8;
  char* const hbuf = smem;
  char* const wbuf = smem + 2 * HALO;

  const uint8_t* const src0 = reinterpret_cast<const uint8_t*>(g.src[0]);
  const uint8_t* const src1 = reinterpret_cast<const uint8_t*>(g.src[1]);
  const uint8_t* const src2 = reinterpret_cast<const uint8_t*>(g.src[2]);
  const int64_t st0 = g.stride[0], st1 = g.stride[1], st2 = g.stride[2];
  const int ce0 = g.cend[0], ce1 = g.nsrc > 2 ? g.cend[1] : (1 << 30);
  struct HaloT { const uint8_t* src; int64_t st; char* hb; int img, y0, x0; };
  auto halo_target = [&](int i, int c) -> HaloT {
    const Tile q = tile_of(i);
    const int cb = c * 64;
    HaloT h;
    if (cb < ce0) {
      h.src = src0 + cb;
      h.st = st0;
    } else if (cb < ce1) {
      h.src = src1 + (cb - ce0);
      h.st = st1;
    } else {
      h.src = src2 + (cb - ce1);
      h.st = st2;
    }
    h.hb = hbuf + ((i * nchunk + c) & 1) * HALO;
    h.img = q.img;
    h.y0 = q.y0;
    h.x0 = q.x0;
    return h;
  };
  auto halo_issue = [&](const HaloT& h, int t) {
#pragma unroll
    for (int k = 0; k < NHP1; ++k) {
      if (t >= 0 && k / PPS1 != t) continue;
      if (k * 256 + gw * 64 >= HPIECES) continue;
      const int P = k * 256 + gt;
      if (P < HPIECES) {
        const int px = P >> 2;
        const int hy = px / HW, hx = px - (px / HW) * HW;
        const int y = h.y0 - 1 + hy, x = h.x0 - 1 + hx;
        const void* gp = zp;
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          gp = h.src + ((int64_t)(h.img * H + y) * W + x) * h.st + pswz(px, P & 3);
        __builtin_amdgcn_global_load_lds(gp, (lds_void*)(h.hb + (k * 256 + gw * 64) * 16), 16, 0, 0);
      }
    }
  };
  int wi_ = 0, ws_ = 0, n0w_ = (lb % ntiles) * BN, wgs_ = 0;
  auto wnext = [&]() {
    ++wgs_;
    if (++ws_ == nk) {
      ws_ = 0;
      ++wi_;
      n0w_ = ((lb + wi_ * G) % ntiles) * BN;
    }
  };
  auto wstage = [&](int k0, int k1) {
    const int c = ws_ / 9, t = ws_ - (ws_ / 9) * 9;
    const int kb = t * g.C + c * 64;
    char* B = wbuf + (wgs_ % NBW) * WSLOT;
#pragma unroll
    for (int k = 0; k < LB0; ++k) {
      if (k < k0 || k >= k1) continue;
      const int P = k * 256 + gt;
      const int row = P >> 2;
      const void* gp = bmat + (int64_t)(n0w_ + row) * p.ldw + kb + pswz(row, P & 3);
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(B + (k * 256 + gw * 64) * 16), 16, 0, 0);
    }
  };

  // ---- fragment addressing -------------------------------------------------
  const int hl = lane >> 5;       // k half of the lane (bytes 32*hl..)
  int prow[4];                    // halo row of this lane's pixel per fragment (tap (0,0))
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = wm * 128 + i * 32 + (lane & 31);
    prow[i] = (m / TW) * HW + (m - (m / TW) * TW);
  }
  const int rho = lane & 31;
  const int wrow = wn * 64 + 16 * ((rho >> 2) & 1) + 4 * (rho >> 3) + (rho & 3);  // + 32*j
  const int cb16 = wn * 64 + 16 * hl;  // acc[i][j][r]: channel cb16 + 32*j + r

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const float xsc = *p.x_scale;
  bf16_t* const out = reinterpret_cast<bf16_t*>(p.out);
  auto epilogue = [&](int ti) {
    const Tile q = tile_of(ti);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c0 = q.n0 + cb16 + 32 * j;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float sc = xsc * p.w_scale[c0 + r];
        const float bv = p.bias ? p.bias[c0 + r] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j][r] = rnd<bf16_t>(fmaf(acc[i][j][r], sc, bv));
      }
    }
    if (p.stat_sum) {
      const int64_t so = (int64_t)(q.mt * WM + wm) * p.ncol + q.n0 + cb16;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          f32x4 sm, m2;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int r = r4 * 4 + u;
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) s += acc[i][j][r];
            s = half32_sum(s);
            const float mean = s * (1.f / 128);
            float v = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float d = acc[i][j][r] - mean;
              v += d * d;
            }
            sm[u] = s;
            m2[u] = half32_sum(v);
          }
          if ((lane & 31) == 0) {
            *reinterpret_cast<f32x4*>(p.stat_sum + so + 32 * j + 4 * r4) = sm;
            *reinterpret_cast<f32x4*>(p.stat_m2 + so + 32 * j + 4 * r4) = m2;
          }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = wm * 128 + i * 32 + (lane & 31);
      const int ty = m / TW, tx = m - (m / TW) * TW;
      const int64_t pix = ((int64_t)q.img * H + q.y0 + ty) * W + q.x0 + tx;
      bf16_t* dst = out + pix * p.out_stride + p.out_coff + q.n0 + cb16;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          u32x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = pack2(acc[i][j][8 * h + 2 * e], acc[i][j][8 * h + 2 * e + 1]);
          *reinterpret_cast<u32x4*>(dst + 32 * j + 8 * h) = pk;
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  };

  // ---- prologue -------------------------------------------------------------
  HaloT hn;
  if (grp) {
    halo_issue(halo_target(0, 0), -1);
  } else {
    wstage(0, LB0);
    wnext();
    if (S > 1) wstage(0, LB0);
    wnext();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  if (grp) pp_barrier();  // the stagger: half 1 runs one barrier behind

  int ti = 0, s = 0;
  for (int gs = 0; gs < S; ++gs) {
    const int c = s / 9, t = s - (s / 9) * 9;
    const char* A = hbuf + ((ti * nchunk + c) & 1) * HALO;
    const int toff = (t / 3) * HW + (t - (t / 3) * 3);
    const char* Bw = wbuf + (gs % NBW) * WSLOT;
    i32x8 wf[2], pf[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) wf[j] = frag32(Bw, wrow + 32 * j, hl);
#pragma unroll
    for (int i = 0; i < 2; ++i) pf[i] = frag32(A, prow[i] + toff, hl);
    if (XM != 2 && !grp && gs + 2 < S) wstage(0, LB0A);
    pp_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (XM == 1)
          acc[i][j][0] += __builtin_bit_cast(float, wf[j][0] ^ pf[i][1]);
        else
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[j], pf[i], acc[i][j], 0, 0, 0, 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
#pragma unroll
    for (int i = 0; i < 2; ++i) pf[i] = frag32(A, prow[2 + i] + toff, hl);
    if (XM == 2) {
      if (!grp) wnext();
    } else if (!grp) {
      if (gs + 2 < S) {
        wstage(LB0A, LB0);
        wnext();
        wait_vm(LB0);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      const bool more = c + 1 < nchunk || ti + 1 < ntl;
      if (more) {
        if (t == 0) hn = c + 1 < nchunk ? halo_target(ti, c + 1) : halo_target(ti + 1, 0);
        if (t * PPS1 < NHP1) halo_issue(hn, t);
        if (t == 8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    pp_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (XM == 1)
          acc[2 + i][j][0] += __builtin_bit_cast(float, wf[j][0] ^ pf[i][1]);
        else
          acc[2 + i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[j], pf[i], acc[2 + i][j], 0, 0, 0, 0, 0,
                                                                          0);
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
    if (++s == nk) {
      epilogue(ti);
      s = 0;
      ++ti;
    }
  }
  if (!grp) pp_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- one tile per block on the bf16 ping-pong step loop (gemm_fwd4.hip) ----
// Round 3: the persistent kernel above spends ~1.8x the cycles per K-step of
// the bf16 ping-pong kernel (experiment modes: without its MFMAs it runs as
// fast; without its loop DMA 35 % faster), so fp8 bought only 1.05x.  This
// is the bf16 kernel's schedule with the fp8 bytes: one block per 8x32 /
// 16x32 / 32x32-pixel tile, the (chunk, tap) step loop with the weight ring
// slot = tap % 3, the next chunk's halo issued at tap 0 by half 1 and awaited
// at tap 8, and the persistent kernel's 32x32x64 fragments, swizzle and
// register epilogue.  A chunk is 64 e4m3 channels (one 64-byte row), so a
// step carries twice the MFMA work of a bf16 step for the same DMA bytes.
// SPLIT: the block index also picks a contiguous range of 64-channel chunks
// (grid = tiles x ksplit); the scaled fp32 tile goes to slab kidx and the
// deterministic split-K finish of gemm_fwd4.hip adds bias, rounds and emits
// the statistics (grids under one block per CU: the 64^2 level at batch 2)
// MM: also the per-tile per-channel min / max of the stored output
// (VuConvFp8.stat_min / stat_max, the just-in-time e4m3 scale of the next
// conv's input: fp8.double_conv_forward)
template <int BN, int XM = 0, bool SPLIT = false, bool MM = false>
__global__ __launch_bounds__(512, 1) void conv3x3_fp8_pp_kernel(VuConvFp8 p) {
  constexpr int NBW = 3;
  constexpr int WM = PP<BN>::WM, WN = PP<BN>::WN, TH = PP<BN>::TH, TW = PP<BN>::TW;
  constexpr int BM = TH * TW;
  static_assert(BM == WM * 128 && BN == WN * 64 && WM * WN == 8, "wave grid");
  constexpr int HW = TW + 2, HP = (TH + 2) * HW;
  constexpr int HPIECES = HP * 4;
  constexpr int NHP1 = (HPIECES + 255) / 256;
  constexpr int HALO = HP * 64;
  constexpr int WPIECES = BN * 4;
  constexpr int LB0 = WPIECES / 256;
  constexpr int LB0A = (LB0 + 1) / 2;
  constexpr int WSLOT = BN * 64;
  constexpr int PD = NBW - 1;
  constexpr int MAIN = 2 * HALO + NBW * WSLOT;
  static_assert(MAIN <= 163840 && LB0 >= 1, "LDS / DMA schedule");
  __shared__ __attribute__((aligned(16))) char smem[MAIN];

  const VuGather& g = p.a;
  const int H = g.H, W = g.W;
  const int tx_n = W / TW, ty_n = H / TH;
  const int mtiles = g.N * ty_n * tx_n;
  const int ntiles = p.ncol / BN;
  const int btiles = mtiles * ntiles;
  const int ks = SPLIT ? (int)(gridDim.x / btiles) : 1;
  const int bid0 = xcd_remap(blockIdx.x, btiles * ks);
  const int kidx = SPLIT ? bid0 / btiles : 0;
  const int bid = bid0 - kidx * btiles;
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int img = mt / (ty_n * tx_n);
  const int trem = mt - img * (ty_n * tx_n);
  const int y0 = (trem / tx_n) * TH, x0 = (trem - (trem / tx_n) * tx_n) * TW;
  const int n0 = nt * BN;
  const int nchunk = g.C / 64;
  const int cbeg = SPLIT ? kidx * nchunk / ks : 0, cend = SPLIT ? (kidx + 1) * nchunk / ks : nchunk;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int grp = wid >> 2;
  const int gt = tid & 255, gw = wid & 3;
  const uint8_t* bmat = reinterpret_cast<const uint8_t*>(p.w);
  const void* zp = (const void*)vu_zero_page8;
  char* const hbuf = smem;
  char* const wbuf = smem + 2 * HALO;

  const uint8_t* const src0 = reinterpret_cast<const uint8_t*>(g.src[0]);
  const uint8_t* const src1 = reinterpret_cast<const uint8_t*>(g.src[1]);
  const uint8_t* const src2 = reinterpret_cast<const uint8_t*>(g.src[2]);
  const int64_t st0 = g.stride[0], st1 = g.stride[1], st2 = g.stride[2];
  const int ce0 = g.cend[0], ce1 = g.nsrc > 2 ? g.cend[1] : (1 << 30);
  auto halo_chunk = [&](int c, int buf) {
    int ib = img, yb = y0, xb = x0;
    asm volatile("" : "+s"(ib), "+s"(yb), "+s"(xb));
    const int cb = c * 64;
    const uint8_t* src;
    int64_t st;
    if (cb < ce0) {
      src = src0 + cb;
      st = st0;
    } else if (cb < ce1) {
      src = src1 + (cb - ce0);
      st = st1;
    } else {
      src = src2 + (cb - ce1);
      st = st2;
    }
    src += (int64_t)ib * H * W * st;
#pragma unroll
    for (int i = 0; i < NHP1; ++i) {
      if (i * 256 + gw * 64 >= HPIECES) continue;  // wave-uniform
      const int P = i * 256 + gt;
      if (P < HPIECES) {
        const int px = P >> 2;
        const int hy = px / HW, hx = px - (px / HW) * HW;
        const int y = yb - 1 + hy, x = xb - 1 + hx;
        const bool ok = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        const void* gp = ok ? (const void*)(src + (int64_t)(y * W + x) * st + pswz(px, P & 3)) : zp;
        __builtin_amdgcn_global_load_lds(gp, (lds_void*)(hbuf + buf * HALO + (i * 256 + gw * 64) * 16), 16, 0, 0);
      }
    }
  };
  const uint8_t* const wrow0 = bmat + (int64_t)n0 * p.ldw;
  auto wstage = [&](int c, int t, int slot, int i0, int i1) {
    const int k0 = t * g.C + c * 64;
    char* B = wbuf + slot * WSLOT;
#pragma unroll
    for (int i = 0; i < LB0; ++i) {
      if (i < i0 || i >= i1) continue;
      const int P = i * 256 + gt;
      const int row = P >> 2;
      const void* gp = (const void*)(wrow0 + (int64_t)row * p.ldw + k0 + pswz(row, P & 3));
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(B + (i * 256 + gw * 64) * 16), 16, 0, 0);
    }
  };

  // fragment addressing (as the persistent kernel)
  const int hl = lane >> 5;
  int prow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = wm * 128 + i * 32 + (lane & 31);
    prow[i] = (m / TW) * HW + (m - (m / TW) * TW);
  }
  const int rho = lane & 31;
  const int wrow = wn * 64 + 16 * ((rho >> 2) & 1) + 4 * (rho >> 3) + (rho & 3);  // + 32*j
  const int cb16 = wn * 64 + 16 * hl;  // acc[i][j][r]: channel cb16 + 32*j + r

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (grp) {
    halo_chunk(cbeg, 0);
  } else {
    wstage(cbeg, 0, 0, 0, LB0);
    wstage(cbeg, 1, 1, 0, LB0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  if (grp) pp_barrier();

  int hb = 0;
  for (int c = cbeg; c < cend; ++c) {
    const bool next_here = c + 1 < cend;
    const char* Ah = hbuf + hb * HALO;
    // not unrolled: the compiler would hoist all nine taps' swizzled fragment
    // addresses out of the loop and spill them
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int ty = (t * 11) >> 5, tx = t - ty * 3;
      const int toff = ty * HW + tx;
      const int slot = tx;
      const char* Bw = wbuf + slot * WSLOT;
      const int pslot = slot == 0 ? 2 : slot - 1;
      const int pt = t + PD < 9 ? t + PD : t + PD - 9;
      const bool pref = t + PD < 9 || next_here;
      const int pc = t + PD < 9 ? c : c + 1;
      i32x8 wf[2], pf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) wf[j] = frag32(Bw, wrow + 32 * j, hl);
#pragma unroll
      for (int i = 0; i < 2; ++i) pf[i] = frag32(Ah, prow[i] + toff, hl);
      if (XM != 2 && !grp && pref) wstage(pc, pt, pslot, 0, LB0A);
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (XM == 1)
            acc[i][j][0] += __builtin_bit_cast(float, wf[j][0] ^ pf[i][1]);
          else
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[j], pf[i], acc[i][j], 0, 0, 0, 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
#pragma unroll
      for (int i = 0; i < 2; ++i) pf[i] = frag32(Ah, prow[2 + i] + toff, hl);
      if (XM == 2) {
      } else if (!grp) {
        if (pref) {
          wstage(pc, pt, pslot, LB0A, LB0);
          wait_vm((PD - 1) * LB0);
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else {
        if (t == 0 && next_here) halo_chunk(c + 1, hb ^ 1);
        if (t == 8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (XM == 1)
            acc[2 + i][j][0] += __builtin_bit_cast(float, wf[j][0] ^ pf[i][1]);
          else
            acc[2 + i][j] =
                __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[j], pf[i], acc[2 + i][j], 0, 0, 0, 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    }
    hb ^= 1;
  }
  if (!grp) pp_barrier();

  // ---- register epilogue (the persistent kernel's) ---------------------------
  const __attribute__((address_space(4))) VuConvFp8* ep =
      (const __attribute__((address_space(4))) VuConvFp8*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ep));
  const float xsc = *ep->x_scale;
  if (SPLIT) {
    // scaled fp32 partial tile -> slab kidx (row = pixel, ncol columns)
    const int64_t M = (int64_t)g.N * H * W;
    float* const slab = ep->workspace + (int64_t)kidx * M * ep->ncol;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = wm * 128 + i * 32 + (lane & 31);
      const int ty = m / TW, tx = m - (m / TW) * TW;
      float* const row = slab + (((int64_t)img * H + y0 + ty) * W + x0 + tx) * ep->ncol + n0 + cb16;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f32x4 v;
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = acc[i][j][4 * q + u] * (xsc * ep->w_scale[n0 + cb16 + 32 * j + 4 * q + u]);
          *reinterpret_cast<f32x4*>(row + 32 * j + 4 * q) = v;
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c0 = n0 + cb16 + 32 * j;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float sc = xsc * ep->w_scale[c0 + r];
      const float bv = ep->bias ? ep->bias[c0 + r] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j][r] = rnd<bf16_t>(fmaf(acc[i][j][r], sc, bv));
    }
  }
  if (ep->stat_sum) {
    const int64_t so = (int64_t)(mt * WM + wm) * ep->ncol + n0 + cb16;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        f32x4 sm, m2;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = r4 * 4 + u;
          float sv = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) sv += acc[i][j][r];
          sv = half32_sum(sv);
          const float mean = sv * (1.f / 128);
          float v = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float d = acc[i][j][r] - mean;
            v += d * d;
          }
          sm[u] = sv;
          m2[u] = half32_sum(v);
        }
        if ((lane & 31) == 0) {
          *reinterpret_cast<f32x4*>(ep->stat_sum + so + 32 * j + 4 * r4) = sm;
          *reinterpret_cast<f32x4*>(ep->stat_m2 + so + 32 * j + 4 * r4) = m2;
        }
      }
  }
  if constexpr (MM) {
    const int64_t so = (int64_t)(mt * WM + wm) * ep->ncol + n0 + cb16;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        f32x4 mn, mx;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = r4 * 4 + u;
          float a = acc[0][j][r], b = acc[0][j][r];
#pragma unroll
          for (int i = 1; i < 4; ++i) {
            a = fminf(a, acc[i][j][r]);
            b = fmaxf(b, acc[i][j][r]);
          }
          mn[u] = half32_min(a);
          mx[u] = half32_max(b);
        }
        if ((lane & 31) == 0) {
          *reinterpret_cast<f32x4*>(ep->stat_min + so + 32 * j + 4 * r4) = mn;
          *reinterpret_cast<f32x4*>(ep->stat_max + so + 32 * j + 4 * r4) = mx;
        }
      }
  }
  bf16_t* const out = reinterpret_cast<bf16_t*>(ep->out);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = wm * 128 + i * 32 + (lane & 31);
    const int ty = m / TW, tx = m - (m / TW) * TW;
    const int64_t pix = ((int64_t)img * H + y0 + ty) * W + x0 + tx;
    bf16_t* dst = out + pix * ep->out_stride + ep->out_coff + n0 + cb16;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u32x4 pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = pack2(acc[i][j][8 * h + 2 * e], acc[i][j][8 * h + 2 * e + 1]);
        *reinterpret_cast<u32x4*>(dst + 32 * j + 8 * h) = pk;
      }
  }
}

// ---- 64 -> 64 channels: resident weights, persistent tile stream ----------
// The two 64-channel 1024^2 layers (inc.2, up4.2) have one 64-byte chunk per
// pixel: on the step loop above a tile is nine steps long and its prologue
// (first halo) and epilogue are not overlapped (0.93x the bf16 kernels).  As
// the bf16 v6 kernel (gemm_fwd6.hip): the 64 x 576-byte weight matrix lands
// in LDS once per block and stays; a block walks 16 x 32-pixel tiles, the
// next tile's halo landing in the other buffer while this one computes; wave
// w owns image rows 2w, 2w+1 (2 pixel x 2 channel 32x32x64 fragments, 36
// MFMAs per tile); the epilogue (scales, bias, bf16, per-wave statistics of
// its 64 pixels, stores) runs from registers.
constexpr int C64_TH = 16, C64_TW = 32;
constexpr int C64_HW = C64_TW + 2;
constexpr int C64_HP = (C64_TH + 2) * C64_HW;       // 612 halo pixels
constexpr int C64_HPIECES = C64_HP * 4;             // 16-byte pieces
constexpr int C64_NHR = (C64_HPIECES + 511) / 512;  // 5 DMA rounds
constexpr int C64_HALO = C64_HP * 64;
constexpr int C64_WBYTES = 9 * 64 * 64;             // [tap][co][64 ci] e4m3
constexpr int C64_WPIECES = C64_WBYTES / 16;
constexpr int C64_NWR = (C64_WPIECES + 511) / 512;
// output staging strip per wave: 32 pixel rows of 128 bytes (+16 B pad)
constexpr int C64_SP = 144, C64_STRIP = 32 * C64_SP;
constexpr int C64_LDS = C64_WBYTES + 2 * C64_HALO + 2 * 64 * 4 + 8 * C64_STRIP;
static_assert(C64_LDS <= 163840, "LDS");
// NCH = 2 (round 4): 128 input channels (two 64-channel chunks, e.g. the
// up4.1 concat of skip + upsampled sources) -> 64: both chunks' weights
// resident (72 KiB), the (tile, chunk) steps share the halo double buffer,
// direct stores (the staging strips do not fit beside the second chunk)
template <int NCH, bool STG>
constexpr int c64_lds() { return NCH * C64_WBYTES + 2 * C64_HALO + 2 * 64 * 4 + (STG ? 8 * C64_STRIP : 0); }
static_assert(c64_lds<2, false>() <= 163840, "LDS");

// STG: the bf16 output goes through a private LDS strip per wave and leaves
// as whole 128-byte pixel rows (1 KiB contiguous per store instruction)
// instead of 16-byte pieces at a 128-byte pixel stride
// XM (A/B timing only, results wrong): 1 no MFMAs, 2 no loop halo DMA, 3 no output stores,
// 4 no statistics
template <bool STATS, bool STG, int XM = 0, int NCH = 1, bool MM = false>
__global__ __launch_bounds__(512, 1) void conv3x3_fp8_c64_kernel(VuConvFp8 p) {
  static_assert(NCH == 1 || !STG, "LDS: no staging strips beside two weight chunks");
  __shared__ __attribute__((aligned(16))) char smem[c64_lds<NCH, STG>()];
  char* const wl = smem;
  char* const hl0 = smem + NCH * C64_WBYTES;
  float* const ssc = reinterpret_cast<float*>(smem + NCH * C64_WBYTES + 2 * C64_HALO);  // x_scale * w_scale[c]
  float* const sbi = ssc + 64;                                                           // bias[c]
  char* const strip = smem + NCH * C64_WBYTES + 2 * C64_HALO + 2 * 64 * 4 + (threadIdx.x >> 6) * C64_STRIP;

  const VuGather& g = p.a;
  const int H = g.H, W = g.W;
  const int txn = W / C64_TW, per_img = txn * (H / C64_TH);
  const int T = g.N * per_img;
  const int G = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, G);
  const int ntile_blk = (T - lb + G - 1) / G;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // 64-channel chunk ch -> its source tensor and channel offset
  auto chunk_src = [&](int ch, const uint8_t*& s, int64_t& stv) {
    const int cb = 64 * ch;
    const int q = (cb >= g.cend[0]) + (g.nsrc > 2 && cb >= g.cend[1]);
    s = reinterpret_cast<const uint8_t*>(g.src[q]) + (cb - (q == 0 ? 0 : g.cend[q - 1]));
    stv = g.stride[q];
  };
  const void* const zp = (const void*)vu_zero_page8;

  // resident weights: chunk ch, tap block t = 64 rows (output channels) of 64
  // bytes, piece q of row n holding logical piece q ^ ((n>>2)&3) (pswz)
  {
    const uint8_t* bm = reinterpret_cast<const uint8_t*>(p.w);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
      for (int i = 0; i < C64_NWR; ++i) {
        if (i * 512 + wid * 64 >= C64_WPIECES) continue;  // wave-uniform
        const int s = i * 512 + tid;
        const int tap = s >> 8, row = (s >> 2) & 63;
        const void* gp = (const void*)(bm + (int64_t)row * p.ldw + tap * 64 * NCH + 64 * ch + pswz(row, s & 3));
        __builtin_amdgcn_global_load_lds(gp, (lds_void*)(wl + ch * C64_WBYTES + (i * 512 + wid * 64) * 16), 16, 0,
                                         0);
      }
  }
  if (tid < 64) {
    ssc[tid] = *p.x_scale * p.w_scale[tid];
    sbi[tid] = p.bias ? p.bias[tid] : 0.f;
  }
  auto halo = [&](int t, int ch, int b) {
    const int img = t / per_img, r = t - (t / per_img) * per_img;
    const int ty = r / txn, tx = r - (r / txn) * txn;
    const int y0 = ty * C64_TH - 1, x0 = tx * C64_TW - 1;
    const uint8_t* src;
    int64_t st;
    chunk_src(ch, src, st);
    const uint8_t* s0 = src + (int64_t)img * H * W * st;
    char* dst = hl0 + b * C64_HALO;
#pragma unroll
    for (int i = 0; i < C64_NHR; ++i) {
      if (i * 512 + wid * 64 >= C64_HPIECES) continue;  // wave-uniform
      const int s = i * 512 + tid;
      if (s < C64_HPIECES) {
        const int px = s >> 2;
        const int hy = px / C64_HW, hx = px - (px / C64_HW) * C64_HW;
        const int y = y0 + hy, x = x0 + hx;
        const bool ok = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        const void* gp = ok ? (const void*)(s0 + (int64_t)(y * W + x) * st + pswz(px, s & 3)) : zp;
        __builtin_amdgcn_global_load_lds(gp, (lds_void*)(dst + (i * 512 + wid * 64) * 16), 16, 0, 0);
      }
    }
  };

  if (ntile_blk > 0) halo(lb, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int hl = lane >> 5, rho = lane & 31;
  const int wrow = 16 * ((rho >> 2) & 1) + 4 * (rho >> 3) + (rho & 3);  // + 32*j: channel 16*hl + 32*j + r
  const int cb16 = 16 * hl;
  int prow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) prow[i] = (2 * wid + i) * C64_HW + rho;

  f32x16 acc[2][2];
  int t = lb, b = 0;
  for (int ti = 0; ti < ntile_blk; ++ti, t += G)
  for (int ch = 0; ch < NCH; ++ch) {
    // the next (tile, chunk) step's halo lands in the other buffer meanwhile
    if (XM != 2) {
      if (ch + 1 < NCH) halo(t, ch + 1, b ^ 1);
      else if (ti + 1 < ntile_blk) halo(t + G, 0, b ^ 1);
    }
    const char* hb = hl0 + (XM == 2 ? 0 : b) * C64_HALO;
    if (ch == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }
    // rolled: unrolled, the compiler hoists the nine taps' fragment reads
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = (tap / 3) * C64_HW + tap % 3;
      const char* wb = wl + ch * C64_WBYTES + tap * 4096;
      i32x8 wf[2], pf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) wf[j] = frag32(wb, wrow + 32 * j, hl);
#pragma unroll
      for (int i = 0; i < 2; ++i) pf[i] = frag32(hb, prow[i] + toff, hl);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (XM == 1)
            acc[i][j][0] += __builtin_bit_cast(float, wf[j][0] ^ pf[i][1]);
          else
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[j], pf[i], acc[i][j], 0, 0, 0, 0, 0, 0);
    }
    if (NCH > 1 && ch + 1 < NCH) {
      // more chunks of this tile: only the next step's halo is in flight
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      pp_barrier();
      b ^= 1;
      continue;
    }
    // ---- epilogue: acc[i][j][r] = pixel (row 2*wid + i, column rho), channel cb16 + 32j + r
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 sc = *reinterpret_cast<const f32x4*>(ssc + cb16 + 32 * j + 4 * q);
        const f32x4 bi = *reinterpret_cast<const f32x4*>(sbi + cb16 + 32 * j + 4 * q);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 2; ++i) acc[i][j][4 * q + u] = rnd<bf16_t>(fmaf(acc[i][j][4 * q + u], sc[u], bi[u]));
      }
    const int img = t / per_img, r0 = t - (t / per_img) * per_img;
    const int ty = r0 / txn, tx = r0 - (r0 / txn) * txn;
    if constexpr (MM) {
      // per-wave min / max of its 64 pixels, the statistics' lane -> channel
      // map (channel 16*hl + 32*j + r with j = the lane's row in its half):
      // per j a 16-slot transpose-reduce over the DPP row, then the two rows
      // of the half combined (a 32-slot one spilled the two-chunk kernel)
      const bool rowhi = (lane >> 4) & 1;
      float mn = 0.f, mx = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = fminf(acc[0][j][r], acc[1][j][r]);
        float m0 = bfly16_op<0>(v, lane);
        const auto a0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m0), __float_as_uint(m0), false, false);
        m0 = fminf(__uint_as_float(a0[0]), __uint_as_float(a0[1]));
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = fmaxf(acc[0][j][r], acc[1][j][r]);
        float m1 = bfly16_op<1>(v, lane);
        const auto a1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(m1), __float_as_uint(m1), false, false);
        m1 = fmaxf(__uint_as_float(a1[0]), __uint_as_float(a1[1]));
        if (j == (int)rowhi) {
          mn = m0;
          mx = m1;
        }
      }
      const int64_t so = (int64_t)(t * (C64_TH / 2) + wid) * p.ncol + 16 * (lane >> 5) + 32 * ((lane >> 4) & 1) +
                         (lane & 15);
      p.stat_min[so] = mn;
      p.stat_max[so] = mx;
    }
    if (STATS && XM != 4) {
      // per-wave (sum, centered M2) of its 64 pixels: slot k = 16j + r of
      // this lane half (channel 16*hl + 32j + r); after the butterfly lane m
      // of a half holds slot m, i.e. lane l owns channel
      // 16*(l>>5) + 32*((l>>4)&1) + (l&15): one 4-byte store per statistic
      float v[32];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) v[16 * j + r] = acc[0][j][r] + acc[1][j][r];
      const float sv = bfly32_reduce(v, lane);
      float mb[32];
      bfly32_bcast(sv * (1.f / 64), lane, mb);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d0 = acc[0][j][r] - mb[16 * j + r], d1 = acc[1][j][r] - mb[16 * j + r];
          v[16 * j + r] = d0 * d0 + d1 * d1;
        }
      const float mq = bfly32_reduce(v, lane);
      const int64_t so = (int64_t)(t * (C64_TH / 2) + wid) * p.ncol + 16 * (lane >> 5) + 32 * ((lane >> 4) & 1) +
                         (lane & 15);
      p.stat_sum[so] = sv;
      p.stat_m2[so] = mq;
    }

    bf16_t* const out = reinterpret_cast<bf16_t*>(p.out);
    if (STG) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        // this wave's image row 2*wid + i: lane (rho, hl) -> strip row rho
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            u32x4 pk;
#pragma unroll
            for (int e = 0; e < 4; ++e) pk[e] = pack2(acc[i][j][8 * h + 2 * e], acc[i][j][8 * h + 2 * e + 1]);
            *reinterpret_cast<u32x4*>(strip + rho * C64_SP + (cb16 + 32 * j + 8 * h) * 2) = pk;
          }
        // (private strip: the wave's own LDS writes complete before its reads)
        const int64_t pix0 = ((int64_t)img * H + ty * C64_TH + 2 * wid + i) * W + tx * C64_TW;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int pr = 8 * k + (lane >> 3), pc = lane & 7;
          const u32x4 v = *reinterpret_cast<const u32x4*>(strip + pr * C64_SP + pc * 16);
          if (XM == 3) {
            if (v[0] == 0x7fc07fc0u && v[3] == 0x12345678u)  // (never: keeps the staging alive)
              *reinterpret_cast<u32x4*>(out + (pix0 + pr) * p.out_stride + p.out_coff + pc * 8) = v;
          } else {
            *reinterpret_cast<u32x4*>(out + (pix0 + pr) * p.out_stride + p.out_coff + pc * 8) = v;
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 2 * !STG; ++i) {
      const int64_t pix = ((int64_t)img * H + ty * C64_TH + 2 * wid + i) * W + tx * C64_TW + rho;
      bf16_t* dst = out + pix * p.out_stride + p.out_coff + cb16;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          u32x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = pack2(acc[i][j][8 * h + 2 * e], acc[i][j][8 * h + 2 * e + 1]);
          *reinterpret_cast<u32x4*>(dst + 32 * j + 8 * h) = pk;
        }
    }
    // the next tile's halo was issued before this tile's stores: wait for it
    // only (2 statistics + 8 output stores may stay in flight)
    if (XM == 3)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (STATS && XM != 4)
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // 2 statistics + 8 output stores
    else
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    pp_barrier();  // (a __syncthreads() would drain the stores too)
    b ^= 1;
  }
}

int g_c64 = 2;  // VU_TUNE_FP8_C64: 2 (default) resident-weight kernel, staged stores; 1 direct stores; 0 off

// 64-channel chunks the resident-weight kernel walks per tile (1 or 2), 0 = not served
int c64_nch(const VuConvFp8& p) {
  const VuGather& g = p.a;
  if (!g_c64 || p.ncol != 64 || (g.C != 64 && g.C != 128)) return 0;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.cend[t] % 64) return 0;
  if (g.H % C64_TH != 0 || g.W % C64_TW != 0) return 0;
  const int64_t T = (int64_t)g.N * (g.H / C64_TH) * (g.W / C64_TW);
  if (T < 2 * (int64_t)cu_count()) return 0;  // a tile stream per block
  return g.C / 64;
}

bool c64_ok(const VuConvFp8& p) {
  const VuGather& g = p.a;
  if (!g_c64 || g.nsrc != 1 || g.C != 64 || g.cend[0] != 64 || p.ncol != 64) return false;
  if (g.H % C64_TH != 0 || g.W % C64_TW != 0) return false;
  const int64_t T = (int64_t)g.N * (g.H / C64_TH) * (g.W / C64_TW);
  return T >= 2 * (int64_t)cu_count();  // a tile stream per block
}

template <int BN>
bool tiles_ok(const VuConvFp8& p) {
  const VuGather& g = p.a;
  return p.ncol % BN == 0 && g.H % PP<BN>::TH == 0 && g.W % PP<BN>::TW == 0;
}

int pick_bn(const VuConvFp8& p) {
  if (tiles_ok<256>(p)) return 256;
  if (p.ncol % 256 != 0 && tiles_ok<128>(p)) return 128;
  if (p.ncol == 64 && tiles_ok<64>(p)) return 64;
  return 0;
}

bool served(const VuConvFp8& p) {
  const VuGather& g = p.a;
  if (g.R != 3 || g.S != 3 || g.sy != 1 || g.sx != 1 || g.dy != 1 || g.dx != 1 || g.oy != -1 || g.ox != -1 ||
      g.Hs != g.H || g.Ws != g.W || g.nsrc < 1 || g.nsrc > 3)
    return false;
  if (g.C % 64 != 0 || g.C < 64) return false;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.cend[t] % 64 != 0 || g.stride[t] % 16 != 0) return false;
  if (p.ldw % 16 != 0 || p.ldw < 9 * (int64_t)g.C || p.out_stride % 8 != 0 || p.out_coff % 8 != 0) return false;
  if (!p.x_scale || !p.w_scale || !p.out) return false;
  if ((int64_t)g.N * g.H * g.W >= (int64_t)1 << 31) return false;
  return pick_bn(p) != 0;
}

int g_pp = 1;  // VU_TUNE_FP8_PP: 1 (default) one tile per block on the ping-pong step loop, 0 persistent (A/B)

int g_split = 1;  // VU_TUNE_FP8_SPLIT: 1 (default) split-K for grids under one block per CU, 0 off

template <int BN>
int64_t bn_tiles(const VuConvFp8& p) {
  const VuGather& g = p.a;
  return (int64_t)g.N * (g.H / PP<BN>::TH) * (g.W / PP<BN>::TW) * (p.ncol / BN);
}

// split factor of the step-loop kernel: tiles < CUs -> ceil(CUs / tiles)
// chunk ranges of >= 8 chunks each (at batch 2 / 1024^2: down4.2, 1024
// channels, 129 -> 117 us; down4.1 with 512 would be 73 -> 87 us -- the slab
// round trip costs more than the idle half of the chip there)
int fp8_ksplit(const VuConvFp8& p) {
  if (!g_split || !g_pp || g_grid != 0 || c64_nch(p)) return 1;
  const int bn = pick_bn(p);
  const int64_t tiles = bn == 256 ? bn_tiles<256>(p) : bn == 128 ? bn_tiles<128>(p) : bn_tiles<64>(p);
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  if (tiles >= cu_count() || M % 128 != 0 || p.ncol % 64 != 0) return 1;
  int ks = (int)((cu_count() + tiles - 1) / tiles);
  const int maxks = p.a.C / 64 / 8;
  if (ks > maxks) ks = maxks;
  return ks < 2 ? 1 : ks;
}

template <int BN>
int launch(const VuConvFp8& p, hipStream_t st) {
  const VuGather& g = p.a;
  const int64_t tiles = bn_tiles<BN>(p);
  const int ks = fp8_ksplit(p);
  if (ks > 1) {
    if (!p.workspace) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((conv3x3_fp8_pp_kernel<BN, 0, true>), dim3((unsigned)(tiles * ks)), dim3(512), 0, st, p);
    VuGemmFwd q;
    memset(&q, 0, sizeof(q));
    q.a = g;
    q.ncol = p.ncol;
    q.out = p.out;
    q.out_stride = p.out_stride;
    q.out_coff = p.out_coff;
    q.bias = p.bias;
    q.stat_sum = p.stat_sum;
    q.stat_m2 = p.stat_m2;
    q.workspace = p.workspace;
    q.ksplit = ks;
    q.out_mode = 0;
    q.accumulate = 0;
    return splitk_finish_launch(q, st);
  }
  if (g_pp && g_grid == 0) {
    if (p.stat_min) {
      if (g_xm != 0) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((conv3x3_fp8_pp_kernel<BN, 0, false, true>), dim3((unsigned)tiles), dim3(512), 0, st, p);
      return (int)hipGetLastError();
    }
    if (g_xm == 1)
      hipLaunchKernelGGL((conv3x3_fp8_pp_kernel<BN, 1>), dim3((unsigned)tiles), dim3(512), 0, st, p);
    else if (g_xm == 2)
      hipLaunchKernelGGL((conv3x3_fp8_pp_kernel<BN, 2>), dim3((unsigned)tiles), dim3(512), 0, st, p);
    else
      hipLaunchKernelGGL((conv3x3_fp8_pp_kernel<BN>), dim3((unsigned)tiles), dim3(512), 0, st, p);
    return (int)hipGetLastError();
  }
  const int64_t cap = g_grid > 0 ? g_grid : cu_count();
  const int64_t nblk = tiles < cap ? tiles : cap;
  if (g_xm == 1)
    hipLaunchKernelGGL((conv3x3_fp8_kernel<BN, 1>), dim3((unsigned)nblk), dim3(512), 0, st, p);
  else if (g_xm == 2)
    hipLaunchKernelGGL((conv3x3_fp8_kernel<BN, 2>), dim3((unsigned)nblk), dim3(512), 0, st, p);
  else
    hipLaunchKernelGGL((conv3x3_fp8_kernel<BN>), dim3((unsigned)nblk), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

// ---- quantisation ------------------------------------------------------------
template <typename T>
__global__ void amax_kernel(const T* x, int64_t xs, int64_t P, int C, unsigned* out) {
  const int cv = C / 8;
  const int64_t n = P * cv;
  float m = 0.f;
  // four 16-byte vectors in flight per thread (clamped, unguarded loads; the
  // extra copies of the last vector leave the max unchanged)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e0 < n; e0 += 4 * stride) {
    Vec8<T> v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int64_t e = e0 + u * stride;
      e = e < n ? e : n - 1;
      const int64_t pix = e / cv;
      const int c8 = (int)(e - pix * cv) * 8;
      v[u].load(x + pix * xs + c8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(v[u].get(k)));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float sh[16];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r = fmaxf(r, sh[w]);
    atomicMax(out, __float_as_uint(r));  // non-negative floats order as their bits
  }
}

VU_DEV float qscale(float amax) { return amax > 0.f ? 448.f / amax : 1.f; }

// 4 floats -> 4 e4m3 bytes (round to nearest even; inputs pre-clamped)
VU_DEV uint32_t e4m3x4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

VU_DEV float clamp448(float v) { return fminf(fmaxf(v, -448.f), 448.f); }

template <typename T>
__global__ void quant_kernel(const T* x, int64_t xs, int64_t P, int C, const float* amax, uint8_t* y, int64_t ys,
                             float* dq) {
  const float s = qscale(*amax);
  if (dq && blockIdx.x == 0 && threadIdx.x == 0) *dq = 1.f / s;
  const int cv = C / 8;
  const int64_t n = P * cv;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = e / cv;
    const int c8 = (int)(e - pix * cv) * 8;
    Vec8<T> v;
    v.load(x + pix * xs + c8);
    float f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = clamp448(v.get(k) * s);
    u32x2 o;
    o[0] = e4m3x4(f[0], f[1], f[2], f[3]);
    o[1] = e4m3x4(f[4], f[5], f[6], f[7]);
    *reinterpret_cast<u32x2*>(y + pix * ys + c8) = o;
  }
}

__global__ void quant_rows_kernel(const float* x, int64_t cols, uint8_t* y, int64_t ldy, float* dq) {
  const float* xr = x + (int64_t)blockIdx.x * cols;
  float m = 0.f;
  for (int64_t k = threadIdx.x; k < cols; k += blockDim.x) m = fmaxf(m, fabsf(xr[k]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float sh[16];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  float am = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) am = fmaxf(am, sh[w]);
  const float s = qscale(am);
  if (threadIdx.x == 0) dq[blockIdx.x] = 1.f / s;
  uint8_t* yr = y + (int64_t)blockIdx.x * ldy;
  for (int64_t k = 4 * (int64_t)threadIdx.x; k < ldy; k += 4 * (int64_t)blockDim.x) {
    float f[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) f[u] = k + u < cols ? clamp448(xr[k + u] * s) : 0.f;
    *reinterpret_cast<uint32_t*>(yr + k) = e4m3x4(f[0], f[1], f[2], f[3]);
  }
}

int nblocks(int64_t n, int per) {
  const int64_t b = (n + per - 1) / per;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

// ---- BatchNorm apply (+ReLU) fused with e4m3 quantisation, delayed scaling --
// z = relu?(x * scale[c] + shift[c]) (two roundings, no FMA contraction, so
// the result is the unfused apply's fp32 value), q = e4m3(clamp(z * s)),
// s = 448 / ring[slot] -- the amax RECORDED BY THE PREVIOUS STEP -- while
// this step's max |z| is max-accumulated into ring[(slot+1)%3] for the next
// one, and ring[(slot+2)%3] (last step's scale slot, read by no one this
// step) is cleared for the step after.  One read of the bf16 conv output,
// one 1-byte write: the bf16 activation, its amax pass and its quantise pass
// of the three-launch path never touch HBM.  scale == nullptr: identity
// affine (quantise a bf16 activation with the delayed scale).
// CALIB: only max-accumulate max |z| into ring[slot] (first step: no
// history), nothing stored.
constexpr int Q8_UNR = 4;

template <typename T, bool CALIB>
__global__ __launch_bounds__(256) void bn_apply_q8_kernel(const T* x, int64_t xs, uint8_t* y, int64_t ys, int64_t P,
                                                          int C, const float* scale, const float* shift, int relu,
                                                          float* ring, int slot, float* dq) {
  const int V = C >> 3;
  const int R = 256 / V;
  const int c = (threadIdx.x & (V - 1)) * 8;
  const int row = threadIdx.x / V;
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = scale ? scale[c + i] : 1.f;
    sh[i] = scale ? shift[c + i] : 0.f;
  }
  float s = 1.f;
  if (!CALIB) {
    s = qscale(ring[slot]);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (dq) dq[0] = 1.f / s;
      ring[(slot + 2) % 3] = 0.f;
    }
  }
  float m = 0.f;
  const int64_t step = (int64_t)gridDim.x * R * Q8_UNR;
  for (int64_t p0 = (int64_t)blockIdx.x * R * Q8_UNR + row; p0 < P; p0 += step) {
    Vec8<T> v[Q8_UNR];
#pragma unroll
    for (int u = 0; u < Q8_UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * R;
      if (p < P) v[u].load(x + p * xs + c);
    }
#pragma unroll
    for (int u = 0; u < Q8_UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * R;
      if (p >= P) continue;
      float f[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        // z = x * scale + shift with two roundings: hipcc contracts a*b+c into
        // an FMA (through __fmul_rn and the fp-contract pragma alike), which
        // moved max|z| by an ulp against the two-op restatement; the empty asm
        // makes the product opaque
        float z = v[u].get(i);
        if (scale) {
          float pr = z * sc[i];
          asm volatile("" : "+v"(pr));
          z = pr + sh[i];
        }
        if (relu) z = fmaxf(z, 0.f);
        m = fmaxf(m, fabsf(z));
        f[i] = clamp448(z * s);
      }
      if (!CALIB) {
        u32x2 o;
        o[0] = e4m3x4(f[0], f[1], f[2], f[3]);
        o[1] = e4m3x4(f[4], f[5], f[6], f[7]);
        *reinterpret_cast<u32x2*>(y + p * ys + c) = o;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float shm[4];
  if ((threadIdx.x & 63) == 0) shm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float r = fmaxf(fmaxf(shm[0], shm[1]), fmaxf(shm[2], shm[3]));
    atomicMax(reinterpret_cast<unsigned*>(ring + (CALIB ? slot : (slot + 1) % 3)), __float_as_uint(r));
  }
}

// max |z| over the pixels of z = relu?(y * scale[c] + shift[c]) from the
// per-tile per-channel min / max of y: the affine map is monotone per channel,
// so the extreme z of a channel is at its min or max y -- computed with the
// two roundings of bn_apply_q8_kernel (the product made opaque), i.e. exactly
// the max |z| that kernel's calibration pass measures over every element.
// Order-independent (integer max of non-negative float bits): deterministic.
__global__ __launch_bounds__(256) void relu_amax_kernel(const float* pmin, const float* pmax, int64_t n, int C,
                                                        const float* scale, const float* shift, int relu,
                                                        unsigned* out) {
  // four consecutive channels per step (C % 4 == 0, host-checked): 16-byte loads
  float m = 0.f;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int c0 = (int)((i << 2) % C);
    const f32x4 lo = reinterpret_cast<const f32x4*>(pmin)[i], hi = reinterpret_cast<const f32x4*>(pmax)[i];
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
    if (scale) {
      sc = *reinterpret_cast<const f32x4*>(scale + c0);
      sh = *reinterpret_cast<const f32x4*>(shift + c0);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float z = k < 4 ? lo[k] : hi[k - 4];
      if (scale) {
        float pr = z * sc[k & 3];
        asm volatile("" : "+v"(pr));
        z = pr + sh[k & 3];
      }
      if (relu) z = fmaxf(z, 0.f);
      m = fmaxf(m, fabsf(z));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float shm[4];
  if ((threadIdx.x & 63) == 0) shm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(fmaxf(fmaxf(shm[0], shm[1]), fmaxf(shm[2], shm[3]))));
}

}  // namespace

int conv_fp8_tune(int key, int value) {
  if (key == VU_TUNE_FP8_SPLIT) {
    g_split = value != 0;
    return 0;
  }
  if (key == VU_TUNE_FP8_GRID) {
    g_grid = value;
    return 0;
  }
  if (key == VU_TUNE_FP8_XM) {
    g_xm = value;
    return 0;
  }
  if (key == VU_TUNE_FP8_PP) {
    g_pp = value != 0;
    return 0;
  }
  if (key == VU_TUNE_FP8_C64) {
    g_c64 = value < 0 ? 0 : value;
    return 0;
  }
  return -1;
}

extern "C" int64_t vu_conv3x3_fp8_row_tile(const VuConvFp8* args) {
  if (!served(*args)) return 0;
  return c64_nch(*args) ? 64 : 128;
}

extern "C" int64_t vu_conv3x3_fp8_workspace_bytes(const VuConvFp8* args) {
  if (!served(*args)) return 0;
  const int ks = fp8_ksplit(*args);
  return ks > 1 ? (int64_t)ks * args->a.N * args->a.H * args->a.W * args->ncol * (int64_t)sizeof(float) : 0;
}

// 1 when the kernel that serves *args emits VuConvFp8.stat_min / stat_max:
// the step-loop kernel (one tile per block, no split-K) and the 64-channel
// resident-weight kernels; not the persistent (VU_TUNE_FP8_PP 0 / capped grid)
// or split-K paths, nor experiment modes
extern "C" int vu_conv3x3_fp8_minmax_ok(const VuConvFp8* args) {
  if (!served(*args) || g_xm != 0) return 0;
  if (c64_nch(*args) == 2) return 1;
  if (c64_ok(*args)) return 1;
  return (g_pp && g_grid == 0 && fp8_ksplit(*args) <= 1) ? 1 : 0;
}

extern "C" int vu_conv3x3_fp8(const VuConvFp8* args, void* stream) {
  if (!served(*args)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (args->stat_min && !vu_conv3x3_fp8_minmax_ok(args)) return (int)hipErrorInvalidValue;
  if (c64_nch(*args) == 2) {
    const VuGather& g = args->a;
    const int64_t T = (int64_t)g.N * (g.H / C64_TH) * (g.W / C64_TW);
    const int64_t grid = T < cu_count() ? T : cu_count();
    if (args->stat_min) {
      if (args->stat_sum)
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, false, 0, 2, true>), dim3((unsigned)grid), dim3(512), 0, st,
                           *args);
      else
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<false, false, 0, 2, true>), dim3((unsigned)grid), dim3(512), 0, st,
                           *args);
      return (int)hipGetLastError();
    }
    if (args->stat_sum)
      hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, false, 0, 2>), dim3((unsigned)grid), dim3(512), 0, st, *args);
    else
      hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<false, false, 0, 2>), dim3((unsigned)grid), dim3(512), 0, st, *args);
    return (int)hipGetLastError();
  }
  if (c64_ok(*args)) {
    const VuGather& g = args->a;
    const int64_t T = (int64_t)g.N * (g.H / C64_TH) * (g.W / C64_TW);
    const int64_t grid = T < cu_count() ? T : cu_count();
    if (g_xm >= 1 && g_xm <= 4 && args->stat_sum) {
      if (g_xm == 4)
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, true, 4>), dim3((unsigned)grid), dim3(512), 0, st, *args);
      else if (g_xm == 1)
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, true, 1>), dim3((unsigned)grid), dim3(512), 0, st, *args);
      else if (g_xm == 2)
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, true, 2>), dim3((unsigned)grid), dim3(512), 0, st, *args);
      else
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, true, 3>), dim3((unsigned)grid), dim3(512), 0, st, *args);
      return (int)hipGetLastError();
    }
    if (args->stat_min) {  // (the staging-strip variant, g_c64 >= 2, has no min / max epilogue)
      if (args->stat_sum)
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, false, 0, 1, true>), dim3((unsigned)grid), dim3(512), 0, st,
                           *args);
      else
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<false, false, 0, 1, true>), dim3((unsigned)grid), dim3(512), 0, st,
                           *args);
      return (int)hipGetLastError();
    }
    if (g_c64 >= 2) {
      if (args->stat_sum)
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, true>), dim3((unsigned)grid), dim3(512), 0, st, *args);
      else
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<false, true>), dim3((unsigned)grid), dim3(512), 0, st, *args);
    } else {
      if (args->stat_sum)
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<true, false>), dim3((unsigned)grid), dim3(512), 0, st, *args);
      else
        hipLaunchKernelGGL((conv3x3_fp8_c64_kernel<false, false>), dim3((unsigned)grid), dim3(512), 0, st, *args);
    }
    return (int)hipGetLastError();
  }
  switch (pick_bn(*args)) {
    case 256: return launch<256>(*args, st);
    case 128: return launch<128>(*args, st);
    default: return launch<64>(*args, st);
  }
}

extern "C" int vu_fp8_relu_amax(const float* pmin, const float* pmax, int64_t rows, int C, const float* scale,
                                const float* shift, int relu, float* amax, void* stream) {
  if (C <= 0 || C % 4 != 0 || rows < 0 || !pmin || !pmax || !amax || (scale && !shift))
    return (int)hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(pmin) | reinterpret_cast<uintptr_t>(pmax) | reinterpret_cast<uintptr_t>(scale) |
       reinterpret_cast<uintptr_t>(shift)) % 16 != 0)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(amax, 0, sizeof(float), st);
  if (e != hipSuccess) return (int)e;
  const int64_t n = rows * (int64_t)C;
  if (n == 0) return 0;
  const int nb = nblocks(n / 4, 256 * 8);
  hipLaunchKernelGGL(relu_amax_kernel, dim3(nb), dim3(256), 0, st, pmin, pmax, n, C, scale, shift, relu,
                     (unsigned*)amax);
  VU_CHECK_LAUNCH();
}

extern "C" int vu_amax(const void* x, int64_t xs, int64_t P, int C, float* amax, int accumulate, int dtype,
                       void* stream) {
  if (C % 8 != 0 || xs % 8 != 0 || P < 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (!accumulate) {
    hipError_t e = hipMemsetAsync(amax, 0, sizeof(float), st);
    if (e != hipSuccess) return (int)e;
  }
  if (P == 0) return 0;
  int nb = nblocks(P * (C / 8), 256 * 8);
  if (nb > 1024) nb = 1024;  // one atomic max per block on one word (see vu_bn_apply_fp8)
  if (dtype == VU_BF16)
    hipLaunchKernelGGL(amax_kernel<bf16_t>, dim3(nb), dim3(256), 0, st, (const bf16_t*)x, xs, P, C, (unsigned*)amax);
  else
    hipLaunchKernelGGL(amax_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)x, xs, P, C, (unsigned*)amax);
  VU_CHECK_LAUNCH();
}

extern "C" int vu_quant_fp8(const void* x, int64_t xs, int64_t P, int C, const float* amax, uint8_t* y, int64_t ys,
                            float* dq, int dtype, void* stream) {
  if (C % 8 != 0 || xs % 8 != 0 || ys % 8 != 0 || P < 0) return (int)hipErrorInvalidValue;
  if (P == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int nb = nblocks(P * (C / 8), 256 * 4);
  if (dtype == VU_BF16)
    hipLaunchKernelGGL(quant_kernel<bf16_t>, dim3(nb), dim3(256), 0, st, (const bf16_t*)x, xs, P, C, amax, y, ys, dq);
  else
    hipLaunchKernelGGL(quant_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)x, xs, P, C, amax, y, ys, dq);
  VU_CHECK_LAUNCH();
}

extern "C" int vu_bn_apply_fp8(const void* x, int64_t xs, uint8_t* y, int64_t ys, int64_t P, int C,
                               const float* scale, const float* shift, int relu, float* amax_ring, int slot,
                               int calibrate, float* dq, int dtype, void* stream) {
  const int V = C / 8;
  if (C % 8 != 0 || V < 1 || V > 256 || (V & (V - 1)) != 0 || xs % 8 != 0 || P < 0 || slot < 0 || slot > 2 ||
      !amax_ring || (!calibrate && (ys % 8 != 0 || !y)) || (scale && !shift) || (dtype != VU_BF16 && dtype != VU_F32))
    return (int)hipErrorInvalidValue;
  if (P == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int64_t R = 256 / V;
  int64_t g = (P + R * 16 - 1) / (R * 16);          // ~16 pixel rows per thread
  const int64_t g1 = (P + R * Q8_UNR - 1) / (R * Q8_UNR);
  if (g < 256) g = g1 < 256 ? g1 : 256;               // small tensors: >= one CU sweep
  // at most 1024 blocks: each block ends with ONE atomic max on the same ring
  // word, and atomics to one address serialise at the memory side (~12 ns
  // each): 4096 blocks made a 268 MB calibration pass run at 3.3 TB/s (round 6)
  if (g > 1024) g = 1024;
  const dim3 grid((unsigned)g);
#define VU_Q8_LAUNCH(T, CAL)                                                                                  \
  hipLaunchKernelGGL((bn_apply_q8_kernel<T, CAL>), grid, dim3(256), 0, st, (const T*)x, xs, y, ys, P, C, scale, \
                     shift, relu, amax_ring, slot, dq)
  if (dtype == VU_BF16) {
    if (calibrate) VU_Q8_LAUNCH(bf16_t, true); else VU_Q8_LAUNCH(bf16_t, false);
  } else {
    if (calibrate) VU_Q8_LAUNCH(float, true); else VU_Q8_LAUNCH(float, false);
  }
#undef VU_Q8_LAUNCH
  VU_CHECK_LAUNCH();
}

extern "C" int vu_quant_rows_fp8(const float* x, int rows, int64_t cols, uint8_t* y, int64_t ldy, float* dq,
                                 void* stream) {
  if (rows < 0 || cols < 0 || ldy < cols || ldy % 4 != 0) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(quant_rows_kernel, dim3(rows), dim3(256), 0, (hipStream_t)stream, x, cols, y, ldy, dq);
  VU_CHECK_LAUNCH();
}
