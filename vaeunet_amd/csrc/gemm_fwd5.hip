// 3x3 / stride-1 / pad-1 convolution, PERSISTENT ping-pong variant ("v5",
// bf16) for the narrow DoubleConv layers (input channels <= 128 by default:
// unet_parts.py:40,43 at the 512^2 / 256^2 levels and their input-gradient
// convs).
//
// Same wave program as v4 (gemm_fwd4.hip: halo-tiled implicit GEMM, waves
// 0-3 / 4-7 one barrier apart, weights and halo streamed by LDS-DMA with the
// two streams split between the halves), but one block per CU walks the
// tiles lb, lb+G, lb+2G, ... and the pipeline never drains between them:
// during the last chunk of a tile, half 1 already streams chunk 0 of the
// block's next tile and half 0 keeps the weight ring two steps ahead across
// the tile boundary.  With K = 9*64 or 9*128 a tile is only 18-36 K-steps,
// so v4's per-block prologue (first halo + weights from HBM) and drain cost
// 15-30 % of the layer; here they are paid once per CU.
//
// The epilogue therefore cannot use LDS (the next tile's halo and weights
// are in flight in it) and runs from registers.  To make that cheap the
// weight rows are read in a permuted order: fragment j of a wave reads the
// LDS rows of channels 16*(r>>2) + 4*j + (r&3) (r = A-operand row), so each
// lane ends up with 16 CONSECUTIVE output channels of one pixel -- two
// 16-byte NHWC stores per fragment row -- and the BatchNorm partials of a
// channel live in one 16-lane DPP row (row_ror reductions, no LDS, no
// cross-row shuffles).
#include "common.h"
#include "../../include/vaeunet.h"

static __device__ __attribute__((aligned(16))) uint32_t vu_zero_page5[16];

namespace {

typedef __attribute__((address_space(3))) void lds_void;

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

// sum over the 16 lanes of a DPP row (every lane receives the total)
template <int R>
VU_DEV float ror_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false));
}
VU_DEV float row16_sum(float v) { return ror_add<1>(ror_add<2>(ror_add<4>(ror_add<8>(v)))); }

VU_DEV uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

int g_max_c = 0;        // VU_TUNE_V5_MAX_C (0 = off: measured no net gain over v4)
int g_min_tiles = -1;   // VU_TUNE_V5_MIN_TILES; -1 = 2 x CU count
int g_grid = 0;         // VU_TUNE_V5_GRID: grid cap (tests); 0 = CU count

template <int BN>
__global__ __launch_bounds__(512, 1) void conv3x3_pers_kernel(VuGemmFwd p) {
  constexpr int WM = PP<BN>::WM, WN = PP<BN>::WN, TH = PP<BN>::TH, TW = PP<BN>::TW;
  constexpr int BM = TH * TW;
  static_assert(BM == WM * 128 && BN == WN * 64 && WM * WN == 8, "wave grid");
  constexpr int HW = TW + 2, HP = (TH + 2) * HW;
  constexpr int HPIECES = HP * 4;                 // 16-byte pieces per chunk halo
  constexpr int NHP1 = (HPIECES + 255) / 256;     // halo DMA slots per half-1 thread
  constexpr int HALO = HP * 64;
  constexpr int WPIECES = BN * 4;
  constexpr int LB0 = WPIECES / 256;              // weight DMA slots per half-0 thread
  constexpr int LB0A = (LB0 + 1) / 2;             // ... issued in phase 1 (rest in phase 2)
  constexpr int WSLOT = BN * 64;
  constexpr int NBW = 3;                          // weight ring (prefetch distance 2)
  constexpr int PPS1 = (NHP1 + 7) / 8;            // halo slots issued per step (steps 0..7)
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
  const int lb = xcd_remap(blockIdx.x, G);        // logical block: tiles lb, lb+G, ...
  const int ntl = (T - lb + G - 1) / G;           // tiles of this block (>= 1)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int grp = wid >> 2;  // ping-pong half (one wave of each half per SIMD)
  const int nchunk = g.C / 32;
  const int nk = nchunk * 9;
  const int S = ntl * nk;                         // steps of the whole launch

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

  // ---- DMA roles (see gemm_fwd4.hip): half 0 streams weights, half 1 halos --
  const int gt = tid & 255;
  const int gw = wid & 3;
  const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
  const void* zp = (const void*)vu_zero_page5;
  char* const hbuf = smem;
  char* const wbuf = smem + 2 * HALO;

  const bf16_t* const src0 = reinterpret_cast<const bf16_t*>(g.src[0]);
  const bf16_t* const src1 = reinterpret_cast<const bf16_t*>(g.src[1]);
  const bf16_t* const src2 = reinterpret_cast<const bf16_t*>(g.src[2]);
  const int64_t st0 = g.stride[0], st1 = g.stride[1], st2 = g.stride[2];
  const int ce0 = g.cend[0], ce1 = g.nsrc > 2 ? g.cend[1] : (1 << 30);
  struct HaloT { const bf16_t* src; int64_t st; char* hb; int img, y0, x0; };
  auto halo_target = [&](int i, int c) -> HaloT {
    const Tile q = tile_of(i);
    const int cb = c * 32;
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
      if (k * 256 + gw * 64 >= HPIECES) continue;  // wave-uniform
      const int P = k * 256 + gt;
      if (P < HPIECES) {
        const int px = P >> 2;
        const int hy = px / HW, hx = px - (px / HW) * HW;
        const int y = h.y0 - 1 + hy, x = h.x0 - 1 + hx;
        const void* gp = zp;
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          gp = h.src + ((int64_t)(h.img * H + y) * W + x) * h.st + (P & 3) * 8;
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
    const int kb = t * g.C + c * 32;
    char* B = wbuf + (wgs_ % NBW) * WSLOT;
#pragma unroll
    for (int k = 0; k < LB0; ++k) {
      if (k < k0 || k >= k1) continue;
      const int P = k * 256 + gt;
      const void* gp = bmat + (int64_t)(n0w_ + (P >> 2)) * p.ldb + kb + (P & 3) * 8;
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(B + (k * 256 + gw * 64) * 16), 16, 0, 0);
    }
  };

  // ---- fragment addressing -------------------------------------------------
  int arow[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = wm * 128 + i * 16 + (lane & 15);
    const int ty = m / TW, tx = m - (m / TW) * TW;
    arow[i] = (ty * HW + tx) * 64 + (lane >> 4) * 16;
  }
  // permuted weight rows: fragment j, A-row r -> channel 16*(r>>2) + 4*j + (r&3)
  const int brow = (wn * 64 + 16 * ((lane & 15) >> 2) + (lane & 3)) * 64 + (lane >> 4) * 16;
  // acc[i][j][r]: pixel wm*128 + i*16 + (lane&15), channel cb16 + 4*j + r
  const int cb16 = wn * 64 + 16 * (lane >> 4);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  bf16_t* const out = reinterpret_cast<bf16_t*>(p.out);
  auto epilogue = [&](int ti) {
    const Tile q = tile_of(ti);
    const int c0 = q.n0 + cb16;
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float bv = p.bias[c0 + 4 * j + r];
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i][j][r] += bv;
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = rnd<bf16_t>(acc[i][j][r]);
    if (p.stat_sum) {
      // per-wave statistics tile: 128 pixels (8 fragments x one DPP row)
      float* ss = p.stat_sum + (int64_t)(q.mt * WM + wm) * p.ncol + c0;
      float* sq = p.stat_m2 + (int64_t)(q.mt * WM + wm) * p.ncol + c0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 sm, m2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) s += acc[i][j][r];
          s = row16_sum(s);
          const float mean = s * (1.f / 128);
          float v = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float d = acc[i][j][r] - mean;
            v += d * d;
          }
          sm[r] = s;
          m2[r] = row16_sum(v);
        }
        if ((lane & 15) == 0) {
          *reinterpret_cast<f32x4*>(ss + 4 * j) = sm;
          *reinterpret_cast<f32x4*>(sq + 4 * j) = m2;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = wm * 128 + i * 16 + (lane & 15);
      const int ty = m / TW, tx = m - (m / TW) * TW;
      const int64_t pix = ((int64_t)q.img * H + q.y0 + ty) * W + q.x0 + tx;
      bf16_t* dst = out + pix * p.out_stride + p.out_coff + c0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 a = acc[i][2 * h], b = acc[i][2 * h + 1];
        if (p.accumulate) {
          const u32x4 o = *reinterpret_cast<const u32x4*>(dst + 8 * h);
          a[0] += __uint_as_float(o[0] << 16);
          a[1] += __uint_as_float(o[0] & 0xffff0000u);
          a[2] += __uint_as_float(o[1] << 16);
          a[3] += __uint_as_float(o[1] & 0xffff0000u);
          b[0] += __uint_as_float(o[2] << 16);
          b[1] += __uint_as_float(o[2] & 0xffff0000u);
          b[2] += __uint_as_float(o[3] << 16);
          b[3] += __uint_as_float(o[3] & 0xffff0000u);
        }
        u32x4 pk;
        pk[0] = pack2(a[0], a[1]);
        pk[1] = pack2(a[2], a[3]);
        pk[2] = pack2(b[0], b[1]);
        pk[3] = pack2(b[2], b[3]);
        *reinterpret_cast<u32x4*>(dst + 8 * h) = pk;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  };

  // ---- prologue: halo of (tile 0, chunk 0), weights of steps 0 and 1 --------
  HaloT hn;
  if (grp) {
    halo_issue(halo_target(0, 0), -1);
  } else {
    wstage(0, LB0);
    wnext();
    if (S > 1) wstage(0, LB0);
    wnext();  // (wi_, ws_) = step 2
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  if (grp) pp_barrier();  // the stagger: half 1 runs one barrier behind

  int ti = 0, s = 0;
  for (int gs = 0; gs < S; ++gs) {
    const int c = s / 9, t = s - (s / 9) * 9;
    const char* A = hbuf + ((ti * nchunk + c) & 1) * HALO + ((t / 3) * HW + (t - (t / 3) * 3)) * 64;
    const char* Bw = wbuf + (gs % NBW) * WSLOT;
    u32x4 bf[4], af[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const u32x4*>(Bw + brow + j * 4 * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const u32x4*>(A + arow[i]);
    if (!grp && gs + 2 < S) wstage(0, LB0A);
    pp_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                            __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const u32x4*>(A + arow[4 + i]);
    if (!grp) {
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
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                                __builtin_bit_cast(bf16x8, af[i]), acc[4 + i][j], 0, 0,
                                                                0);
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
    if (++s == nk) {
      epilogue(ti);
      s = 0;
      ++ti;
    }
  }
  if (!grp) pp_barrier();  // re-align the halves
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BN>
int launch(const VuGemmFwd& p, hipStream_t st) {
  const VuGather& g = p.a;
  const int64_t mt = (int64_t)g.N * (g.H / PP<BN>::TH) * (g.W / PP<BN>::TW);
  const int64_t tiles = mt * (p.ncol / BN);
  const int64_t cap = g_grid > 0 ? g_grid : cu_count();
  const int64_t nblk = tiles < cap ? tiles : cap;  // one block per CU
  hipLaunchKernelGGL((conv3x3_pers_kernel<BN>), dim3((unsigned)nblk), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

template <int BN>
bool tiles_ok(const VuGemmFwd& p) {
  const VuGather& g = p.a;
  return p.ncol % BN == 0 && g.H % PP<BN>::TH == 0 && g.W % PP<BN>::TW == 0;
}

// Output-column tile for this problem (0 = not served): by default every CU
// gets at least two tiles, otherwise persistence buys nothing over v4.
int pick_bn(const VuGemmFwd& p) {
  const VuGather& g = p.a;
  if (g.C > g_max_c) return 0;
  const int64_t pix = (int64_t)g.N * g.H * g.W;
  const int64_t need = g_min_tiles >= 0 ? g_min_tiles : 2 * (int64_t)cu_count();
  if (tiles_ok<256>(p) && (pix / 256) * (p.ncol / 256) >= need) return 256;
  if (p.ncol % 256 != 0 && tiles_ok<128>(p) && (pix / 512) * (p.ncol / 128) >= need) return 128;
  if (p.ncol == 64 && tiles_ok<64>(p) && pix / 1024 >= need) return 64;
  return 0;
}

}  // namespace

// Row tile of the BatchNorm partials (128: one per wave tile) when v5 serves
// this problem, else 0.  Same operand contract as gemm_fwd_v4_bm.
int gemm_fwd_v5_bm(const VuGemmFwd& p, int dtype) {
  const VuGather& g = p.a;
  if (dtype != VU_BF16 || p.out_mode != 0) return 0;
  if (g.R != 3 || g.S != 3 || g.sy != 1 || g.sx != 1 || g.dy != 1 || g.dx != 1 || g.oy != -1 ||
      g.ox != -1 || g.Hs != g.H || g.Ws != g.W)
    return 0;
  if (g.C % 32 != 0) return 0;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.cend[t] % 32 != 0 || g.stride[t] % 8 != 0) return 0;
  if (p.out_stride % 8 != 0 || p.out_coff % 8 != 0 || p.ldb % 8 != 0) return 0;
  if ((int64_t)g.N * g.H * g.W >= (int64_t)1 << 31) return 0;
  return pick_bn(p) ? 128 : 0;
}

int gemm_fwd_v5_launch(const VuGemmFwd& p, hipStream_t st) {
  switch (pick_bn(p)) {
    case 256: return launch<256>(p, st);
    case 128: return launch<128>(p, st);
    case 64: return launch<64>(p, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// vu_gemm_set_tuning keys owned by v5 (gemm_fwd4.hip forwards them); 0 if handled
int gemm_fwd_v5_tune(int key, int value) {
  switch (key) {
    case VU_TUNE_V5_MAX_C: g_max_c = value; return 0;
    case VU_TUNE_V5_MIN_TILES: g_min_tiles = value; return 0;
    case VU_TUNE_V5_GRID: g_grid = value; return 0;
    default: return -1;
  }
}
