// 3x3 / stride-1 / pad-1 convolution WEIGHT gradient over halo tiles ("v3",
// bf16): slab[s][co][tap*C + ci] = sum_{pixels p of split s} dy[p][co] *
// x[p + tap][ci].  Serves every DoubleConv / DecoderBlock 3x3 conv weight
// gradient of the hot path (unet_parts.py:40,43) and of the ResNet34 encoder
// (unet_resnet.py:131-137) whose image width is a multiple of 16.
//
// Why: the v2 kernel treats the nine taps as nine independent K columns and
// gathers the shifted input separately for each, so every x pixel crosses
// L2 -> LDS nine times (and dy once per column tile).  Here a block owns
// (BI output channels) x (all 9 taps) x (one 64-channel input chunk) and
// walks 4x32-pixel tiles of its pixel split; per tile it DMA-loads dy once
// and the 6x34 x halo once, and all nine taps read the halo in place.
//
//   * 8 waves, 16x16x32 bf16 MFMA, both operands read with the transposed
//     ds_read_b64_tr_b16 (pixels are the reduction dim);
//   * halo rows are laid out with a 48-pixel pitch (34 used) so that a tap
//     shift of r rows moves the address by a multiple of 16 rows: the 32-byte
//     block swizzle (a function of the row's low 4 bits) is then unchanged and
//     every tap / k-step offset is a compile-time immediate of the LDS read;
//   * operands land by LDS-DMA with the swizzle applied to the SOURCE column,
//     double-buffered per pixel tile; fp32 accumulators stay in registers
//     across the split, then one slab write (vu_slab_reduce sums the splits in
//     a fixed order: deterministic).
#include "common.h"
#include "../../include/vaeunet.h"

static __device__ __attribute__((aligned(16))) uint32_t vu_zero_page_w3[16];

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// pixel tile: 128 pixels = 4 x 32, or 8 x 16 for 16-pixel-wide images (the
// ResNet34 encoder's 16^2 level); the halo row pitch (TW + 2 used) is a
// multiple of 16 rows so that a tap / tile-row shift keeps the swizzle
constexpr int TP = 128;
template <int TW> struct WT {
  static constexpr int TH = TP / TW, HWP = TW == 32 ? 48 : 32, HROWS = TH + 2;
};

template <int RB> VU_DEV int fsw(int m) {
  return RB >= 256 ? ((m & 3) | ((m >> 1) & 4)) : (((m >> 1) & 1) | ((m >> 2) & 2));
}
template <int RB> VU_DEV int tr_off(int m, int col) {
  return m * RB + (((col >> 4) ^ fsw<RB>(m)) << 5) + ((col & 15) << 1);
}
// logical column of the 16-byte physical chunk pc of row m (source-side swizzle)
template <int RB> VU_DEV int swz_col(int m, int pc) {
  return ((((pc >> 1) ^ fsw<RB>(m)) << 1) | (pc & 1)) * 8;
}

// Transposed LDS reads as inline asm: through the builtin the compiler cannot
// tell them from the next tile's LDS-DMA destinations and inserts an
// s_waitcnt vmcnt(0) before the first read of a tile -- right after that
// tile's successor was issued -- which serialises DMA and MFMA (the double
// buffer never overlapped).  Ordering is explicit instead: vmcnt + barrier
// for DMA -> reads, lgkm_wait() + tie() for reads -> MFMAs.
VU_DEV u32x2 tr_read(const char* p) {
  u32x2 r;
  const uint32_t a = (uint32_t)(uintptr_t)(const lds_void*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

VU_DEV u32x4 tr_frag(const char* base, int off_lo, int off_hi) {
  u32x2 l2 = tr_read(base + off_lo), h2 = tr_read(base + off_hi);
  return u32x4{l2[0], l2[1], h2[0], h2[1]};
}

// The same read from a per-lane LDS byte address held in a VGPR plus a
// compile-time byte offset in the instruction's 16-bit offset field: the
// tap / k-step shifts of a tile cost no address arithmetic (off folds to a
// constant once the group loop is unrolled).
VU_DEV u32x2 tr_read_o(uint32_t a, const int off) {
  u32x2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(off));
  return r;
}
VU_DEV u32x4 tr_frag_o(uint32_t lo, uint32_t hi, const int off) {
  u32x2 l2 = tr_read_o(lo, off), h2 = tr_read_o(hi, off);
  return u32x4{l2[0], l2[1], h2[0], h2[1]};
}
VU_DEV u32x4 tr_frag_o2(uint32_t a, const int off_lo, const int off_hi) {
  u32x2 l2 = tr_read_o(a, off_lo), h2 = tr_read_o(a, off_hi);
  return u32x4{l2[0], l2[1], h2[0], h2[1]};
}
VU_DEV uint32_t lds_addr(const char* p) { return (uint32_t)(uintptr_t)(const lds_void*)p; }

// at most n LDS operations outstanding (n folds to a constant after unrolling)
VU_DEV void lgkm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt lgkmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt lgkmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory"); break;
    default: asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory"); break;
  }
}
VU_DEV void tie(u32x4& v) { asm volatile("" : "+v"(v)); }

// FAST (round 4, the default): per tile, the fragment-read base addresses of
// the tile's LDS stage are formed once (14 VGPRs) and every (k-step, tap)
// read uses the instruction offset field; the tile walk advances its
// (image, row, column) counters instead of dividing; interior tiles (halo
// inside the image) take precomputed 32-bit per-lane halo offsets with no
// bounds test.  The round-3 loop formed every read address with a VALU add
// and recomputed the DMA addresses per tile: ~190 VALU + ~110 SALU per
// 144-MFMA tile per wave (1.3 VALU per MFMA at BI = 128, 2.6 at BI = 64;
// profiles/r3e_sq_timing_unet.txt).
template <int BI, int TJ, int TW, int FASTM>
__global__ __launch_bounds__(512, 1) void wgrad3x3_halo_kernel(VuGemmWgrad p) {
  constexpr bool FAST = FASTM != 0, PRIO = FASTM != 2;   // FASTM 2: no s_setprio around the MFMA groups
  constexpr int TH = WT<TW>::TH, HWP = WT<TW>::HWP, HROWS = WT<TW>::HROWS;
  constexpr int NT = 512;
  constexpr int RBP = BI * 2, CPI = BI / 8;
  constexpr int LP = TP * CPI / NT;                       // dy DMA instrs per thread per tile
  constexpr int NH = (HROWS * HWP * 8 + NT - 1) / NT;     // halo DMA instrs per thread per tile
  constexpr int PB = TP * RBP, QB = NH * NT * 16;
  constexpr int STAGE = PB + QB;
  // TJ = 1: a wave owns 4 (BI=128) or 2 (BI=64) co tiles x one 16-channel ci tile,
  // the fewest transposed LDS reads per MFMA (A fragments reused over 9 taps)
  constexpr int WCI = 4 / TJ;                             // waves along ci (TJ ci tiles per wave)
  constexpr int TI = BI / 16 / (8 / WCI);                 // co tiles per wave
  static_assert(LP >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const VuGather& gp = p.p;   // dy, 1x1
  const VuGather& gq = p.q;   // x, 3x3 halo
  const int H = gq.H, W = gq.W;
  const int tiles_w = W / TW, tiles_img = (H / TH) * tiles_w;
  const int T = gq.N * tiles_img;
  const int itiles = (p.ni + BI - 1) / BI, jch = gq.C / 64;
  const int ntile = itiles * jch;
  const int bid = xcd_remap(blockIdx.x, ntile * p.splits);
  const int split = bid / ntile, tile = bid - split * ntile;
  const int it = tile / jch, jc = tile - it * jch;
  const int i0 = it * BI;
  const int tps = (int)(p.m_per_split / TP);
  const int t_beg = split * tps;
  const int t_end = t_beg + tps < T ? t_beg + tps : T;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const void* zp = (const void*)vu_zero_page_w3;

  // source of this block's 64-channel x chunk
  const int cb = jc * 64;
  const int qs = (cb >= gq.cend[0]) + (gq.nsrc > 2 && cb >= gq.cend[1]);
  const bf16_t* xsrc = reinterpret_cast<const bf16_t*>(gq.src[qs]) + (cb - (qs == 0 ? 0 : gq.cend[qs - 1]));
  const int64_t xst = gq.stride[qs];
  const bf16_t* dsrc = reinterpret_cast<const bf16_t*>(gp.src[0]);
  const int64_t dst_ = gp.stride[0];

  // fixed per-thread DMA slots, one register each (the accumulators leave
  // little room): dy slot = element offset from the tile's first pixel (-1:
  // channel past ni, zero page); halo slot = hy | hx << 4 | col << 10 (-1:
  // pitch padding / past the last row, no load)
  int p_off[LP];
#pragma unroll
  for (int k = 0; k < LP; ++k) {
    int e = k * NT + tid, row = e / CPI, pc = e - row * CPI;
    const int ty = row / TW, tx = row - ty * TW, col = i0 + swz_col<RBP>(row, pc);
    p_off[k] = col < p.ni ? (int)((int64_t)(ty * W + tx) * dst_ + col) : -1;
  }
  int q_pk[NH];
#pragma unroll
  for (int k = 0; k < NH; ++k) {
    int e = k * NT + tid, hp = e >> 3, pc = e & 7;
    const int hy = hp / HWP, hx = hp - hy * HWP;
    q_pk[k] = (hy < HROWS && hx < TW + 2) ? (hy | hx << 4 | swz_col<128>(hp, pc) << 10) : -1;
  }

  // FAST: 32-bit offset of each halo slot's source element from the tile's
  // first pixel (interior tiles), INT32_MIN for a slot that loads nothing;
  // border tiles re-derive the slot geometry from the thread id
  int q_rel[FAST ? NH : 1];
  if constexpr (FAST) {
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int q = q_pk[k];
      q_rel[k] = q >= 0 ? (int)((int64_t)(((q & 15) - 1) * W + ((q >> 4) & 63) - 1) * xst + (q >> 10)) : INT32_MIN;
    }
  }
  // Tiles are numbered down the columns of tiles of an image (t -> image,
  // tile column, tile row): a split's consecutive tiles are vertically
  // adjacent, so the two halo rows a tile shares with its predecessor are
  // still in L2 and each tile fetches TH new x rows from HBM instead of TH + 2
  // (raster order revisited them a whole tile row = 16 tiles later, long
  // evicted: the 512^2 64-channel launch read 1.5x its algorithmic bytes).
  const int tiles_h = H / TH;
  // tile walk counters (FAST): image, tile row, tile column of the next stage
  int w_img = 0, w_ty = 0, w_tx = 0;
  if constexpr (FAST) {
    w_img = t_beg / tiles_img;
    const int tr = t_beg - w_img * tiles_img;
    w_tx = tr / tiles_h;
    w_ty = tr - w_tx * tiles_h;
  }

  auto stage_fast = [&](int buf) {
    const int img = w_img, y0 = w_ty * TH, x0 = w_tx * TW;
    if (++w_ty == tiles_h) {
      w_ty = 0;
      if (++w_tx == tiles_w) { w_tx = 0; ++w_img; }
    }
    char* Pb = smem + buf * STAGE;
    char* Qb = Pb + PB;
    const int64_t pix0 = ((int64_t)img * H + y0) * W + x0;
    const bf16_t* dtile = dsrc + pix0 * dst_;
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const void* s = p_off[k] >= 0 ? (const void*)(dtile + p_off[k]) : zp;
      __builtin_amdgcn_global_load_lds(s, (lds_void*)(Pb + (k * NT + wid * 64) * 16), 16, 0, 0);
    }
    if (y0 > 0 && y0 + TH < H && x0 > 0 && x0 + TW < W) {
      const bf16_t* xtile = xsrc + pix0 * xst;
#pragma unroll
      for (int k = 0; k < NH; ++k)
        if (q_rel[k] != INT32_MIN)
          __builtin_amdgcn_global_load_lds((const void*)(xtile + q_rel[k]), (lds_void*)(Qb + (k * NT + wid * 64) * 16),
                                           16, 0, 0);
    } else {
      const bf16_t* ximg = xsrc + (int64_t)img * H * W * xst;
#pragma unroll
      for (int k = 0; k < NH; ++k) {
        const int e = k * NT + tid, hp = e >> 3, pc = e & 7;
        const int hy = hp / HWP, hx = hp - hy * HWP;
        if (hy < HROWS && hx < TW + 2) {
          const int y = y0 - 1 + hy, x = x0 - 1 + hx;
          const void* s = zp;
          if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
            s = ximg + (int64_t)(y * W + x) * xst + swz_col<128>(hp, pc);
          __builtin_amdgcn_global_load_lds(s, (lds_void*)(Qb + (k * NT + wid * 64) * 16), 16, 0, 0);
        }
      }
    }
  };

  auto stage = [&](int t, int buf) {
    const int img = t / tiles_img, tr = t - img * tiles_img;
    const int y0 = (tr - (tr / tiles_h) * tiles_h) * TH, x0 = (tr / tiles_h) * TW;
    char* Pb = smem + buf * STAGE;
    char* Qb = Pb + PB;
    const bf16_t* dtile = dsrc + (((int64_t)img * H + y0) * W + x0) * dst_;
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const void* s = p_off[k] >= 0 ? (const void*)(dtile + p_off[k]) : zp;
      __builtin_amdgcn_global_load_lds(s, (lds_void*)(Pb + (k * NT + wid * 64) * 16), 16, 0, 0);
    }
    // halo: only the 34 used pixels of each 48-pixel row are loaded (lanes on
    // the pitch padding or past the last row issue nothing; a wave whose
    // lanes are all padding skips the instruction)
    const bf16_t* ximg = xsrc + (int64_t)img * H * W * xst;
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int q = q_pk[k];
      if (q >= 0) {
        const int y = y0 - 1 + (q & 15), x = x0 - 1 + ((q >> 4) & 63);
        const void* s = zp;
        if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
          s = ximg + (int64_t)(y * W + x) * xst + (q >> 10);
        __builtin_amdgcn_global_load_lds(s, (lds_void*)(Qb + (k * NT + wid * 64) * 16), 16, 0, 0);
      }
    }
  };

  // fragment read offsets (bytes; every k-step / tap shift is an immediate)
  const int g4 = lane >> 4, li = lane & 15, qd = li >> 2, pp = li & 3;
  const int wco = wid / WCI, wci = wid - (wid / WCI) * WCI;   // co pair, ci group of this wave
  int offA[TI][2];   // (FAST uses [a][0] only: [a][1] = [a][0] + 4 * RBP, rows m and m + 4 share the swizzle)
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      offA[a][h] = tr_off<RBP>(8 * g4 + qd + 4 * h, (wco * TI + a) * 16 + 4 * pp);
  int offB[TJ][2][3];
#pragma unroll
  for (int b = 0; b < TJ; ++b)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int s = 0; s < 3; ++s)
        // pixel k of a 32-pixel k-step = tile row k / TW (of the step's
        // 32 / TW rows), column k % TW; tap column shift s
        offB[b][h][s] = tr_off<128>(((8 * g4 + qd + 4 * h) / TW) * HWP + (8 * g4 + qd + 4 * h) % TW + s,
                                    (wci * TJ + b) * 16 + 4 * pp);

  f32x4 acc[TI][TJ][9];
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int b = 0; b < TJ; ++b)
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[a][b][t] = f32x4{0, 0, 0, 0};

  const int nsteps = t_end > t_beg ? t_end - t_beg : 0;
  if (nsteps > 0) {
    if constexpr (FAST) stage_fast(0);
    else stage(t_beg, 0);
  }
  for (int st = 0; st < nsteps; ++st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + 1 < nsteps) {
      if constexpr (FAST) stage_fast((st + 1) & 1);
      else stage(t_beg + st + 1, (st + 1) & 1);
    }
    const char* Pb = smem + (st & 1) * STAGE;
    const char* Qb = Pb + PB;
    // FAST: this stage's per-lane fragment base addresses (the +4-row half
    // of an A fragment keeps the swizzle: an immediate 4 * RBP)
    uint32_t bA[TI], bB[TJ][2][3];
    if constexpr (FAST) {
      const uint32_t pa = lds_addr(Pb), qa = lds_addr(Qb);
#pragma unroll
      for (int a = 0; a < TI; ++a) bA[a] = pa + offA[a][0];
#pragma unroll
      for (int b = 0; b < TJ; ++b)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int s = 0; s < 3; ++s) bB[b][h][s] = qa + offB[b][h][s];
    }
    // software-pipelined fragment reads over the 36 (k-step, tap) MFMA groups
    // of a tile: group g's B fragments are read two groups ahead (and a
    // k-step's A fragments two groups before its first tap), so an MFMA group
    // never waits on a just-issued transposed LDS read
    constexpr int NG = TP / 32 * 9;
    u32x4 aq[2][TI], bq[3][TJ];
    auto load_b = [&](int g, u32x4* dst) {
      const int ks = g / 9, q = g - (g / 9) * 9, r = q / 3, s = q - (q / 3) * 3;
#pragma unroll
      for (int b = 0; b < TJ; ++b) {
        if constexpr (FAST) dst[b] = tr_frag_o(bB[b][0][s], bB[b][1][s], (ks * (32 / TW) + r) * HWP * 128);
        else dst[b] = tr_frag(Qb + (ks * (32 / TW) + r) * HWP * 128, offB[b][0][s], offB[b][1][s]);
      }
    };
    auto load_a = [&](int ks, u32x4* dst) {
#pragma unroll
      for (int a = 0; a < TI; ++a) {
        if constexpr (FAST) dst[a] = tr_frag_o2(bA[a], ks * 32 * RBP, ks * 32 * RBP + 4 * RBP);
        else dst[a] = tr_frag(Pb + ks * 32 * RBP, offA[a][0], offA[a][1]);
      }
    };
    load_a(0, aq[0]);
    load_b(0, bq[0]);
    load_b(1, bq[1]);
    // LDS reads issued for group x (its B fragments, plus a k-step's A
    // fragments ahead of its first tap)
    auto nreads = [&](int x) { return x >= NG ? 0 : 2 * TJ + ((x % 9 == 0 && x > 0) ? 2 * TI : 0); };
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int ks = g / 9, t = g - (g / 9) * 9;
      if (g + 2 < NG) {
        if ((g + 2) % 9 == 0) load_a((g + 2) / 9, aq[((g + 2) / 9) & 1]);
        load_b(g + 2, bq[(g + 2) % 3]);
      }
      // group g's fragments (and every older read) are complete once only the
      // reads of groups g+1 and g+2 may still be outstanding
      lgkm_wait(nreads(g + 1) + nreads(g + 2));
#pragma unroll
      for (int a = 0; a < TI; ++a) tie(aq[ks & 1][a]);
#pragma unroll
      for (int b = 0; b < TJ; ++b) tie(bq[g % 3][b]);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < TI; ++a)
#pragma unroll
        for (int b = 0; b < TJ; ++b)
          acc[a][b][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, aq[ks & 1][a]), __builtin_bit_cast(bf16x8, bq[g % 3][b]), acc[a][b][t], 0, 0, 0);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    }
  }

  float* out = p.out + (int64_t)split * p.ni * p.nj;
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int b = 0; b < TJ; ++b)
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int j = t * gq.C + cb + (wci * TJ + b) * 16 + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + (wco * TI + a) * 16 + 4 * g4 + r;
          if (i < p.ni) out[(int64_t)i * p.nj + j] = acc[a][b][t][r];
        }
      }
}

// vu_gemm_set_tuning(VU_TUNE_W3_FAST, ...): 1 (default) the round-4 main loop,
// 0 the round-3 loop, 2 the round-4 loop without s_setprio (A/B runs)
int g_w3_fast = 1;

template <int BI, int TW>
int launch(const VuGemmWgrad& p, hipStream_t st) {
  int64_t nblk = (int64_t)((p.ni + BI - 1) / BI) * (p.q.C / 64) * p.splits;
  if (nblk <= 0) return 0;
  if (g_w3_fast == 1)
    hipLaunchKernelGGL((wgrad3x3_halo_kernel<BI, 1, TW, 1>), dim3((unsigned)nblk), dim3(512), 0, st, p);
  else if (g_w3_fast == 2)
    hipLaunchKernelGGL((wgrad3x3_halo_kernel<BI, 1, TW, 2>), dim3((unsigned)nblk), dim3(512), 0, st, p);
  else
    hipLaunchKernelGGL((wgrad3x3_halo_kernel<BI, 1, TW, 0>), dim3((unsigned)nblk), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

// Output-channel tile: 128 unless the grid is small -- fewer than 256 blocks
// even at the finest split (4 pixel tiles per block) -- where 64-channel tiles
// double the blocks (the ResNet34 encoder's 64^2 / 32^2 / 16^2 levels: 128
// blocks, half the chip, with 128-channel tiles)
int g_w3_small = 1;  // vu_gemm_set_tuning(VU_TUNE_W3_SMALL, ...): 0 = round-2 behaviour (A/B runs)

int pick_bi(const VuGemmWgrad& p) {
  if (p.ni <= 64 || p.q.W % 32 != 0) return 64;  // (128 x 16-wide tiles would spill)
  if (!g_w3_small) return 128;
  const int64_t T = (int64_t)p.q.N * p.q.H * p.q.W / TP;
  const int64_t blocks128 = (int64_t)((p.ni + 127) / 128) * (p.q.C / 64) * (T / 4 > 0 ? T / 4 : 1);
  return blocks128 < 256 ? 64 : 128;
}

}  // namespace

// (BI, BJ = 9*64) when the halo kernel serves this problem, else 0: bf16, dy
// a plain 1x1 NHWC map, x a 3x3 stride-1 pad-1 gather of 64-channel aligned
// sources over an image whose width is a multiple of 32 and height of 4 (or
// width a multiple of 16 and height of 8).
// Splits must then be whole 128-pixel tiles (m_per_split % 128 == 0).
int gemm_wgrad_v3_tile(const VuGemmWgrad& p, int dtype, int* bi, int* bj) {
  const VuGather& a = p.p;
  const VuGather& g = p.q;
  if (dtype != VU_BF16) return 0;
  if (a.nsrc != 1 || a.R != 1 || a.S != 1 || a.oy != 0 || a.ox != 0 || a.stride[0] % 8 || a.C != p.ni ||
      p.ni % 8)
    return 0;
  if (g.R != 3 || g.S != 3 || g.sy != 1 || g.sx != 1 || g.dy != 1 || g.dx != 1 || g.oy != -1 || g.ox != -1 ||
      g.Hs != g.H || g.Ws != g.W || a.N != g.N || a.H != g.H || a.W != g.W)
    return 0;
  if (g.C % 64 || p.nj != 9 * g.C) return 0;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.cend[t] % 64 || g.stride[t] % 8) return 0;
  const int tw = g.W % 32 == 0 ? 32 : (g.W % 16 == 0 && g_w3_small ? 16 : 0);
  if (!tw || g.H % (TP / tw)) return 0;
  if ((int64_t)g.N * g.H * g.W >= (int64_t)1 << 31) return 0;
  if ((int64_t)(TP / tw) * g.W * a.stride[0] >= (int64_t)1 << 31) return 0;   // 32-bit dy slot offsets
  for (int t = 0; t < g.nsrc; ++t)                                               // 32-bit halo slot offsets
    if ((int64_t)(TP / tw + 2) * (g.W + 2) * g.stride[t] >= (int64_t)1 << 31) return 0;
  *bi = pick_bi(p);
  *bj = 9 * 64;
  return 1;
}

int gemm_wgrad_v3_launch(const VuGemmWgrad& p, hipStream_t st) {
  if (p.m_per_split % TP) return (int)hipErrorInvalidValue;
  if (p.q.W % 32 != 0) return launch<64, 16>(p, st);
  if (pick_bi(p) == 64) return launch<64, 32>(p, st);
  return launch<128, 32>(p, st);
}

int gemm_wgrad_v3_tune(int key, int value) {
  if (key == VU_TUNE_W3_SMALL) {
    g_w3_small = value != 0;
    return 0;
  }
  if (key == VU_TUNE_W3_FAST) {
    if (value < 0 || value > 2) return (int)hipErrorInvalidValue;
    g_w3_fast = value;
    return 0;
  }
  return -1;
}
