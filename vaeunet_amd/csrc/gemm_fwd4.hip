// 3x3 / stride-1 / pad-1 convolution as a halo-tiled implicit GEMM with a
// PING-PONG wave schedule ("v4", bf16).  Serves the DoubleConv forward convs
// (unet_parts.py:40,43) and their stride-1 input-gradient convs (flipped
// weights) when the output-channel count is a multiple of 64/128/256.
//
// Why another kernel: v3 (gemm_fwd3.hip) runs all eight waves of a block in
// lockstep -- every wave reads its fragments, then every wave issues MFMAs --
// so each SIMD's matrix pipe idles while both of its waves wait on LDS, and
// rocprof shows ~35 % of wave time parked at barriers.  Here the two halves
// of the block (waves 0-3 and 4-7, one of each per SIMD) run the same
// program one barrier apart: while one half streams its fragments out of LDS
// the other half issues MFMAs, so the pipe sees back-to-back 16-MFMA
// segments from alternating waves (cdna_hip_programming.md "256^2 8-phase
// template"; MI355X_MICROARCH.md "Two waves per SIMD").
//
//   * every wave owns a 128-pixel x 64-channel output tile (8 x 4 fragments
//     of v_mfma_f32_16x16x32_bf16, 128 accumulator registers); the block is
//     256 x 256 (8x32 pixels), 512 x 128 (16x32) or 1024 x 64 (32x32);
//   * K is walked in steps of one tap x 32 input channels; per 32-channel
//     chunk the (TH+2) x (TW+2) halo lands ONCE in LDS (64-byte pixel rows,
//     contiguous 1 KiB fragment reads -- no swizzle needed) and the nine taps
//     read it in place at a shifted row;
//   * weights stream per step into a 3-slot ring (prefetch distance 2), the
//     next chunk's halo streams in during the first steps of the current
//     chunk, both by LDS-DMA (global_load_lds_dwordx4) with counted vmcnt
//     waits and raw s_barrier so DMA stays in flight across barriers;
//   * MFMA operands are (weights, pixels): each lane's accumulator holds 4
//     consecutive output channels of one pixel, which makes the BatchNorm
//     partial statistics a register + 16-lane reduction and the bf16 output
//     staging 8-byte LDS writes;
//   * epilogue: bias, storage rounding, per-wave (sum, centered M2) of the
//     rounded values (same contract as v1-v3) by DPP row sums, then each
//     wave stages its tile 32 pixels at a time through a private LDS strip
//     and stores whole 128-byte pixel rows (16 bytes per lane);
//   * the step loop is (chunk, tap) with the weight ring slot = tap % 3 and
//     the halo slot addresses recomputed per chunk: no per-step divisions and
//     no per-slot register arrays live across the MFMAs (measured 6 % faster
//     than a flat step loop with precomputed slots);
//   * split-K for grids under one block per CU (the 32x32 and 64x64 levels:
//     down4 convs and their input gradients have 64-128 256x256 tiles for
//     256 CUs): each block walks a contiguous range of 32-channel chunks and
//     writes its fp32 tile to a slab; splitk_finish_kernel sums the slabs in
//     a fixed order and applies the epilogue above (deterministic).
#include "common.h"
#include "../../include/vaeunet.h"

static __device__ __attribute__((aligned(16))) uint32_t vu_zero_page4[16];

namespace {

typedef __attribute__((address_space(3))) void lds_void;

template <int BN> struct PP;
template <> struct PP<256> { static constexpr int WM = 2, WN = 4, TH = 8, TW = 32; };
template <> struct PP<128> { static constexpr int WM = 4, WN = 2, TH = 16, TW = 32; };
template <> struct PP<64> { static constexpr int WM = 8, WN = 1, TH = 32, TW = 32; };

// at most N vector-memory operations of this wave outstanding (loads AND
// stores: CDNA counts both in vmcnt, in issue order)
template <int N>
VU_DEV void wait_vm_c() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// A workgroup barrier nothing is scheduled across (the ping-pong relies on
// the exact placement of reads, DMA issues and MFMAs between barriers).
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

// RELU: epilogue ReLU (VuGemmFwd.relu).  FULL: one read segment + one
// 32-MFMA segment per step (2 barriers) instead of two 16-MFMA halves (4
// barriers): twice the matrix work per barrier interval, 16 more fragment
// registers (VU_TUNE_PP_FULL, A/B).
// ZB: the latent-shortcut epilogue (VuGemmFwd.zbias) as its own
// instantiation -- a runtime branch pushed the others to 256 VGPRs + scratch.
// PERS (round 5, VU_TUNE_PP_PERSIST): a persistent grid (<= one block per CU)
// walks its tiles; the next tile's first halo and first two weight slots are
// issued before the current tile's epilogue (which stages through its own LDS
// strips), so the per-tile prologue wait overlaps the epilogue.
template <int BN, bool SPLIT, bool BNB, bool RELU = false, bool FULL = false, bool ZB = false, bool PERS = false>
__global__ __launch_bounds__(512, 1) void conv3x3_pp_kernel(VuGemmFwd p) {
  constexpr int NBW = 3;                          // weight ring slots
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
  constexpr int PD = NBW - 1;                     // weight prefetch distance (steps)
  constexpr int MAIN = 2 * HALO + NBW * WSLOT;
  // epilogue: each wave stages 32-pixel rows of its tile through a private
  // LDS strip (the main-loop buffers, free by then) and stores whole 128-byte
  // pixel rows
  constexpr int SPITCH = 144;                     // staged pixel row (128 B + pad)
  constexpr int STG = 32 * SPITCH;
  constexpr int SMEM = PERS ? MAIN + 8 * STG : MAIN;
  static_assert(SMEM <= 163840 && 8 * STG <= MAIN, "LDS");
  static_assert(!(PERS && SPLIT), "persistent walk: whole-K tiles only");
  static_assert(LB0 >= 1, "DMA schedule");
  static_assert(9 % NBW == 0, "ring slot = tap % NBW");
  static_assert(TW == 32, "fragment geometry");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const VuGather& g = p.a;
  const int H = g.H, W = g.W;
  const int tx_n = W / TW, ty_n = H / TH;
  const int mtiles = g.N * ty_n * tx_n;
  const int ntiles = p.ncol / BN;
  const int btiles = mtiles * ntiles;
  // split-K (SPLIT): the block index also picks a K range (kidx); a separate
  // instantiation so the plain kernel carries none of it (register pressure)
  const int ksplit = SPLIT ? p.ksplit : 1;
  const int bid0 = xcd_remap(blockIdx.x, btiles * ksplit);
  const int kidx = SPLIT ? bid0 / btiles : 0;
  // the tile this block computes (mt, img, y0, x0, n0: epilogue) and the one
  // its DMA streams (d*: the same, or -- PERS, during the epilogue -- the next)
  int mt, img, y0, x0, n0, dimg, dy0, dx0, dn0;
  auto tile_coords = [&](int b, int& m_, int& im_, int& y_, int& x_, int& n_) {
    m_ = b / ntiles;
    const int nt_ = b - m_ * ntiles;
    im_ = m_ / (ty_n * tx_n);
    const int tr = m_ - im_ * (ty_n * tx_n);
    y_ = (tr / tx_n) * TH;
    x_ = (tr - (tr / tx_n) * tx_n) * TW;
    n_ = nt_ * BN;
  };
  int cur = SPLIT ? bid0 - kidx * btiles : bid0;
  {
    int mdum;
    tile_coords(cur, mdum, dimg, dy0, dx0, dn0);
  }
  // this block's contiguous range of 32-channel chunks
  const int call = g.C / 32;
  const int cbeg = SPLIT ? kidx * call / ksplit : 0, cend = SPLIT ? (kidx + 1) * call / ksplit : call;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int grp = wid >> 2;  // ping-pong half (one wave of each half per SIMD)

  // ---- DMA roles ------------------------------------------------------------
  // vmcnt counts a wave's loads in issue order, so a wave that mixes slow
  // (HBM) halo loads with fast (L2) weight loads would have every weight wait
  // also drain the halo.  The halves therefore split the streams: waves 0-3
  // stream the weights (and wait for them every step), waves 4-7 stream the
  // next chunk's halo (and wait for it once per chunk).
  const int gt = tid & 255;        // thread index inside the half
  const int gw = wid & 3;          // wave index inside the half
  const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
  const void* zp = (const void*)vu_zero_page4;
  char* const hbuf = smem;
  char* const wbuf = smem + 2 * HALO;

  // channel sources (concat inputs) held in registers: no per-chunk kernarg loads
  const bf16_t* const src0 = reinterpret_cast<const bf16_t*>(g.src[0]);
  const bf16_t* const src1 = reinterpret_cast<const bf16_t*>(g.src[1]);
  const bf16_t* const src2 = reinterpret_cast<const bf16_t*>(g.src[2]);
  const int64_t st0 = g.stride[0], st1 = g.stride[1], st2 = g.stride[2];
  const int ce0 = g.cend[0], ce1 = g.nsrc > 2 ? g.cend[1] : (1 << 30);
  // (half 1) the whole halo of chunk c into buffer buf; slot geometry is
  // recomputed per chunk (a per-slot register array would stay live through
  // the MFMA loop: 19 registers at BN = 64)
  auto halo_chunk = [&](int c, int buf) {
    int ib = dimg, yb = dy0, xb = dx0;
    asm volatile("" : "+s"(ib), "+s"(yb), "+s"(xb));  // keep the slot math inside the loop
    const int cb = c * 32;
    const bf16_t* src;
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
    src += (int64_t)ib * H * W * st + (gt & 3) * 8;
#pragma unroll
    for (int i = 0; i < NHP1; ++i) {
      if (i * 256 + gw * 64 >= HPIECES) continue;  // wave-uniform
      const int P = i * 256 + gt;
      if (P < HPIECES) {
        const int px = P >> 2;
        const int hy = px / HW, hx = px - (px / HW) * HW;
        const int y = yb - 1 + hy, x = xb - 1 + hx;
        const bool ok = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        const void* gp = ok ? (const void*)(src + (int64_t)(y * W + x) * st) : zp;
        char* dst = hbuf + buf * HALO + (i * 256 + gw * 64) * 16;
        __builtin_amdgcn_global_load_lds(gp, (lds_void*)dst, 16, 0, 0);
      }
    }
  };
  // (half 0) weight slots [i0, i1) of (chunk c, tap t) into ring slot `slot`
  auto wstage = [&](int c, int t, int slot, int i0, int i1) {
    const int k0 = t * g.C + c * 32;
    char* B = wbuf + slot * WSLOT;
#pragma unroll
    for (int i = 0; i < LB0; ++i) {
      if (i < i0 || i >= i1) continue;
      const int P = i * 256 + gt;
      const int row = P >> 2;
      const void* gp = (const void*)(bmat + (int64_t)(dn0 + row) * p.ldb + k0 + (P & 3) * 8);
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(B + (i * 256 + gw * 64) * 16), 16, 0, 0);
    }
  };

  // ---- fragment addressing -------------------------------------------------
  // A fragment i of a wave covers tile pixels wm*128 + i*16 + (0..15): row
  // wm*4 + i/2, columns (i&1)*16 + (0..15) (TW = 32), so its halo byte offset
  // (tap (0,0)) is one per-lane base plus a compile-time constant
  const int abase = ((wm * 4) * HW + (lane & 15)) * 64 + (lane >> 4) * 16;
  auto arow = [&](int i) { return abase + ((i >> 1) * HW + (i & 1) * 16) * 64; };
  const int brow = (wn * 64 + (lane & 15)) * 64 + (lane >> 4) * 16;
  const int cbase = wn * 64 + 4 * (lane >> 4);

  // ---- prologue: halo of chunk 0, weights of steps 0 and 1 -----------------
  if (grp) {
    halo_chunk(cbeg, 0);
  } else {
    wstage(cbeg, 0, 0, 0, LB0);
    wstage(cbeg, 1, 1, 0, LB0);
  }
  int kt = 0;  // PERS: tiles walked
  for (;;) {
  tile_coords(cur, mt, img, y0, x0, n0);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  if (grp) pp_barrier();  // the stagger: half 1 runs one barrier behind

  // steps = (chunk c, tap t); a chunk has 9 = 3 x NBW taps, so the weight
  // ring slot of tap t is t % 3 in every chunk
  int hb = 0;  // halo buffer of the current chunk
  for (int c = cbeg; c < cend; ++c) {
    const bool next_here = c + 1 < cend;
    const char* Ah = hbuf + hb * HALO;
    for (int t = 0; t < 9; ++t) {
      const int ty = (t * 11) >> 5, tx = t - ty * 3;  // t / 3, t % 3 (t < 9)
      const char* A = Ah + (ty * HW + tx) * 64;
      const int slot = tx;                             // t % NBW (= t % 3)
      const char* Bw = wbuf + slot * WSLOT;
      const int pslot = slot == 0 ? 2 : slot - 1;      // (t + 2) % NBW
      const int pt = t + PD < 9 ? t + PD : t + PD - 9;
      const bool pref = t + PD < 9 || next_here;      // the step two ahead exists
      const int pc = t + PD < 9 ? c : c + 1;
      if constexpr (FULL) {
        // -- one read segment: weights + all 8 pixel fragments; half 0
        //    prefetches the weights two steps ahead and waits for the next
        //    step's, half 1 streams the next chunk's halo (waits at tap 8)
        u32x4 bq[4], aq[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) bq[j] = *reinterpret_cast<const u32x4*>(Bw + brow + j * 16 * 64);
#pragma unroll
        for (int i = 0; i < 8; ++i) aq[i] = *reinterpret_cast<const u32x4*>(A + arow(i));
        if (!grp) {
          if (pref) {
            wstage(pc, pt, pslot, 0, LB0);
            wait_vm_c<(PD - 1) * LB0>();
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
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bq[j]),
                                                                __builtin_bit_cast(bf16x8, aq[i]), acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        pp_barrier();
        continue;
      }
      u32x4 bf[4], af[4];
      // -- phase 1: weights + pixel fragments 0..3; half 0 prefetches the
      //    weights two steps ahead
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const u32x4*>(Bw + brow + j * 16 * 64);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const u32x4*>(A + arow(i));
      if (!grp && pref) wstage(pc, pt, pslot, 0, LB0A);
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
      // -- phase 2: pixel fragments 4..7; half 0 finishes the prefetch and
      //    waits for the next step's weights; half 1 streams the next chunk's
      //    halo and waits for it at the chunk's last tap
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const u32x4*>(A + arow(4 + i));
      if (!grp) {
        if (pref) {
          wstage(pc, pt, pslot, LB0A, LB0);
          wait_vm_c<(PD - 1) * LB0>();  // only the prefetch just issued may be in flight
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
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                                  __builtin_bit_cast(bf16x8, af[i]), acc[4 + i][j], 0,
                                                                  0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    }
    hb ^= 1;
  }
  if (!grp) pp_barrier();  // re-align the halves
  // PERS: every wave is past its last fragment read -- the next tile's first
  // halo (buffer 0) and weight slots 0, 1 stream in during this epilogue
  bool more = false;
  if constexpr (PERS) {
    ++kt;
    const int vb = (int)blockIdx.x + kt * (int)gridDim.x;
    more = vb < btiles;
    if (more) {
      cur = xcd_remap(vb, btiles);
      int mdum;
      tile_coords(cur, mdum, dimg, dy0, dx0, dn0);
      if (grp) {
        halo_chunk(cbeg, 0);
      } else {
        wstage(cbeg, 0, 0, 0, LB0);
        wstage(cbeg, 1, 1, 0, LB0);
      }
    }
  }

  // ---- epilogue -------------------------------------------------------------
  // acc[i][j][r]: pixel wm*128 + i*16 + (lane&15), channel n0 + cbase + j*16 + r
  // Epilogue-only arguments are re-read from the kernarg segment through an
  // opaque pointer so that they are not held in SGPRs across the MFMA loop.
  const __attribute__((address_space(4))) VuGemmFwd* ep =
      (const __attribute__((address_space(4))) VuGemmFwd*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ep));
  if (SPLIT) {
    // split-K: raw fp32 partial tile -> slab kidx (16-byte stores of 4 channels)
    float* const sbase = ep->workspace + (int64_t)kidx * ((int64_t)g.N * H * W) * ep->ncol + n0 + cbase +
                         (((int64_t)img * H + y0 + wm * 4) * W + x0 + (lane & 15)) * ep->ncol;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float* row = sbase + ((i >> 1) * (int64_t)W + (i & 1) * 16) * ep->ncol;
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4*>(row + j * 16) = acc[i][j];
    }
    return;
  }
  if constexpr (ZB) {
    // the latent-broadcast shortcut (VuGemmFwd.zbias): fragment i's pixel is
    // tile row wm*4 + i/2, column (i&1)*16 + (lane&15); its border class picks
    // one of the sample's 9 bias rows (4 channels per 16-byte load).  One
    // fragment at a time, its loads fenced: batched, they spilled.
    // (lane-derived values made opaque here, so that nothing of this address
    // math is hoisted above the MFMA loop and held live through it)
    int lz = lane;
    asm volatile("" : "+v"(lz));
    const float* const zb0 = ep->zbias + (int64_t)img * 9 * ep->ncol + n0 + wn * 64 + 4 * (lz >> 4);
    const int cx0 = zb_class(x0 + (lz & 15), W), cx1 = zb_class(x0 + 16 + (lz & 15), W);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int zo = (3 * zb_class(y0 + wm * 4 + (i >> 1), H) + ((i & 1) ? cx1 : cx0)) * ep->ncol;
      f32x4 zv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) zv[j] = *reinterpret_cast<const f32x4*>(zb0 + zo + j * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += zv[j];
      asm volatile("" ::: "memory");
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float bv = ep->bias ? ep->bias[n0 + cbase + j * 16 + r] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i][j][r] = rnd<bf16_t>(acc[i][j][r] + bv);
    }
  }
  if constexpr (RELU)
#pragma unroll
    for (int i = 0; i < 8; ++i) epi_relu(acc[i]);
  if (ep->stat_sum) {
    // per-wave statistics tile: its 128 pixels (8 fragments x one 16-lane DPP
    // row), two-pass (sum, centered M2) of the rounded values; lane (g4, x)
    // keeps column (x/4)*16 + 4*g4 + x%4 of the wave's 64, so the tile's 64
    // columns go out in one store per statistic
    // The in-lane passes run on channel PAIRS with packed fp32 ops (v_pk_add /
    // v_pk_fma: half the VALU issue of the scalar form, the same roundings in
    // the same order -- bit-identical); a wave64 VALU op occupies its SIMD 4
    // cycles and this epilogue runs with the matrix pipe idle.
    float ms = 0.f, mq = 0.f;
    const int x = lane & 15;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x2 sv = f32x2{0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 8; ++i) sv += f32x2{acc[i][j][2 * h], acc[i][j][2 * h + 1]};
        // (the opaque copy keeps the two DPP reductions scalar: packed, each
        // step became two DPP moves + zero inits + a packed add)
        float s0 = row16_sum(sv[0]), s1 = row16_sum(sv[1]);
        asm volatile("" : "+v"(s0), "+v"(s1));
        sv = f32x2{s0, s1};
        const f32x2 mean = sv * (1.f / 128);  // exact (power-of-two scale)
        f32x2 q = f32x2{0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const f32x2 d = f32x2{acc[i][j][2 * h], acc[i][j][2 * h + 1]} - mean;
          q = __builtin_elementwise_fma(d, d, q);
        }
        float q0 = row16_sum(q[0]), q1 = row16_sum(q[1]);
        asm volatile("" : "+v"(q0), "+v"(q1));
        q = f32x2{q0, q1};
        if (x == j * 4 + 2 * h) {
          ms = sv[0];
          mq = q[0];
        }
        if (x == j * 4 + 2 * h + 1) {
          ms = sv[1];
          mq = q[1];
        }
      }
    const int64_t so = (int64_t)(mt * WM + wm) * ep->ncol + n0 + wn * 64 + (x >> 2) * 16 + 4 * (lane >> 4) + (x & 3);
    ep->stat_sum[so] = ms;
    ep->stat_m2[so] = mq;
  }
  u32x2 pk[8][4];  // bf16 pairs: channels (4*g4 + j*16) + {0,1}, {2,3}
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pk[i][j][0] = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
      pk[i][j][1] = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
    }
  // BatchNorm-backward partials (bnb_part) are taken in the staged-row layout
  // below: a lane holds channels (lane & 7) * 8 .. +7 of the wave's 64 for
  // pixels q * 8 + (lane >> 3) of each 32-pixel row h.  The BN input x of
  // those 16 pixels is loaded now (all 16 loads in flight at once) and
  // consumed row by row.
  constexpr bool bnb = BNB;
  const int bc = n0 + wn * 64 + (lane & 7) * 8;
  float bsc[8], bsf[8], bmu[8], bis[8], bs0[8], bs1[8];
  u32x4 bx[2][4];  // rows h (even/odd): row h + 1 is loaded while row h is used
  const bf16_t* xr = nullptr;
  if (bnb) {
    xr = reinterpret_cast<const bf16_t*>(ep->bnb_x) + bc +
         (((int64_t)img * H + y0 + wm * 4) * W + x0 + (lane >> 3)) * ep->bnb_xstride;
#pragma unroll
    for (int q = 0; q < 4; ++q) bx[0][q] = *reinterpret_cast<const u32x4*>(xr + (int64_t)q * 8 * ep->bnb_xstride);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bsc[e] = ep->bnb_scale[bc + e];
      bsf[e] = ep->bnb_shift[bc + e];
      bmu[e] = ep->bnb_mean[bc + e];
      bis[e] = ep->bnb_invstd[bc + e];
      bs0[e] = 0.f;
      bs1[e] = 0.f;
    }
  }
  // the main-loop buffers are free once every wave is past its last fragment
  // read: an LDS wait + raw barrier, NOT __syncthreads() -- that also waits
  // vmcnt(0), i.e. for the acknowledgement of the statistics stores just
  // issued (measured: the 17 forward layers 2.65 ms with statistics against
  // 2.44 ms without)
  if constexpr (!PERS) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_barrier();
  }
  // fragments 2h and 2h+1 are the 32 pixels of tile row wm*4 + h
  bf16_t* const orow0 = reinterpret_cast<bf16_t*>(ep->out) + ep->out_coff + n0 + wn * 64 +
                        (((int64_t)img * H + y0 + wm * 4) * W + x0) * ep->out_stride;
  const int64_t orow_y = (int64_t)W * ep->out_stride;
  char* const stg = smem + (PERS ? MAIN : 0) + wid * STG;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<u32x2*>(stg + (ii * 16 + (lane & 15)) * SPITCH + (j * 16 + 4 * (lane >> 4)) * 2) =
            pk[2 * h + ii][j];
    u32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = q * 64 + lane;
      v[q] = *reinterpret_cast<const u32x4*>(stg + (e >> 3) * SPITCH + (e & 7) * 16);
    }
    if (bnb && h + 1 < 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bx[(h + 1) & 1][q] =
            *reinterpret_cast<const u32x4*>(xr + ((int64_t)(h + 1) * W + q * 8) * ep->bnb_xstride);
    }
    bf16_t* const orow = orow0 + h * orow_y;
    if (ep->accumulate) {
      // out += result, rounded once more (a bf16 tensor add)
      u32x4 old[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = q * 64 + lane;
        old[q] = *reinterpret_cast<const u32x4*>(orow + (e >> 3) * ep->out_stride + (e & 7) * 8);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float lo = __uint_as_float(old[q][w] << 16) + __uint_as_float(v[q][w] << 16);
          const float hi = __uint_as_float(old[q][w] & 0xffff0000u) + __uint_as_float(v[q][w] & 0xffff0000u);
          v[q][w] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = q * 64 + lane;
      *reinterpret_cast<u32x4*>(orow + (e >> 3) * ep->out_stride + (e & 7) * 8) = v[q];
    }
    if (bnb) {
      // dz = stored output, masked by the forward ReLU; sums as vu_bn_bwd_reduce
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf) {
            const int e = 2 * w + hf;
            const float xv = __uint_as_float(hf ? (bx[h & 1][q][w] & 0xffff0000u) : (bx[h & 1][q][w] << 16));
            float dz = __uint_as_float(hf ? (v[q][w] & 0xffff0000u) : (v[q][w] << 16));
            if (ep->bnb_relu && !(xv * bsc[e] + bsf[e] > 0.f)) dz = 0.f;
            bs0[e] += dz;
            bs1[e] += dz * ((xv - bmu[e]) * bis[e]);
          }
    }
  }
  if (bnb) {
    // lanes sharing (lane & 7) hold the same 8 channels: fold over lane bits 3-5
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        bs0[e] += __shfl_xor(bs0[e], o, 64);
        bs1[e] += __shfl_xor(bs1[e], o, 64);
      }
    }
    if (lane < 8) {
      float* pr = ep->bnb_part + (int64_t)(mt * WM + wm) * 2 * ep->ncol + bc;
      *reinterpret_cast<f32x4*>(pr) = f32x4{bs0[0], bs0[1], bs0[2], bs0[3]};
      *reinterpret_cast<f32x4*>(pr + 4) = f32x4{bs0[4], bs0[5], bs0[6], bs0[7]};
      *reinterpret_cast<f32x4*>(pr + ep->ncol) = f32x4{bs1[0], bs1[1], bs1[2], bs1[3]};
      *reinterpret_cast<f32x4*>(pr + ep->ncol + 4) = f32x4{bs1[4], bs1[5], bs1[6], bs1[7]};
    }
  }
  if (!more) break;
  }  // tile walk (one pass unless PERS)
}

// split-K epilogue: out = round(sum_k slab[k] + bias) (+ out if accumulate),
// BatchNorm (sum, centered M2) per 128-row tile of the rounded values.  Block:
// 128 rows x 64 columns, 256 threads (8 column groups of 8 x 32 row lanes).
__global__ __launch_bounds__(256) void splitk_finish_kernel(VuGemmFwd p) {
  __shared__ float red[32][65];
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  const int ctiles = p.ncol / 64;
  const int rb = blockIdx.x / ctiles, cb = blockIdx.x - (blockIdx.x / ctiles) * ctiles;
  const int t = threadIdx.x, cg = t & 7, rs = t >> 3;
  const int c0 = cb * 64 + cg * 8;
  const int64_t slab = M * p.ncol;
  float v[4][8];
  float bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = p.bias ? p.bias[c0 + e] : 0.f;
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
  // slab sums in k order; the 4 row groups x 2 splits of loads are issued
  // together (a per-row k loop waits one memory round trip per load)
  f32x4 sa[4], sb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) sa[q] = sb[q] = f32x4{0, 0, 0, 0};
  const float* src0 = p.workspace + ((int64_t)rb * 128 + rs) * p.ncol + c0;
  const int64_t qs = 32 * (int64_t)p.ncol;
  int k = 0;
  for (; k + 2 <= p.ksplit; k += 2) {
    f32x4 ta[2][4], tb[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float* src = src0 + (k + h) * slab + q * qs;
        ta[h][q] = *reinterpret_cast<const f32x4*>(src);
        tb[h][q] = *reinterpret_cast<const f32x4*>(src + 4);
      }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sa[q] += ta[h][q];
        sb[q] += tb[h][q];
      }
  }
  if (k < p.ksplit) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float* src = src0 + k * slab + q * qs;
      sa[q] += *reinterpret_cast<const f32x4*>(src);
      sb[q] += *reinterpret_cast<const f32x4*>(src + 4);
    }
  }
  // The epilogue's loads -- the old output rows (accumulate) and the BN-
  // backward operands (bnb_part) -- issued together before the first store:
  // behind the stores they may alias they were ~12 serial round trips.
  bf16_t* dstq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t m = (int64_t)rb * 128 + rs + 32 * q;
    int64_t orow = m;
    if (p.out_mode == 2) {  // stride-2 sub-lattice (parity-class input gradients)
      const int64_t hw = (int64_t)p.a.H * p.a.W;
      const int64_t n = m / hw, rem = m - n * hw;
      const int h = (int)(rem / p.a.W), w = (int)(rem - (int64_t)h * p.a.W);
      orow = ((int64_t)n * p.oH + 2 * h + p.opy) * p.oW + 2 * w + p.opx;
    }
    dstq[q] = out + orow * p.out_stride + p.out_coff + c0;
  }
  Vec8<bf16_t> old[4], xq[4];
  float bsc[8], bsf[8], bmu[8], bis[8];
  f32x4 za[4], zb[4];  // VuGemmFwd.zbias of the 4 rows (latent shortcut)
#pragma unroll
  for (int q = 0; q < 4; ++q) za[q] = zb[q] = f32x4{0, 0, 0, 0};
  if (p.zbias) {
    const int hw = p.a.H * p.a.W;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t m = (int64_t)rb * 128 + rs + 32 * q;
      const int n = (int)(m / hw), rem = (int)(m - (int64_t)n * hw);
      const int h = rem / p.a.W, w = rem - (rem / p.a.W) * p.a.W;
      const float* z = p.zbias + ((int64_t)n * 9 + 3 * zb_class(h, p.a.H) + zb_class(w, p.a.W)) * p.ncol + c0;
      za[q] = *reinterpret_cast<const f32x4*>(z);
      zb[q] = *reinterpret_cast<const f32x4*>(z + 4);
    }
  }
  if (p.accumulate) {
#pragma unroll
    for (int q = 0; q < 4; ++q) old[q].load(dstq[q]);
  }
  if (p.bnb_part) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      xq[q].load(reinterpret_cast<const bf16_t*>(p.bnb_x) + ((int64_t)rb * 128 + rs + 32 * q) * p.bnb_xstride + c0);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bsc[e] = p.bnb_scale[c0 + e];
      bsf[e] = p.bnb_shift[c0 + e];
      bmu[e] = p.bnb_mean[c0 + e];
      bis[e] = p.bnb_invstd[c0 + e];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 a = p.zbias ? sa[q] + za[q] : sa[q], b = p.zbias ? sb[q] + zb[q] : sb[q];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[q][e] = rnd<bf16_t>(a[e] + bv[e]);
      v[q][4 + e] = rnd<bf16_t>(b[e] + bv[4 + e]);
    }
    if (p.relu)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[q][e] = fmaxf(v[q][e], 0.f);
    Vec8<bf16_t> o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.set(e, v[q][e]);
    if (p.accumulate) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o.set(e, old[q].get(e) + v[q][e]);
    }
    o.store(dstq[q]);
  }
  if (p.bnb_part) {
    // BatchNorm-backward partials of this 128-row tile (see VuGemmFwd.bnb_part)
    float s0[8], s1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s0[e] = s1[e] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = xq[q].get(e);
        float dz = v[q][e];
        if (p.bnb_relu && !(xv * bsc[e] + bsf[e] > 0.f)) dz = 0.f;
        s0[e] += dz;
        s1[e] += dz * ((xv - bmu[e]) * bis[e]);
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[rs][cg * 8 + e] = k ? s1[e] : s0[e];
      __syncthreads();
      if (rs == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float sm = 0.f;
          for (int r = 0; r < 32; ++r) sm += red[r][cg * 8 + e];
          p.bnb_part[((int64_t)rb * 2 + k) * p.ncol + c0 + e] = sm;
        }
      }
      __syncthreads();
    }
  }
  if (!p.stat_sum) return;
  // two-pass (sum, centered M2) of the 128 rows of each column
  float mean[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rs][cg * 8 + e] = (v[0][e] + v[1][e]) + (v[2][e] + v[3][e]);
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float sm = 0.f;
    for (int r = 0; r < 32; ++r) sm += red[r][cg * 8 + e];
    mean[e] = sm;
  }
  __syncthreads();
  if (rs == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) p.stat_sum[(int64_t)rb * p.ncol + c0 + e] = mean[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] *= 1.f / 128;
    float q2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float d = v[q][e] - mean[e];
      q2 += d * d;
    }
    red[rs][cg * 8 + e] = q2;
  }
  __syncthreads();
  if (rs == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float sm = 0.f;
      for (int r = 0; r < 32; ++r) sm += red[r][cg * 8 + e];
      p.stat_m2[(int64_t)rb * p.ncol + c0 + e] = sm;
    }
  }
}

template <int BN>
bool tiles_ok(const VuGemmFwd& p) {
  const VuGather& g = p.a;
  return p.ncol % BN == 0 && g.H % PP<BN>::TH == 0 && g.W % PP<BN>::TW == 0;
}

int g_min_blocks = 256;  // vu_gemm_set_tuning(VU_TUNE_V4_MIN_BLOCKS, ...)
int g_splitk = 1;        // vu_gemm_set_tuning(VU_TUNE_V4_SPLITK, ...): 0 off, 1 auto, k >= 2 forced
int g_pp_full = 1;       // VU_TUNE_PP_FULL: one phase per step (conv3x3_pp_kernel FULL; 0 = two halves)
int g_pp_persist = 0;    // VU_TUNE_PP_PERSIST: persistent tile walk for 128/256-column tiles (PERS);
                         // 1 = grids over one block per CU, k >= 2 = always, grid capped at k (tests)

// Output-column tile the ping-pong kernel uses for this problem (0 = not served).
int pick_bn(const VuGemmFwd& p) {
  const VuGather& g = p.a;
  const int64_t pix = (int64_t)g.N * g.H * g.W;
  const int mb = g_min_blocks;
  // at least ~one block per CU, else the v3 tiles (more, smaller blocks) win
  if (tiles_ok<256>(p) && (pix / 256) * (p.ncol / 256) >= mb) return 256;
  if (p.ncol % 256 != 0 && tiles_ok<128>(p) && (pix / 512) * (p.ncol / 128) >= mb) return 128;
  // 64 x 64 problems (18 K steps) are prologue/epilogue bound at 1 block/CU: v3 wins
  if (p.ncol == 64 && (g.C > 64 || mb < 256) && tiles_ok<64>(p) && pix / 1024 >= mb) return 64;
  // column counts that are 64- but not 128-multiples (padded decoder concats:
  // 704, 832): 1024 x 64 tiles, several column tiles per pixel tile
  if (p.ncol % 128 != 0 && p.ncol > 64 && tiles_ok<64>(p) && (pix / 1024) * (p.ncol / 64) >= mb) return 64;
  return 0;
}

struct Plan {
  int bn, ks;
};

// Tile and K-split.  A grid under one block per CU gets the widest column
// tile that divides the output and the smallest split that reaches one block
// per CU (down4: 128 256x256 tiles -> 2, its input gradient: 64 tiles -> 4;
// the ResNet34 encoder's 64^2 / 32^2 levels: 64 512x128 / 32 256x256 tiles),
// at least g_split_min_chunks 32-channel chunks per split.
int g_split_min_chunks = 2;  // vu_gemm_set_tuning(VU_TUNE_V4_SPLIT_CHUNKS, ...)

}  // namespace
int gemm_fwd_v2_small(const VuGemmFwd& p, int dtype);  // gemm_fwd2.hip
int gemm_fwd_v7_bm(const VuGemmFwd& p, int dtype);     // gemm_fwd7.hip
int cu_count4() {  // compute units of the current device (persistent grid)
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}
namespace {

template <int BN>
int64_t tile_count(const VuGemmFwd& p) {
  const VuGather& g = p.a;
  return (int64_t)g.N * (g.H / PP<BN>::TH) * (g.W / PP<BN>::TW) * (p.ncol / BN);
}

Plan plan(const VuGemmFwd& p) {
  const VuGather& g = p.a;
  const int chunks = g.C / 32;
  Plan r{pick_bn(p), 1};
  if (r.bn) {
    if (g_splitk >= 2) r.ks = g_splitk < chunks ? g_splitk : chunks;
    return r;
  }
  const int maxks = chunks / (g_split_min_chunks > 0 ? g_split_min_chunks : 1);
  if (g_splitk == 0 || maxks < 2) return r;
  // small grids the 128x64 v2 tiles fill go there -- unless K is long
  // (>= 512 input channels: the UNet down4 input gradient, 1024 -> 512 at
  // 32^2, ran 201 us on v2 tiles vs 80 us split 4 ways here, tools/enc_bench.py)
  if (g_splitk == 1 && g.C < 512 && gemm_fwd_v2_small(p, VU_BF16)) return r;
  // ... and those the small-grid kernel takes (gemm_fwd7.hip, VU_TUNE_V7)
  if (g_splitk == 1 && gemm_fwd_v7_bm(p, VU_BF16)) return r;
  int bn = 0;
  int64_t blocks = 0;
  if (tiles_ok<256>(p)) {
    bn = 256;
    blocks = tile_count<256>(p);
  } else if (tiles_ok<128>(p)) {
    bn = 128;
    blocks = tile_count<128>(p);
  } else if (p.ncol % 128 != 0 && tiles_ok<64>(p)) {
    // 64- but not 128-multiple column counts (the 832-column decoder concat
    // gradient at 32^2: it fell to the v2 small-grid gather, 377 TFLOP/s)
    bn = 64;
    blocks = tile_count<64>(p);
  } else {
    return r;
  }
  if (blocks < 16) return r;
  int ks = (int)((g_min_blocks + blocks - 1) / blocks);
  if (g_splitk >= 2) ks = g_splitk;
  if (ks > maxks) ks = maxks;
  if (ks < 2) return r;
  return Plan{bn, ks};
}

template <int BN>
int launch(const VuGemmFwd& p, int ks, hipStream_t st) {
  const VuGather& g = p.a;
  const int64_t mt = (int64_t)g.N * (g.H / PP<BN>::TH) * (g.W / PP<BN>::TW);
  const int64_t tiles = mt * (p.ncol / BN);
  if (ks <= 1) {
    VuGemmFwd q = p;
    q.ksplit = 1;
    if (p.zbias && p.relu)  // folded eval-BN DecoderBlock conv1 (inference): bias table + ReLU epilogue
      hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, false, true, BN != 64, true>), dim3((unsigned)tiles),
                         dim3(512), 0, st, q);
    else if (p.zbias)
      hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, false, false, BN != 64, true>), dim3((unsigned)tiles),
                         dim3(512), 0, st, q);
    else if (p.bnb_part) {
      // (the 64-column tiles spill with the FULL step's extra fragments)
      if constexpr (BN != 64) {
        if (g_pp_full)
          hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, true, false, true>), dim3((unsigned)tiles), dim3(512), 0, st,
                             q);
        else
          hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, true>), dim3((unsigned)tiles), dim3(512), 0, st, q);
      } else {
        hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, true>), dim3((unsigned)tiles), dim3(512), 0, st, q);
      }
    }
    else if (p.relu)
      hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, false, true>), dim3((unsigned)tiles), dim3(512), 0, st, q);
    else if (BN != 64 && g_pp_full && (g_pp_persist >= 2 || (g_pp_persist == 1 && tiles > cu_count4()))) {
      // persistent walk: one block per CU (g_pp_persist >= 2: the grid capped at that many blocks, tests)
      const int64_t grid = g_pp_persist >= 2 ? (tiles < g_pp_persist ? tiles : g_pp_persist) : cu_count4();
      hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, false, false, BN != 64, false, BN != 64>),
                         dim3((unsigned)grid), dim3(512), 0, st, q);
    }
    else if (BN != 64 && g_pp_full)  // (BN = 64 FULL spills 11 VGPRs: up4.1 fwd 341 -> 389 us, profiles/r6z_ab_pp64_full.txt)
      hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, false, false, BN != 64>), dim3((unsigned)tiles), dim3(512), 0,
                         st, q);

    else
      hipLaunchKernelGGL((conv3x3_pp_kernel<BN, false, false>), dim3((unsigned)tiles), dim3(512), 0, st, q);
    return (int)hipGetLastError();
  }
  const dim3 grid((unsigned)(tiles * ks));
  if (!p.workspace) return (int)hipErrorInvalidValue;
  VuGemmFwd q = p;
  q.ksplit = ks;
  if (BN == 256 && g_pp_full)  // (the 128-column split variant spills with the extra fragments)
    hipLaunchKernelGGL((conv3x3_pp_kernel<BN, true, false, false, BN == 256>), grid, dim3(512), 0, st, q);
  else
    hipLaunchKernelGGL((conv3x3_pp_kernel<BN, true, false>), grid, dim3(512), 0, st, q);
  const int64_t M = (int64_t)g.N * g.H * g.W;
  hipLaunchKernelGGL(splitk_finish_kernel, dim3((unsigned)((M / 128) * (p.ncol / 64))), dim3(256), 0, st, q);
  return (int)hipGetLastError();
}

bool operands_ok(const VuGemmFwd& p, int dtype) {
  const VuGather& g = p.a;
  if (dtype != VU_BF16 || p.out_mode != 0) return false;
  if (g.R != 3 || g.S != 3 || g.sy != 1 || g.sx != 1 || g.dy != 1 || g.dx != 1 || g.oy != -1 ||
      g.ox != -1 || g.Hs != g.H || g.Ws != g.W)
    return false;
  if (g.C % 32 != 0) return false;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.cend[t] % 32 != 0 || g.stride[t] % 8 != 0) return false;
  if (p.out_stride % 8 != 0 || p.out_coff % 8 != 0 || p.ldb % 8 != 0) return false;
  if ((int64_t)g.N * g.H * g.W >= (int64_t)1 << 31) return false;
  return true;
}

}  // namespace

// Row tile (BM) when the ping-pong kernel serves this problem, else 0: bf16,
// 3x3 stride-1 pad-1 gather over same-size sources, 32-channel aligned source
// groups, plain NHWC output with 8-element aligned strides.  BatchNorm
// statistics come per 128 pixels (one wave tile, or one finish-kernel tile).
int gemm_fwd_v4_bm(const VuGemmFwd& p, int dtype) {
  return operands_ok(p, dtype) && plan(p).bn ? 128 : 0;
}

// BatchNorm-backward partial row tile (128: one wave tile, or one finish
// tile) when the ping-pong kernel serves the problem and its output is a
// whole plain tensor (no accumulate, no channel offset), else 0.
int gemm_fwd_v4_bnb_tile(const VuGemmFwd& p, int dtype) {
  if (!gemm_fwd_v4_bm(p, dtype) || p.accumulate || p.out_coff != 0) return 0;
  if (p.bnb_xstride % 8 != 0) return 0;
  return 128;
}

// fp32 split-K slab bytes the ping-pong kernel needs for this problem (0 = none)
// the deterministic split-K finish over p.ksplit fp32 slabs in p.workspace
// (also used by the v2 small-grid split, gemm_fwd2.hip)
int splitk_finish_launch(const VuGemmFwd& p, hipStream_t st) {
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  if (M % 128 != 0 || p.ncol % 64 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(splitk_finish_kernel, dim3((unsigned)((M / 128) * (p.ncol / 64))), dim3(256), 0, st, p);
  return (int)hipGetLastError();
}

int64_t gemm_fwd_v4_workspace(const VuGemmFwd& p, int dtype) {
  if (!operands_ok(p, dtype)) return 0;
  const Plan r = plan(p);
  if (!r.bn || r.ks <= 1) return 0;
  return (int64_t)r.ks * p.a.N * p.a.H * p.a.W * p.ncol * (int64_t)sizeof(float);
}

int gemm_fwd_v4_launch(const VuGemmFwd& p, hipStream_t st) {
  const Plan r = plan(p);
  switch (r.bn) {
    case 256: return launch<256>(p, r.ks, st);
    case 128: return launch<128>(p, r.ks, st);
    case 64: return launch<64>(p, r.ks, st);
    default: return (int)hipErrorInvalidValue;
  }
}

int conv_fp8_tune(int key, int value);     // conv_fp8.hip
int gemm_stream_tune(int key, int value);  // gemm_stream.hip
int gemm_fwd_v2_tune(int key, int value);  // gemm_fwd2.hip
int gemm_fwd_v5_tune(int key, int value);  // gemm_fwd5.hip
int gemm_fwd_v6_tune(int key, int value);  // gemm_fwd6.hip
int gemm_fwd_v7_tune(int key, int value);  // gemm_fwd7.hip
int gemm_wgrad_v3_tune(int key, int value);  // gemm_wgrad3.hip
int gemm_wgrad_v2_tune(int key, int value);  // gemm_wgrad2.hip
int bn_tune(int key, int value);           // bn.hip
int attn_tune(int key, int value);         // attention.hip
extern int g_tune_gen;                     // gemm_fwd.hip
extern int g_tune_slab4;                   // gemm_wgrad.hip
extern int g_v2_cfg;                       // gemm_fwd2.hip

namespace {
int g_tune_unsafe = 0;  // VU_TUNE_UNSAFE
int g_xm_modes = 0;     // vu_gemm_experiment_modes()
int xm_bit(int key) {
  return key == VU_TUNE_V6_XM ? 1 : key == VU_TUNE_V7_XM ? 2 : key == VU_TUNE_FP8_XM ? 4 : 0;
}
int set_tuning(int key, int value);
}  // namespace

// Experiment modes (timing decompositions, several with wrong results by
// design) are refused unless VU_TUNE_UNSAFE was set first, and
// tracked so that a benchmark can refuse to report while one is active.
extern "C" int vu_gemm_set_tuning(int key, int value) {
  if (key == VU_TUNE_UNSAFE) {
    g_tune_unsafe = value != 0;
    return 0;
  }
  const int bit = xm_bit(key);
  if (bit && value != 0 && !g_tune_unsafe) return (int)hipErrorInvalidValue;
  const int r = set_tuning(key, value);
  if (r == 0 && bit) g_xm_modes = value != 0 ? (g_xm_modes | bit) : (g_xm_modes & ~bit);
  return r;
}

extern "C" int vu_gemm_experiment_modes(void) { return g_xm_modes; }

namespace {
int set_tuning(int key, int value) {
  if (key == VU_TUNE_V4_MIN_BLOCKS) {
    g_min_blocks = value;
    return 0;
  }
  if (key == VU_TUNE_V4_SPLITK) {
    g_splitk = value;
    return 0;
  }
  if (key == VU_TUNE_PP_FULL) {
    g_pp_full = value;
    return 0;
  }
  if (key == VU_TUNE_PP_PERSIST) {
    g_pp_persist = value;
    return 0;
  }
  if (key == VU_TUNE_V4_SPLIT_CHUNKS) {
    g_split_min_chunks = value;
    return 0;
  }
  if (key == VU_TUNE_GEN) {
    if (value < 1 || value > 4) return (int)hipErrorInvalidValue;
    g_tune_gen = value;
    return 0;
  }
  if (key == VU_TUNE_SLAB4) {
    g_tune_slab4 = value;
    return 0;
  }
  if (key == VU_TUNE_V2_CFG) {
    if (value < 0 || value > 2) return (int)hipErrorInvalidValue;
    g_v2_cfg = value;
    return 0;
  }
  if (conv_fp8_tune(key, value) == 0 || gemm_stream_tune(key, value) == 0 || gemm_fwd_v2_tune(key, value) == 0 ||
      gemm_fwd_v5_tune(key, value) == 0 || gemm_fwd_v6_tune(key, value) == 0 || gemm_fwd_v7_tune(key, value) == 0 ||
      gemm_wgrad_v3_tune(key, value) == 0 || gemm_wgrad_v2_tune(key, value) == 0 || bn_tune(key, value) == 0 ||
      attn_tune(key, value) == 0)
    return 0;
  return (int)hipErrorInvalidValue;
}
}  // namespace
