// 3x3 / stride-1 / pad-1 convolution with 64 input and 64 output channels
// ("v6", bf16): the second conv of the 512^2-level DoubleConvs (inc, up4:
// unet_parts.py:43) and the input gradient of every 64 -> 64 conv (the same
// shape with flipped weights).
//
// Why a separate kernel: with K = 576 a tile of these layers is 9-18 K-steps
// long, so the halo / ping-pong kernels (one tile per block) spend a large
// part of every tile in its prologue (first halo), its weight stream and its
// LDS-staged epilogue: 740-820 TFLOP/s in the bench step against
// 1,100-1,500 on the deeper layers.  Here the whole weight matrix (64 x 576
// bf16 = 72 KiB) is loaded into LDS ONCE per block and stays resident, and a
// persistent block walks its tiles as one stream of (tile, 32-channel chunk)
// groups:
//
//   * tile = 16 x 32 pixels x 64 channels; wave w owns image rows 2w, 2w+1
//     (4 pixel fragments x 4 channel fragments of v_mfma_f32_16x16x32_bf16,
//     64 accumulator registers);
//   * the only DMA stream is the halo: while a group computes from one
//     18 x 34-pixel chunk buffer, the next group's chunk (the second chunk of
//     this tile or the first of the next tile) lands in the other one
//     (global_load_lds_dwordx4), so the pipeline never drains at a tile seam;
//   * MFMA operands are (weights, pixels) with the weight rows read in a
//     permuted order, so a lane's accumulators hold 16 consecutive output
//     channels of one pixel, stored straight from registers (no LDS staging,
//     no barrier; 64 contiguous bytes per pixel and store), with the BatchNorm partial
//     statistics of each wave's 64 pixels from a DPP butterfly transpose-
//     reduce (same contract as the other kernels: per-tile sum + centered M2
//     of the rounded values);
//   * LDS images are conflict-free for every fragment read: weight rows XOR
//     their 16-byte pieces with wswz(row); halo pixel P keeps its piece k at
//     position (k + 2 * ((P >> 2) & 1)) & 3, which spreads the 16 lanes of
//     every ds_read_b128 lane group over distinct banks for any tap shift.
#include "common.h"
#include "../../include/vaeunet.h"

static __device__ __attribute__((aligned(16))) uint32_t v6_zero_page[16];

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int TH = 16, TW = 32;
constexpr int HWD = TW + 2;                  // halo row (pixels)
constexpr int HP = (TH + 2) * HWD;           // 612 halo pixels
constexpr int HPIECES = HP * 4;              // 16-byte pieces of one 32-channel chunk
constexpr int NHR = (HPIECES + 511) / 512;   // DMA rounds per chunk (5)
constexpr int HBUF = NHR * 512 * 16;         // chunk buffer, padded to whole DMA rounds
constexpr int WROW = 576 * 2;                // one output channel's weights (bytes)
constexpr int WBYTES = 64 * WROW;            // 72 KiB, resident
constexpr int WROUNDS = WBYTES / 16 / 512;   // 9
constexpr int LDS_BYTES = WBYTES + 2 * HBUF;
static_assert(LDS_BYTES <= 163840, "LDS");
static_assert(WROUNDS * 512 * 16 == WBYTES, "weight DMA rounds");

template <int N>
VU_DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// a workgroup barrier that neither drains the memory counters nor lets the
// compiler move LDS reads, DMA issues or MFMAs across it
VU_DEV void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// weight-row piece swizzle: with the permuted fragment rows below (lane row
// rr of fragment j = channel 16*(rr>>2) + 4j + (rr&3)) every ds_read_b128
// lane group touches 16 distinct 4-bank groups (checked for all j, tap, c)
VU_DEV int wswz(int n) { return (n + (n >> 2)) & 7; }


// ---- butterfly transpose-reduce over the 16 lanes of a DPP row ----------
// v[k] (16 slots per lane) -> lane m of the row holds the sum over the row's
// lanes of slot m: each step pairs lanes across one lane bit and halves the
// array (15 lane moves instead of 16 four-step rotate-add reductions, 64)
template <int CTRL>
VU_DEV float dmov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
VU_DEV float lx1(float v) { return dmov<0xB1>(v); }               // lane ^ 1
VU_DEV float lx2(float v) { return dmov<0x4E>(v); }               // lane ^ 2
VU_DEV float lx4(float v) { return dmov<0x1B>(dmov<0x141>(v)); }  // lane ^ 4
VU_DEV float lx8(float v) { return dmov<0x128>(v); }              // lane ^ 8 (row_ror:8)

VU_DEV float bfly16_reduce(const float (&v)[16], int lane) {
  const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
  float x[8], y[4], z[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = (b3 ? v[k + 8] : v[k]) + lx8(b3 ? v[k] : v[k + 8]);
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = (b2 ? x[k + 4] : x[k]) + lx4(b2 ? x[k] : x[k + 4]);
#pragma unroll
  for (int k = 0; k < 2; ++k) z[k] = (b1 ? y[k + 2] : y[k]) + lx2(b1 ? y[k] : y[k + 2]);
  return (b0 ? z[1] : z[0]) + lx1(b0 ? z[0] : z[1]);
}

// inverse: lane m of a row holds the value of slot m -> every lane gets all 16
VU_DEV void bfly16_bcast(float m, int lane, float (&out)[16]) {
  const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
  float z[2], y[4], x[8];
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
    out[k] = b3 ? q : x[k];
    out[k + 8] = b3 ? x[k] : q;
  }
}

// RELU: the epilogue ReLU (VuGemmFwd.relu) as a separate instantiation: the
// runtime block spilled the statistics variant (+16 % in the training step)
// XM (experiment modes, VU_TUNE_V6_XM; A/B timing only, 0 in production):
// 1 = s_setprio(1) around each tap's 16 MFMAs (the two waves of a SIMD
// otherwise free-run in the same phase); 2 = no halo DMA after the first
// (every group computes on stale buffers: the DMA-latency share); 3 = no
// statistics and the output stores predicated off by a value test the
// compiler cannot fold (the MFMAs stay live: the epilogue's share); 4 = the
// fragments read once per group, not per tap (the LDS-read share); results
// wrong in 2-4; 5 = the output stores non-temporal (results exact)
template <bool STATS, bool RELU = false, int XM = 0>
__global__ __launch_bounds__(512, 1) void conv3x3_c64_kernel(VuGemmFwd p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  char* const wl = smem;
  char* const hl = smem + WBYTES;

  const VuGather& g = p.a;
  const int H = g.H, W = g.W;
  const int txn = W / TW, per_img = txn * (H / TH);
  const int T = g.N * per_img;
  const int G = gridDim.x;  // <= T (host)
  const int lb = xcd_remap(blockIdx.x, G);
  const int ngroups = 2 * ((T - lb + G - 1) / G);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kg = lane >> 4;
  const bf16_t* const src = reinterpret_cast<const bf16_t*>(g.src[0]);
  const int64_t st = g.stride[0];
  const void* const zp = (const void*)v6_zero_page;
  // bias of this lane's channels, loaded up front: a load in the epilogue
  // would wait for the in-flight halo DMA (vmcnt is in order)
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    bv[j] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + 16 * kg + 4 * j) : f32x4{0, 0, 0, 0};

  // ---- resident weights: row n (output channel) = 576 bf16; 16-byte piece
  //      pc of row n lives at piece pc ^ wswz(n) ----
  {
    const bf16_t* bm = reinterpret_cast<const bf16_t*>(p.b);
#pragma unroll
    for (int i = 0; i < WROUNDS; ++i) {
      const int s = i * 512 + tid;
      const int n = s / 72, pc = s - (s / 72) * 72;
      const void* gp = (const void*)(bm + (int64_t)n * p.ldb + (pc ^ wswz(n)) * 8);
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(wl + (i * 512 + wid * 64) * 16), 16, 0, 0);
    }
  }
  // ---- halo of (tile t, chunk c) into buffer b ----
  auto halo = [&](int t, int c, int b) {
    const int img = t / per_img, r = t - (t / per_img) * per_img;
    const int ty = r / txn, tx = r - (r / txn) * txn;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
    const bf16_t* s0 = src + (int64_t)img * H * W * st + c * 32;
    char* dst = hl + b * HBUF;
#pragma unroll
    for (int i = 0; i < NHR; ++i) {
      if (i * 512 + wid * 64 >= HPIECES) continue;  // wave-uniform
      const int s = i * 512 + tid;
      const int P = s >> 2, pos = s & 3;
      const int hy = P / HWD, hx = P - (P / HWD) * HWD;
      const int y = y0 + hy, x = x0 + hx;
      const int k = (pos - ((P >> 1) & 2)) & 3;  // the global piece stored at position pos
      const bool ok = s < HPIECES && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      const void* gp = ok ? (const void*)(s0 + (int64_t)(y * W + x) * st + k * 8) : zp;
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(dst + (i * 512 + wid * 64) * 16), 16, 0, 0);
    }
  };

  halo(lb, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  raw_barrier();

  // B fragment j, lane row l16 = output channel n_j = 16*(l16>>2) + 4j + (l16&3),
  // so that a lane's accumulators hold 16 consecutive channels (16*kg ..):
  // K piece (tap, c, kg) of row n_j sits at piece tap*8 + ((c*4 + kg) ^ wswz(n_j))
  int boff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = 16 * (l16 >> 2) + 4 * j + (l16 & 3);
    boff[j] = n * WROW + ((kg ^ wswz(n)) << 4);
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  // the previous tile's packed output, stored one piece per tap during the
  // next group's MFMAs (a burst of stores at the group end idled the MFMA pipe)
  u32x4 pend[8];
  bf16_t* pdst = nullptr;
  bool have_pend = false;
  // ... and its BatchNorm partials (stored after the 8 output pieces: a store
  // issued before the next group's halo DMA would be waited for with it)
  float pst_sum = 0.f, pst_m2 = 0.f;
  int64_t pst_so = 0;
  auto store_stats = [&]() {
    p.stat_sum[pst_so] = pst_sum;
    p.stat_m2[pst_so] = pst_m2;
  };
  auto store_pend = [&](int q) {  // piece q = 2 * fragment + half
    bf16_t* o = pdst + ((q >> 2) * (int64_t)W + ((q >> 1) & 1) * 16) * p.out_stride + 32 * (q & 1);
    if constexpr (XM == 5)
      __builtin_nontemporal_store(pend[q], reinterpret_cast<u32x4*>(o));
    else if (XM != 3 || pend[q][0] == 0x7fc17fc1u)
      *reinterpret_cast<u32x4*>(o) = pend[q];
  };

  // the 9 taps of one group over halo buffer b, chunk c; `pending` stores
  // the previous tile's output pieces one per tap
  auto taps = [&](int b, int c, bool pending) {
    const char* hb = hl + b * HBUF;
    const int cx = c << 6;  // (c*4) XORed into the piece index: 4 pieces = 64 bytes
    u32x4 bf[4], af[4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ty = tap / 3, tx = tap - (tap / 3) * 3;
      if (tap < 8 && pending) store_pend(tap);
      if (STATS && XM != 3 && tap == 8 && pending) store_stats();
      if (XM != 4 || tap == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const u32x4*>(wl + (boff[j] ^ cx) + tap * 128);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int P = (2 * wid + (i >> 1) + ty) * HWD + (i & 1) * 16 + tx + l16;
          af[i] = *reinterpret_cast<const u32x4*>(hb + P * 64 + (((kg + ((P >> 1) & 2)) & 3) << 4));
        }
      }
      if constexpr (XM == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                              __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0);
      if constexpr (XM == 1) __builtin_amdgcn_s_setprio(0);
    }
  };

  // a block walks its tiles as (chunk 0, chunk 1) group pairs; one halo
  // buffer flip and one barrier per group
  const int ntile_blk = ngroups / 2;
  int t = lb, b = 0;
  for (int ti = 0; ti < ntile_blk; ++ti) {
    // ---- group (t, chunk 0): the other buffer takes chunk 1 of this tile ----
    if (XM != 2) halo(t, 1, b ^ 1);
    taps(b, 0, have_pend);
    // the halo was issued before the previous tile's 8 stores
    if (have_pend && XM != 3) {
      have_pend = false;
      if (STATS) wait_vm<10>(); else wait_vm<8>();
    } else {
      have_pend = false;
      wait_vm<0>();
    }
    raw_barrier();
    b ^= 1;
    // ---- group (t, chunk 1): the other buffer takes chunk 0 of the next tile ----
    const int img = t / per_img, r0 = t - (t / per_img) * per_img;
    const int ty = r0 / txn, tx = r0 - (r0 / txn) * txn;
    if (ti + 1 < ntile_blk && XM != 2) halo(t + G, 0, b ^ 1);
    taps(b, 1, false);
    // ---- epilogue of tile t from registers: acc[i][j][r] = pixel fragment
    //      i (row 2*wid + i/2, column (i&1)*16 + l16), channel 16kg + 4j + r ----
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] += bv[j];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = rnd<bf16_t>(acc[i][j][r]);
    if constexpr (RELU)
#pragma unroll
      for (int i = 0; i < 4; ++i) epi_relu(acc[i]);
    if (STATS && XM != 3) {
      // per-wave (sum, centered M2) of its 64 pixels: slot 4j + r of a lane
      // is channel 16*kg + 4j + r; after the butterfly lane (kg, l16) holds
      // slot l16, i.e. channel lane: one store per statistic
      float v[16];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[4 * j + r] = (acc[0][j][r] + acc[1][j][r]) + (acc[2][j][r] + acc[3][j][r]);
      const float ms = bfly16_reduce(v, lane);
      float mb[16];
      bfly16_bcast(ms * (1.f / 64), lane, mb);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float q = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float d = acc[i][j][r] - mb[4 * j + r];
            q += d * d;
          }
          v[4 * j + r] = q;
        }
      const float mq = bfly16_reduce(v, lane);
      pst_so = (int64_t)(t * 8 + wid) * p.ncol + lane;
      pst_sum = ms;
      pst_m2 = mq;
    }
    // stores: a lane holds channels 16kg .. 16kg+15 of its pixel (two 16-byte
    // pieces); a permlane16 + permlane32 swap regroups them so that store h
    // of lane kg writes channels 32h + 8kg .. +7: 64 contiguous bytes per
    // pixel and instruction.  Issued during the next group (store_pend).
    pdst = reinterpret_cast<bf16_t*>(p.out) + p.out_coff + 8 * kg +
           (((int64_t)img * H + ty * TH + 2 * wid) * W + tx * TW + l16) * p.out_stride;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      u32x4 cv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = acc[i][2 * h], e = acc[i][2 * h + 1];
        cv[h] = u32x4{(uint32_t)f2bf(a[0]) | ((uint32_t)f2bf(a[1]) << 16), (uint32_t)f2bf(a[2]) | ((uint32_t)f2bf(a[3]) << 16),
                      (uint32_t)f2bf(e[0]) | ((uint32_t)f2bf(e[1]) << 16), (uint32_t)f2bf(e[2]) | ((uint32_t)f2bf(e[3]) << 16)};
      }
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const auto r1 = __builtin_amdgcn_permlane16_swap(cv[0][w], cv[1][w], false, false);
        const auto r2 = __builtin_amdgcn_permlane32_swap(r1[0], r1[1], false, false);
        cv[0][w] = r2[0];
        cv[1][w] = r2[1];
      }
      pend[2 * i] = cv[0];
      pend[2 * i + 1] = cv[1];
    }
    have_pend = true;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    // the next group's halo was issued before this tile's statistics stores
    wait_vm<0>();
    raw_barrier();
    b ^= 1;
    t += G;
  }
  if (have_pend) {
#pragma unroll
    for (int q = 0; q < 8; ++q) store_pend(q);
    if (STATS && XM != 3) store_stats();
  }
}

// ---- the same tile stream with the two wave halves' epilogues staggered ----
//
// In conv3x3_c64_kernel all eight waves run the epilogue of a tile (bias,
// rounding, packing, the statistics butterflies: VALU only) together at the
// end of the chunk-1 group, so the matrix pipe of every SIMD idles through it
// while the two waves of the SIMD contend for VALU issue.  Here it is split:
//
//   * light part, end of the chunk-1 group (all waves): bias, rounding, ReLU,
//     bf16 packing into the 8 output pieces (the same registers the round-5
//     kernel kept its deferred stores in), accumulators cleared;
//   * heavy part, in the NEXT tile's chunk-0 group: the 8 output stores and
//     the BatchNorm statistics computed from the packed pieces -- placed at
//     opposite ends by the two waves of a SIMD (w and w + 4):
//
//       waves 4-7:  [heavy part of t] [chunk-0 taps of t+1]
//       waves 0-3:  [chunk-0 taps of t+1] [heavy part of t]
//
//     so each half's heavy part runs beside the partner's MFMAs
//     (MI355X_MICROARCH.md "Two waves per SIMD" item 9: split roles by wave
//     number >= 4).
//
// After the permlane regroup a lane holds channels 32h + 8kg + e (piece h,
// element e) of its pixel, 16 channels as before, so the butterfly over the 16
// lanes of a row gives lane m the sums of slot m = channel 32(m >> 3) + 8kg +
// (m & 7): the same additions in the same tree order as the round-5 kernel
// (which kept slot m = channel 16kg + m) -- bit-identical outputs and
// statistics, only the statistics' store addresses are permuted.
template <bool STATS, bool RELU = false>
__global__ __launch_bounds__(512, 1) void conv3x3_c64s_kernel(VuGemmFwd p) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES + 64 * 4];
  char* const wl = smem;
  char* const hl = smem + WBYTES;
  float* const bias_l = reinterpret_cast<float*>(smem + LDS_BYTES);

  const VuGather& g = p.a;
  const int H = g.H, W = g.W;
  const int txn = W / TW, per_img = txn * (H / TH);
  const int T = g.N * per_img;
  const int G = gridDim.x;  // <= T (host)
  const int lb = xcd_remap(blockIdx.x, G);
  const int ntile_blk = (T - lb + G - 1) / G;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool late = wid >= 4;  // waves 4-7: heavy part first in the chunk-0 group
  const int l16 = lane & 15, kg = lane >> 4;
  const bf16_t* const src = reinterpret_cast<const bf16_t*>(g.src[0]);
  const int64_t st = g.stride[0];
  const void* const zp = (const void*)v6_zero_page;
  const bool has_bias = p.bias != nullptr;
  if (tid < 64) bias_l[tid] = has_bias ? p.bias[tid] : 0.f;  // read from LDS in the epilogue

  {
    const bf16_t* bm = reinterpret_cast<const bf16_t*>(p.b);
#pragma unroll
    for (int i = 0; i < WROUNDS; ++i) {
      const int s = i * 512 + tid;
      const int n = s / 72, pc = s - (s / 72) * 72;
      const void* gp = (const void*)(bm + (int64_t)n * p.ldb + (pc ^ wswz(n)) * 8);
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(wl + (i * 512 + wid * 64) * 16), 16, 0, 0);
    }
  }
  auto halo = [&](int t, int c, int b) {
    const int img = t / per_img, r = t - (t / per_img) * per_img;
    const int ty = r / txn, tx = r - (r / txn) * txn;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
    const bf16_t* s0 = src + (int64_t)img * H * W * st + c * 32;
    char* dst = hl + b * HBUF;
#pragma unroll
    for (int i = 0; i < NHR; ++i) {
      if (i * 512 + wid * 64 >= HPIECES) continue;  // wave-uniform
      const int s = i * 512 + tid;
      const int P = s >> 2, pos = s & 3;
      const int hy = P / HWD, hx = P - (P / HWD) * HWD;
      const int y = y0 + hy, x = x0 + hx;
      const int k = (pos - ((P >> 1) & 2)) & 3;
      const bool ok = s < HPIECES && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      const void* gp = ok ? (const void*)(s0 + (int64_t)(y * W + x) * st + k * 8) : zp;
      __builtin_amdgcn_global_load_lds(gp, (lds_void*)(dst + (i * 512 + wid * 64) * 16), 16, 0, 0);
    }
  };

  halo(lb, 0, 0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // (+ the bias_l stores)
  raw_barrier();

  int boff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = 16 * (l16 >> 2) + 4 * j + (l16 & 3);
    boff[j] = n * WROW + ((kg ^ wswz(n)) << 4);
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
  u32x4 pend[8];  // tile t's packed output pieces (q = 2 * fragment + half)

  auto taps = [&](int b, int c) {
    const char* hb = hl + b * HBUF;
    const int cx = c << 6;
    u32x4 bf[4], af[4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ty = tap / 3, tx = tap - (tap / 3) * 3;
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const u32x4*>(wl + (boff[j] ^ cx) + tap * 128);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int P = (2 * wid + (i >> 1) + ty) * HWD + (i & 1) * 16 + tx + l16;
        af[i] = *reinterpret_cast<const u32x4*>(hb + P * 64 + (((kg + ((P >> 1) & 2)) & 3) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                              __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0);
    }
  };

  // light part: acc -> pend (bias, bf16 rounding, ReLU, 64-byte regroup); acc cleared
  auto light = [&]() {
    if (has_bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 bvj = *reinterpret_cast<const f32x4*>(bias_l + 16 * kg + 4 * j);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] += bvj;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (RELU) {
        f32x4 z[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) z[j][r] = rnd<bf16_t>(acc[i][j][r]);
        epi_relu(z);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = z[j];
      }
      u32x4 cv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = acc[i][2 * h], e = acc[i][2 * h + 1];
        cv[h] = u32x4{(uint32_t)f2bf(a[0]) | ((uint32_t)f2bf(a[1]) << 16), (uint32_t)f2bf(a[2]) | ((uint32_t)f2bf(a[3]) << 16),
                      (uint32_t)f2bf(e[0]) | ((uint32_t)f2bf(e[1]) << 16), (uint32_t)f2bf(e[2]) | ((uint32_t)f2bf(e[3]) << 16)};
      }
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const auto r1 = __builtin_amdgcn_permlane16_swap(cv[0][w], cv[1][w], false, false);
        const auto r2 = __builtin_amdgcn_permlane32_swap(r1[0], r1[1], false, false);
        cv[0][w] = r2[0];
        cv[1][w] = r2[1];
      }
      pend[2 * i] = cv[0];
      pend[2 * i + 1] = cv[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    }
  };

  // heavy part of tile t from pend: the 8 output stores, then the statistics
  auto heavy = [&](int t) {
    const int img = t / per_img, r0 = t - (t / per_img) * per_img;
    const int ty = r0 / txn, tx = r0 - (r0 / txn) * txn;
    bf16_t* const pdst = reinterpret_cast<bf16_t*>(p.out) + p.out_coff + 8 * kg +
                         (((int64_t)img * H + ty * TH + 2 * wid) * W + tx * TW + l16) * p.out_stride;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      bf16_t* o = pdst + ((q >> 2) * (int64_t)W + ((q >> 1) & 1) * 16) * p.out_stride + 32 * (q & 1);
      *reinterpret_cast<u32x4*>(o) = pend[q];
    }
    if (STATS) {
      // slot 8h + e of a lane = channel 32h + 8kg + e of its pixel, pixel
      // fragments i = q >> 1 (piece q = 2i + h)
      auto val = [&](int i, int h, int e) {
        const uint32_t w = pend[2 * i + h][e >> 1];
        return __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
      };
      float v[16];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[8 * h + e] = (val(0, h, e) + val(1, h, e)) + (val(2, h, e) + val(3, h, e));
      const float ms = bfly16_reduce(v, lane);
      float mb[16];
      bfly16_bcast(ms * (1.f / 64), lane, mb);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float q = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float d = val(i, h, e) - mb[8 * h + e];
            q += d * d;
          }
          v[8 * h + e] = q;
        }
      const float mq = bfly16_reduce(v, lane);
      const int ch = 32 * (l16 >> 3) + 8 * kg + (l16 & 7);
      const int64_t so = (int64_t)(t * 8 + wid) * p.ncol + ch;
      p.stat_sum[so] = ms;
      p.stat_m2[so] = mq;
    }
  };

  int t = lb, b = 0;
  for (int ti = 0; ti < ntile_blk; ++ti) {
    // ---- chunk-0 group (+ the previous tile's heavy part) ----
    halo(t, 1, b ^ 1);
    const bool ep = ti > 0;
    if (ep && late) heavy(t - G);
    taps(b, 0);
    if (ep && !late) heavy(t - G);
    // the halo was issued before the heavy part's 8 output (+ 2 statistics) stores
    if (ep) {
      if (STATS) wait_vm<10>(); else wait_vm<8>();
    } else {
      wait_vm<0>();
    }
    raw_barrier();
    b ^= 1;
    // ---- chunk-1 group, then the light part of this tile ----
    if (ti + 1 < ntile_blk) halo(t + G, 0, b ^ 1);
    taps(b, 1);
    light();
    wait_vm<0>();
    raw_barrier();
    b ^= 1;
    t += G;
  }
  if (ntile_blk > 0) heavy(t - G);
}

int cu_count6() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

int g_v6_xm = 0;  // VU_TUNE_V6_XM (experiment modes of conv3x3_c64_kernel)
int g_v6_stag = 1;  // VU_TUNE_V6_STAG: 1 = the staggered-epilogue kernel (conv3x3_c64s_kernel)
int g_v6 = 1;  // VU_TUNE_V6: 0 off, 1 on (grids of >= 1 tile per CU), k >= 2 on with the grid capped at k

}  // namespace

// Statistics row tile (64) when v6 serves this problem, else 0.
int gemm_fwd_v6_bm(const VuGemmFwd& p, int dtype) {
  if (g_v6 == 0 || dtype != VU_BF16 || p.out_mode != 0 || p.accumulate) return 0;
  const VuGather& g = p.a;
  if (g.R != 3 || g.S != 3 || g.sy != 1 || g.sx != 1 || g.dy != 1 || g.dx != 1 || g.oy != -1 || g.ox != -1 ||
      g.Hs != g.H || g.Ws != g.W)
    return 0;
  if (g.nsrc != 1 || g.C != 64 || g.cend[0] != 64) return 0;
  // wider outputs without statistics (the input gradient of a 128 -> 64 concat
  // conv, up4.1: 64 -> 128 channels at 512^2) as one launch per 64-column
  // slice: K = 576 is too short for the ping-pong tiles (922 TFLOP/s there)
  if (p.ncol != 64 && (p.ncol % 64 != 0 || p.ncol > 256 || p.stat_sum || p.bnb_part || p.bias)) return 0;
  if (g.H % TH != 0 || g.W % TW != 0) return 0;
  if (g.stride[0] % 8 != 0 || p.out_stride % 8 != 0 || p.out_coff % 8 != 0 || p.ldb % 8 != 0 || p.ldb < 576)
    return 0;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  if (M >= ((int64_t)1 << 31)) return 0;
  const int64_t T = M / (TH * TW);
  // at least one tile per block (ResNet34 layer1: 64 -> 64 at 128^2, B = 8:
  // 256 tiles, 3-4 % faster per launch than the v3 halo kernel; round 5)
  if (g_v6 == 1 && T < (int64_t)cu_count6()) return 0;
  return 64;
}

// BatchNorm-backward partials are not emitted here (0): at 512^2 with 64
// channels this kernel already moves ~3.7 TB/s, and reading the BN input in
// its epilogue (+268 MB per launch) plus the partial sums cost more than the
// separate reduction pass they replace (measured: +100 us per launch against
// the 97 us pass; profiles/r3_prof_bnb_fusion.txt).
int gemm_fwd_v6_bnb_tile(const VuGemmFwd& p, int dtype) {
  (void)p;
  (void)dtype;
  return 0;
}

int gemm_fwd_v6_launch(const VuGemmFwd& p, hipStream_t st) {
  const int64_t T = (int64_t)p.a.N * p.a.H * p.a.W / (TH * TW);
  int64_t grid = T < cu_count6() ? T : cu_count6();
  if (g_v6 >= 2 && grid > g_v6) grid = g_v6;
  if (p.bnb_part) return (int)hipErrorInvalidValue;
  if (p.ncol > 64) {
    // one launch per 64-column slice: weight rows and output channels offset
    for (int c0 = 0; c0 < p.ncol; c0 += 64) {
      VuGemmFwd q = p;
      q.ncol = 64;
      q.b = reinterpret_cast<const bf16_t*>(p.b) + (int64_t)c0 * p.ldb;
      q.out_coff = p.out_coff + c0;
      if (int e = gemm_fwd_v6_launch(q, st)) return e;
    }
    return 0;
  }
  if (g_v6_stag && g_v6_xm == 0) {
    if (p.stat_sum) {
      if (p.relu) hipLaunchKernelGGL((conv3x3_c64s_kernel<true, true>), dim3((unsigned)grid), dim3(512), 0, st, p);
      else hipLaunchKernelGGL(conv3x3_c64s_kernel<true>, dim3((unsigned)grid), dim3(512), 0, st, p);
    } else {
      if (p.relu) hipLaunchKernelGGL((conv3x3_c64s_kernel<false, true>), dim3((unsigned)grid), dim3(512), 0, st, p);
      else hipLaunchKernelGGL(conv3x3_c64s_kernel<false>, dim3((unsigned)grid), dim3(512), 0, st, p);
    }
    return (int)hipGetLastError();
  }
  if (p.stat_sum)
    if (p.relu) hipLaunchKernelGGL((conv3x3_c64_kernel<true, true>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 1) hipLaunchKernelGGL((conv3x3_c64_kernel<true, false, 1>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 2) hipLaunchKernelGGL((conv3x3_c64_kernel<true, false, 2>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 3) hipLaunchKernelGGL((conv3x3_c64_kernel<true, false, 3>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 4) hipLaunchKernelGGL((conv3x3_c64_kernel<true, false, 4>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 5) hipLaunchKernelGGL((conv3x3_c64_kernel<true, false, 5>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else hipLaunchKernelGGL(conv3x3_c64_kernel<true>, dim3((unsigned)grid), dim3(512), 0, st, p);
  else
    if (p.relu) hipLaunchKernelGGL((conv3x3_c64_kernel<false, true>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 1) hipLaunchKernelGGL((conv3x3_c64_kernel<false, false, 1>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 2) hipLaunchKernelGGL((conv3x3_c64_kernel<false, false, 2>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 3) hipLaunchKernelGGL((conv3x3_c64_kernel<false, false, 3>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 4) hipLaunchKernelGGL((conv3x3_c64_kernel<false, false, 4>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else if (g_v6_xm == 5) hipLaunchKernelGGL((conv3x3_c64_kernel<false, false, 5>), dim3((unsigned)grid), dim3(512), 0, st, p);
    else hipLaunchKernelGGL(conv3x3_c64_kernel<false>, dim3((unsigned)grid), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

int gemm_fwd_v6_tune(int key, int value) {
  if (key == VU_TUNE_V6_XM) {
    if (value < 0 || value > 5) return (int)hipErrorInvalidValue;
    g_v6_xm = value;
    return 0;
  }
  if (key == VU_TUNE_V6) {
    g_v6 = value < 0 ? 0 : value;
    return 0;
  }
  if (key == VU_TUNE_V6_STAG) {
    g_v6_stag = value != 0;
    return 0;
  }
  return -1;
}
