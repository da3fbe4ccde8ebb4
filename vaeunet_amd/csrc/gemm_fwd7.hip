// 3x3 / stride-1 / pad-1 convolution for SMALL GRIDS ("v7", bf16): the
// ResNet34 encoder of UNetResNet (unet_resnet.py:131-137, torchvision-style
// BasicBlocks at 64^2 / 32^2 / 16^2 for a 512^2 input) and the other 3x3
// layers whose 256-pixel tiles do not fill the chip.
//
// What bounds these layers is not the MFMA rate but the bytes a CU must move
// into LDS per flop.  The round-2 small-grid mode (v2, 128 x 64 tiles of an
// im2col gather) loads every input pixel nine times (once per tap): 24 KB per
// 64-deep K step per block, ~94 B/clk per CU at the MFMA rate against the
// ~30-37 B/clk a CU's L2 -> LDS DMA sustains (MI355X_MICROARCH.md "Indexed
// rows", "ldsdma-fill"), so it ran at 0.10-0.13 of the bf16 roof.  Here:
//
//   * halo tiling as the ping-pong kernel (gemm_fwd4.hip): a block owns 128
//     output pixels (4 x 32, or 8 x 16 for 16-pixel-wide images) x BN output
//     channels; per 32-channel chunk the (TH+2) x (TW+2) halo lands in LDS
//     once and the nine taps read it in place (1.4-1.6x instead of 9x the
//     input bytes), weights stream per tap through an NBW-slot ring;
//   * a 128-pixel tile keeps enough blocks to fill 256 CUs without split-K
//     (64^2: 512 blocks, 32^2: 256) -- and without its fp32 slabs -- but one
//     4-wave tile per CU leaves each SIMD a single MFMA stream.  So the block
//     has 8 waves in two K GROUPS: group 0 takes the even chunks of the
//     block's K range, group 1 the odd ones, each with its own halo and
//     weight images, on the SAME output tile; the groups run one barrier
//     apart (group 1 reads fragments while group 0 issues MFMAs and vice
//     versa: the ping-pong of gemm_fwd4.hip) and their fp32 accumulators are
//     summed through LDS once at the end (fixed order: deterministic);
//   * DMA roles as gemm_fwd4.hip (vmcnt is in-order per wave): group 0's
//     waves stream both groups' weights and wait for them per step, group
//     1's waves stream both groups' next-chunk halos and wait once per chunk
//     pair;
//   * each wave owns 32 pixels x BN channels (2 x BN/16 fragments of
//     v_mfma_f32_16x16x32_bf16, operands (weights, pixels): a lane's
//     accumulator holds 4 consecutive channels of one pixel);
//   * epilogue (group 0): bias, storage rounding, BatchNorm (sum, centered
//     M2) per 128-pixel tile (per-wave DPP row sums combined with Chan's
//     formula across the four waves), optional accumulate, 16-byte stores of
//     whole pixel rows staged through LDS; or (SPLIT) the fp32 tile to a
//     split-K slab for splitk_finish_kernel (gemm_fwd4.hip), for the 16^2
//     level whose 128 tiles are half a chip.
#include "common.h"
#include "../../include/vaeunet.h"

static __device__ __attribute__((aligned(16))) uint32_t vu_zero_page7[16];
// XM 5 (timing diagnostic): per wave of blocks < SG_DBG_BLOCKS, cycle totals of
// the phases [prologue, fragment reads + DMA waits, barrier 1, MFMA issue,
// barrier 2, epilogue, steps, 0] (tools/enc_bench.py --phases)
constexpr int SG_DBG_BLOCKS = 64;
static __device__ unsigned long long vu_sg_dbg[SG_DBG_BLOCKS * 8 * 8];

namespace {

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
VU_DEV void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

VU_DEV void sg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Fragment reads as inline asm: through plain LDS loads the compiler's
// waitcnt pass, which cannot see the explicit lgkmcnt wait of phase 1, puts an
// s_waitcnt lgkmcnt(0) in front of the first MFMA of phase 2 -- right after
// the NEXT step's reads were issued -- and the read latency is exposed again.
// Ordering is explicit instead: lgkmcnt wait + tie() before the barrier.
VU_DEV u32x4 lds_rd(uint32_t a) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
template <int OFF>
VU_DEV u32x4 lds_rd_off(uint32_t a) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}
VU_DEV void tie(u32x4& v) { asm volatile("" : "+v"(v)); }
VU_DEV uint32_t lds_addr(const char* p) { return (uint32_t)(uintptr_t)(const lds_void*)p; }

template <int R>
VU_DEV float ror_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xf, 0xf, false));
}
VU_DEV float row16_sum(float v) { return ror_add<1>(ror_add<2>(ror_add<4>(ror_add<8>(v)))); }

template <int TW, int BN, int NBW>
struct SG {
  static constexpr int TH = 128 / TW;
  static constexpr int HW = TW + 2, HP = (TH + 2) * HW;
  static constexpr int HALO = HP * 64;           // one group's chunk halo (bytes)
  static constexpr int HPIECES = HP * 4;         // its 16-byte pieces
  static constexpr int NH = (2 * HPIECES + 255) / 256;  // halo DMA slots per loader thread
  static constexpr int WTAP = BN * 64;           // one group's weights of one tap
  static constexpr int SLOT = 3 * 2 * WTAP;      // ring slot: a tap row (3 taps) of both groups
  static constexpr int LB = SLOT / 16 / 256;     // weight DMA slots per loader thread per step
  static constexpr int NJ = BN / 16;
  static constexpr int MAIN = 4 * HALO + NBW * SLOT;
  // epilogue: group 1's accumulators, 4 staging strips, BN statistics
  // epilogue (round 4): each of the 8 waves finalizes one 16-pixel fragment
  static constexpr int RED = 8 * (NJ * 4) * 64 * 4;
  static constexpr int SPITCH = BN * 2 + 16;
  static constexpr int STG = 16 * SPITCH;
  static constexpr int STAT = 8 * BN * 2 * 4;
  static constexpr int EPI = RED + 8 * STG + STAT;
  static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
};

// XM (experiment modes, A/B runs only; 0 in production): 2 = no DMA inside
// the loop, 4 = no loop (launch + prologue + epilogue), 5 = production
// schedule with per-phase cycle counters (vu_sg_dbg)
template <int TW, int BN, int NBW, bool SPLIT, int XM = 0, bool RELU = false>  // RELU: epilogue ReLU
__global__ __launch_bounds__(512, 1) void conv3x3_sg_kernel(VuGemmFwd p) {
  constexpr bool TMR = XM == 5;
  unsigned long long tph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;
  auto tmark = [&](int k) {
    if constexpr (TMR) {
      const unsigned long long t = __builtin_readcyclecounter();
      tph[k] += t - tlast;
      tlast = t;
    }
  };
  if constexpr (TMR) tlast = __builtin_readcyclecounter();
  using G = SG<TW, BN, NBW>;
  constexpr int TH = G::TH, HW = G::HW, HALO = G::HALO, HPIECES = G::HPIECES, NH = G::NH;
  constexpr int WTAP = G::WTAP, SLOT = G::SLOT, LB = G::LB, NJ = G::NJ;
  constexpr int PD = NBW - 1;  // weight prefetch distance (steps)
  static_assert(G::LDS <= 163840, "LDS");
  static_assert(LB == 6 && (PD - 1) * LB <= 63 && PD <= 3, "DMA schedule");
  static_assert(TW == 16 || TW == 32, "tile geometry");
  __shared__ __attribute__((aligned(16))) char smem[G::LDS];

  const VuGather& g = p.a;
  const int H = g.H, W = g.W;
  const int tx_n = W / TW, ty_n = H / TH;
  const int mtiles = g.N * ty_n * tx_n;
  const int ntiles = p.ncol / BN;
  const int btiles = mtiles * ntiles;
  const int ksplit = SPLIT ? p.ksplit : 1;
  const int bid0 = xcd_remap(blockIdx.x, btiles * ksplit);
  const int kidx = SPLIT ? bid0 / btiles : 0;
  const int bid = SPLIT ? bid0 - kidx * btiles : bid0;
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int img = mt / (ty_n * tx_n);
  const int trem = mt - img * (ty_n * tx_n);
  const int y0 = (trem / tx_n) * TH, x0 = (trem - (trem / tx_n) * tx_n) * TW;
  const int n0 = nt * BN;
  // this block's chunk range (an even count: the host guarantees it); pair k
  // = chunks cbeg + 2k (group 0) and cbeg + 2k + 1 (group 1)
  const int call = g.C / 32;
  const int cbeg = SPLIT ? kidx * call / ksplit : 0, cend = SPLIT ? (kidx + 1) * call / ksplit : call;
  const int npair = XM == 4 ? 0 : (cend - cbeg) >> 1;
  const int S = npair * 3;  // steps: tap rows

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;  // K group
  const int q = wid & 3;     // pixel quarter (32 pixels) of the tile
  const int gt = tid & 255;
  const bf16_t* bmat = reinterpret_cast<const bf16_t*>(p.b);
  const void* zp = (const void*)vu_zero_page7;
  char* const hbuf = smem;                 // [2 buffers][2 groups][HALO]
  char* const wbuf = smem + 4 * HALO;      // [NBW slots][3 taps][2 groups][WTAP]

  const bf16_t* const src0 = reinterpret_cast<const bf16_t*>(g.src[0]);
  const bf16_t* const src1 = reinterpret_cast<const bf16_t*>(g.src[1]);
  const bf16_t* const src2 = reinterpret_cast<const bf16_t*>(g.src[2]);
  const int64_t st0 = g.stride[0], st1 = g.stride[1], st2 = g.stride[2];
  const int ce0 = g.cend[0], ce1 = g.nsrc > 2 ? g.cend[1] : (1 << 30);

  // LDS images: 64-byte pixel (weight) rows whose 16-byte pieces are stored
  // at piece ^ (2 * ((row >> 2) & 1)) -- every ds_read_b128 fragment read of
  // 16 consecutive rows is then conflict-free at any start row (4 LDS cycles
  // instead of 8), i.e. for every tap shift of the halo (applied on the DMA
  // source side; the reads below undo it per tap).
  //
  // (group 1) DMA slots of the two halos of a chunk pair, resolved ONCE: the
  // geometry does not change between pairs, only the source chunk (measured:
  // recomputing the slot geometry per pair -- a division by the halo width,
  // bounds tests, 64-bit products for 7 slots -- stalled the whole block at
  // every pair start).  hv = pixel index in the image << 3 | group << 2 |
  // logical piece; -1: outside the image (zero page); -2: no piece.
  int hv[NH];
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    const int P = i * 256 + gt;
    const int gg = P >= HPIECES;
    const int Pl = P - gg * HPIECES;
    const int px = Pl >> 2;
    const int hy = px / HW, hx = px - (px / HW) * HW;
    const int y = y0 - 1 + hy, x = x0 - 1 + hx;
    const bool ok = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    const int kl = (Pl & 3) ^ ((px >> 1) & 2);  // logical piece landing in physical slot Pl & 3
    hv[i] = P >= 2 * HPIECES ? -2 : (ok ? ((y * W + x) << 3 | gg << 2 | kl) : -1);
  }
  const int64_t img_px = (int64_t)img * H * W;
  auto chunk_src = [&](int c, const bf16_t*& src, int64_t& st) {
    const int cb = c * 32;
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
    src += img_px * st;
  };
  auto halo_pair = [&](int k, int buf) {
    const bf16_t *sa, *sb;
    int64_t ta, tb;
    chunk_src(cbeg + 2 * k, sa, ta);
    chunk_src(cbeg + 2 * k + 1, sb, tb);
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      if (i * 256 + (wid & 3) * 64 >= 2 * HPIECES) continue;  // wave-uniform
      const int v = hv[i];
      if (v != -2) {
        const bool g1 = (v >> 2) & 1;
        const void* gp = v >= 0 ? (const void*)((g1 ? sb : sa) + (int64_t)(v >> 3) * (g1 ? tb : ta) + (v & 3) * 8)
                                : zp;
        char* dst = hbuf + buf * 2 * HALO + (i * 256 + (wid & 3) * 64) * 16;
        __builtin_amdgcn_global_load_lds(gp, (lds_void*)dst, 16, 0, 0);
      }
    }
  };
  // (group 0) both groups' weights of step (pair k, tap row r) into ring slot
  // sl: DMA i = tap 3r + i/2 of group i%2, 64 rows x 4 pieces; the per-lane
  // row pointer is resolved once
  const bf16_t* const wrow = bmat + (int64_t)(n0 + (gt >> 2)) * p.ldb + ((gt & 3) ^ ((gt >> 3) & 2)) * 8;
  auto wstage = [&](int k, int r, int sl) {
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int tx = i >> 1, gg = i & 1;
      const int k0 = (3 * r + tx) * g.C + (cbeg + 2 * k + gg) * 32;
      char* dst = wbuf + sl * SLOT + (tx * 2 + gg) * WTAP + (wid & 3) * 64 * 16;
      __builtin_amdgcn_global_load_lds((const void*)(wrow + k0), (lds_void*)dst, 16, 0, 0);
    }
  };

  // fragment i (0, 1) of this wave = tile pixels (2q + i) * 16 + (lane & 15):
  // its halo pixel at tap (0, 0)
  auto apix = [&](int i) {
    const int tp = (2 * q + i) * 16;
    return (tp / TW) * HW + (tp % TW) + (lane & 15);
  };
  const int pa0 = apix(0), pa1 = apix(1), kq = lane >> 4;
  auto aoff = [&](int P) { return P * 64 + ((kq ^ ((P >> 1) & 2)) << 4); };
  const int brow = (lane & 15) * 64 + ((kq ^ (((lane & 15) >> 1) & 2)) << 4);
  // fragments of (tap row r, halo buffer b, ring slot sl): per tap x of the
  // row, fr[6x .. 6x+3] weights, fr[6x+4], fr[6x+5] pixels
  auto read_frags = [&](int r, int b, int sl, u32x4* fr) {
    const char* Ah = hbuf + (b * 2 + grp) * HALO;
    static_assert(NJ == 4, "fragment read list");
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      const uint32_t bw = lds_addr(wbuf + sl * SLOT + (x * 2 + grp) * WTAP + brow);
      fr[6 * x + 0] = lds_rd_off<0>(bw);
      fr[6 * x + 1] = lds_rd_off<1024>(bw);
      fr[6 * x + 2] = lds_rd_off<2048>(bw);
      fr[6 * x + 3] = lds_rd_off<3072>(bw);
      fr[6 * x + 4] = lds_rd(lds_addr(Ah + aoff(pa0 + r * HW + x)));
      fr[6 * x + 5] = lds_rd(lds_addr(Ah + aoff(pa1 + r * HW + x)));
    }
  };

  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  // ---- prologue: pair 0's halos, weights of steps 0 .. PD-1 ----------------
  if (grp) {
    halo_pair(0, 0);
  } else {
    for (int s = 0; s < PD && s < S; ++s) wstage(0, s, s);  // PD <= 3: the tap rows of pair 0
  }
  // group 0 waits for step 0's weights only (steps 1 .. PD-1 keep landing
  // while step 0 runs; step 0's phase 1 waits for step 1 as every step does)
  if (!grp && S >= PD) wait_vm<(PD - 1) * LB>();
  else wait_vm<0>();
  sg_barrier();
  if (grp) sg_barrier();  // the stagger: group 1 runs one barrier behind

  // ---- main loop ------------------------------------------------------------
  // Step s = tap row r (three taps, 24 MFMAs per wave) of chunk pair k.  Two
  // phases per step, separated by barriers, the groups one phase apart
  // (ping-pong):
  //   phase 1: the step's 18 fragments are read; group 0 issues the weights
  //     of step s + PD and waits for step s + 1's; group 1 issues the next
  //     pair's halos at r = 0 and waits for them at r = 2;
  //   phase 2: the MFMAs.
  // (One tap per step measured 2.5x slower: 8 MFMAs between two barriers do
  // not cover the barrier and LDS-latency cost of a phase.)
  tmark(0);
  u32x4 fr[18];
  int r = 0, k = 0, hb = 0, slot = 0;
  int pk = PD / 3, pr = PD % 3;  // (pair, row) of step s + PD
  for (int s = 0; s < S; ++s) {
    read_frags(r, hb, slot, fr);
    if (XM != 2) {
      if (!grp) {
        if (s + PD < S) {
          wstage(pk, pr, slot == 0 ? NBW - 1 : slot - 1);  // ring slot (s + PD) % NBW
          wait_vm<(PD - 1) * LB>();  // step s + 1's weights have landed
        } else {
          wait_vm<0>();
        }
      } else {
        if (r == 0 && k + 1 < npair) halo_pair(k + 1, hb ^ 1);
        if (r == 2) wait_vm<0>();
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < 18; ++j) tie(fr[j]);
    tmark(1);
    sg_barrier();
    tmark(2);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int x = 0; x < 3; ++x)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fr[6 * x + j]),
                                                              __builtin_bit_cast(bf16x8, fr[6 * x + 4 + i]), acc[i][j],
                                                              0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    tmark(3);
    sg_barrier();
    tmark(4);
    if constexpr (TMR) tph[6] += 1;
    slot = slot == NBW - 1 ? 0 : slot + 1;
    if (++r == 3) {
      r = 0;
      ++k;
      hb ^= 1;
    }
    if (++pr == 3) {
      pr = 0;
      ++pk;
    }
  }
  if (!grp) sg_barrier();  // re-align the groups
  __syncthreads();

  // ---- sum the two K groups; every wave finalizes one fragment -------------
  // Wave (grp, q) owns fragment i = grp of its pixel quarter q and hands its
  // partial of the other fragment to the partner wave (grp ^ 1, q): both
  // groups share the epilogue (round 4: it was group 0's alone, group 1
  // idling; part of v7's per-launch fixed cost).  The sums are the same two
  // partials as before (fp32 addition commutes): bit-identical outputs.
  const __attribute__((address_space(4))) VuGemmFwd* ep =
      (const __attribute__((address_space(4))) VuGemmFwd*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(ep));
  float* const red = reinterpret_cast<float*>(smem);
  const int w8 = grp * 4 + q, pw8 = (grp ^ 1) * 4 + q;
  f32x4 mine[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const f32x4 o = grp ? acc[0][j] : acc[1][j];
    mine[j] = grp ? acc[1][j] : acc[0][j];
#pragma unroll
    for (int r = 0; r < 4; ++r) red[((w8 * NJ + j) * 4 + r) * 64 + lane] = o[r];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) mine[j][r] += red[((pw8 * NJ + j) * 4 + r) * 64 + lane];
  // this wave's pixels: tile pixel (2q + grp) * 16 + (lane & 15)
  const int tp0 = (2 * q + grp) * 16;
  const int cl = 4 * (lane >> 4);  // first of this lane's 4 channels in a 16-channel fragment
  if (SPLIT) {
    const int64_t M = (int64_t)g.N * H * W;
    float* const slab = ep->workspace + (int64_t)kidx * M * ep->ncol + n0 + cl;
    const int tp = tp0 + (lane & 15), row = tp / TW, col = tp - (tp / TW) * TW;
    float* const dst = slab + (((int64_t)img * H + y0 + row) * W + x0 + col) * ep->ncol;
#pragma unroll
    for (int j = 0; j < NJ; ++j) *reinterpret_cast<f32x4*>(dst + j * 16) = mine[j];
    return;
  }
  char* const stg = smem + G::RED + w8 * G::STG;
  float* const stat = reinterpret_cast<float*>(smem + G::RED + 8 * G::STG);  // [8 waves][BN] sum, then m2
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float bv = ep->bias ? ep->bias[n0 + j * 16 + cl + r] : 0.f;
      mine[j][r] = rnd<bf16_t>(mine[j][r] + bv);
    }
  if constexpr (RELU) epi_relu(mine);
  if (ep->stat_sum) {
    // per-wave (sum, centered M2) over its 16 pixels for every channel
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sv = row16_sum(mine[j][r]);
        const float d = mine[j][r] - sv * (1.f / 16);
        const float qv = row16_sum(d * d);
        if ((lane & 15) == 0) {
          stat[w8 * BN + j * 16 + cl + r] = sv;
          stat[(8 + w8) * BN + j * 16 + cl + r] = qv;
        }
      }
  }
  // stage the wave's 16 pixels x BN channels (bf16, a private strip) and
  // store whole pixel rows
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    u32x2 v;
    v[0] = (uint32_t)f2bf(mine[j][0]) | ((uint32_t)f2bf(mine[j][1]) << 16);
    v[1] = (uint32_t)f2bf(mine[j][2]) | ((uint32_t)f2bf(mine[j][3]) << 16);
    *reinterpret_cast<u32x2*>(stg + (lane & 15) * G::SPITCH + (j * 16 + cl) * 2) = v;
  }
  __syncthreads();   // the statistics of all eight waves (and each wave's strip) are in LDS
  {
    constexpr int PPR = BN / 8;  // 16-byte pieces per pixel row
    bf16_t* const out = reinterpret_cast<bf16_t*>(ep->out) + ep->out_coff + n0;
#pragma unroll
    for (int e0 = 0; e0 < 16 * PPR; e0 += 64) {
      const int e = e0 + lane;
      const int pl = e / PPR, pc = e - (e / PPR) * PPR;
      const int tp = tp0 + pl;
      const int row = tp / TW, col = tp - (tp / TW) * TW;
      u32x4 v = *reinterpret_cast<const u32x4*>(stg + pl * G::SPITCH + pc * 16);
      bf16_t* const dst = out + (((int64_t)img * H + y0 + row) * W + x0 + col) * ep->out_stride + pc * 8;
      if (ep->accumulate) {
        const u32x4 old = *reinterpret_cast<const u32x4*>(dst);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float lo = __uint_as_float(old[w] << 16) + __uint_as_float(v[w] << 16);
          const float hi = __uint_as_float(old[w] & 0xffff0000u) + __uint_as_float(v[w] & 0xffff0000u);
          v[w] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
        }
      }
      *reinterpret_cast<u32x4*>(dst) = v;
    }
  }
  if (ep->stat_sum && tid < BN) {
    // combine the eight waves' 16-pixel statistics (Chan, fixed order)
    float sw[8], tot = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      sw[w] = stat[w * BN + tid];
      tot += sw[w];
    }
    const float mean = tot * (1.f / 128);
    float m2 = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const float d = sw[w] * (1.f / 16) - mean;
      m2 += stat[(8 + w) * BN + tid] + 16.f * d * d;
    }
    ep->stat_sum[(int64_t)mt * ep->ncol + n0 + tid] = tot;
    ep->stat_m2[(int64_t)mt * ep->ncol + n0 + tid] = m2;
  }
  if constexpr (TMR) {
    tmark(5);
    if (blockIdx.x < SG_DBG_BLOCKS && lane == 0) {
      unsigned long long* d = vu_sg_dbg + ((int64_t)blockIdx.x * 8 + wid) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = tph[i];
    }
  }
}

int g_v7 = 1;      // vu_gemm_set_tuning(VU_TUNE_V7, ...): 0 off, 1 auto, 2 every small grid incl. C >= 512
int g_v7_nbw = 3;  // VU_TUNE_V7_NBW: weight ring slots (tap rows: 3 or 4; 3 measured 2-4 % faster)
int g_v7_xm = 0;   // VU_TUNE_V7_XM: experiment mode of unsplit 6-slot launches (A/B runs only)

struct Plan7 {
  int tw, bn, ks;
};

Plan7 plan7(const VuGemmFwd& p, int dtype) {
  Plan7 r{0, 0, 0};
  const VuGather& g = p.a;
  if (g_v7 == 0 || dtype != VU_BF16 || p.out_mode != 0) return r;
  if (g.R != 3 || g.S != 3 || g.sy != 1 || g.sx != 1 || g.dy != 1 || g.dx != 1 || g.oy != -1 || g.ox != -1 ||
      g.Hs != g.H || g.Ws != g.W)
    return r;
  if (g.C % 64 != 0 || p.ncol % 64 != 0) return r;
  for (int t = 0; t < g.nsrc; ++t)
    if (g.cend[t] % 32 != 0 || g.stride[t] % 8 != 0) return r;
  if (p.out_stride % 8 != 0 || p.out_coff % 8 != 0 || p.ldb % 8 != 0) return r;
  const int tw = g.W % 32 == 0 ? 32 : (g.W % 16 == 0 ? 16 : 0);
  if (!tw || g.H % (128 / tw) != 0) return r;
  const int64_t M = (int64_t)g.N * g.H * g.W;
  if (M >= ((int64_t)1 << 31)) return r;
  const int64_t tiles = (M / 128) * (p.ncol / 64);
  if (tiles < 64) return r;
  const int chunks = g.C / 32;
  if (chunks < 4) return r;  // one chunk pair per block: the halo kernels' 256-pixel tiles do better
  int ks = 1;
  while (tiles * ks < 256 && chunks % (4 * ks) == 0 && chunks / (2 * ks) >= 4) ks *= 2;
  r.tw = tw;
  r.bn = 64;
  r.ks = ks;
  return r;
}

template <int TW>
int launch7(const VuGemmFwd& p, const Plan7& r, hipStream_t st) {
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  const int64_t tiles = (M / 128) * (p.ncol / 64);
  VuGemmFwd q = p;
  q.ksplit = r.ks;
  const dim3 gr((unsigned)(r.ks <= 1 ? tiles : tiles * r.ks));
  if (r.ks > 1 && !p.workspace) return (int)hipErrorInvalidValue;
  if (r.ks <= 1 && g_v7_xm == 2)
    hipLaunchKernelGGL((conv3x3_sg_kernel<TW, 64, 4, false, 2>), gr, dim3(512), 0, st, q);
  else if (r.ks <= 1 && g_v7_xm == 4)
    hipLaunchKernelGGL((conv3x3_sg_kernel<TW, 64, 4, false, 4>), gr, dim3(512), 0, st, q);
  else if (r.ks <= 1 && g_v7_xm == 5 && !p.relu)
    hipLaunchKernelGGL((conv3x3_sg_kernel<TW, 64, 3, false, 5>), gr, dim3(512), 0, st, q);
  else if (r.ks <= 1 && p.relu)
    hipLaunchKernelGGL((conv3x3_sg_kernel<TW, 64, 3, false, 0, true>), gr, dim3(512), 0, st, q);
  else if (r.ks <= 1 && g_v7_nbw == 3)
    hipLaunchKernelGGL((conv3x3_sg_kernel<TW, 64, 3, false>), gr, dim3(512), 0, st, q);
  else if (r.ks <= 1)
    hipLaunchKernelGGL((conv3x3_sg_kernel<TW, 64, 4, false>), gr, dim3(512), 0, st, q);
  else if (g_v7_nbw == 3)
    hipLaunchKernelGGL((conv3x3_sg_kernel<TW, 64, 3, true>), gr, dim3(512), 0, st, q);
  else
    hipLaunchKernelGGL((conv3x3_sg_kernel<TW, 64, 4, true>), gr, dim3(512), 0, st, q);
  return (int)hipGetLastError();
}

}  // namespace

int splitk_finish_launch(const VuGemmFwd& p, hipStream_t st);  // gemm_fwd4.hip

// Row tile (128) when the small-grid kernel serves this problem, else 0.  It
// is asked only after the resident-weight (v6) and unsplit ping-pong (v4)
// kernels declined (gemm_fwd.hip's dispatch order); mode 1 leaves the long-K
// (>= 512 input channels) 32-pixel-wide grids to the ping-pong split-K.
int gemm_fwd_v7_bm(const VuGemmFwd& p, int dtype) {
  const Plan7 r = plan7(p, dtype);
  if (!r.tw) return 0;
  // >= 512 input channels on 32-wide images: the v4 split-K measured faster
  if (g_v7 == 1 && p.a.C >= 512 && r.tw == 32) return 0;
  return 128;
}

int64_t gemm_fwd_v7_workspace(const VuGemmFwd& p, int dtype) {
  const Plan7 r = plan7(p, dtype);
  return r.ks > 1 ? (int64_t)r.ks * p.a.N * p.a.H * p.a.W * p.ncol * (int64_t)sizeof(float) : 0;
}

int gemm_fwd_v7_launch(const VuGemmFwd& p, hipStream_t st) {
  const Plan7 r = plan7(p, VU_BF16);
  if (!r.tw) return (int)hipErrorInvalidValue;
  const int64_t M = (int64_t)p.a.N * p.a.H * p.a.W;
  if (M % 128 != 0) return (int)hipErrorInvalidValue;
  const int e = r.tw == 32 ? launch7<32>(p, r, st) : launch7<16>(p, r, st);
  if (e || r.ks <= 1) return e;
  VuGemmFwd q = p;
  q.ksplit = r.ks;
  return splitk_finish_launch(q, st);
}

// XM 5's counters: n = 8 phases x 8 waves x SG_DBG_BLOCKS blocks max
extern "C" int vu_sg_debug_read(unsigned long long* out, int n) {
  if (n > SG_DBG_BLOCKS * 64) n = SG_DBG_BLOCKS * 64;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(vu_sg_dbg), (size_t)n * sizeof(unsigned long long));
}

int gemm_fwd_v7_tune(int key, int value) {
  if (key == VU_TUNE_V7) {
    if (value < 0 || value > 2) return (int)hipErrorInvalidValue;
    g_v7 = value;
    return 0;
  }
  if (key == VU_TUNE_V7_XM) {
    g_v7_xm = value;
    return 0;
  }
  if (key == VU_TUNE_V7_NBW) {
    if (value != 3 && value != 4) return (int)hipErrorInvalidValue;
    g_v7_nbw = value;
    return 0;
  }
  return -1;
}
