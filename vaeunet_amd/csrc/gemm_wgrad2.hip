// Weight-gradient GEMM, large-tile bf16 variant ("v2") — same contract as
// gemm_wgrad.hip: slab[s][i][j] = sum_{m in split s} P[m][i] * Q[m][j].
//
//   * 8 waves (512 threads); output tile 128 x 256 (waves 2x4, 64x64 each)
//     or 64 x 256 for the 64-channel layers (waves 1x8, 64x32 each);
//   * 64 pixels per step, both operand images [m][col] filled by LDS-DMA
//     (global_load_lds_dwordx4); each lane's (pixel, column chunk) is fixed
//     for the whole launch, so its tap / channel / source decode is done once
//     and only the pixel coordinates advance (by 64) per step;
//   * the 32-byte-block XOR swizzle that makes the transposed
//     ds_read_b64_tr_b16 fragment reads conflict-free is applied to the
//     SOURCE column of each lane (the LDS image stays lane-linear);
//   * deterministic split-K over pixels into fp32 slabs (vu_slab_reduce).
#include "common.h"
#include "../../include/vaeunet.h"

static __device__ __attribute__((aligned(16))) uint32_t vu_zero_page[16];  // per code object

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// 32-byte block swizzle: a 32-lane half of a transposed read touches 8 rows
// (4 consecutive + 4 rows 8 apart), one 32-byte block each; f(m) spreads them
// over the 8 bank blocks of the 256-byte bank window.  Rows >= 256 B: all
// three row bits; 128-B rows (4 blocks): pairs by parity; 64-B rows (2
// blocks): the two row quads.
template <int RB> VU_DEV int fsw(int m) {
  return RB >= 256 ? ((m & 3) | ((m >> 1) & 4))
                   : RB == 128 ? (((m >> 1) & 1) | ((m >> 2) & 2)) : ((m >> 3) & 1);
}

template <int RB> VU_DEV int tr_off(int m, int col) {
  return m * RB + (((col >> 4) ^ fsw<RB>(m)) << 5) + ((col & 15) << 1);
}

// Transposed 16-bit LDS read as inline asm.  Through the builtin, the
// compiler cannot tell these reads from the LDS-DMA destinations still in
// flight and puts an s_waitcnt vmcnt(0) in front of them, which drains the
// whole DMA ring every step; here the ring's counted vmcnt waits + barriers
// order DMA and reads, and lgkm_wait() below orders reads and MFMAs.
VU_DEV u32x2 tr_read(const char* p) {
  u32x2 r;
  const uint32_t a = (uint32_t)(uintptr_t)(const lds_void*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}

// wait until at most N LDS reads are outstanding; the fragments passed are
// tied to the wait so their consumers cannot be scheduled above it
template <int N> VU_DEV void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N > 15 ? 15 : N) : "memory");
}
VU_DEV void tie(u32x4& v) { asm volatile("" : "+v"(v)); }

// A DMA slot's fixed column: tap, source and channel, with the source's base
// pointer (channel offset applied) and pixel stride resolved ONCE into
// registers.  Indexing the kernel-argument arrays g.src[t] / g.stride[t] with
// a per-lane t inside the step loop makes the compiler fetch them with vector
// loads and wait for them with s_waitcnt vmcnt(0) -- which, vmcnt being in
// order, also drains every LDS-DMA stage in flight and serialises the ring
// (measured: ~12 GB/s per CU).
struct Col {
  int r, s;
  const bf16_t* base;
  int64_t stride;
  bool ok;
};

VU_DEV Col decode_col(const VuGather& g, int col, int ncols) {
  Col d;
  d.ok = col < ncols;
  int cc = d.ok ? col : 0;
  int tap = cc / g.C, ch = cc - tap * g.C;
  d.r = tap / g.S;
  d.s = tap - d.r * g.S;
  const int t = (ch >= g.cend[0]) + (g.nsrc > 2 && ch >= g.cend[1]);
  const int coff = ch - (t == 0 ? 0 : (t == 1 ? g.cend[0] : g.cend[1]));
  const void* src = t == 0 ? g.src[0] : (t == 1 ? g.src[1] : g.src[2]);
  d.stride = t == 0 ? g.stride[0] : (t == 1 ? g.stride[1] : g.stride[2]);
  d.base = reinterpret_cast<const bf16_t*>(src) + coff;
  return d;
}

// wait until at most K*NL vector-memory operations are outstanding, K the
// number of younger ring stages in flight (a runtime 0 .. NS-1)
template <int NL, int K>
VU_DEV void vm_wait_stages(int k) {
  if constexpr (K <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (k >= K) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K * NL) : "memory");
    else vm_wait_stages<NL, K - 1>(k);
  }
}

// NS: LDS ring slots (NS - 1 stages in flight while a step computes)
template <int BI, int BJ, int WI, int WJ, int BMR, int NS = 3>
__global__ __launch_bounds__(WI * WJ * 64, 1) void gemm_wgrad_v2_kernel(VuGemmWgrad p) {
  constexpr int NT = WI * WJ * 64;
  constexpr int RBP = BI * 2, RBQ = BJ * 2;          // LDS row bytes
  constexpr int CPI = BI / 8, CPJ = BJ / 8;          // 16-byte chunks per row
  constexpr int LI = BMR * CPI / NT, LJ = BMR * CPJ / NT;
  constexpr int TI = BI / WI / 16, TJ = BJ / WJ / 16;
  constexpr int STAGE = BMR * (RBP + RBQ);
  static_assert(LI >= 1 && LJ >= 1, "tile too small");
  constexpr int NSTAGE = NS;  // LDS ring, DMA NS - 1 steps ahead
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];

  const VuGather& gp = p.p;
  const VuGather& gq = p.q;
  const int64_t M = (int64_t)gp.N * gp.H * gp.W;
  const int itiles = (p.ni + BI - 1) / BI, jtiles = (p.nj + BJ - 1) / BJ;
  const int ntile = itiles * jtiles;
  const int bid = xcd_remap(blockIdx.x, ntile * p.splits);
  const int split = bid / ntile;
  const int tile = bid - split * ntile;
  const int it = tile / jtiles, jt = tile - it * jtiles;
  const int i0 = it * BI, j0 = jt * BJ;
  const int64_t mbeg = (int64_t)split * p.m_per_split;
  const int64_t mend = (mbeg + p.m_per_split < M) ? mbeg + p.m_per_split : M;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wi = wid / WJ, wj = wid - (wid / WJ) * WJ;
  const void* zp = (const void*)vu_zero_page;

  // per-thread fixed (row-in-step, column) assignment of every DMA slot
  int prow[LI], qrow[LJ];
  Col pcd[LI], qcd[LJ];
#pragma unroll
  for (int k = 0; k < LI; ++k) {
    int q = k * NT + tid;
    prow[k] = q / CPI;
    int pc = q - prow[k] * CPI;
    int lcol = ((((pc >> 1) ^ fsw<RBP>(prow[k])) << 1) | (pc & 1)) * 8;
    pcd[k] = decode_col(gp, i0 + lcol, p.ni);
  }
#pragma unroll
  for (int k = 0; k < LJ; ++k) {
    int q = k * NT + tid;
    qrow[k] = q / CPJ;
    int pc = q - qrow[k] * CPJ;
    int lcol = ((((pc >> 1) ^ fsw<RBQ>(qrow[k])) << 1) | (pc & 1)) * 8;
    qcd[k] = decode_col(gq, j0 + lcol, p.nj);
  }
  int pn[LI], ph[LI], pw[LI], qn[LJ], qh[LJ], qw[LJ];
  auto decode = [&](int64_t m, int& n, int& h, int& w) {
    int hw = gp.H * gp.W;
    int64_t mm = m < M ? m : 0;
    n = (int)(mm / hw);
    int rem = (int)(mm - (int64_t)n * hw);
    h = rem / gp.W;
    w = rem - h * gp.W;
  };
  auto advance = [&](int& n, int& h, int& w) {
    w += BMR;
    while (w >= gp.W) { w -= gp.W; if (++h == gp.H) { h = 0; ++n; } }
  };
#pragma unroll
  for (int k = 0; k < LI; ++k) decode(mbeg + prow[k], pn[k], ph[k], pw[k]);
#pragma unroll
  for (int k = 0; k < LJ; ++k) decode(mbeg + qrow[k], qn[k], qh[k], qw[k]);

  auto src_of = [&](const VuGather& g, const Col& d, int n, int h, int w, bool mok) -> const void* {
    if (!mok || !d.ok) return zp;
    int hs = h * g.sy + d.r * g.dy + g.oy;
    int ws = w * g.sx + d.s * g.dx + g.ox;
    if ((unsigned)hs >= (unsigned)g.Hs || (unsigned)ws >= (unsigned)g.Ws) return zp;
    return d.base + (((int64_t)n * g.Hs + hs) * g.Ws + ws) * d.stride;
  };

  // Linear gathers (every 1x1 and unpadded ConvT operand): no tap reads
  // outside the source image and Hs == sy * H, with W | BMR or BMR | W and
  // the split starting on a step boundary.  Then each DMA slot's source
  // pointer advances per step by a fixed increment -- BMR / W source rows,
  // or BMR pixels within a row and a row change every W / BMR steps
  // (block-uniform) -- instead of the per-step decode + 64-bit address
  // arithmetic + bounds branches (~290 VALU per step and wave, which left the
  // MFMA pipe idle most of the step).
  auto linear = [&](const VuGather& g) {
    if (g.oy < 0 || g.ox < 0 || g.dy < 0 || g.dx < 0 || g.Hs != g.H * g.sy) return false;
    if ((g.H - 1) * g.sy + (g.R - 1) * g.dy + g.oy >= g.Hs) return false;
    if ((g.W - 1) * g.sx + (g.S - 1) * g.dx + g.ox >= g.Ws) return false;
    return BMR % g.W == 0 || g.W % BMR == 0;
  };
  const bool lin = linear(gp) && linear(gq) && mbeg % BMR == 0;
  const bool multirow = BMR % gp.W == 0;  // a step covers BMR / W whole rows
  int wcnt = (int)(mbeg % gp.W);          // column of the step start (BMR | W case)
  const bf16_t* pptr[LI];
  const bf16_t* qptr[LJ];
  int pinc[LI], pwrap[LI], qinc[LJ], qwrap[LJ];
  auto lin_init = [&](const VuGather& g, const Col& d, int n, int h, int w, const bf16_t*& ptr, int& inc,
                      int& wrap) {
    ptr = d.ok ? d.base + (((int64_t)n * g.Hs + h * g.sy + d.r * g.dy + g.oy) * g.Ws + w * g.sx + d.s * g.dx + g.ox) *
                               d.stride
               : nullptr;
    const int64_t row = (int64_t)g.sy * g.Ws;  // source pixels per grid row
    inc = (int)((multirow ? (BMR / g.W) * row : (int64_t)BMR * g.sx) * d.stride);
    wrap = (int)((multirow ? (BMR / g.W) * row : row - (int64_t)(g.W - BMR) * g.sx) * d.stride);
  };
  if (lin) {
#pragma unroll
    for (int k = 0; k < LI; ++k) lin_init(gp, pcd[k], pn[k], ph[k], pw[k], pptr[k], pinc[k], pwrap[k]);
#pragma unroll
    for (int k = 0; k < LJ; ++k) lin_init(gq, qcd[k], qn[k], qh[k], qw[k], qptr[k], qinc[k], qwrap[k]);
  }

  auto stage = [&](int64_t mb, int buf) {
    char* Pb = smem + buf * STAGE;
    char* Qb = Pb + BMR * RBP;
    if (lin) {
      wcnt += BMR;
      const bool wrapped = wcnt >= gp.W;  // block-uniform
      if (wrapped) wcnt -= gp.W;
#pragma unroll
      for (int k = 0; k < LI; ++k) {
        const void* s = (pptr[k] != nullptr && mb + prow[k] < mend) ? (const void*)pptr[k] : zp;
        __builtin_amdgcn_global_load_lds(s, (lds_void*)(Pb + (k * NT + wid * 64) * 16), 16, 0, 0);
        if (pptr[k] != nullptr) pptr[k] += wrapped ? pwrap[k] : pinc[k];
      }
#pragma unroll
      for (int k = 0; k < LJ; ++k) {
        const void* s = (qptr[k] != nullptr && mb + qrow[k] < mend) ? (const void*)qptr[k] : zp;
        __builtin_amdgcn_global_load_lds(s, (lds_void*)(Qb + (k * NT + wid * 64) * 16), 16, 0, 0);
        if (qptr[k] != nullptr) qptr[k] += wrapped ? qwrap[k] : qinc[k];
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < LI; ++k) {
      const void* s = src_of(gp, pcd[k], pn[k], ph[k], pw[k], mb + prow[k] < mend);
      __builtin_amdgcn_global_load_lds(s, (lds_void*)(Pb + (k * NT + wid * 64) * 16), 16, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < LJ; ++k) {
      const void* s = src_of(gq, qcd[k], qn[k], qh[k], qw[k], mb + qrow[k] < mend);
      __builtin_amdgcn_global_load_lds(s, (lds_void*)(Qb + (k * NT + wid * 64) * 16), 16, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < LI; ++k) advance(pn[k], ph[k], pw[k]);
#pragma unroll
    for (int k = 0; k < LJ; ++k) advance(qn[k], qh[k], qw[k]);
  };

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int b = 0; b < TJ; ++b) acc[a][b] = f32x4{0, 0, 0, 0};

  const int nsteps = mend > mbeg ? (int)((mend - mbeg + BMR - 1) / BMR) : 0;
  // counted-vmcnt ring, two stages in flight WHILE waiting: at step st the
  // block first agrees that slot (st-1)%3 has been read (barrier), refills
  // it with stage st+2, and only then waits for stage st (vmcnt leaves the
  // two younger stages outstanding) and publishes it (barrier).  These
  // kernels are HBM/L2-latency bound (SQ_WAIT_ANY 65 % with one stage in
  // flight at the wait), so the bytes in flight are what sets the rate.
  constexpr int NL = LI + LJ;
#pragma unroll
  for (int s0 = 0; s0 < NSTAGE - 1; ++s0)
    if (nsteps > s0) stage(mbeg + (int64_t)s0 * BMR, s0);
  const int g4 = lane >> 4, li = lane & 15, qd = li >> 2, pp = li & 3;
  for (int st = 0; st < nsteps; ++st) {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + NSTAGE - 1 < nsteps) stage(mbeg + (int64_t)(st + NSTAGE - 1) * BMR, (st + NSTAGE - 1) % NSTAGE);
    // stage st has landed once only the younger stages may be outstanding
    const int younger = nsteps - 1 - st < NSTAGE - 1 ? nsteps - 1 - st : NSTAGE - 1;
    vm_wait_stages<NL, NSTAGE - 1>(younger);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int cur = st % NSTAGE;
    const char* Pb = smem + cur * STAGE;
    const char* Qb = Pb + BMR * RBP;
    // fragments of k-step ks+1 are read while k-step ks's MFMAs issue
    auto load = [&](int ks, u32x4* af, u32x4* bf) {
      const int m = ks * 32 + 8 * g4 + qd;
#pragma unroll
      for (int a = 0; a < TI; ++a) {
        int col = wi * (BI / WI) + a * 16 + 4 * pp;
        u32x2 l2 = tr_read(Pb + tr_off<RBP>(m, col)), h2 = tr_read(Pb + tr_off<RBP>(m + 4, col));
        af[a] = u32x4{l2[0], l2[1], h2[0], h2[1]};
      }
#pragma unroll
      for (int b = 0; b < TJ; ++b) {
        int col = wj * (BJ / WJ) + b * 16 + 4 * pp;
        u32x2 l2 = tr_read(Qb + tr_off<RBQ>(m, col)), h2 = tr_read(Qb + tr_off<RBQ>(m + 4, col));
        bf[b] = u32x4{l2[0], l2[1], h2[0], h2[1]};
      }
    };
    u32x4 af[2][TI], bf[2][TJ];
    load(0, af[0], bf[0]);
#pragma unroll
    for (int ks = 0; ks < BMR / 32; ++ks) {
      if (ks + 1 < BMR / 32) {
        load(ks + 1, af[(ks + 1) & 1], bf[(ks + 1) & 1]);
        lgkm_wait<2 * (TI + TJ)>();  // k-step ks's reads done, ks+1's may fly
      } else {
        lgkm_wait<0>();
      }
#pragma unroll
      for (int a = 0; a < TI; ++a) tie(af[ks & 1][a]);
#pragma unroll
      for (int b = 0; b < TJ; ++b) tie(bf[ks & 1][b]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < TI; ++a)
#pragma unroll
        for (int b = 0; b < TJ; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, af[ks & 1][a]), __builtin_bit_cast(bf16x8, bf[ks & 1][b]), acc[a][b], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  float* out = p.out + (int64_t)split * p.ni * p.nj;
#pragma unroll
  for (int a = 0; a < TI; ++a)
#pragma unroll
    for (int b = 0; b < TJ; ++b) {
      int j = j0 + wj * (BJ / WJ) + b * 16 + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int i = i0 + wi * (BI / WI) + a * 16 + 4 * g4 + r;
        if (i < p.ni && j < p.nj) out[(int64_t)i * p.nj + j] = acc[a][b][r];
      }
    }
}

template <int BI, int BJ, int WI, int WJ, int BMR, int NS = 3>
int launch(const VuGemmWgrad& p, hipStream_t st) {
  int itiles = (p.ni + BI - 1) / BI, jtiles = (p.nj + BJ - 1) / BJ;
  int64_t nblk = (int64_t)itiles * jtiles * p.splits;
  if (nblk <= 0) return 0;
  hipLaunchKernelGGL((gemm_wgrad_v2_kernel<BI, BJ, WI, WJ, BMR, NS>), dim3((unsigned)nblk), dim3(WI * WJ * 64), 0, st,
                     p);
  return (int)hipGetLastError();
}

// VU_TUNE_W2_BIG: 256 x 256 output tiles (32 pixels per step, 4-slot ring)
// for the large 1x1 / ConvT weight gradients (both dims >= 256): 1.5x the
// MFMA work per LDS byte of the 128 x 256 tile, whose blocks wait on the
// L2 -> LDS feed (~16 GB/s per CU on the UNet ConvT gradients)
int g_w2_big = 0;
bool big_tile(const VuGemmWgrad& p) { return g_w2_big && p.ni >= 256 && p.nj >= 256; }

}  // namespace

int gemm_wgrad_v2_tune(int key, int value) {
  if (key == VU_TUNE_W2_BIG) {
    g_w2_big = value;
    return 0;
  }
  return -1;
}

// Output tile (BI, BJ) of the v2 kernel for this problem, or 0 if it does not apply.
int gemm_wgrad_v2_tile(const VuGemmWgrad& p, int dtype, int* bi, int* bj) {
  if (dtype != VU_BF16) return 0;
  const VuGather* gs[2] = {&p.p, &p.q};
  for (auto g : gs)
    for (int t = 0; t < g->nsrc; ++t)
      if (g->cend[t] % 8 || g->stride[t] % 8) return 0;
  int64_t M = (int64_t)p.p.N * p.p.H * p.p.W;
  // (round 4: was 4096, which sent the ResNet34 16^2 level (M = 2048 at
  // batch 8) to the generic register-staged kernel at ~90 TFLOP/s)
  if (M < 512) return 0;
  // small outputs (the attention gates' 1x1 convs) get a tile that fits them
  // instead of streaming zero columns through a 256-wide one
  if (p.ni <= 32 && p.nj <= 64) { *bi = 32; *bj = 64; return 1; }
  if (p.ni <= 64 && p.nj <= 128) { *bi = 64; *bj = 128; return 1; }
  if (big_tile(p)) { *bi = 256; *bj = 256; return 1; }
  *bi = p.ni <= 64 ? 64 : 128;
  *bj = 256;
  return 1;
}

int gemm_wgrad_v2_launch(const VuGemmWgrad& p, hipStream_t st) {
  if (p.ni <= 32 && p.nj <= 64) return launch<32, 64, 2, 4, 128>(p, st);
  if (p.ni <= 64 && p.nj <= 128) return launch<64, 128, 2, 4, 128>(p, st);
  if (p.ni <= 64) return launch<64, 256, 1, 8, 64>(p, st);
  if (big_tile(p)) return launch<256, 256, 2, 4, 32, 4>(p, st);
  return launch<128, 256, 2, 4, 64>(p, st);
}
