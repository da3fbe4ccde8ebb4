// BatchNorm2d (train/eval), fused ReLU, and per-channel reductions over NHWC.
//
// Reference semantics: nn.BatchNorm2d in train mode (unet_parts.py:41,44 and
// the attention-gate BNs :12,16,20): batch mean and biased variance over
// (N,H,W), y = gamma*(x-mean)/sqrt(var+eps) + beta, running stats updated with
// momentum 0.1 and the UNBIASED variance, then nn.ReLU(inplace=True)
// (unet_parts.py:42,45) whose backward masks by output > 0.
//
// Statistics come from the producing GEMM's epilogue as per-row-tile (sum,
// centered M2) pairs; vu_bn_finalize combines them about the group mean in
// fp64 in a fixed order, so results are bitwise reproducible.
// Backward needs two per-channel sums (sum dz, sum dz*xhat): a two-stage
// deterministic reduction (fp32 per block, fp64 across blocks).
//
// Memory-bound layout rule used by every kernel here: a thread owns one
// fixed 8-channel vector (16 B bf16 / 32 B fp32) for its whole life, so the
// per-channel coefficients live in registers and the pixel loop is a pure
// load-FMA-store stream; a block covers 256/V pixels per pass (V = C/8).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "../../include/vaeunet.h"

namespace {

// Combining per-tile (sum, centered M2) pairs without a division per tile:
// for a group of tiles with mean m, M2 = sum_t [M2_t + n_t (m_t - m)^2]
// (exact, and as stable as Chan's pairwise update since every deviation is
// taken from the group mean).  Both stages hold their inputs in registers and
// make the two passes (group mean, then M2 about it) over the registers: the
// loads of a lane are independent and issue back to back (these launches are
// latency-bound, not bandwidth-bound).
constexpr int STATS_TPB = 32;   // tiles per stage-1 block (8 per lane)
constexpr int STATS_MAXS = 256; // stage-1 blocks per channel group (8 per stage-2 lane)

// stage 1: grid (ceil(C/64), S), 256 threads = 64 channels x 4 tile lanes.
// A block reduces its tiles in rounds of STATS_TPB (one round unless the
// problem has more than STATS_TPB * STATS_MAXS tiles); rounds merge with
// Chan's pairwise update.
__global__ void bn_stats_stage1(const float* psum, const float* pm2, int tiles, int64_t tile_rows,
                                int64_t rows, int C, int S, double* ws) {
  __shared__ double sh[4][64];
  const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const bool ok = c < C;
  const int per = (tiles + S - 1) / S;
  const int tb0 = blockIdx.y * per, te0 = min(tiles, tb0 + per);
  constexpr int U = STATS_TPB / 4;
  double N = 0, Mn = 0, Q = 0;   // running (n, mean, M2) of the rounds so far
  for (int tb = tb0; tb < te0; tb += STATS_TPB) {
    const int te = min(te0, tb + STATS_TPB);
    const int64_t n_r = min(rows, (int64_t)te * tile_rows) - (int64_t)tb * tile_rows;
    // clamped addresses and unconditional loads, selected afterwards (a
    // guarded load compiles to a branch + vmcnt(0) each: serial round trips)
    float sv[U], mv[U];
    double nv[U];
    const int cc = ok ? c : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(tb + tl + 4 * u, te - 1);
      sv[u] = psum[(int64_t)t * C + cc];
      mv[u] = pm2[(int64_t)t * C + cc];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = tb + tl + 4 * u;
      const bool in = ok && t < te;
      sv[u] = in ? sv[u] : 0.f;
      mv[u] = in ? mv[u] : 0.f;
      int64_t nt = rows - (int64_t)t * tile_rows;
      nv[u] = in ? (double)(nt > tile_rows ? tile_rows : nt) : 0.0;
    }
    double s = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) s += (double)sv[u];
    sh[tl][cl] = s;
    __syncthreads();
    const double m = (sh[0][cl] + sh[1][cl] + sh[2][cl] + sh[3][cl]) / (double)n_r;
    __syncthreads();
    double q = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (nv[u] > 0) {
        const double d = (double)sv[u] / nv[u] - m;
        q += (double)mv[u] + nv[u] * d * d;
      }
    }
    sh[tl][cl] = q;
    __syncthreads();
    const double q_r = sh[0][cl] + sh[1][cl] + sh[2][cl] + sh[3][cl];
    __syncthreads();
    const double nn = N + (double)n_r, d = m - Mn;
    Q += q_r + d * d * N * (double)n_r / nn;
    Mn += d * (double)n_r / nn;
    N = nn;
  }
  if (tl == 0 && ok) {
    double* o = ws + ((int64_t)blockIdx.y * C + c) * 3;
    o[0] = N; o[1] = Mn; o[2] = Q;
  }
}

// stage 2: 1024 threads = 32 channels x 32 lanes, <= 8 stage-1 partials per lane
__global__ void bn_stats_stage2(const double* ws, int S, int C, const float* gamma, const float* beta,
                                float* rmean, float* rvar, float momentum, float eps, float* scale,
                                float* shift, float* smean, float* sinvstd, int64_t* nbt) {
  __shared__ double sh[2][32][33];
  const int cl = threadIdx.x & 31, q = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  const bool ok = c < C;
  // the per-channel operands first: issued with the partial loads below, not
  // after the trees behind the stores they may alias (4 serial round trips)
  const int cc = ok ? c : 0;
  const float g = gamma ? gamma[cc] : 1.f, b = beta ? beta[cc] : 0.f;
  const bool upd = rmean && momentum != 0.f;
  const float rm0 = upd ? rmean[cc] : 0.f, rv0 = upd ? rvar[cc] : 0.f;
  const int64_t nb0 = nbt ? nbt[0] : 0;
  constexpr int U = STATS_MAXS / 32;
  double nv[U], mv[U], qv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const double* o = ws + ((int64_t)min(q + 32 * u, S - 1) * C + (ok ? c : 0)) * 3;
    nv[u] = o[0];
    mv[u] = o[1];
    qv[u] = o[2];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool in = ok && q + 32 * u < S;
    nv[u] = in ? nv[u] : 0.0;
    mv[u] = in ? mv[u] : 0.0;
    qv[u] = in ? qv[u] : 0.0;
  }
  double n = 0, sm = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) { n += nv[u]; sm += nv[u] * mv[u]; }
  sh[0][q][cl] = n; sh[1][q][cl] = sm;
  __syncthreads();
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1) {
    if (q < w) { sh[0][q][cl] += sh[0][q + w][cl]; sh[1][q][cl] += sh[1][q + w][cl]; }
    __syncthreads();
  }
  n = sh[0][0][cl];
  const double m = n > 0 ? sh[1][0][cl] / n : 0.0;
  __syncthreads();
  double M2 = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) { const double d = mv[u] - m; M2 += qv[u] + nv[u] * d * d; }
  sh[0][q][cl] = M2;
  __syncthreads();
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1) {
    if (q < w) sh[0][q][cl] += sh[0][q + w][cl];
    __syncthreads();
  }
  if (q != 0 || !ok) return;
  M2 = sh[0][0][cl];
  double var = n > 0 ? M2 / n : 0.0;
  float invstd = (float)(1.0 / sqrt(var + (double)eps));
  float mean = (float)m;
  scale[c] = g * invstd;
  shift[c] = b - mean * g * invstd;
  if (smean) smean[c] = mean;
  if (sinvstd) sinvstd[c] = invstd;
  if (nbt && c == 0) nbt[0] = nb0 + 1;
  if (upd) {
    double unb = n > 1 ? M2 / (n - 1) : var;
    rmean[c] = (1.f - momentum) * rm0 + momentum * mean;
    rvar[c] = (1.f - momentum) * rv0 + momentum * (float)unb;
  }
}

// Round 6: the statistics finalize as ONE launch (VU_TUNE_BN_STATS1).  First
// built with __threadfence() release / acquire in every block: 45 us per
// launch against ~12 us for the two launches (UNet -5.6 %, VAE -4.5 %,
// profiles/r6s1_*: each fence writes the XCD's L2 back and invalidates).  Now
// fence-free, on the guide's measured sc1 hand-off (below): still UNet
// -0.6/-0.7 %, VAE -0.9/-1.1 % (profiles/r6s2_*): the last block's serial
// tail (atomic round trip, write-through loads) costs more than the second
// launch it saves inside a graph replay.  Kept opt-in.  Stage 1 as bn_stats_stage1 with 64 channels x 16 tile lanes per
// 1024-thread block (64 tiles per round); each block publishes its (mean, M2)
// per channel, and the last block of its channel group to arrive -- counted
// on a per-group device counter, which that block resets for the next launch
// -- combines the group's S <= 256 partials (<= 16 per lane, about the group
// mean in fp64, as stage 2) and writes the coefficients.  Saves stage 2's
// launch per BatchNorm, a latency-bound ~6 us kernel (rocprof,
// profiles/r6a5_unet_kernel_stats_attn_pair.csv: 25 per UNet step) -- in
// principle.
// The counters assume the launches of one device do not overlap one another
// (one stream, as every caller runs them).
constexpr int FST_LANES = 16, FST_U = 4, FST_TPB = FST_LANES * FST_U, FST_MAXS = 256, FST_MAXG = 64;
constexpr int FST_PL = FST_MAXS / FST_LANES;   // partials per lane in the last block
__device__ unsigned int g_fst_count[FST_MAXG];

VU_DEV double fst_block_rows(int s, int per, int tiles, int64_t tile_rows, int64_t rows) {
  const int tb = s * per;
  if (tb >= tiles) return 0.0;
  const int te = min(tiles, tb + per);
  return (double)(min(rows, (int64_t)te * tile_rows) - (int64_t)tb * tile_rows);
}

__global__ __launch_bounds__(1024) void bn_stats_fused_kernel(
    const float* psum, const float* pm2, int tiles, int64_t tile_rows, int64_t rows, int C, int S, double* ws,
    const float* gamma, const float* beta, float* rmean, float* rvar, float momentum, float eps, float* scale,
    float* shift, float* smean, float* sinvstd, int64_t* nbt) {
  __shared__ double sh[2][FST_LANES][64];
  __shared__ int is_last;
  const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const bool ok = c < C;
  const int cc = ok ? c : 0;
  const int per = (tiles + S - 1) / S;
  const int tb0 = blockIdx.y * per, te0 = min(tiles, tb0 + per);
  double N = 0, Mn = 0, Q = 0;
  for (int tb = tb0; tb < te0; tb += FST_TPB) {
    const int te = min(te0, tb + FST_TPB);
    const int64_t n_r = min(rows, (int64_t)te * tile_rows) - (int64_t)tb * tile_rows;
    float sv[FST_U], mv[FST_U];
    double nv[FST_U];
#pragma unroll
    for (int u = 0; u < FST_U; ++u) {
      const int t = min(tb + tl + FST_LANES * u, te - 1);
      sv[u] = psum[(int64_t)t * C + cc];
      mv[u] = pm2[(int64_t)t * C + cc];
    }
#pragma unroll
    for (int u = 0; u < FST_U; ++u) {
      const int t = tb + tl + FST_LANES * u;
      const bool in = ok && t < te;
      sv[u] = in ? sv[u] : 0.f;
      mv[u] = in ? mv[u] : 0.f;
      const int64_t nt = rows - (int64_t)t * tile_rows;
      nv[u] = in ? (double)(nt > tile_rows ? tile_rows : nt) : 0.0;
    }
    double s = 0;
#pragma unroll
    for (int u = 0; u < FST_U; ++u) s += (double)sv[u];
    sh[0][tl][cl] = s;
    __syncthreads();
    double st = 0;
#pragma unroll
    for (int l = 0; l < FST_LANES; ++l) st += sh[0][l][cl];
    const double m = st / (double)n_r;
    double q = 0;
#pragma unroll
    for (int u = 0; u < FST_U; ++u) {
      if (nv[u] > 0) {
        const double d = (double)sv[u] / nv[u] - m;
        q += (double)mv[u] + nv[u] * d * d;
      }
    }
    sh[1][tl][cl] = q;
    __syncthreads();
    double q_r = 0;
#pragma unroll
    for (int l = 0; l < FST_LANES; ++l) q_r += sh[1][l][cl];
    __syncthreads();
    const double nn = N + (double)n_r, d = m - Mn;
    Q += q_r + d * d * N * (double)n_r / nn;
    Mn += d * (double)n_r / nn;
    N = nn;
  }
  // publish and count without fences (MI355X_MICROARCH.md, hand-off table,
  // first row: write-through sc1 stores by the storing wave, its vmcnt(0)
  // wait, ONE agent-scope atomic add per workgroup; the workgroup whose add
  // returned S - 1 reads every handed-off byte with sc1 loads behind a
  // workgroup barrier).  Wave 0 (tl == 0) is the only storing wave.
  if (tl == 0) {
    if (ok) {
      double* o = ws + ((int64_t)blockIdx.y * C + c) * 2;
      __hip_atomic_store(o, Mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 1, Q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) {
      const unsigned prev =
          __hip_atomic_fetch_add(&g_fst_count[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      is_last = prev == (unsigned)(S - 1);
      if (is_last) __hip_atomic_store(&g_fst_count[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!is_last) return;
  const float g = gamma ? gamma[cc] : 1.f, b = beta ? beta[cc] : 0.f;
  const bool upd = rmean && momentum != 0.f;
  const float rm0 = upd ? rmean[cc] : 0.f, rv0 = upd ? rvar[cc] : 0.f;
  const int64_t nb0 = nbt ? nbt[0] : 0;
  double pm[FST_PL], pq[FST_PL], pn[FST_PL];
#pragma unroll
  for (int u = 0; u < FST_PL; ++u) {
    double* o = ws + ((int64_t)min(tl + FST_LANES * u, S - 1) * C + cc) * 2;
    pm[u] = __hip_atomic_load(o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pq[u] = __hip_atomic_load(o + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int u = 0; u < FST_PL; ++u) {
    const int s = tl + FST_LANES * u;
    const bool in = ok && s < S;
    pn[u] = in ? fst_block_rows(s, per, tiles, tile_rows, rows) : 0.0;
    pm[u] = in ? pm[u] : 0.0;
    pq[u] = in ? pq[u] : 0.0;
  }
  double n = 0, sm = 0;
#pragma unroll
  for (int u = 0; u < FST_PL; ++u) { n += pn[u]; sm += pn[u] * pm[u]; }
  sh[0][tl][cl] = n;
  sh[1][tl][cl] = sm;
  __syncthreads();
  n = 0;
  sm = 0;
#pragma unroll
  for (int l = 0; l < FST_LANES; ++l) { n += sh[0][l][cl]; sm += sh[1][l][cl]; }
  const double m = n > 0 ? sm / n : 0.0;
  __syncthreads();
  double M2 = 0;
#pragma unroll
  for (int u = 0; u < FST_PL; ++u) { const double d = pm[u] - m; M2 += pq[u] + pn[u] * d * d; }
  sh[0][tl][cl] = M2;
  __syncthreads();
  if (tl != 0 || !ok) return;
  M2 = 0;
#pragma unroll
  for (int l = 0; l < FST_LANES; ++l) M2 += sh[0][l][cl];
  const double var = n > 0 ? M2 / n : 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float mean = (float)m;
  scale[c] = g * invstd;
  shift[c] = b - mean * g * invstd;
  if (smean) smean[c] = mean;
  if (sinvstd) sinvstd[c] = invstd;
  if (nbt && c == 0) nbt[0] = nb0 + 1;
  if (upd) {
    const double unb = n > 1 ? M2 / (n - 1) : var;
    rmean[c] = (1.f - momentum) * rm0 + momentum * mean;
    rvar[c] = (1.f - momentum) * rv0 + momentum * (float)unb;
  }
}

__global__ void bn_eval_kernel(const float* gamma, const float* beta, const float* rm, const float* rv,
                               float eps, int C, float* scale, float* shift, float* smean, float* sinvstd) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float invstd = 1.f / sqrtf(rv[c] + eps);
  float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * invstd;
  shift[c] = b - rm[c] * g * invstd;
  if (smean) smean[c] = rm[c];
  if (sinvstd) sinvstd[c] = invstd;
}

// Fixed-channel mapping: V = C/8 vectors per pixel, V a power of two <= 256.
struct ChanMap {
  int V, R, cv, row;
  VU_DEV ChanMap(int C) {
    V = C >> 3;
    R = 256 / V;
    cv = threadIdx.x & (V - 1);
    row = threadIdx.x / V;
  }
};

// Streaming kernels issue UNR independent 16-byte rows per thread before
// using any of them (a grid-stride loop with one load in flight per thread
// leaves HBM at ~60% of its bandwidth).
constexpr int UNR = 4;

template <typename T, bool NT>
__global__ void bn_apply_kernel(const T* x, int64_t xs, T* y, int64_t ys, int64_t P, int C,
                                const float* scale, const float* shift, int relu) {
  ChanMap cm(C);
  const int c = cm.cv * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sc[i] = scale[c + i]; sh[i] = shift[c + i]; }
  const int64_t step = (int64_t)gridDim.x * cm.R * UNR;
  for (int64_t p0 = (int64_t)blockIdx.x * cm.R * UNR + cm.row; p0 < P; p0 += step) {
    Vec8<T> v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * cm.R;
      if (p < P) { if (NT) v[u].load_nt(x + p * xs + c); else v[u].load(x + p * xs + c); }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * cm.R;
      if (p >= P) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float z = v[u].get(i) * sc[i] + sh[i];
        v[u].set(i, relu ? fmaxf(z, 0.f) : z);
      }
      v[u].store(y + p * ys + c);
    }
  }
}

// ---- per-channel partial reductions ----
// MODE 0: s0 = sum x (over an optional pixel window)
// MODE 1: s0 = sum dz, s1 = sum dz*xhat; dz = dy*(z>0 if relu), xhat=(x-mean)*invstd
constexpr int RED_MAXBLK = 1024;

struct RedArgs {
  const void* a; int64_t as;   // x (mode 0) or dy (mode 1)
  const void* b; int64_t bs;   // x (mode 1)
  int64_t P; int C;
  const float* scale; const float* shift; const float* mean; const float* invstd;
  int relu;
  float* part;                 // [nblk][2][C]
  int H, W, y0, x0, Hr, Wr;    // pixel window (mode 0); Hr == 0: dense
};

VU_DEV int64_t win_pix(const RedArgs& r, int64_t p) {
  if (r.Hr == 0) return p;
  int64_t j = p % r.Wr, t = p / r.Wr;
  int64_t i = t % r.Hr, n = t / r.Hr;
  return (n * r.H + r.y0 + i) * r.W + r.x0 + j;
}

template <typename T, int MODE, bool NT>
__global__ void chan_partial_kernel(RedArgs r) {
  __shared__ float sh[2][256 * 8];
  ChanMap cm(r.C);
  const int c = cm.cv * 8;
  float s0[8], s1[8], sc[8], sf[8], mu[8], is[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s0[i] = 0.f; s1[i] = 0.f;
    if (MODE == 1) {
      sc[i] = r.scale[c + i]; sf[i] = r.shift[c + i]; mu[i] = r.mean[c + i]; is[i] = r.invstd[c + i];
    }
  }
  const int64_t step = (int64_t)gridDim.x * cm.R * UNR;
  for (int64_t p0 = (int64_t)blockIdx.x * cm.R * UNR + cm.row; p0 < r.P; p0 += step) {
    Vec8<T> va[UNR], vb[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * cm.R;
      if (p < r.P) {
        const T* pa = reinterpret_cast<const T*>(r.a) + (MODE == 0 ? win_pix(r, p) : p) * r.as + c;
        const T* pb = reinterpret_cast<const T*>(r.b) + p * r.bs + c;
        if (NT) {
          va[u].load_nt(pa);
          if (MODE == 1) vb[u].load_nt(pb);
        } else {
          va[u].load(pa);
          if (MODE == 1) vb[u].load(pb);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (p0 + (int64_t)u * cm.R >= r.P) continue;
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) s0[i] += va[u].get(i);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float xv = vb[u].get(i);
          float dz = va[u].get(i);
          if (r.relu && !(fmaf(xv, sc[i], sf[i]) > 0.f)) dz = 0.f;
          s0[i] += dz;
          s1[i] += dz * ((xv - mu[i]) * is[i]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { sh[0][cm.row * r.C + c + i] = s0[i]; sh[1][cm.row * r.C + c + i] = s1[i]; }
  __syncthreads();
  for (int cc = threadIdx.x; cc < r.C; cc += 256) {
    float a0 = 0.f, a1 = 0.f;
    a0 = lds_sum(&sh[0][cc], cm.R, r.C);
    a1 = lds_sum(&sh[1][cc], cm.R, r.C);
    r.part[((int64_t)blockIdx.x * 2 + 0) * r.C + cc] = a0;
    if (MODE == 1) r.part[((int64_t)blockIdx.x * 2 + 1) * r.C + cc] = a1;
  }
}

// scalar fallback for channel counts that are not 8 x power-of-two (C <= 256)
template <typename T, int MODE>
__global__ void chan_partial_scalar(RedArgs r) {
  __shared__ float sh[2][256];
  const int R = 256 / r.C;
  const int t = threadIdx.x, c = t % r.C, row = t / r.C;
  const bool act = row < R;
  float s0 = 0.f, s1 = 0.f;
  if (act) {
    const int64_t step = (int64_t)gridDim.x * R;
    // SU rows per round, loaded from clamped pixel indices before any is used
    // (a guarded load per row serialised the round trips: the 1-channel psi
    // maps ran at ~1.2 TB/s); then summed in row order, as before
    constexpr int SU = 4;
    for (int64_t p0 = (int64_t)blockIdx.x * R + row; p0 < r.P; p0 += SU * step) {
      float av[SU], xv[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int64_t p = p0 + u * step < r.P ? p0 + u * step : r.P - 1;
        av[u] = ld1<T>(reinterpret_cast<const T*>(r.a) + win_pix(r, p) * r.as + c);
        if (MODE != 0) xv[u] = ld1<T>(reinterpret_cast<const T*>(r.b) + p * r.bs + c);
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        if (p0 + u * step >= r.P) break;
        if (MODE == 0) s0 += av[u];
        else {
          float dz = av[u];
          if (r.relu && !(xv[u] * r.scale[c] + r.shift[c] > 0.f)) dz = 0.f;
          s0 += dz;
          s1 += dz * (xv[u] - r.mean[c]) * r.invstd[c];
        }
      }
    }
    sh[0][row * r.C + c] = s0;
    sh[1][row * r.C + c] = s1;
  }
  __syncthreads();
  if (t < r.C) {
    float a0 = 0.f, a1 = 0.f;
    a0 = lds_sum(&sh[0][t], R, r.C);
    a1 = lds_sum(&sh[1][t], R, r.C);
    r.part[((int64_t)blockIdx.x * 2 + 0) * r.C + t] = a0;
    r.part[((int64_t)blockIdx.x * 2 + 1) * r.C + t] = a1;
  }
}

// stage 2: fp64 column sums of the [nblk][2][C] partials (colsum32, fixed order)
__global__ void chan_final_sum(const float* part, int nblk, int C, float* out, int accumulate) {
  int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const float o0 = accumulate ? out[c < C ? c : C - 1] : 0.f;   // before the sums (bn_bwd_final)
  double s[1];
  colsum32<1>(part, nblk, 2 * (int64_t)C, C, c, c < C, s);
  if (threadIdx.x < 32 && c < C) out[c] = accumulate ? o0 + (float)s[0] : (float)s[0];
}

__global__ void bn_bwd_final(const float* part, int nblk, int C, int64_t P, const float* gamma,
                             const float* invstd, float* dgamma, float* dbeta, int accumulate,
                             float* coef, int train) {
  int c = blockIdx.x * 32 + (threadIdx.x & 31);
  // the per-channel operands (and the gradients accumulated into) are loaded
  // BEFORE the column sums, which they do not depend on: after them, behind
  // the coef stores they may alias, they were 3 more serial round trips
  const int cl = c < C ? c : C - 1;
  const float g = gamma ? gamma[cl] : 1.f;
  const float is = invstd[cl];
  const float dg0 = (dgamma && accumulate) ? dgamma[cl] : 0.f;
  const float db0 = (dbeta && accumulate) ? dbeta[cl] : 0.f;
  double s[2];
  colsum32<2>(part, nblk, 2 * (int64_t)C, C, c, c < C, s);
  if (threadIdx.x >= 32 || c >= C) return;
  float k1 = g * is;
  coef[c] = k1;
  coef[C + c] = train ? (float)(-(double)k1 * is * s[1] / (double)P) : 0.f;
  coef[2 * C + c] = train ? (float)(-(double)k1 * s[0] / (double)P) : 0.f;
  if (dgamma) dgamma[c] = accumulate ? dg0 + (float)s[1] : (float)s[1];
  if (dbeta) dbeta[c] = accumulate ? db0 + (float)s[0] : (float)s[0];
}

template <typename T, bool NT>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* dy, int64_t dys, const T* x, int64_t xs, int64_t P, int C,
                                    const float* scale, const float* shift, const float* mean,
                                    const float* coef, int relu, T* dx, int64_t dxs) {
  ChanMap cm(C);
  const int c = cm.cv * 8;
  float sc[8], sf[8], mu[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = scale[c + i]; sf[i] = shift[c + i]; mu[i] = mean[c + i];
    k1[i] = coef[c + i]; k2[i] = coef[C + c + i]; k3[i] = coef[2 * C + c + i];
  }
  const int64_t step = (int64_t)gridDim.x * cm.R * UNR;
  for (int64_t p0 = (int64_t)blockIdx.x * cm.R * UNR + cm.row; p0 < P; p0 += step) {
    Vec8<T> vd[UNR], vx[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * cm.R;
      if (p < P) {
        if (NT) {
          vd[u].load_nt(dy + p * dys + c);
          vx[u].load_nt(x + p * xs + c);
        } else {
          vd[u].load(dy + p * dys + c);
          vx[u].load(x + p * xs + c);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * cm.R;
      if (p >= P) continue;
      Vec8<T> vo;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float xv = vx[u].get(i), dz = vd[u].get(i);
        if (relu && !(fmaf(xv, sc[i], sf[i]) > 0.f)) dz = 0.f;
        vo.set(i, fmaf(k1[i], dz, k2[i] * (xv - mu[i])) + k3[i]);
      }
      vo.store(dx + p * dxs + c);
    }
  }
}

// Round 6: the backward apply of TWO BatchNorms (no ReLU) fed by the SAME
// output gradient -- the attention gate's W_g and W_x BatchNorms, whose
// output gradient is the psi backward's ds (unet_parts.py:11-20): dz read
// once, both input gradients written; per element exactly
// bn_bwd_apply_kernel's arithmetic.
template <typename T, bool NT>
__global__ __launch_bounds__(256) void bn_bwd_apply2_kernel(const T* dy, int64_t dys, const T* x1, int64_t x1s, const T* x2, int64_t x2s,
                                     int64_t P, int C, const float* mean1, const float* coef1, const float* mean2,
                                     const float* coef2, T* dx1, int64_t dx1s, T* dx2, int64_t dx2s) {
  ChanMap cm(C);
  const int c = cm.cv * 8;
  float mu1[8], a1[8], b1[8], e1[8], mu2[8], a2[8], b2[8], e2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu1[i] = mean1[c + i]; a1[i] = coef1[c + i]; b1[i] = coef1[C + c + i]; e1[i] = coef1[2 * C + c + i];
    mu2[i] = mean2[c + i]; a2[i] = coef2[c + i]; b2[i] = coef2[C + c + i]; e2[i] = coef2[2 * C + c + i];
  }
  const int64_t step = (int64_t)gridDim.x * cm.R * UNR;
  for (int64_t p0 = (int64_t)blockIdx.x * cm.R * UNR + cm.row; p0 < P; p0 += step) {
    Vec8<T> vd[UNR], v1[UNR], v2[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * cm.R;
      if (p < P) {
        if (NT) {
          vd[u].load_nt(dy + p * dys + c);
          v1[u].load_nt(x1 + p * x1s + c);
          v2[u].load_nt(x2 + p * x2s + c);
        } else {
          vd[u].load(dy + p * dys + c);
          v1[u].load(x1 + p * x1s + c);
          v2[u].load(x2 + p * x2s + c);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * cm.R;
      if (p >= P) continue;
      Vec8<T> o1, o2;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float dz = vd[u].get(i);
        o1.set(i, fmaf(a1[i], dz, b1[i] * (v1[u].get(i) - mu1[i])) + e1[i]);
        o2.set(i, fmaf(a2[i], dz, b2[i] * (v2[u].get(i) - mu2[i])) + e2[i]);
      }
      o1.store(dx1 + p * dx1s + c);
      o2.store(dx2 + p * dx2s + c);
    }
  }
}

template <typename T>
__global__ void bn_bwd_apply_scalar(const T* dy, int64_t dys, const T* x, int64_t xs, int64_t P, int C,
                                    const float* scale, const float* shift, const float* mean,
                                    const float* coef, int relu, T* dx, int64_t dxs) {
  int64_t tot = P * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = e / C;
    int c = (int)(e - p * C);
    float xv = ld1<T>(x + p * xs + c), dz = ld1<T>(dy + p * dys + c);
    if (relu && !(fmaf(xv, scale[c], shift[c]) > 0.f)) dz = 0.f;
    st1<T>(dx + p * dxs + c, fmaf(coef[c], dz, coef[C + c] * (xv - mean[c])) + coef[2 * C + c]);
  }
}

template <typename T>
__global__ void bn_apply_scalar(const T* x, int64_t xs, T* y, int64_t ys, int64_t P, int C,
                                const float* scale, const float* shift, int relu) {
  int64_t tot = P * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = e / C;
    int c = (int)(e - p * C);
    float z = ld1<T>(x + p * xs + c) * scale[c] + shift[c];
    st1<T>(y + p * ys + c, relu ? fmaxf(z, 0.f) : z);
  }
}

// ---- BatchNorm(+ReLU) fused with MaxPool2d(2) (Down, unet_parts.py:51-63;
//      the encoder DoubleConv outputs feed the pool and the skip) ----
// a = relu(y*scale + shift) rounded to T is written (the skip
// connection and the max-pool backward read it) and the 2x2 max of the
// rounded values goes to the pooled tensor in the same pass -- one read of
// y instead of y, then a.  A thread owns 8 channels; a row is one pooled pixel
// (its 2x2 window = 4 loads in flight).
template <typename T>
__global__ void bn_apply_maxpool_kernel(const T* y, int64_t ys, T* a, int64_t as, T* pool, int64_t ps, int N,
                                        int H, int W, int C, const float* scale, const float* shift, int relu) {
  ChanMap cm(C);
  const int c = cm.cv * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { sc[i] = scale[c + i]; sh[i] = shift[c + i]; }
  const int Ho = H >> 1, Wo = W >> 1;
  const int64_t Q = (int64_t)N * Ho * Wo;
  for (int64_t q = (int64_t)blockIdx.x * cm.R + cm.row; q < Q; q += (int64_t)gridDim.x * cm.R) {
    const int j = (int)(q % Wo);
    const int64_t t = q / Wo;
    const int i = (int)(t % Ho), n = (int)(t / Ho);
    const int64_t p00 = ((int64_t)n * H + 2 * i) * W + 2 * j;
    Vec8<T> v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k].load(y + (p00 + (k >> 1) * W + (k & 1)) * ys + c);
    float best[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) best[e] = -INFINITY;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float z = v[k].get(e) * sc[e] + sh[e];
        v[k].set(e, relu ? fmaxf(z, 0.f) : z);
        const float f = v[k].get(e);  // the stored (rounded) value
        if (f > best[e] || isnan(f)) best[e] = f;
      }
      v[k].store(a + (p00 + (k >> 1) * W + (k & 1)) * as + c);
    }
    Vec8<T> o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.set(e, best[e]);
    o.store(pool + q * ps + c);
  }
}

// ---- BatchNorm(+ReLU) backward THROUGH the 2x2 max-pool (round 4) ----------
// The encoder DoubleConvs' BN2 output a = relu(BN(y)) feeds the next Down's
// max-pool and the decoder's skip concat.  Its backward used to be: max-pool
// backward (reads a, the skip gradient and the pooled gradient, writes the
// full-size gradient of a), then the BN backward reduce (reads that gradient
// and y) and apply (reads both again, writes dy): 8.25 full-size passes.  Here
// neither a nor its gradient is touched: each pass recomputes, per 2x2
// window, a = T(relu(fma(y, scale, shift))) exactly as vu_bn_apply_maxpool2
// stored it, its first-max argmax, and the gradient of a as the max-pool
// backward stored it, T(skip + [argmax] pooled) -- bit-identical inputs to
// the BN backward -- from y, the skip gradient and the pooled gradient:
// 5.5 passes.  A thread owns 8 channels of one pooled pixel (its window).
struct PoolBnArgs {
  const void* y; int64_t ys;       // BN input (the conv output), full size
  const void* dp; int64_t dps;     // gradient of the pooled output
  const void* add; int64_t adds;   // skip-connection gradient (full size) or null
  int N, H, W, C;
  const float* scale; const float* shift; const float* mean; const float* invstd;
  int relu;
  float* part;                     // partial pass: [nblk][2][C]
  const float* coef;               // apply pass: k1, k2, k3 [3][C] (bn_bwd_final)
  void* dx; int64_t dxs;           // apply pass: gradient of y
};

template <typename T, bool NT>
VU_DEV void pool_window(const PoolBnArgs& r, int64_t q, int c, const float (&sc)[8], const float (&sf)[8],
                        float (&yv)[4][8], float (&dz)[4][8], int64_t& p00) {
  const int Wo = r.W >> 1, Ho = r.H >> 1;
  const int j = (int)(q % Wo);
  const int64_t t = q / Wo;
  const int i = (int)(t % Ho), n = (int)(t / Ho);
  p00 = ((int64_t)n * r.H + 2 * i) * r.W + 2 * j;
  const T* y = reinterpret_cast<const T*>(r.y);
  const T* ad = reinterpret_cast<const T*>(r.add);
  Vec8<T> vy[4], va[4], vg;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t pix = p00 + (k >> 1) * r.W + (k & 1);
    if (NT) vy[k].load_nt(y + pix * r.ys + c); else vy[k].load(y + pix * r.ys + c);
    if (ad) { if (NT) va[k].load_nt(ad + pix * r.adds + c); else va[k].load(ad + pix * r.adds + c); }
  }
  vg.load(reinterpret_cast<const T*>(r.dp) + q * r.dps + c);
  float best[8];
  int arg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      yv[k][e] = vy[k].get(e);
      const float z = fmaf(yv[k][e], sc[e], sf[e]);
      const float f = rnd<T>(r.relu ? fmaxf(z, 0.f) : z);  // the stored activation
      if (f > best[e] || isnan(f)) { best[e] = f; arg[e] = k; }
    }
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float o = ad ? va[k].get(e) : 0.f;
      if (arg[e] == k) o += vg.get(e);
      float d = rnd<T>(o);                                   // the stored pool-input gradient
      if (r.relu && !(fmaf(yv[k][e], sc[e], sf[e]) > 0.f)) d = 0.f;
      dz[k][e] = d;
    }
}

template <typename T, bool NT>
__global__ void pool_bn_partial_kernel(PoolBnArgs r) {
  __shared__ float sh[2][256 * 8];
  ChanMap cm(r.C);
  const int c = cm.cv * 8;
  float s0[8], s1[8], sc[8], sf[8], mu[8], is[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s0[e] = 0.f; s1[e] = 0.f;
    sc[e] = r.scale[c + e]; sf[e] = r.shift[c + e]; mu[e] = r.mean[c + e]; is[e] = r.invstd[c + e];
  }
  const int64_t Q = (int64_t)r.N * (r.H >> 1) * (r.W >> 1);
  for (int64_t q = (int64_t)blockIdx.x * cm.R + cm.row; q < Q; q += (int64_t)gridDim.x * cm.R) {
    float yv[4][8], dz[4][8];
    int64_t p00;
    pool_window<T, NT>(r, q, c, sc, sf, yv, dz, p00);
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s0[e] += dz[k][e];
        s1[e] += dz[k][e] * ((yv[k][e] - mu[e]) * is[e]);
      }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { sh[0][cm.row * r.C + c + e] = s0[e]; sh[1][cm.row * r.C + c + e] = s1[e]; }
  __syncthreads();
  for (int cc = threadIdx.x; cc < r.C; cc += 256) {
    float a0 = 0.f, a1 = 0.f;
    a0 = lds_sum(&sh[0][cc], cm.R, r.C);
    a1 = lds_sum(&sh[1][cc], cm.R, r.C);
    r.part[((int64_t)blockIdx.x * 2 + 0) * r.C + cc] = a0;
    r.part[((int64_t)blockIdx.x * 2 + 1) * r.C + cc] = a1;
  }
}

template <typename T, bool NT>
__global__ void pool_bn_apply_kernel(PoolBnArgs r) {
  ChanMap cm(r.C);
  const int c = cm.cv * 8;
  float sc[8], sf[8], mu[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = r.scale[c + e]; sf[e] = r.shift[c + e]; mu[e] = r.mean[c + e];
    k1[e] = r.coef[c + e]; k2[e] = r.coef[r.C + c + e]; k3[e] = r.coef[2 * r.C + c + e];
  }
  T* dx = reinterpret_cast<T*>(r.dx);
  const int64_t Q = (int64_t)r.N * (r.H >> 1) * (r.W >> 1);
  for (int64_t q = (int64_t)blockIdx.x * cm.R + cm.row; q < Q; q += (int64_t)gridDim.x * cm.R) {
    float yv[4][8], dz[4][8];
    int64_t p00;
    pool_window<T, NT>(r, q, c, sc, sf, yv, dz, p00);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      Vec8<T> vo;
#pragma unroll
      for (int e = 0; e < 8; ++e) vo.set(e, k1[e] * dz[k][e] + k2[e] * (yv[k][e] - mu[e]) + k3[e]);
      vo.store(dx + (p00 + (k >> 1) * r.W + (k & 1)) * r.dxs + c);
    }
  }
}

// ---- BatchNorm forward for SMALL tensors: finalize + apply in one launch ----
// The ResNet34 encoder's 64^2-16^2 levels (and the U-Net's 32^2 level) have
// 16-256 partial-statistics tiles; there the two finalize launches and the
// apply are each latency-bound (~5-10 us for a few MB), so a layer spent more
// time in its BatchNorm than in its convolution.  Here a block owns 32
// channels x a pixel range: it combines the (sum, centered M2) partials of its
// 32 channels itself (fp64, the exact group-mean form of bn_stats_stage1 /
// stage2), then applies out = [relu](y*scale + shift [+ residual]) to its
// pixels.  The blocks of one channel group repeat the (small) combine; the
// first writes the coefficients (scale, shift, mean, invstd) and the running
// statistics.  256 threads = 32 channels x 8 tile lanes (combine), then 4
// lanes x 8 channels x 64 pixel rows (apply).
constexpr int BNF_MAXT = 256;  // tiles a block combines (8 tile lanes x 32)

struct BnFusedArgs {
  const float* psum; const float* pm2; int tiles; int64_t tile_rows; int64_t P; int C;
  const float* gamma; const float* beta; float* rmean; float* rvar; int64_t* nbt; float momentum; float eps;
  float* coef;                               // [4][C]: scale, shift, mean, invstd
  const void* y; int64_t ys;
  const void* res; int64_t rs; const float* rsc; const float* rsh;   // optional residual (+ its BN)
  void* out; int64_t os; int relu; int split;
};

template <typename T>
__global__ __launch_bounds__(256) void bn_fwd_fused_kernel(BnFusedArgs a) {
  __shared__ double shd[8][32];
  __shared__ float ssc[32], ssh[32];
  const int cg = blockIdx.x / a.split, sp = blockIdx.x - cg * a.split;
  const int tid = threadIdx.x;
  // ---- combine: lane (cl, tl) takes tiles tl, tl + 8, ... of channel cg*32 + cl
  {
    const int cl = tid & 31, tl = tid >> 5;
    const int c = cg * 32 + cl;
    // the per-channel operands first (bn_stats_stage2)
    const float g = a.gamma ? a.gamma[c] : 1.f, b = a.beta ? a.beta[c] : 0.f;
    const bool upd = sp == 0 && a.rmean && a.momentum != 0.f;
    const float rm0 = upd ? a.rmean[c] : 0.f, rv0 = upd ? a.rvar[c] : 0.f;
    const int64_t nb0 = (sp == 0 && a.nbt) ? a.nbt[0] : 0;
    constexpr int U = BNF_MAXT / 8;
    float sv[U], mv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = min(tl + 8 * u, a.tiles - 1);  // clamped, unconditional loads
      sv[u] = a.psum[(int64_t)t * a.C + c];
      mv[u] = a.pm2[(int64_t)t * a.C + c];
    }
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) s += tl + 8 * u < a.tiles ? (double)sv[u] : 0.0;
    shd[tl][cl] = s;
    __syncthreads();
    double tot = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) tot += shd[k][cl];
    const double m = tot / (double)a.P;
    __syncthreads();
    double q = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = tl + 8 * u;
      if (t < a.tiles) {
        const int64_t nt64 = a.P - (int64_t)t * a.tile_rows;
        const double nt = (double)(nt64 > a.tile_rows ? a.tile_rows : nt64);
        const double d = (double)sv[u] / nt - m;
        q += (double)mv[u] + nt * d * d;
      }
    }
    shd[tl][cl] = q;
    __syncthreads();
    if (tl == 0) {
      double M2 = 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k) M2 += shd[k][cl];
      const double n = (double)a.P;
      const double var = M2 / n;
      const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
      const float mean = (float)m;
      const float scale = g * invstd, shift = b - mean * g * invstd;
      ssc[cl] = scale;
      ssh[cl] = shift;
      if (sp == 0) {
        a.coef[c] = scale;
        a.coef[a.C + c] = shift;
        a.coef[2 * a.C + c] = mean;
        a.coef[3 * a.C + c] = invstd;
        if (a.nbt && c == 0) a.nbt[0] = nb0 + 1;
        if (upd) {
          const double unb = n > 1 ? M2 / (n - 1) : var;
          a.rmean[c] = (1.f - a.momentum) * rm0 + a.momentum * mean;
          a.rvar[c] = (1.f - a.momentum) * rv0 + a.momentum * (float)unb;
        }
      }
    }
    __syncthreads();
  }
  // ---- apply over this block's pixel range
  const int cv = tid & 3, row = tid >> 2;
  const int c = cg * 32 + cv * 8;
  float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = ssc[cv * 8 + i];
    sh[i] = ssh[cv * 8 + i];
    rsc[i] = 1.f;
    rsh[i] = 0.f;
  }
  if (a.rsc) {   // one uniform branch around all 16 loads: they issue together
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      rsc[i] = a.rsc[c + i];
      rsh[i] = a.rsh[c + i];
    }
  }
  const int64_t per = (a.P + a.split - 1) / a.split;
  const int64_t p_beg = (int64_t)sp * per, p_end = min(a.P, p_beg + per);
  const T* y = reinterpret_cast<const T*>(a.y);
  const T* r = reinterpret_cast<const T*>(a.res);
  T* out = reinterpret_cast<T*>(a.out);
  for (int64_t p0 = p_beg + row; p0 < p_end; p0 += 64 * UNR) {
    // clamped, unguarded loads (a guarded pair per row sat behind its own
    // vmcnt(0): UNR serial round trips per iteration)
    Vec8<T> vy[UNR], vr[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * 64 < p_end ? p0 + (int64_t)u * 64 : p_end - 1;
      vy[u].load(y + p * a.ys + c);
    }
    if (r) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int64_t p = p0 + (int64_t)u * 64 < p_end ? p0 + (int64_t)u * 64 : p_end - 1;
        vr[u].load(r + p * a.rs + c);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * 64;
      if (p >= p_end) continue;
      Vec8<T> vo;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float z = vy[u].get(i) * sc[i] + sh[i];
        if (r) {
          float rr = vr[u].get(i);
          if (a.rsc) rr = rr * rsc[i] + rsh[i];
          z = z + rr;
        }
        vo.set(i, a.relu ? fmaxf(z, 0.f) : z);
      }
      vo.store(out + p * a.os + c);
    }
  }
}

// ---- BatchNorm backward for SMALL tensors: the fp64 finish of the per-channel
//      sums folded into the apply pass (bn_bwd_final + bn_bwd_apply in one
//      launch; the partial pass chan_partial_kernel stays) ----
// A block owns 32 channels x a pixel range; it sums the <= 128 partial rows
// of its channels itself (fp64), forms k1 = gamma*invstd, k2 = -k1*invstd*
// sum(dz*xhat)/P, k3 = -k1*sum(dz)/P exactly as bn_bwd_final, and applies
// dx = k1*dz + k2*(x - mean) + k3; the first block of a channel group writes
// dgamma / dbeta.
constexpr int BNB_FUSED_MAXBLK = 128;

struct BnBwdFusedArgs {
  const void* dy; int64_t dys; const void* x; int64_t xs; int64_t P; int C;
  const float* scale; const float* shift; const float* mean; const float* invstd; const float* gamma;
  int relu; int train; const float* part; int nblk;
  float* dgamma; float* dbeta; int accumulate;
  void* dx; int64_t dxs; int split;
};

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_fused_apply_kernel(BnBwdFusedArgs a) {
  __shared__ double shd[2][8][32];
  __shared__ float sk[3][32];
  const int cg = blockIdx.x / a.split, sp = blockIdx.x - cg * a.split;
  const int tid = threadIdx.x;
  {
    const int cl = tid & 31, tl = tid >> 5;
    const int c = cg * 32 + cl;
    // the per-channel operands first (after the trees, behind the stores
    // they may alias, they were 3 serial round trips)
    const float g = a.gamma ? a.gamma[c] : 1.f;
    const float is = a.invstd[c];
    const bool wr = sp == 0 && a.accumulate;
    const float dg0 = (wr && a.dgamma) ? a.dgamma[c] : 0.f;
    const float db0 = (wr && a.dbeta) ? a.dbeta[c] : 0.f;
    double s0 = 0.0, s1 = 0.0;
    for (int r0 = tl; r0 < a.nblk; r0 += 64) {
      float v0[8], v1[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = min(r0 + 8 * u, a.nblk - 1);  // clamped, unconditional loads
        v0[u] = a.part[((int64_t)r * 2 + 0) * a.C + c];
        v1[u] = a.part[((int64_t)r * 2 + 1) * a.C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (r0 + 8 * u < a.nblk) {
          s0 += (double)v0[u];
          s1 += (double)v1[u];
        }
    }
    shd[0][tl][cl] = s0;
    shd[1][tl][cl] = s1;
    __syncthreads();
    if (tl == 0) {
      double S0 = 0.0, S1 = 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        S0 += shd[0][k][cl];
        S1 += shd[1][k][cl];
      }
      const float k1 = g * is;
      sk[0][cl] = k1;
      sk[1][cl] = a.train ? (float)(-(double)k1 * is * S1 / (double)a.P) : 0.f;
      sk[2][cl] = a.train ? (float)(-(double)k1 * S0 / (double)a.P) : 0.f;
      if (sp == 0) {
        if (a.dgamma) a.dgamma[c] = a.accumulate ? dg0 + (float)S1 : (float)S1;
        if (a.dbeta) a.dbeta[c] = a.accumulate ? db0 + (float)S0 : (float)S0;
      }
    }
    __syncthreads();
  }
  const int cv = tid & 3, row = tid >> 2;
  const int c = cg * 32 + cv * 8;
  float sc[8], sf[8], mu[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = a.scale[c + i];
    sf[i] = a.shift[c + i];
    mu[i] = a.mean[c + i];
    k1[i] = sk[0][cv * 8 + i];
    k2[i] = sk[1][cv * 8 + i];
    k3[i] = sk[2][cv * 8 + i];
  }
  const int64_t per = (a.P + a.split - 1) / a.split;
  const int64_t p_beg = (int64_t)sp * per, p_end = min(a.P, p_beg + per);
  const T* dy = reinterpret_cast<const T*>(a.dy);
  const T* x = reinterpret_cast<const T*>(a.x);
  T* dx = reinterpret_cast<T*>(a.dx);
  for (int64_t p0 = p_beg + row; p0 < p_end; p0 += 64 * UNR) {
    Vec8<T> vd[UNR], vx[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * 64;
      if (p < p_end) {
        vd[u].load(dy + p * a.dys + c);
        vx[u].load(x + p * a.xs + c);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = p0 + (int64_t)u * 64;
      if (p >= p_end) continue;
      Vec8<T> vo;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xv = vx[u].get(i);
        float dz = vd[u].get(i);
        if (a.relu && !(fmaf(xv, sc[i], sf[i]) > 0.f)) dz = 0.f;
        vo.set(i, fmaf(k1[i], dz, k2[i] * (xv - mu[i])) + k3[i]);
      }
      vo.store(dx + p * a.dxs + c);
    }
  }
}

inline unsigned ew_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

inline bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

// vectorised fixed-channel path: C = 8 * 2^k <= 2048, strides multiples of 8
inline bool chanmap_ok(int C, int64_t s0, int64_t s1, int64_t s2 = 0) {
  return C % 8 == 0 && pow2(C / 8) && C / 8 <= 256 && s0 % 8 == 0 && s1 % 8 == 0 && s2 % 8 == 0;
}

// blocks for a fixed-channel stream over P pixels: ~16 pixel rows per thread
// (the size class the fused small-tensor paths are admitted by)
inline unsigned chan_grid16(int64_t P, int C, int maxblk) {
  int R = 256 / (C / 8);
  int64_t g = (P + (int64_t)R * 16 - 1) / ((int64_t)R * 16);
  if (g > maxblk) g = maxblk;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Launch grid of the streaming kernels: ~16 pixel rows per thread on large
// tensors, but on small ones at least g_bn_minblk blocks (down to one UNR-deep
// load round per thread): a 64-block grid whose threads each wait out four
// dependent load rounds was latency-bound (9 us for the 4 MB of a ResNet34
// layer3 BN backward).  VU_TUNE_BN_MINBLK, 0 = the 16-row grid only.
int g_bn_minblk = 256;
int g_bn_onepass = 0;  // VU_TUNE_BN_ONEPASS (vu_bn_bwd_fused below; measured slower, off)
int g_bn_stats1 = 0;   // VU_TUNE_BN_STATS1 (vu_bn_finalize as one launch; measured slower, off)
inline unsigned chan_grid(int64_t P, int C, int maxblk) {
  int R = 256 / (C / 8);
  int64_t g = (P + (int64_t)R * 16 - 1) / ((int64_t)R * 16);
  const int64_t g1 = (P + (int64_t)R * UNR - 1) / ((int64_t)R * UNR);
  const int64_t lo = g1 < g_bn_minblk ? g1 : g_bn_minblk;
  if (g < lo) g = lo;
  if (g > maxblk) g = maxblk;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Non-temporal loads for the streams of a large tensor: those bytes cannot
// stay in the 256 MB Infinity Cache until their next use anyway, and keeping
// them out leaves it to the smaller tensors.  Same-box A/B
// (profiles/r2_ab_bn_nt.log): UNet 483 -> 491 img/s for any threshold of
// 0-128 MB; VAE 708 at -1 (never), 701-703 at 0 (always), 708 at 32 MB.
// Threshold in MB per streamed tensor (VU_TUNE_BN_NT_MB, for A/B runs; -1 = never).
int g_bn_nt_mb = 32;
inline bool bn_nt(int64_t P, int C, int esize) {
  const int64_t mb = g_bn_nt_mb;
  return mb >= 0 && P * C * esize >= mb * 1000000;
}

typedef void (*ApplyFn)(const bf16_t*, int64_t, bf16_t*, int64_t, int64_t, int, const float*, const float*, int);
typedef void (*BwdApplyFn)(const bf16_t*, int64_t, const bf16_t*, int64_t, int64_t, int, const float*,
                           const float*, const float*, const float*, int, bf16_t*, int64_t);
inline ApplyFn bn_apply_bf16(int64_t P, int C) {
  return bn_nt(P, C, 2) ? bn_apply_kernel<bf16_t, true> : bn_apply_kernel<bf16_t, false>;
}
inline BwdApplyFn bn_bwd_apply_bf16(int64_t P, int C) {
  return bn_nt(P, C, 2) ? bn_bwd_apply_kernel<bf16_t, true> : bn_bwd_apply_kernel<bf16_t, false>;
}

template <typename T, int MODE>
int launch_partial(const RedArgs& r, hipStream_t st, int& nblk, int maxblk = RED_MAXBLK) {
  bool vec = chanmap_ok(r.C, r.as, MODE == 0 ? 8 : r.bs);
  if (vec) {
    nblk = (int)chan_grid(r.P, r.C, maxblk);
    if (std::is_same<T, bf16_t>::value && bn_nt(r.P, r.C, 2))
      hipLaunchKernelGGL((chan_partial_kernel<T, MODE, true>), dim3(nblk), dim3(256), 0, st, r);
    else
      hipLaunchKernelGGL((chan_partial_kernel<T, MODE, false>), dim3(nblk), dim3(256), 0, st, r);
  } else if (r.C <= 256) {
    int R = 256 / r.C;
    int64_t g = (r.P + (int64_t)R * 16 - 1) / ((int64_t)R * 16);
    nblk = (int)(g > RED_MAXBLK ? RED_MAXBLK : (g < 1 ? 1 : g));
    hipLaunchKernelGGL((chan_partial_scalar<T, MODE>), dim3(nblk), dim3(256), 0, st, r);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace

int bn_tune(int key, int value) {
  if (key == VU_TUNE_BN_NT_MB) {
    g_bn_nt_mb = value;
    return 0;
  }
  if (key == VU_TUNE_BN_ONEPASS) {
    g_bn_onepass = value ? 1 : 0;
    return 0;
  }
  if (key == VU_TUNE_BN_STATS1) {
    g_bn_stats1 = value ? 1 : 0;
    return 0;
  }
  if (key == VU_TUNE_BN_MINBLK) {
    g_bn_minblk = value < 0 ? 0 : value;
    return 0;
  }
  return -1;
}

extern "C" int64_t vu_reduce_workspace_bytes(int64_t P, int C) {
  (void)P;
  return (int64_t)RED_MAXBLK * 2 * C * (int64_t)sizeof(float);
}

static int stats_blocks(int tiles) {
  int S = (tiles + STATS_TPB - 1) / STATS_TPB;
  if (S > STATS_MAXS) S = STATS_MAXS;
  if (S < 1) S = 1;
  return S;
}

extern "C" int64_t vu_bn_finalize_workspace_bytes(int tiles, int C) {
  int S = stats_blocks(tiles);
  return (int64_t)S * C * 3 * sizeof(double);
}

extern "C" int vu_bn_finalize(const float* psum, const float* pm2, int tiles, int64_t tile_rows,
                              int64_t rows, int C, const float* gamma, const float* beta,
                              float* running_mean, float* running_var, float momentum, float eps,
                              float* scale, float* shift, float* save_mean, float* save_invstd,
                              int64_t* num_batches_tracked, float* workspace, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  double* ws = reinterpret_cast<double*>(workspace);
  if (g_bn_stats1 && C <= 64 * FST_MAXG && tiles >= 1) {
    // (its S * C * 2 doubles fit in stats_blocks' S * C * 3: fewer blocks of more tiles)
    int S2 = (tiles + FST_TPB - 1) / FST_TPB;
    S2 = S2 > FST_MAXS ? FST_MAXS : S2;
    hipLaunchKernelGGL(bn_stats_fused_kernel, dim3((C + 63) / 64, S2), dim3(1024), 0, st, psum, pm2, tiles,
                       tile_rows, rows, C, S2, ws, gamma, beta, running_mean, running_var, momentum, eps, scale,
                       shift, save_mean, save_invstd, num_batches_tracked);
    return (int)hipGetLastError();
  }
  int S = stats_blocks(tiles);
  hipLaunchKernelGGL(bn_stats_stage1, dim3((C + 63) / 64, S), dim3(256), 0, st, psum, pm2, tiles,
                     tile_rows, rows, C, S, ws);
  hipLaunchKernelGGL(bn_stats_stage2, dim3((C + 31) / 32), dim3(1024), 0, st, ws, S, C, gamma, beta,
                     running_mean, running_var, momentum, eps, scale, shift, save_mean, save_invstd,
                     num_batches_tracked);
  return (int)hipGetLastError();
}

extern "C" int vu_bn_eval_coeffs(const float* gamma, const float* beta, const float* running_mean,
                                 const float* running_var, float eps, int C, float* scale,
                                 float* shift, float* save_mean, float* save_invstd, void* stream) {
  hipLaunchKernelGGL(bn_eval_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, gamma,
                     beta, running_mean, running_var, eps, C, scale, shift, save_mean, save_invstd);
  return (int)hipGetLastError();
}

extern "C" int vu_bn_apply(const void* x, int64_t xs, void* y, int64_t ys, int64_t P, int C,
                           const float* scale, const float* shift, int relu, int dtype,
                           void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (P * C == 0) return 0;
  bool vec = chanmap_ok(C, xs, ys);
  if (dtype == VU_BF16) {
    if (vec)
      hipLaunchKernelGGL(bn_apply_bf16(P, C), dim3(chan_grid(P, C, 8192)), dim3(256), 0, st,
                         (const bf16_t*)x, xs, (bf16_t*)y, ys, P, C, scale, shift, relu);
    else
      hipLaunchKernelGGL(bn_apply_scalar<bf16_t>, dim3(ew_grid(P * C)), dim3(256), 0, st,
                         (const bf16_t*)x, xs, (bf16_t*)y, ys, P, C, scale, shift, relu);
  } else {
    if (vec)
      hipLaunchKernelGGL((bn_apply_kernel<float, false>), dim3(chan_grid(P, C, 8192)), dim3(256), 0, st,
                         (const float*)x, xs, (float*)y, ys, P, C, scale, shift, relu);
    else
      hipLaunchKernelGGL(bn_apply_scalar<float>, dim3(ew_grid(P * C)), dim3(256), 0, st,
                         (const float*)x, xs, (float*)y, ys, P, C, scale, shift, relu);
  }
  return (int)hipGetLastError();
}

extern "C" int vu_bn_bwd_reduce(const void* dy, int64_t dys, const void* x, int64_t xs, int64_t P,
                                int C, const float* scale, const float* shift, const float* mean,
                                const float* invstd, const float* gamma, int relu, int train,
                                float* dgamma, float* dbeta, int accumulate, float* coef,
                                float* workspace, int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  RedArgs r{dy, dys, x, xs, P, C, scale, shift, mean, invstd, relu, workspace, 0, 0, 0, 0, 0, 0};
  int nblk = 0, rc;
  rc = dtype == VU_BF16 ? launch_partial<bf16_t, 1>(r, st, nblk) : launch_partial<float, 1>(r, st, nblk);
  if (rc) return rc;
  hipLaunchKernelGGL(bn_bwd_final, dim3((C + 31) / 32), dim3(COLSUM_THREADS), 0, st, workspace, nblk, C, P,
                     gamma, invstd, dgamma, dbeta, accumulate, coef, train);
  return (int)hipGetLastError();
}

// GEMM-epilogue partials come per 64-128-pixel row tile (16k-32k rows at
// 512^2): folded first by a grid of (channel group, row range) blocks into at
// most FOLD_MAXS rows (fp64 sums rounded once to fp32), then the fixed-order
// colsum32 of bn_bwd_final.  A single colsum32 pass over 32k rows runs on
// C/32 blocks: 2 blocks for 64 channels, 3-4x the time of both passes here.
constexpr int FOLD_MAXS = 256, FOLD_DIRECT = 1024;
static int fold_blocks(int nblk) {
  int S = (nblk + 63) / 64;
  return S > FOLD_MAXS ? FOLD_MAXS : (S < 1 ? 1 : S);
}

namespace {
__global__ void bnb_fold_kernel(const float* part, int nblk, int C, int S, float* ws) {
  __shared__ double sh[2][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const bool ok = c < C;
  const int per = (nblk + S - 1) / S;
  const int r0 = blockIdx.y * per, r1 = min(nblk, r0 + per);
  double s0 = 0.0, s1 = 0.0;
  const int cc = ok ? c : 0;
  for (int r = r0 + rl; r < r1; r += 4) {
    s0 += (double)part[((int64_t)r * 2 + 0) * C + cc];
    s1 += (double)part[((int64_t)r * 2 + 1) * C + cc];
  }
  sh[0][rl][cl] = s0;
  sh[1][rl][cl] = s1;
  __syncthreads();
  if (rl == 0 && ok) {
    ws[((int64_t)blockIdx.y * 2 + 0) * C + c] = (float)(((sh[0][0][cl] + sh[0][1][cl]) + sh[0][2][cl]) + sh[0][3][cl]);
    ws[((int64_t)blockIdx.y * 2 + 1) * C + c] = (float)(((sh[1][0][cl] + sh[1][1][cl]) + sh[1][2][cl]) + sh[1][3][cl]);
  }
}
}  // namespace

extern "C" int64_t vu_bn_bwd_finish_workspace_bytes(int nblk, int C) {
  return nblk <= FOLD_DIRECT ? 0 : (int64_t)fold_blocks(nblk) * 2 * C * (int64_t)sizeof(float);
}

extern "C" int vu_bn_bwd_finish(const float* part, int nblk, int64_t P, int C, const float* gamma,
                                const float* invstd, int train, float* dgamma, float* dbeta, int accumulate,
                                float* coef, float* workspace, void* stream) {
  if (nblk < 1 || C < 1) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (nblk > FOLD_DIRECT) {
    if (!workspace) return (int)hipErrorInvalidValue;
    const int S = fold_blocks(nblk);
    hipLaunchKernelGGL(bnb_fold_kernel, dim3((C + 63) / 64, S), dim3(256), 0, st, part, nblk, C, S, workspace);
    part = workspace;
    nblk = S;
  }
  hipLaunchKernelGGL(bn_bwd_final, dim3((C + 31) / 32), dim3(COLSUM_THREADS), 0, st, part, nblk, C, P, gamma,
                     invstd, dgamma, dbeta, accumulate, coef, train);
  return (int)hipGetLastError();
}

extern "C" int vu_bn_bwd_apply(const void* dy, int64_t dys, const void* x, int64_t xs, int64_t P,
                               int C, const float* scale, const float* shift, const float* mean,
                               const float* coef, int relu, void* dx, int64_t dxs, int dtype,
                               void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (P * C == 0) return 0;
  bool vec = chanmap_ok(C, dys, xs, dxs);
  if (dtype == VU_BF16) {
    if (vec)
      hipLaunchKernelGGL(bn_bwd_apply_bf16(P, C), dim3(chan_grid(P, C, 8192)), dim3(256), 0, st,
                         (const bf16_t*)dy, dys, (const bf16_t*)x, xs, P, C, scale, shift, mean, coef,
                         relu, (bf16_t*)dx, dxs);
    else
      hipLaunchKernelGGL(bn_bwd_apply_scalar<bf16_t>, dim3(ew_grid(P * C)), dim3(256), 0, st,
                         (const bf16_t*)dy, dys, (const bf16_t*)x, xs, P, C, scale, shift, mean, coef,
                         relu, (bf16_t*)dx, dxs);
  } else {
    if (vec)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<float, false>), dim3(chan_grid(P, C, 8192)), dim3(256), 0, st,
                         (const float*)dy, dys, (const float*)x, xs, P, C, scale, shift, mean, coef,
                         relu, (float*)dx, dxs);
    else
      hipLaunchKernelGGL(bn_bwd_apply_scalar<float>, dim3(ew_grid(P * C)), dim3(256), 0, st,
                         (const float*)dy, dys, (const float*)x, xs, P, C, scale, shift, mean, coef,
                         relu, (float*)dx, dxs);
  }
  return (int)hipGetLastError();
}

extern "C" int vu_bn_bwd_apply2_ok(int C, int64_t dys, int64_t x1s, int64_t x2s, int64_t dx1s, int64_t dx2s) {
  return chanmap_ok(C, dys, x1s, x2s) && chanmap_ok(C, dx1s, dx2s, 8) ? 1 : 0;
}

extern "C" int vu_bn_bwd_apply2(const void* dy, int64_t dys, const void* x1, int64_t x1s, const void* x2,
                                int64_t x2s, int64_t P, int C, const float* mean1, const float* coef1,
                                const float* mean2, const float* coef2, void* dx1, int64_t dx1s, void* dx2,
                                int64_t dx2s, int dtype, void* stream) {
  if (!vu_bn_bwd_apply2_ok(C, dys, x1s, x2s, dx1s, dx2s)) return (int)hipErrorInvalidValue;
  if (P * C == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = chan_grid(P, C, 8192);
  if (dtype == VU_BF16) {
    if (bn_nt(P, C, 2))
      hipLaunchKernelGGL((bn_bwd_apply2_kernel<bf16_t, true>), dim3(grid), dim3(256), 0, st, (const bf16_t*)dy, dys,
                         (const bf16_t*)x1, x1s, (const bf16_t*)x2, x2s, P, C, mean1, coef1, mean2, coef2,
                         (bf16_t*)dx1, dx1s, (bf16_t*)dx2, dx2s);
    else
      hipLaunchKernelGGL((bn_bwd_apply2_kernel<bf16_t, false>), dim3(grid), dim3(256), 0, st, (const bf16_t*)dy,
                         dys, (const bf16_t*)x1, x1s, (const bf16_t*)x2, x2s, P, C, mean1, coef1, mean2, coef2,
                         (bf16_t*)dx1, dx1s, (bf16_t*)dx2, dx2s);
  } else {
    hipLaunchKernelGGL((bn_bwd_apply2_kernel<float, false>), dim3(grid), dim3(256), 0, st, (const float*)dy, dys,
                       (const float*)x1, x1s, (const float*)x2, x2s, P, C, mean1, coef1, mean2, coef2, (float*)dx1,
                       dx1s, (float*)dx2, dx2s);
  }
  return (int)hipGetLastError();
}

extern "C" int vu_chan_sum(const void* x, int64_t stride, int N, int H, int W, int y0, int x0, int Hr,
                           int Wr, int C, float* out, int accumulate, float* workspace, int dtype,
                           void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int64_t P = (int64_t)N * Hr * Wr;
  RedArgs r{x, stride, nullptr, 0, P, C, nullptr, nullptr, nullptr, nullptr, 0, workspace, H, W, y0, x0, Hr, Wr};
  int nblk = 0, rc;
  rc = dtype == VU_BF16 ? launch_partial<bf16_t, 0>(r, st, nblk) : launch_partial<float, 0>(r, st, nblk);
  if (rc) return rc;
  hipLaunchKernelGGL(chan_final_sum, dim3((C + 31) / 32), dim3(COLSUM_THREADS), 0, st, workspace, nblk, C, out,
                     accumulate);
  return (int)hipGetLastError();
}

// MaxPool2d(2) fusion (even H, W; C = 8 * 2^k <= 2048; 8-element strides)
static bool pool_fusable(int H, int W, int C, int64_t s0, int64_t s1, int64_t s2) {
  return H % 2 == 0 && W % 2 == 0 && chanmap_ok(C, s0, s1, s2);
}

extern "C" int vu_bn_apply_maxpool2(const void* y, int64_t ys, void* a, int64_t as, void* pool, int64_t ps, int N,
                                    int H, int W, int C, const float* scale, const float* shift, int relu, int dtype,
                                    void* stream) {
  if (!pool_fusable(H, W, C, ys, as, ps)) return (int)hipErrorInvalidValue;
  const int64_t Q = (int64_t)N * (H / 2) * (W / 2);
  if (Q == 0) return 0;
  const unsigned grid = chan_grid(Q * 4, C, 8192);  // ~4 pooled pixels per thread
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VU_BF16)
    hipLaunchKernelGGL(bn_apply_maxpool_kernel<bf16_t>, dim3(grid), dim3(256), 0, st, (const bf16_t*)y, ys,
                       (bf16_t*)a, as, (bf16_t*)pool, ps, N, H, W, C, scale, shift, relu);
  else
    hipLaunchKernelGGL(bn_apply_maxpool_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)y, ys,
                       (float*)a, as, (float*)pool, ps, N, H, W, C, scale, shift, relu);
  return (int)hipGetLastError();
}

// BatchNorm(+ReLU) backward through the 2x2 max-pool: partial pass, fp64
// finish (dgamma, dbeta, k1..k3 into coef [3][C]), apply pass -> dx (the
// gradient of y).  1 when served (even H and W, the vectorised channel map).
extern "C" int vu_bn_bwd_pool_supported(int H, int W, int C, int64_t ys, int64_t dps, int64_t adds, int64_t dxs) {
  return H % 2 == 0 && W % 2 == 0 && H > 0 && W > 0 && chanmap_ok(C, ys, dps, adds) && dxs % 8 == 0;
}

extern "C" int vu_bn_bwd_pool(const void* y, int64_t ys, const void* dp, int64_t dps, const void* add, int64_t adds,
                              int N, int H, int W, int C, const float* scale, const float* shift, const float* mean,
                              const float* invstd, const float* gamma, int relu, int train, float* dgamma,
                              float* dbeta, int accumulate, float* coef, float* workspace, void* dx, int64_t dxs,
                              int dtype, void* stream) {
  if (!vu_bn_bwd_pool_supported(H, W, C, ys, dps, add ? adds : 8, dxs) || N < 1) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int64_t P = (int64_t)N * H * W;
  PoolBnArgs r{y, ys, dp, dps, add, adds, N, H, W, C, scale, shift, mean, invstd, relu, workspace, coef, dx, dxs};
  const int nblk = (int)chan_grid(P, C, RED_MAXBLK);  // rows = pooled pixels: ~4 windows per thread
  const bool nt = bn_nt(P, C, dtype == VU_BF16 ? 2 : 4);
  const unsigned agrid = chan_grid(P, C, 8192);
  if (dtype == VU_BF16) {
    if (nt) hipLaunchKernelGGL((pool_bn_partial_kernel<bf16_t, true>), dim3(nblk), dim3(256), 0, st, r);
    else hipLaunchKernelGGL((pool_bn_partial_kernel<bf16_t, false>), dim3(nblk), dim3(256), 0, st, r);
  } else {
    hipLaunchKernelGGL((pool_bn_partial_kernel<float, false>), dim3(nblk), dim3(256), 0, st, r);
  }
  hipLaunchKernelGGL(bn_bwd_final, dim3((C + 31) / 32), dim3(COLSUM_THREADS), 0, st, workspace, nblk, C, P, gamma,
                     invstd, dgamma, dbeta, accumulate, coef, train);
  if (dtype == VU_BF16) {
    if (nt) hipLaunchKernelGGL((pool_bn_apply_kernel<bf16_t, true>), dim3(agrid), dim3(256), 0, st, r);
    else hipLaunchKernelGGL((pool_bn_apply_kernel<bf16_t, false>), dim3(agrid), dim3(256), 0, st, r);
  } else {
    hipLaunchKernelGGL((pool_bn_apply_kernel<float, false>), dim3(agrid), dim3(256), 0, st, r);
  }
  return (int)hipGetLastError();
}

// Single-launch train-mode BatchNorm forward (finalize + apply [+ residual] [+ ReLU])
// for small tensors: vu_bn_fwd_fused_supported() says when it applies.
extern "C" int vu_bn_fwd_fused_supported(int tiles, int C, int64_t ys, int64_t rs, int64_t os) {
  return tiles >= 1 && tiles <= BNF_MAXT && C % 32 == 0 && ys % 8 == 0 && rs % 8 == 0 && os % 8 == 0;
}

extern "C" int vu_bn_fwd_fused(const float* psum, const float* pm2, int tiles, int64_t tile_rows, int64_t P, int C,
                               const float* gamma, const float* beta, float* running_mean, float* running_var,
                               int64_t* num_batches_tracked, float momentum, float eps, float* coef, const void* y,
                               int64_t ys, const void* res, int64_t rs, const float* rscale, const float* rshift,
                               void* out, int64_t os, int relu, int dtype, void* stream) {
  if (!vu_bn_fwd_fused_supported(tiles, C, ys, res ? rs : 0, os) || P < 1) return (int)hipErrorInvalidValue;
  if ((rscale == nullptr) != (rshift == nullptr)) return (int)hipErrorInvalidValue;
  BnFusedArgs a{psum, pm2, tiles, tile_rows, P, C, gamma, beta, running_mean, running_var, num_batches_tracked,
                momentum, eps, coef, y, ys, res, rs, rscale, rshift, out, os, relu, 1};
  // pixel splits per 32-channel group: ~256 blocks in all, >= 128 pixels each
  const int groups = C / 32;
  int64_t split = (256 + groups - 1) / groups;
  const int64_t maxs = (P + 127) / 128;
  if (split > maxs) split = maxs;
  if (split < 1) split = 1;
  a.split = (int)split;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VU_BF16)
    hipLaunchKernelGGL(bn_fwd_fused_kernel<bf16_t>, dim3((unsigned)(groups * split)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(bn_fwd_fused_kernel<float>, dim3((unsigned)(groups * split)), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// BatchNorm(+ReLU) backward for small tensors in two launches (the partial
// pass, then the fused fp64 finish + apply) instead of three.
// ---- one-launch BatchNorm(+ReLU) backward of a small tensor ---------------
// (P <= ONEPASS_MAXP: ResNet34 layer3 / layer4 and the 32^2 / 16^2 decoder
// levels of config 3, where the two launches of the fused path were ~7 us
// each of mostly latency; bf16): one 512-thread block per 8 channels
// reduces sum dz and sum dz * xhat over all P pixels (thread t: pixels
// t + 512 k; fp32 per thread, a fixed-order lane butterfly per wave, fp64
// across the 8 waves), writes dgamma / dbeta and applies dx.  Deterministic;
// the same per-element formulas as chan_partial_kernel<.., 1> +
// bn_bwd_fused_apply_kernel.  MEASURED SLOWER (VAE -12 %, off by default,
// profiles/r5w_ab_bn_onepass.txt): a block per 8 channels of a channels-last
// tensor reads 16 bytes per 128-byte line per pixel (every line fetched by
// C / 8 blocks), and wider channel slices leave C / 64 = 4-8 blocks -- the
// reduction needs the cross-block stage of the two-launch path.
constexpr int ONEPASS_T = 512, ONEPASS_B = 8, ONEPASS_MAXP = 8192;
constexpr int ONEPASS_W = ONEPASS_T / 64;

VU_DEV float bfly_sum64(float v) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m, 64);
  return v;
}

template <typename T>
__global__ __launch_bounds__(ONEPASS_T) void bn_bwd_onepass_kernel(BnBwdFusedArgs a) {
  __shared__ float wsum[2][ONEPASS_W][8];
  __shared__ float sk[3][8];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = blockIdx.x * 8;
  // 32-bit element offsets from the uniform bases (P * stride < 2^31, host
  // check) and clamped unconditional loads, ONEPASS_B pixels per thread in
  // flight; the apply pass re-reads its pixels (L2-resident: <= 256 KB per
  // block) rather than holding all of them in registers (that spilled)
  const int P = (int)a.P, dys = (int)a.dys, xs = (int)a.xs;
  const T* dyc = reinterpret_cast<const T*>(a.dy) + c;
  const T* xc = reinterpret_cast<const T*>(a.x) + c;
  float sc[8], sf[8], mu[8], is[8], s0[8], s1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = a.scale[c + i]; sf[i] = a.shift[c + i]; mu[i] = a.mean[c + i]; is[i] = a.invstd[c + i];
    s0[i] = 0.f; s1[i] = 0.f;
  }
  const bool wr = a.accumulate && tid < 8;
  const float g = tid < 8 ? (a.gamma ? a.gamma[c + tid] : 1.f) : 0.f;
  const float dg0 = (wr && a.dgamma) ? a.dgamma[c + tid] : 0.f;
  const float db0 = (wr && a.dbeta) ? a.dbeta[c + tid] : 0.f;
  for (int p0 = tid; p0 < P; p0 += ONEPASS_T * ONEPASS_B) {
    Vec8<T> vd[ONEPASS_B], vx[ONEPASS_B];
#pragma unroll
    for (int k = 0; k < ONEPASS_B; ++k) {
      const int p = min(p0 + k * ONEPASS_T, P - 1);
      vd[k].load(dyc + p * dys);
      vx[k].load(xc + p * xs);
    }
#pragma unroll
    for (int k = 0; k < ONEPASS_B; ++k) {
      if (p0 + k * ONEPASS_T >= P) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xv = vx[k].get(i);
        float dz = vd[k].get(i);
        if (a.relu && !(fmaf(xv, sc[i], sf[i]) > 0.f)) dz = 0.f;
        s0[i] += dz;
        s1[i] += dz * ((xv - mu[i]) * is[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float t0 = bfly_sum64(s0[i]), t1 = bfly_sum64(s1[i]);
    if (lane == 0) {
      wsum[0][wv][i] = t0;
      wsum[1][wv][i] = t1;
    }
  }
  __syncthreads();
  if (tid < 8) {
    double S0 = 0.0, S1 = 0.0;
#pragma unroll
    for (int w = 0; w < ONEPASS_W; ++w) {
      S0 += (double)wsum[0][w][tid];
      S1 += (double)wsum[1][w][tid];
    }
    const float isc = a.invstd[c + tid];
    const float k1 = g * isc;
    sk[0][tid] = k1;
    sk[1][tid] = a.train ? (float)(-(double)k1 * isc * S1 / (double)a.P) : 0.f;
    sk[2][tid] = a.train ? (float)(-(double)k1 * S0 / (double)a.P) : 0.f;
    if (a.dgamma) a.dgamma[c + tid] = a.accumulate ? dg0 + (float)S1 : (float)S1;
    if (a.dbeta) a.dbeta[c + tid] = a.accumulate ? db0 + (float)S0 : (float)S0;
  }
  __syncthreads();
  float k1[8], k2[8], k3[8];   // block-uniform: scalar registers
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    k1[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sk[0][i])));
    k2[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sk[1][i])));
    k3[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sk[2][i])));
  }
  T* dxc = reinterpret_cast<T*>(a.dx) + c;
  const int dxs = (int)a.dxs;
  for (int p0 = tid; p0 < P; p0 += ONEPASS_T * ONEPASS_B) {
    Vec8<T> vd[ONEPASS_B], vx[ONEPASS_B];
#pragma unroll
    for (int k = 0; k < ONEPASS_B; ++k) {
      const int p = min(p0 + k * ONEPASS_T, P - 1);
      vd[k].load(dyc + p * dys);
      vx[k].load(xc + p * xs);
    }
#pragma unroll
    for (int k = 0; k < ONEPASS_B; ++k) {
      const int p = p0 + k * ONEPASS_T;
      if (p >= P) continue;
      Vec8<T> vo;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xv = vx[k].get(i);
        float dz = vd[k].get(i);
        if (a.relu && !(fmaf(xv, sc[i], sf[i]) > 0.f)) dz = 0.f;
        vo.set(i, fmaf(k1[i], dz, k2[i] * (xv - mu[i])) + k3[i]);
      }
      vo.store(dxc + p * dxs);
    }
  }
}

extern "C" int vu_bn_bwd_fused_supported(int64_t P, int C, int64_t dys, int64_t xs, int64_t dxs) {
  return C % 32 == 0 && chanmap_ok(C, dys, xs) && dxs % 8 == 0 && P >= 1 &&
         (int)chan_grid16(P, C, RED_MAXBLK) <= BNB_FUSED_MAXBLK;
}

extern "C" int vu_bn_bwd_fused(const void* dy, int64_t dys, const void* x, int64_t xs, int64_t P, int C,
                               const float* scale, const float* shift, const float* mean, const float* invstd,
                               const float* gamma, int relu, int train, float* dgamma, float* dbeta,
                               int accumulate, void* dx, int64_t dxs, float* workspace, int dtype, void* stream) {
  if (!vu_bn_bwd_fused_supported(P, C, dys, xs, dxs)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (g_bn_onepass && dtype == VU_BF16 && P <= ONEPASS_MAXP && dys % 8 == 0 && xs % 8 == 0 && P * (dys > xs ? (dys > dxs ? dys : dxs) : (xs > dxs ? xs : dxs)) < ((int64_t)1 << 31)) {
    BnBwdFusedArgs a{dy, dys, x, xs, P, C, scale, shift, mean, invstd, gamma, relu, train, nullptr, 0,
                     dgamma, dbeta, accumulate, dx, dxs, 1};
    hipLaunchKernelGGL(bn_bwd_onepass_kernel<bf16_t>, dim3((unsigned)(C / 8)), dim3(ONEPASS_T), 0, st, a);
    return (int)hipGetLastError();
  }
  RedArgs r{dy, dys, x, xs, P, C, scale, shift, mean, invstd, relu, workspace, 0, 0, 0, 0, 0, 0};
  int nblk = 0, rc;
  rc = dtype == VU_BF16 ? launch_partial<bf16_t, 1>(r, st, nblk, BNB_FUSED_MAXBLK)
                        : launch_partial<float, 1>(r, st, nblk, BNB_FUSED_MAXBLK);
  if (rc) return rc;
  if (nblk > BNB_FUSED_MAXBLK) return (int)hipErrorInvalidValue;
  BnBwdFusedArgs a{dy, dys, x, xs, P, C, scale, shift, mean, invstd, gamma, relu, train, workspace, nblk,
                   dgamma, dbeta, accumulate, dx, dxs, 1};
  const int groups = C / 32;
  int64_t split = (256 + groups - 1) / groups;
  const int64_t maxs = (P + 127) / 128;
  if (split > maxs) split = maxs;
  if (split < 1) split = 1;
  a.split = (int)split;
  if (dtype == VU_BF16)
    hipLaunchKernelGGL(bn_bwd_fused_apply_kernel<bf16_t>, dim3((unsigned)(groups * split)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(bn_bwd_fused_apply_kernel<float>, dim3((unsigned)(groups * split)), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}
