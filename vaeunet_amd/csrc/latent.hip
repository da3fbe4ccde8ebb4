// The VAE bottleneck of UNetResNet (unet/unet_resnet.py:140-154, 191-194,
// 217-229) and the latent injection of its DecoderBlocks (:37-41, 93-94) as
// four launches per training step instead of ~50.
//
// Everything downstream of z is spatially constant per sample: z_spatial =
// interpolate(z[..., None, None], align_corners=True) is an exact broadcast,
// a bilinear resize of a constant map is the same constant, and a 1x1 conv +
// BatchNorm + ReLU of a per-sample constant map is again per-sample constant.
// Over the N*HW pixels of such a map the batch statistics are those of the N
// sample vectors (each counted HW times), so z_initial (32 -> 512) and every
// z_proj (32 -> 32) reduce to [N x L] vector arithmetic, and the maps are
// written once, already activated (the channel-padded concat source of a
// DecoderBlock's conv1 included).  The backward needs only the per-sample
// pixel sums of each map's gradient.
//
//   vu_vae_heads_fwd   one block per sample: channel mean of f[-1] (fixed
//                      order), both heads (one wave per output group, lanes
//                      over the 512-long dot product, DPP-free shuffle tree),
//                      reparameterize;
//   vu_latent_fwd      per (consumer, 64-channel group, pixel chunk) block:
//                      the consumer's conv + BN (+running statistics) + ReLU
//                      on the N vectors, then its map stores;
//   vu_latent_bwd_sums per-sample partial pixel sums of the maps' gradients;
//   vu_latent_bwd      one block: BN / ReLU / conv backward of every consumer
//                      on the vectors (weight, bias, gamma, beta gradients),
//                      dz, reparameterize backward, both heads' backward ->
//                      dpooled (the caller broadcasts dpooled / HW into
//                      d f[-1] with vu_sample_broadcast).
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int LAT_PCH = 1024;   // pixels per vu_latent_fwd block
constexpr int LAT_CG = 64;      // channels per vu_latent_fwd block
constexpr int LAT_SPLITS = 32;  // pixel splits per sample of vu_latent_bwd_sums
constexpr int LAT_MAXN = 64;    // samples
constexpr int LAT_MAXJ = 8;     // consumers per launch
#define VU_LATENT_BWD_MAX_LDS (64 * 1024)

// the job table travels BY VALUE in the kernel arguments (~1.7 KB): no device
// table to upload, so a captured HIP graph replays it as is
struct LatentJobs {
  VuLatentJob j[LAT_MAXJ];
};

VU_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one block per (sample n, group of LAT_HG latent dims): the channel mean of
// f[-1] for sample n (every group block recomputes it: 256 KB from L2 at the
// bottleneck; group 0 writes it), then the 2 * LAT_HG head dot products of
// its dims (one wave per dot, lanes over the C channels, weight loads
// unrolled), then reparameterize for those dims.  (Round 4 first version:
// one 256-thread block per sample with a serial 64-deep load chain and 16
// serial dots per wave -- 72 us per step.)
constexpr int LAT_HG = 8;     // latent dims per heads block
constexpr int LAT_HT = 512;   // heads block threads
template <typename T>
__global__ __launch_bounds__(LAT_HT) void heads_fwd_kernel(const T* f4, int64_t fs, int HW, int C, const float* w_mu,
                                                           const float* b_mu, const float* w_lv, const float* b_lv,
                                                           int L, const float* eps, float* pooled, float* mu,
                                                           float* logvar, float* z) {
  extern __shared__ float sm[];            // [rows][C] partial sums, then pooled [C], then 2*LAT_HG head outputs
  const int n = blockIdx.x, grp = blockIdx.y, tid = threadIdx.x;
  const int V = C >> 3;                    // 8-channel vectors per pixel (C % 8 == 0)
  const int rows = LAT_HT / V;             // pixel rows in flight per block (V <= LAT_HT)
  const int cv = tid % V, row = tid / V;
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  if (row < rows) {
    const T* base = f4 + (int64_t)n * HW * fs + cv * 8;
    int p = row;
    for (; p + 3 * rows < HW; p += 4 * rows) {   // 4 loads in flight per thread
      Vec8<T> v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u].load(base + (int64_t)(p + u * rows) * fs);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += v[u].get(k);
    }
    for (; p < HW; p += rows) {
      Vec8<T> v;
      v.load(base + (int64_t)p * fs);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v.get(k);
    }
  }
  float* part = sm;                        // [rows][C]
  if (row < rows)
#pragma unroll
    for (int k = 0; k < 8; ++k) part[row * C + cv * 8 + k] = s[k];
  __syncthreads();
  float* pm = sm + rows * C;               // pooled mean [C]
  const float inv = 1.f / (float)HW;
  for (int c = tid; c < C; c += LAT_HT) {
    float t = 0.f;
    for (int q = 0; q < rows; ++q) t += part[q * C + c];
    pm[c] = t * inv;
    if (grp == 0) pooled[(int64_t)n * C + c] = t * inv;
  }
  __syncthreads();
  // dot d < 2*LAT_HG of this group: mu[l0 + d] (d < LAT_HG) or logvar[l0 + d - LAT_HG]; wave w takes d = w, w + 8
  float* hout = pm + C;
  const int lane = tid & 63, wv = tid >> 6, l0 = grp * LAT_HG;
  for (int d = wv; d < 2 * LAT_HG; d += LAT_HT / 64) {
    const int l = l0 + (d < LAT_HG ? d : d - LAT_HG);
    if (l >= L) continue;                  // wave-uniform
    const float* w = d < LAT_HG ? w_mu + (int64_t)l * C : w_lv + (int64_t)l * C;
    float a = 0.f;
    for (int c = lane; c < C; c += 256) {  // 4 loads in flight per lane
      float wr[4], pr[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int cc = c + 64 * u;
        wr[u] = cc < C ? w[cc] : 0.f;
        pr[u] = cc < C ? pm[cc] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) a += wr[u] * pr[u];
    }
    a = wave_sum(a);
    if (lane == 0) {
      if (d < LAT_HG) {
        a += b_mu ? b_mu[l] : 0.f;
        mu[(int64_t)n * L + l] = a;
      } else {
        a += b_lv ? b_lv[l] : 0.f;
        logvar[(int64_t)n * L + l] = a;
      }
      hout[d] = a;
    }
  }
  __syncthreads();
  if (tid < LAT_HG && l0 + tid < L) {
    const int l = l0 + tid;
    const float m = hout[tid];
    z[(int64_t)n * L + l] = eps ? m + eps[(int64_t)n * L + l] * expf(0.5f * hout[LAT_HG + tid]) : m;
  }
}

// ---- consumers: 1x1 conv + BatchNorm + ReLU of a broadcast latent ----------
template <typename T>
__global__ __launch_bounds__(256) void latent_fwd_kernel(const LatentJobs jobs, int njobs, const float* z, int N,
                                                         int L) {
  __shared__ float zs[LAT_MAXN * 64];      // z [N][L] (L <= 64)
  __shared__ float act[LAT_MAXN * LAT_CG];  // a[n][c] of this block's channels
  int j = 0;
  while (j + 1 < njobs && (int64_t)blockIdx.x >= jobs.j[j + 1].block0) ++j;
  const VuLatentJob& J = jobs.j[j];
  const int64_t lb = (int64_t)blockIdx.x - J.block0;
  const int cg = (int)(lb % J.cgroups);
  const int64_t pc = lb / J.cgroups;
  const int tid = threadIdx.x;
  for (int e = tid; e < N * L; e += 256) zs[e] = z[e];
  __syncthreads();
  const int c0 = cg * LAT_CG;
  const int64_t M = (int64_t)N * J.HW;
  if (tid < LAT_CG) {
    const int c = c0 + tid;
    if (c < J.co) {
      const float* w = J.w + (int64_t)c * L;
      const float b = J.bias ? J.bias[c] : 0.f;
      double s = 0.0;
      for (int n = 0; n < N; ++n) {
        float y = b;
        for (int l = 0; l < L; ++l) y += w[l] * zs[n * L + l];
        act[n * LAT_CG + tid] = y;
        s += y;
      }
      float scale, shift, mean, invstd;
      if (J.train) {
        const double m = s / N;
        double q = 0.0;
        for (int n = 0; n < N; ++n) {
          const double d = (double)act[n * LAT_CG + tid] - m;
          q += d * d;
        }
        const double var = q / N;
        const double is = 1.0 / sqrt(var + (double)J.eps);
        mean = (float)m;
        invstd = (float)is;
        scale = (float)((double)J.gamma[c] * is);
        shift = (float)((double)J.beta[c] - m * (double)J.gamma[c] * is);
        if (pc == 0 && J.running_mean) {
          J.running_mean[c] = (float)((1.0 - J.momentum) * J.running_mean[c] + J.momentum * m);
          J.running_var[c] = (float)((1.0 - J.momentum) * J.running_var[c] +
                                     J.momentum * var * (double)M / (double)(M > 1 ? M - 1 : 1));
        }
      } else {
        mean = J.running_mean[c];
        invstd = (float)(1.0 / sqrt((double)J.running_var[c] + (double)J.eps));
        scale = J.gamma[c] * invstd;
        shift = J.beta[c] - mean * scale;
      }
      if (pc == 0) {
        J.coef[c] = scale;
        J.coef[J.co + c] = shift;
        J.coef[2 * J.co + c] = mean;
        J.coef[3 * J.co + c] = invstd;
        for (int n = 0; n < N; ++n) J.y[(int64_t)n * J.co + c] = act[n * LAT_CG + tid];
      }
      for (int n = 0; n < N; ++n) {
        const float a = fmaxf(act[n * LAT_CG + tid] * scale + shift, 0.f);
        act[n * LAT_CG + tid] = rnd<T>(a);
      }
    } else {
      for (int n = 0; n < N; ++n) act[n * LAT_CG + tid] = 0.f;  // channel padding of the concat source
    }
  }
  if (J.train && pc == 0 && cg == 0 && tid == 0 && J.num_batches_tracked) *J.num_batches_tracked += 1;
  __syncthreads();
  // map stores: pixels [pc*PCH, (pc+1)*PCH) of the flattened (n, p) range,
  // this block's channels [c0, min(c0 + 64, cpad)) as 8-channel vectors
  const int nch = min(LAT_CG, J.cpad - c0);
  const int vpp = nch >> 3;                // vectors per pixel (cpad % 8 == 0)
  const int64_t e0 = pc * LAT_PCH, e1 = min(M, e0 + LAT_PCH);
  T* out = reinterpret_cast<T*>(J.out);
  // (n, pixel, vector) decodes by multiply-shift: the 64-bit divisions per
  // 16-byte store were the kernel's cost (pixel counts < 2^31: host check)
  const FastDiv dv((uint32_t)vpp), dhw((uint32_t)J.HW);
  for (int64_t e = e0 * vpp + tid; e < e1 * vpp; e += 256) {
    const int64_t pix = (int64_t)dv.div((uint32_t)e);
    const int v = (int)(e - pix * vpp);
    const int n = (int)dhw.div((uint32_t)pix);
    Vec8<T> o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o.set(k, act[n * LAT_CG + v * 8 + k]);
    o.store(out + pix * J.out_stride + c0 + v * 8);
  }
}

// part[job][n][split][c] = sum of dmap over the split's pixels (fixed order)
template <typename T>
__global__ __launch_bounds__(256) void latent_sums_kernel(const LatentJobs jobs, int njobs, int N) {
  int j = 0;
  while (j + 1 < njobs && (int64_t)blockIdx.x >= jobs.j[j + 1].sblock0) ++j;
  const VuLatentJob& J = jobs.j[j];
  const int64_t lb = (int64_t)blockIdx.x - J.sblock0;
  const int n = (int)(lb / LAT_SPLITS), sp = (int)(lb - (int64_t)n * LAT_SPLITS);
  const int C = J.co;                       // % 8 == 0
  const int V = C >> 3, rows = 256 / V;     // V <= 256
  const int tid = threadIdx.x, cv = tid % V, row = tid / V;
  const int per = (J.HW + LAT_SPLITS - 1) / LAT_SPLITS;
  const int p0 = sp * per, p1 = min(J.HW, p0 + per);
  const T* d = reinterpret_cast<const T*>(J.dmap);
  __shared__ float sh[2048];
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  if (row < rows) {
    const T* base = d + (int64_t)n * J.HW * J.dmap_stride + cv * 8;
    int p = p0 + row;
    for (; p + 3 * rows < p1; p += 4 * rows) {   // 4 loads in flight per thread
      Vec8<T> v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u].load(base + (int64_t)(p + u * rows) * J.dmap_stride);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += v[u].get(k);
    }
    for (; p < p1; p += rows) {
      Vec8<T> v;
      v.load(base + (int64_t)p * J.dmap_stride);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v.get(k);
    }
  }
  if (row < rows)
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[row * C + cv * 8 + k] = s[k];
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float t = 0.f;
    for (int q = 0; q < rows; ++q) t += sh[q * C + c];
    J.part[((int64_t)n * LAT_SPLITS + sp) * C + c] = t;
  }
}

// One block (1024 threads): every consumer's backward on the vectors, then
// the bottleneck's.  The work is ~1 MFLOP; what costs is latency, so every
// phase runs its global loads in parallel across the block and keeps the
// intermediate vectors in LDS (the first version walked 256-512-long
// dependent global-load chains per thread: 510 us per step).  LDS (floats):
//   sdy [N][CT]   map-gradient sums, then the consumers' pre-BN gradients
//                 (CT = sum of co over the consumers, job j at column off_j)
//   sz, sdmu, sdlv [N][L]
//   su            [max(16 N L, N C)]: the dz partials of the 16 waves, then
//                 pooled [N][C]
// All sums run in a fixed order (reproducible).
constexpr int LAT_BT = 1024;
// Global-address-space pointers: through plain (generic) pointers the
// compiler emits flat loads / stores, which also count in lgkmcnt -- every
// LDS wait of the loops below then waited for the outstanding global loads
// too (99 flat memory instructions in the first builds of this kernel).
typedef __attribute__((address_space(1))) float gfloat;
template <typename P> VU_DEV gfloat* gf(P* p) { return (gfloat*)(float*)p; }
template <typename P> VU_DEV const gfloat* gfc(const P* p) { return (const gfloat*)(const float*)p; }

struct LJob {   // the fields of a VuLatentJob the backward reads, in LDS
  const gfloat* part;
  const gfloat* coef;
  const gfloat* y;
  const gfloat* gamma;
  gfloat* dgamma;
  gfloat* dbeta;
  gfloat* dbias;
  gfloat* dw;
  const gfloat* w;
  int co, grad_acc, train;
};
constexpr int LAT_RMW = 8;    // gradient elements per thread per round (phases 3a, 4)

__host__ __device__ inline int64_t latent_bwd_lds_floats(int N, int L, int CT, int C) {
  const int64_t u = (int64_t)16 * N * L > (int64_t)N * C ? (int64_t)16 * N * L : (int64_t)N * C;
  return (int64_t)N * CT + 3LL * N * L + u;
}

__global__ __launch_bounds__(LAT_BT) void latent_bwd_kernel(const LatentJobs jobs, int njobs, VuLatentHeads hb,
                                                            int N, int L, float* ws) {
  // ws (optional, A/B diagnostics only): thread 0 records the real-time
  // counter (100 MHz) at each phase boundary into ws[0 .. 7] as uint64
  uint64_t* const tsv = reinterpret_cast<uint64_t*>(ws);
  int tsk = 0;
  auto stamp = [&]() {
    if (tsv && threadIdx.x == 0) tsv[tsk] = __builtin_amdgcn_s_memrealtime();
    ++tsk;
  };
  stamp();
  extern __shared__ float lsm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int joff[LAT_MAXJ + 1];
  joff[0] = 0;
  for (int j = 0; j < njobs; ++j) joff[j + 1] = joff[j] + jobs.j[j].co;
  const int CT = joff[njobs];
  const int C = hb.C;
  float* sdy = lsm;
  float* sz = sdy + (int64_t)N * CT;
  float* sdmu = sz + N * L;
  float* sdlv = sdmu + N * L;
  float* su = sdlv + N * L;

  // The consumers' fields live in an LDS job table so that the loops below
  // can run over the concatenated (job, channel) space -- all consumers'
  // work in one round instead of one latency-bound round per consumer -- with
  // a per-lane job lookup that costs an LDS read, not a per-lane load from
  // the kernel-argument segment (one memory round trip before every address:
  // the first version's 510 us).
  __shared__ LJob lj[LAT_MAXJ];
  __shared__ int loff[LAT_MAXJ + 1];
  if (tid < njobs) {
    const VuLatentJob& J = jobs.j[tid];
    lj[tid] = LJob{gfc(J.part), gfc(J.coef), gfc(J.y), gfc(J.gamma), gf(J.dgamma), gf(J.dbeta), gf(J.dbias),
                   gf(J.dw), gfc(J.w), J.co, J.grad_acc, J.train};
  }
  if (tid <= njobs) loff[tid] = joff[tid];
  __syncthreads();
  stamp();
  auto job_of = [&](int cc) {
    int j = 0;
    while (j + 1 < njobs && cc >= loff[j + 1]) ++j;
    return j;
  };

  // phase 1: map-gradient sums S[n][c] = sum over the LAT_SPLITS partials
  // (all 32 loads of a thread in flight), z -> LDS
  for (int e = tid; e < N * CT; e += LAT_BT) {
    const int n = e / CT, cc = e - n * CT;
    const int j = job_of(cc);
    const int co = lj[j].co, c = cc - loff[j];
    const gfloat* pp = lj[j].part + (int64_t)n * LAT_SPLITS * co + c;
    float v[LAT_SPLITS];
#pragma unroll
    for (int q = 0; q < LAT_SPLITS; ++q) v[q] = pp[(int64_t)q * co];
    float S = 0.f;
#pragma unroll
    for (int q = 0; q < LAT_SPLITS; ++q) S += v[q];
    sdy[e] = S;
  }
  for (int e = tid; e < N * L; e += LAT_BT) sz[e] = gfc(hb.z)[e];
  __syncthreads();
  stamp();

  // phase 2: BatchNorm (+ReLU) backward per consumer channel on the N vectors
  for (int cc = tid; cc < CT; cc += LAT_BT) {
    const int j = job_of(cc);
    const LJob& J = lj[j];
    const int co = J.co, c = cc - loff[j];
    const float scale = J.coef[c], shift = J.coef[co + c], mean = J.coef[2 * co + c], invstd = J.coef[3 * co + c];
    const float gamma = J.gamma[c];
    float yv[16];
    double db = 0.0, dg = 0.0;
    for (int n0 = 0; n0 < N; n0 += 16) {
      const int nn = N - n0 < 16 ? N - n0 : 16;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < nn) yv[k] = J.y[(int64_t)(n0 + k) * co + c];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k >= nn) break;
        const int n = n0 + k;
        const float y = yv[k];
        const float G = (y * scale + shift > 0.f) ? sdy[n * CT + cc] : 0.f;
        sdy[n * CT + cc] = G;
        db += G;
        dg += (double)G * ((y - mean) * invstd);
      }
    }
    if (J.dgamma) J.dgamma[c] = J.grad_acc ? J.dgamma[c] + (float)dg : (float)dg;
    if (J.dbeta) J.dbeta[c] = J.grad_acc ? J.dbeta[c] + (float)db : (float)db;
    const float gi = gamma * invstd;
    const float rM = 1.f / (float)N;   // HW / (N * HW)
    double dbias = 0.0;
    for (int n0 = 0; n0 < N; n0 += 16) {
      const int nn = N - n0 < 16 ? N - n0 : 16;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < nn) yv[k] = J.y[(int64_t)(n0 + k) * co + c];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k >= nn) break;
        const int n = n0 + k;
        const float G = sdy[n * CT + cc];
        const float v = J.train ? gi * (G - rM * ((float)db + (yv[k] - mean) * invstd * (float)dg)) : gi * G;
        sdy[n * CT + cc] = v;
        dbias += v;
      }
    }
    // the conv bias of a train-mode BatchNorm has an exactly zero gradient
    // (the batch mean absorbs it; engine.bias_grad)
    if (J.dbias) {
      const float b = J.train ? 0.f : (float)dbias;
      J.dbias[c] = J.grad_acc ? J.dbias[c] + b : b;
    }
  }
  __syncthreads();
  stamp();

  // phase 3a: conv weight gradients dW_j[c][l] (+)= sum_n DY[n][c] z[n][l];
  // LAT_RMW elements per thread per round so that the read-modify-write
  // loads of a round are in flight together
  for (int e0 = tid; e0 < CT * L; e0 += LAT_RMW * LAT_BT) {
    gfloat* dst[LAT_RMW];
    float old[LAT_RMW], s[LAT_RMW];
#pragma unroll
    for (int u = 0; u < LAT_RMW; ++u) {
      const int e = e0 + u * LAT_BT;
      dst[u] = nullptr;
      old[u] = 0.f;
      s[u] = 0.f;
      if (e >= CT * L) continue;
      const int cc = e / L, l = e - cc * L;
      const int j = job_of(cc);
      if (!lj[j].dw) continue;
      dst[u] = lj[j].dw + (int64_t)(cc - loff[j]) * L + l;
      if (lj[j].grad_acc) old[u] = *dst[u];
      for (int n = 0; n < N; ++n) s[u] += sdy[n * CT + cc] * sz[n * L + l];
    }
#pragma unroll
    for (int u = 0; u < LAT_RMW; ++u)
      if (dst[u]) *dst[u] = old[u] + s[u];
  }
  // phase 3b: dz[n][l] = sum_j sum_c W_j[c][l] DY_j[n][c]: wave w takes the
  // slice [w CT/16, (w+1) CT/16) of the concatenated channels, lane =
  // (n-half, l) over 32 l; the 16 wave partials are summed in wave order
  const int nw = LAT_BT / 64;
  const int nh = lane >> 5;
  const int cb = (int)((int64_t)wv * CT / nw), ce = (int)((int64_t)(wv + 1) * CT / nw);
  for (int l0 = 0; l0 < L; l0 += 32)
  for (int n0 = 0; n0 < N; n0 += 8) {       // 8 samples x 32 dims per pass: 4 accumulators per lane
    const int l = l0 + (lane & 31);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (l < L) {
      for (int c0 = cb; c0 < ce; c0 += 8) {   // 8 weight loads in flight per lane
        float wcl[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int cc = c0 + u;
          wcl[u] = 0.f;
          if (cc < ce) {
            const int j = job_of(cc);
            wcl[u] = lj[j].w[(int64_t)(cc - loff[j]) * L + l];
          }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (c0 + u >= ce) break;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int n = n0 + 2 * k + nh;
            if (n < N) acc[k] += wcl[u] * sdy[n * CT + c0 + u];
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int n = n0 + 2 * k + nh;
      if (n < N && l < L) su[((int64_t)wv * N + n) * L + l] = acc[k];
    }
  }
  __syncthreads();
  stamp();
  for (int e = tid; e < N * L; e += LAT_BT) {
    float s = hb.dz_in ? gfc(hb.dz_in)[e] : 0.f;
    for (int w = 0; w < nw; ++w) s += su[(int64_t)w * N * L + e];
    // reparameterize backward (unet_resnet.py:191-194): z = mu + eps * exp(lv / 2)
    const float gm = hb.dmu_in ? gfc(hb.dmu_in)[e] : 0.f;
    const float gl = hb.dlv_in ? gfc(hb.dlv_in)[e] : 0.f;
    sdmu[e] = gm + s;
    sdlv[e] = gl + (hb.eps ? s * gfc(hb.eps)[e] * 0.5f * expf(0.5f * gfc(hb.logvar)[e]) : 0.f);
  }
  __syncthreads();
  stamp();
  // pooled -> LDS (over the dz partials)
  float* spool = su;
  for (int e = tid; e < N * C; e += LAT_BT) spool[e] = gfc(hb.pooled)[e];
  __syncthreads();
  stamp();

  // phase 4: heads. dW[jj][c] (+)= sum_n d[n][jj] pooled[n][c]; db[jj] (+)= sum_n d[n][jj]
  for (int e0 = tid; e0 < 2 * L * C; e0 += LAT_RMW * LAT_BT) {
    gfloat* dst[LAT_RMW];
    float old[LAT_RMW], s[LAT_RMW];
#pragma unroll
    for (int u = 0; u < LAT_RMW; ++u) {
      const int e = e0 + u * LAT_BT;
      dst[u] = nullptr;
      old[u] = 0.f;
      s[u] = 0.f;
      if (e >= 2 * L * C) continue;
      const int h = e / (L * C), r = e - h * (L * C), jj = r / C, c = r - jj * C;
      const float* d = h ? sdlv : sdmu;
      gfloat* dw = gf(h ? hb.dw_lv : hb.dw_mu);
      if (!dw) continue;
      dst[u] = dw + r;
      if (hb.grad_acc) old[u] = dw[r];
      for (int n = 0; n < N; ++n) s[u] += d[n * L + jj] * spool[n * C + c];
    }
#pragma unroll
    for (int u = 0; u < LAT_RMW; ++u)
      if (dst[u]) *dst[u] = old[u] + s[u];
  }
  for (int e = tid; e < 2 * L; e += LAT_BT) {
    const int h = e / L, jj = e - h * L;
    const float* d = h ? sdlv : sdmu;
    gfloat* db = gf(h ? hb.db_lv : hb.db_mu);
    if (!db) continue;
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += d[n * L + jj];
    db[jj] = hb.grad_acc ? db[jj] + s : s;
  }
  // dpooled[n][c] = sum_jj w_mu[jj][c] dmu[n][jj] + w_lv[jj][c] dlv[n][jj]:
  // a thread per (c, 8-sample group), the 2L weight loads in flight in 8s
  for (int e = tid; e < C * ((N + 7) / 8); e += LAT_BT) {
    const int c = e % C, n0 = (e / C) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j0 = 0; j0 < L; j0 += 8) {
      float wm[8], wl[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        wm[u] = j0 + u < L ? gfc(hb.w_mu)[(int64_t)(j0 + u) * C + c] : 0.f;
        wl[u] = j0 + u < L ? gfc(hb.w_lv)[(int64_t)(j0 + u) * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (j0 + u >= L) break;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (n0 + k < N) acc[k] += wm[u] * sdmu[(n0 + k) * L + j0 + u] + wl[u] * sdlv[(n0 + k) * L + j0 + u];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (n0 + k < N) gf(hb.dpooled)[(int64_t)(n0 + k) * C + c] = acc[k];
  }
  stamp();
}

}  // namespace

#define DISPATCH_T(dtype, ...) \
  if ((dtype) == VU_BF16) { using T = bf16_t; __VA_ARGS__; } else { using T = float; __VA_ARGS__; }

static bool pow2_ok(int C) { int v = C / 8; return C % 8 == 0 && v > 0 && v <= 256 && (v & (v - 1)) == 0; }

extern "C" int vu_vae_heads_fwd(const void* f4, int64_t fs, int N, int HW, int C, const float* w_mu,
                                const float* b_mu, const float* w_lv, const float* b_lv, int L, const float* eps,
                                float* pooled, float* mu, float* logvar, float* z, int dtype, void* stream) {
  if (!pow2_ok(C) || fs % 8 || L < 1) return (int)hipErrorInvalidValue;
  if (N == 0) return 0;
  const int rows = LAT_HT / (C / 8);
  if (rows < 1) return (int)hipErrorInvalidValue;
  const size_t shm = ((size_t)(rows + 1) * C + 2 * LAT_HG) * sizeof(float);
  if (shm > 64 * 1024) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)N, (unsigned)((L + LAT_HG - 1) / LAT_HG));
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((heads_fwd_kernel<T>), grid, dim3(LAT_HT), shm, st, (const T*)f4, fs, HW, C, w_mu, b_mu, w_lv,
                       b_lv, L, eps, pooled, mu, logvar, z);
  })
  return (int)hipGetLastError();
}

extern "C" int64_t vu_latent_fwd_blocks(int N, int HW, int cpad) {
  const int64_t M = (int64_t)N * HW;
  return (int64_t)((cpad + LAT_CG - 1) / LAT_CG) * ((M + LAT_PCH - 1) / LAT_PCH);
}

extern "C" int vu_latent_check_job(int co, int cpad, int64_t out_stride, int dtype) {
  (void)dtype;
  if (co < 1 || cpad < co || cpad % 8 || out_stride % 8 || !pow2_ok(co)) return (int)hipErrorInvalidValue;
  return 0;
}

static int pack(const VuLatentJob* jobs, int njobs, int N, LatentJobs& J, int64_t& fblocks, int64_t& sblocks) {
  if (njobs < 1 || njobs > LAT_MAXJ) return (int)hipErrorInvalidValue;
  fblocks = sblocks = 0;
  for (int j = 0; j < njobs; ++j) {
    J.j[j] = jobs[j];
    VuLatentJob& q = J.j[j];
    if (vu_latent_check_job(q.co, q.cpad, q.out_stride, 0) != 0 || q.HW < 1) return (int)hipErrorInvalidValue;
    if ((int64_t)N * q.HW * 8 >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;  // 32-bit decodes
    q.cgroups = (q.cpad + LAT_CG - 1) / LAT_CG;
    q.block0 = fblocks;
    q.sblock0 = sblocks;
    fblocks += vu_latent_fwd_blocks(N, q.HW, q.cpad);
    sblocks += (int64_t)N * LAT_SPLITS;
  }
  return 0;
}

extern "C" int vu_latent_fwd(const VuLatentJob* jobs, int njobs, const float* z, int N, int L, int dtype,
                             void* stream) {
  if (N < 1 || N > LAT_MAXN || L < 1 || L > 64) return (int)hipErrorInvalidValue;
  LatentJobs J;
  int64_t fb, sb;
  if (int rc = pack(jobs, njobs, N, J, fb, sb)) return rc;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((latent_fwd_kernel<T>), dim3((unsigned)fb), dim3(256), 0, st, J, njobs, z, N, L);
  })
  return (int)hipGetLastError();
}

extern "C" int64_t vu_latent_part_floats(int N, int co) { return (int64_t)N * LAT_SPLITS * co; }

extern "C" int vu_latent_bwd_supported(int N, int L, int64_t sum_co, int C) {
  return N >= 1 && N <= LAT_MAXN && L >= 1 && L <= 64 && sum_co >= 0 &&
         latent_bwd_lds_floats(N, L, (int)sum_co, C) * (int64_t)sizeof(float) <= VU_LATENT_BWD_MAX_LDS;
}

extern "C" int vu_latent_bwd_sums(const VuLatentJob* jobs, int njobs, int N, int dtype, void* stream) {
  if (N < 1 || N > LAT_MAXN) return (int)hipErrorInvalidValue;
  LatentJobs J;
  int64_t fb, sb;
  if (int rc = pack(jobs, njobs, N, J, fb, sb)) return rc;
  for (int j = 0; j < njobs; ++j)
    if (!J.j[j].dmap || J.j[j].dmap_stride % 8 || !J.j[j].part) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((latent_sums_kernel<T>), dim3((unsigned)sb), dim3(256), 0, st, J, njobs, N);
  })
  return (int)hipGetLastError();
}

extern "C" int64_t vu_latent_bwd_workspace_bytes(int N, int L, int64_t sum_co) {
  return ((int64_t)N * sum_co + 3LL * N * L) * (int64_t)sizeof(float);
}

extern "C" int vu_latent_bwd(const VuLatentJob* jobs, int njobs, const VuLatentHeads* heads, int N, int L,
                             float* workspace, void* stream) {
  if (N < 1 || N > LAT_MAXN || L < 1 || L > 64) return (int)hipErrorInvalidValue;
  LatentJobs J;
  int64_t fb = 0, sb = 0;
  if (njobs > 0) {
    if (int rc = pack(jobs, njobs, N, J, fb, sb)) return rc;
  } else if (njobs < 0) {
    return (int)hipErrorInvalidValue;
  }
  int64_t ct = 0;
  for (int j = 0; j < njobs; ++j) ct += J.j[j].co;
  const int64_t shm = latent_bwd_lds_floats(N, L, (int)ct, heads->C) * (int64_t)sizeof(float);
  if (shm > VU_LATENT_BWD_MAX_LDS) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(latent_bwd_kernel, dim3(1), dim3(LAT_BT), (size_t)shm, (hipStream_t)stream, J, njobs, *heads, N,
                     L, workspace);
  return (int)hipGetLastError();
}
