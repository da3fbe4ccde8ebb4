// The VAE bottleneck of UNetResNet (unet/unet_resnet.py:140-154, 191-194,
// 217-229) and the latent injection of its DecoderBlocks (:37-41, 93-94) as
// five launches per training step instead of ~50.
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
//   vu_latent_bwd      two launches: BN / ReLU / conv backward of every
//                      consumer on the vectors (weight, bias, gamma, beta
//                      gradients, dz partials), then dz, reparameterize
//                      backward, both heads' backward -> dpooled (the caller
//                      broadcasts dpooled / HW into d f[-1] with
//                      vu_sample_broadcast).
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int LAT_PCH = 1024;   // pixels per vu_latent_fwd block
constexpr int LAT_CG = 64;      // channels per vu_latent_fwd block
constexpr int LAT_SPLITS = 32;  // pixel splits per sample of vu_latent_bwd_sums
constexpr int LAT_MAXN = 64;    // samples
constexpr int LAT_MAXJ = 8;     // consumers per launch

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
        // the activated vectors (the latent shortcut's c_n: zbias.hip)
        if (pc == 0 && J.act) J.act[(int64_t)n * J.co + c] = rnd<T>(a);
      }
    } else {
      for (int n = 0; n < N; ++n) act[n * LAT_CG + tid] = 0.f;  // channel padding of the concat source
    }
  }
  if (J.train && pc == 0 && cg == 0 && tid == 0 && J.num_batches_tracked) *J.num_batches_tracked += 1;
  if (!J.out) return;  // the latent shortcut: vectors only, no map (block-uniform, before the barrier)
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
    t = lds_sum(sh + c, rows, C);
    J.part[((int64_t)n * LAT_SPLITS + sp) * C + c] = t;
  }
}

// The backward on the vectors, as two launches that spread over the CUs.
// (Round 4 first: one 1024-thread block for everything -- a ~1 MFLOP job
// whose time was all latency chains inside one CU: 510 us in its first form,
// 95-105 us after keeping its vectors in LDS.)  Nothing here depends on
// anything but the split sums, so each block issues every load it needs up
// front and then works from LDS:
//   latent_bwd_bn    one block per (consumer, 32-channel group): the split
//                    sums of its channels, the BatchNorm (+ReLU) backward on
//                    the N vectors (gamma / beta / bias gradients), the conv
//                    weight gradient dW[c][l] (+)= sum_n dy[n][c] z[n][l] of
//                    its rows, and its partial of dz[n][l] = sum_c W[c][l]
//                    dy[n][c] into the workspace;
//   latent_bwd_heads one block per 8 encoder channels: dz = the partials
//                    summed in block order, reparameterize backward (every
//                    block redoes this N x L step), the heads' weight
//                    gradients of its channels, dpooled of its channels;
//                    block 0 the heads' bias gradients.
// Every sum runs in a fixed order (reproducible run to run).
constexpr int LB_T = 256;
constexpr int LB_CW = 32;   // consumer channels per latent_bwd_bn block
constexpr int LB_NCH = 8;   // samples per split-sum round
constexpr int LB_ODW = 8;   // weight-gradient rows held per thread (LB_CW * 64 / LB_T)
constexpr int LH_CW = 8;    // encoder channels per latent_bwd_heads block
constexpr int LH_ODW = 4;   // head weight-gradient elements per thread (2 * 64 * LH_CW / LB_T)
// latent_bwd_bn's split-sum phase: thread (q8, c) adds splits 4 q8 .. 4 q8 + 3
// of sample k = q8 -- i.e. the 8 thread groups cover exactly LAT_SPLITS splits
// and the block is exactly LB_NCH sample rows of LB_CW channels
static_assert(LAT_SPLITS == 4 * (LB_T / LB_CW), "latent_bwd_bn: split sums assume 4 splits per thread group");
static_assert(LB_T == LB_NCH * LB_CW, "latent_bwd_bn: one sample row per thread group");

// Global-address-space pointers: through plain (generic) pointers the
// compiler emits flat loads / stores, which also count in lgkmcnt, so every
// LDS wait would wait for the outstanding global loads too.
typedef __attribute__((address_space(1))) float gfloat;
template <typename P> VU_DEV gfloat* gf(P* p) { return (gfloat*)(float*)p; }
template <typename P> VU_DEV const gfloat* gfc(const P* p) { return (const gfloat*)(const float*)p; }

__host__ __device__ inline int lb_blocks(int co) { return (co + LB_CW - 1) / LB_CW; }
__host__ __device__ inline int64_t lb_lds_floats(int N, int L) {
  return (int64_t)8 * LB_NCH * LB_CW + 2LL * N * LB_CW + (int64_t)N * L + (int64_t)LB_CW * L;
}
__host__ __device__ inline int64_t lh_lds_floats(int N, int L) {
  return 2LL * N * L + (int64_t)N * LH_CW + 2LL * L * LH_CW;
}

__global__ __launch_bounds__(LB_T) void latent_bwd_bn_kernel(const LatentJobs jobs, int njobs, const float* z_, int N,
                                                             int L, float* dzp_) {
  extern __shared__ float lsm[];
  // block -> (consumer, channel group): a wave-uniform walk of the kernarg table
  int b = blockIdx.x, j = 0;
  for (; j + 1 < njobs; ++j) {
    const int nb = lb_blocks(jobs.j[j].co);
    if (b < nb) break;
    b -= nb;
  }
  j = __builtin_amdgcn_readfirstlane(j);
  b = __builtin_amdgcn_readfirstlane(b);
  const VuLatentJob& J = jobs.j[j];
  const int co = J.co, c0 = b * LB_CW, cw = co - c0 < LB_CW ? co - c0 : LB_CW;
  const int tid = threadIdx.x, c = tid & (LB_CW - 1), q8 = tid >> 5;
  float* red = lsm;                          // [8][LB_NCH][LB_CW]
  float* sy = red + 8 * LB_NCH * LB_CW;      // [N][LB_CW] BN input y
  float* sdy = sy + N * LB_CW;               // [N][LB_CW] map-gradient sums, then pre-BN gradients
  float* sz = sdy + N * LB_CW;               // [N][L]
  float* sw = sz + N * L;                    // [cw][L] the conv weight rows
  const gfloat* part = gfc(J.part);
  const gfloat* z = gfc(z_);
  const gfloat* W = gfc(J.w) + (int64_t)c0 * L;
  gfloat* dw = J.dw ? gf(J.dw) + (int64_t)c0 * L : nullptr;

  // the loads that depend on nothing: y, z, the weight rows, the old
  // gradients (read-modify-write when grad_acc), the BN coefficients
  for (int e = tid; e < N * LB_CW; e += LB_T) {
    const int n = e / LB_CW, cc = e % LB_CW;
    if (cc < cw) sy[e] = gfc(J.y)[(int64_t)n * co + c0 + cc];
  }
  for (int e = tid; e < N * L; e += LB_T) sz[e] = z[e];
  for (int e = tid; e < cw * L; e += LB_T) sw[e] = W[e];
  float odw[LB_ODW];
#pragma unroll
  for (int k = 0; k < LB_ODW; ++k) {
    const int e = tid + k * LB_T;
    odw[k] = (dw && J.grad_acc && e < cw * L) ? dw[e] : 0.f;
  }
  float scale = 0.f, shift = 0.f, mean = 0.f, invstd = 0.f, gamma = 0.f, og = 0.f, ob = 0.f, obias = 0.f;
  if (tid < cw) {
    const gfloat* cf = gfc(J.coef) + c0 + tid;
    scale = cf[0];
    shift = cf[co];
    mean = cf[2 * co];
    invstd = cf[3 * co];
    gamma = gfc(J.gamma)[c0 + tid];
    if (J.grad_acc) {
      if (J.dgamma) og = gfc(J.dgamma)[c0 + tid];
      if (J.dbeta) ob = gfc(J.dbeta)[c0 + tid];
      if (J.dbias) obias = gfc(J.dbias)[c0 + tid];
    }
  }

  // phase 1: S[n][c] = sum of the LAT_SPLITS partials: thread (q8, c) adds
  // splits 4 q8 .. 4 q8 + 3 for LB_NCH samples (32 loads in flight), then the
  // 8 group sums in q8 order
  for (int n0 = 0; n0 < N; n0 += LB_NCH) {
    const int nn = N - n0 < LB_NCH ? N - n0 : LB_NCH;
    float v[LB_NCH][4];
#pragma unroll
    for (int k = 0; k < LB_NCH; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[k][u] = (k < nn && c < cw) ? part[((int64_t)(n0 + k) * LAT_SPLITS + 4 * q8 + u) * co + c0 + c] : 0.f;
#pragma unroll
    for (int k = 0; k < LB_NCH; ++k) red[(q8 * LB_NCH + k) * LB_CW + c] = ((v[k][0] + v[k][1]) + v[k][2]) + v[k][3];
    __syncthreads();
    {
      const int k = q8;   // LB_T = LB_NCH * LB_CW
      if (k < nn && c < cw) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) s += red[(q * LB_NCH + k) * LB_CW + c];
        sdy[(n0 + k) * LB_CW + c] = s;
      }
    }
    __syncthreads();
  }

  // phase 2: BatchNorm (+ReLU) backward per channel on the N vectors
  if (tid < cw) {
    double db = 0.0, dg = 0.0;
    for (int n = 0; n < N; ++n) {
      const float y = sy[n * LB_CW + tid];
      const float G = (y * scale + shift > 0.f) ? sdy[n * LB_CW + tid] : 0.f;
      sdy[n * LB_CW + tid] = G;
      db += G;
      dg += (double)G * ((y - mean) * invstd);
    }
    if (J.dgamma) gf(J.dgamma)[c0 + tid] = og + (float)dg;
    if (J.dbeta) gf(J.dbeta)[c0 + tid] = ob + (float)db;
    const float gi = gamma * invstd;
    const float rM = 1.f / (float)N;   // HW / (N * HW)
    double dbias = 0.0;
    for (int n = 0; n < N; ++n) {
      const float G = sdy[n * LB_CW + tid];
      const float y = sy[n * LB_CW + tid];
      const float v = J.train ? gi * (G - rM * ((float)db + (y - mean) * invstd * (float)dg)) : gi * G;
      sdy[n * LB_CW + tid] = v;
      dbias += v;
    }
    // the conv bias of a train-mode BatchNorm has an exactly zero gradient
    // (the batch mean absorbs it; engine.bias_grad)
    if (J.dbias) gf(J.dbias)[c0 + tid] = obias + (J.train ? 0.f : (float)dbias);
  }
  __syncthreads();

  // phase 3: this block's weight-gradient rows and its dz partial
  if (dw) {
#pragma unroll
    for (int k = 0; k < LB_ODW; ++k) {
      const int e = tid + k * LB_T;
      if (e >= cw * L) break;
      const int cc = e / L, l = e - cc * L;
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += sdy[n * LB_CW + cc] * sz[n * L + l];
      dw[e] = odw[k] + s;
    }
  }
  gfloat* dzp = gf(dzp_) + (int64_t)blockIdx.x * N * L;
  for (int e = tid; e < N * L; e += LB_T) {
    const int n = e / L, l = e - n * L;
    float s = 0.f;
    for (int cc = 0; cc < cw; ++cc) s += sw[cc * L + l] * sdy[n * LB_CW + cc];
    dzp[e] = s;
  }
}

__global__ __launch_bounds__(LB_T) void latent_bwd_heads_kernel(VuLatentHeads hb, int N, int L, const float* dzp_,
                                                                int nbp) {
  extern __shared__ float lsm[];
  const int C = hb.C, c0 = blockIdx.x * LH_CW, tid = threadIdx.x;
  float* sdmu = lsm;                  // [N][L]
  float* sdlv = sdmu + N * L;         // [N][L]
  float* spool = sdlv + N * L;        // [N][LH_CW]
  float* swm = spool + N * LH_CW;     // [L][LH_CW]
  float* swl = swm + L * LH_CW;       // [L][LH_CW]
  const gfloat* dzp = gfc(dzp_);
  gfloat* dwm = gf(hb.dw_mu);
  gfloat* dwl = gf(hb.dw_lv);

  // independent loads: pooled and both heads' weights for this block's
  // channels, the old weight gradients (grad_acc)
  for (int e = tid; e < N * LH_CW; e += LB_T) spool[e] = gfc(hb.pooled)[(int64_t)(e / LH_CW) * C + c0 + e % LH_CW];
  for (int e = tid; e < L * LH_CW; e += LB_T) {
    const int64_t g = (int64_t)(e / LH_CW) * C + c0 + e % LH_CW;
    swm[e] = gfc(hb.w_mu)[g];
    swl[e] = gfc(hb.w_lv)[g];
  }
  float odw[LH_ODW];
#pragma unroll
  for (int k = 0; k < LH_ODW; ++k) {
    const int e = tid + k * LB_T;
    odw[k] = 0.f;
    if (hb.grad_acc && e < 2 * L * LH_CW) {
      const int h = e / (L * LH_CW), r = e - h * L * LH_CW;
      const gfloat* d = h ? dwl : dwm;
      if (d) odw[k] = d[(int64_t)(r / LH_CW) * C + c0 + r % LH_CW];
    }
  }
  // dz = incoming + the consumers' partials (block order, 16 loads in flight),
  // then reparameterize backward (unet_resnet.py:191-194): z = mu + eps * exp(lv / 2)
  for (int e = tid; e < N * L; e += LB_T) {
    float s = hb.dz_in ? gfc(hb.dz_in)[e] : 0.f;
    const float gm = hb.dmu_in ? gfc(hb.dmu_in)[e] : 0.f;
    const float gl = hb.dlv_in ? gfc(hb.dlv_in)[e] : 0.f;
    const float ep = hb.eps ? gfc(hb.eps)[e] : 0.f;
    const float lv = hb.eps ? gfc(hb.logvar)[e] : 0.f;
    for (int b0 = 0; b0 < nbp; b0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = b0 + u < nbp ? dzp[(int64_t)(b0 + u) * N * L + e] : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (b0 + u < nbp) s += v[u];
    }
    sdmu[e] = gm + s;
    sdlv[e] = gl + (hb.eps ? s * ep * 0.5f * expf(0.5f * lv) : 0.f);
  }
  __syncthreads();

  // heads: dW[jj][c] (+)= sum_n d[n][jj] pooled[n][c]
#pragma unroll
  for (int k = 0; k < LH_ODW; ++k) {
    const int e = tid + k * LB_T;
    if (e >= 2 * L * LH_CW) break;
    const int h = e / (L * LH_CW), r = e - h * L * LH_CW, jj = r / LH_CW, cc = r % LH_CW;
    gfloat* d = h ? dwl : dwm;
    if (!d) continue;
    const float* dv = h ? sdlv : sdmu;
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += dv[n * L + jj] * spool[n * LH_CW + cc];
    d[(int64_t)jj * C + c0 + cc] = odw[k] + s;
  }
  // dpooled[n][c] = sum_jj w_mu[jj][c] dmu[n][jj] + w_lv[jj][c] dlv[n][jj]
  for (int e = tid; e < N * LH_CW; e += LB_T) {
    const int n = e / LH_CW, cc = e % LH_CW;
    float acc = 0.f;
    for (int jj = 0; jj < L; ++jj) acc += swm[jj * LH_CW + cc] * sdmu[n * L + jj] + swl[jj * LH_CW + cc] * sdlv[n * L + jj];
    gf(hb.dpooled)[(int64_t)n * C + c0 + cc] = acc;
  }
  // db[jj] (+)= sum_n d[n][jj]
  if (blockIdx.x == 0) {
    for (int e = tid; e < 2 * L; e += LB_T) {
      const int h = e / L, jj = e - h * L;
      gfloat* db = gf(h ? hb.db_lv : hb.db_mu);
      if (!db) continue;
      const float* dv = h ? sdlv : sdmu;
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += dv[n * L + jj];
      db[jj] = hb.grad_acc ? db[jj] + s : s;
    }
  }
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
    if (!q.out && (!q.act || q.cpad != q.co)) return (int)hipErrorInvalidValue;  // shortcut: vectors only
    q.cgroups = (q.cpad + LAT_CG - 1) / LAT_CG;
    q.block0 = fblocks;
    q.sblock0 = sblocks;
    fblocks += q.out ? vu_latent_fwd_blocks(N, q.HW, q.cpad) : q.cgroups;
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
  return N >= 1 && N <= LAT_MAXN && L >= 1 && L <= 64 && sum_co >= 0 && C >= LH_CW && C % LH_CW == 0;
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

// the dz partials of the latent_bwd_bn blocks: at most sum_co / 8 blocks
// (co = 8 * 2^k: ceil(co / 32) <= co / 8)
extern "C" int64_t vu_latent_bwd_workspace_bytes(int N, int L, int64_t sum_co) {
  return (sum_co / 8 + 1) * N * L * (int64_t)sizeof(float);
}

extern "C" int vu_latent_bwd(const VuLatentJob* jobs, int njobs, const VuLatentHeads* heads, int N, int L,
                             float* workspace, void* stream) {
  if (N < 1 || N > LAT_MAXN || L < 1 || L > 64) return (int)hipErrorInvalidValue;
  if (heads->C < LH_CW || heads->C % LH_CW) return (int)hipErrorInvalidValue;
  LatentJobs J;
  int64_t fb = 0, sb = 0;
  if (njobs > 0) {
    if (int rc = pack(jobs, njobs, N, J, fb, sb)) return rc;
  } else if (njobs < 0) {
    return (int)hipErrorInvalidValue;
  }
  int nbp = 0;
  for (int j = 0; j < njobs; ++j) nbp += lb_blocks(J.j[j].co);
  if (nbp > 0 && workspace == nullptr) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (nbp > 0)
    hipLaunchKernelGGL(latent_bwd_bn_kernel, dim3((unsigned)nbp), dim3(LB_T),
                       (size_t)(lb_lds_floats(N, L) * sizeof(float)), st, J, njobs, heads->z, N, L, workspace);
  hipLaunchKernelGGL(latent_bwd_heads_kernel, dim3((unsigned)(heads->C / LH_CW)), dim3(LB_T),
                     (size_t)(lh_lds_floats(N, L) * sizeof(float)), st, *heads, N, L, workspace, nbp);
  return (int)hipGetLastError();
}
