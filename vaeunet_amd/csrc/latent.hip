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

template <typename T>
__global__ __launch_bounds__(256) void heads_fwd_kernel(const T* f4, int64_t fs, int HW, int C, const float* w_mu,
                                                        const float* b_mu, const float* w_lv, const float* b_lv, int L,
                                                        const float* eps, float* pooled, float* mu, float* logvar,
                                                        float* z) {
  extern __shared__ float sm[];            // [4][C] partial sums, then pooled [C]
  const int n = blockIdx.x, tid = threadIdx.x;
  const int V = C >> 3;                    // 8-channel vectors per pixel (C % 8 == 0)
  const int rows = 256 / V;                // pixel rows in flight per block (V <= 256)
  const int cv = tid % V, row = tid / V;
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  if (row < rows)
    for (int p = row; p < HW; p += rows) {
      Vec8<T> v;
      v.load(f4 + ((int64_t)n * HW + p) * fs + cv * 8);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v.get(k);
    }
  float* part = sm;                        // [rows][C]
  if (row < rows)
#pragma unroll
    for (int k = 0; k < 8; ++k) part[row * C + cv * 8 + k] = s[k];
  __syncthreads();
  float* pm = sm + rows * C;               // pooled mean [C]
  const float inv = 1.f / (float)HW;
  for (int c = tid; c < C; c += 256) {
    float t = 0.f;
    for (int q = 0; q < rows; ++q) t += part[q * C + c];
    pm[c] = t * inv;
    pooled[(int64_t)n * C + c] = t * inv;
  }
  __syncthreads();
  // heads: output o < L is mu[o], else logvar[o - L]; wave w takes o = w, w+4, ...
  const int lane = tid & 63, wv = tid >> 6;
  for (int o = wv; o < 2 * L; o += 4) {
    const float* w = o < L ? w_mu + (int64_t)o * C : w_lv + (int64_t)(o - L) * C;
    float a = 0.f;
    for (int c = lane; c < C; c += 64) a += w[c] * pm[c];
    a = wave_sum(a);
    if (lane == 0) {
      if (o < L) {
        a += b_mu ? b_mu[o] : 0.f;
        mu[(int64_t)n * L + o] = a;
      } else {
        a += b_lv ? b_lv[o - L] : 0.f;
        logvar[(int64_t)n * L + o - L] = a;
      }
    }
  }
  __syncthreads();
  __threadfence_block();
  for (int j = tid; j < L; j += 256) {
    const float m = mu[(int64_t)n * L + j];
    z[(int64_t)n * L + j] = eps ? m + eps[(int64_t)n * L + j] * expf(0.5f * logvar[(int64_t)n * L + j]) : m;
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
  for (int64_t e = e0 * vpp + tid; e < e1 * vpp; e += 256) {
    const int64_t pix = e / vpp;
    const int v = (int)(e - pix * vpp);
    const int n = (int)(pix / J.HW);
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
  if (row < rows)
    for (int p = p0 + row; p < p1; p += rows) {
      Vec8<T> v;
      v.load(d + ((int64_t)n * J.HW + p) * J.dmap_stride + cv * 8);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v.get(k);
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

// one block: every consumer's backward on the vectors, then the bottleneck's
__global__ __launch_bounds__(1024) void latent_bwd_kernel(const LatentJobs jobs, int njobs, VuLatentHeads hb,
                                                          int N, int L, float* ws) {
  // ws: DY [sum_j N * co_j] floats, then dz [N][L], dmu [N][L], dlv [N][L]
  const int tid = threadIdx.x;
  int64_t off = 0;
  for (int j = 0; j < njobs; ++j) {
    const VuLatentJob& J = jobs.j[j];
    float* DY = ws + off;
    off += (int64_t)N * J.co;
    const float rM = 1.f / (float)N;   // HW / (N * HW)
    for (int c = tid; c < J.co; c += 1024) {
      const float scale = J.coef[c], shift = J.coef[J.co + c], mean = J.coef[2 * J.co + c],
                  invstd = J.coef[3 * J.co + c];
      double db = 0.0, dg = 0.0;
      for (int n = 0; n < N; ++n) {
        float S = 0.f;
        for (int s = 0; s < LAT_SPLITS; ++s) S += J.part[((int64_t)n * LAT_SPLITS + s) * J.co + c];
        const float y = J.y[(int64_t)n * J.co + c];
        const float G = (y * scale + shift > 0.f) ? S : 0.f;
        DY[(int64_t)n * J.co + c] = G;
        db += G;
        dg += (double)G * ((y - mean) * invstd);
      }
      if (J.dgamma) J.dgamma[c] = J.grad_acc ? J.dgamma[c] + (float)dg : (float)dg;
      if (J.dbeta) J.dbeta[c] = J.grad_acc ? J.dbeta[c] + (float)db : (float)db;
      const float gi = J.gamma[c] * invstd;
      double dbias = 0.0;
      for (int n = 0; n < N; ++n) {
        const float y = J.y[(int64_t)n * J.co + c];
        const float G = DY[(int64_t)n * J.co + c];
        const float v = J.train ? gi * (G - rM * ((float)db + (y - mean) * invstd * (float)dg)) : gi * G;
        DY[(int64_t)n * J.co + c] = v;
        dbias += v;
      }
      // the conv bias of a train-mode BatchNorm has an exactly zero gradient
      // (the batch mean absorbs it; engine.bias_grad)
      if (J.dbias) {
        const float b = J.train ? 0.f : (float)dbias;
        J.dbias[c] = J.grad_acc ? J.dbias[c] + b : b;
      }
    }
  }
  __syncthreads();
  // conv weight gradients: dW[co][l] (+)= sum_n DY[n][co] z[n][l]
  off = 0;
  for (int j = 0; j < njobs; ++j) {
    const VuLatentJob& J = jobs.j[j];
    const float* DY = ws + off;
    off += (int64_t)N * J.co;
    if (!J.dw) continue;
    for (int e = tid; e < J.co * L; e += 1024) {
      const int c = e / L, l = e - c * L;
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += DY[(int64_t)n * J.co + c] * hb.z[(int64_t)n * L + l];
      J.dw[e] = J.grad_acc ? J.dw[e] + s : s;
    }
  }
  // dz[n][l] = sum_j sum_co W_j[co][l] DY_j[n][co]
  float* dz = ws + off;
  float* dmu = dz + N * L;
  float* dlv = dmu + N * L;
  for (int e = tid; e < N * L; e += 1024) {
    const int n = e / L, l = e - n * L;
    float s = hb.dz_in ? hb.dz_in[e] : 0.f;
    int64_t o2 = 0;
    for (int j = 0; j < njobs; ++j) {
      const VuLatentJob& J = jobs.j[j];
      const float* DY = ws + o2;
      o2 += (int64_t)N * J.co;
      for (int c = 0; c < J.co; ++c) s += J.w[(int64_t)c * L + l] * DY[(int64_t)n * J.co + c];
    }
    dz[e] = s;
    // reparameterize backward (unet_resnet.py:191-194): z = mu + eps * exp(lv / 2)
    const float gm = hb.dmu_in ? hb.dmu_in[e] : 0.f;
    const float gl = hb.dlv_in ? hb.dlv_in[e] : 0.f;
    dmu[e] = gm + s;
    dlv[e] = gl + (hb.eps ? s * hb.eps[e] * 0.5f * expf(0.5f * hb.logvar[e]) : 0.f);
  }
  __syncthreads();
  // heads: dW[j][c] (+)= sum_n d[n][j] pooled[n][c]; db[j] (+)= sum_n d[n][j]
  const int C = hb.C;
  for (int e = tid; e < 2 * L * C; e += 1024) {
    const int h = e / (L * C), r = e - h * (L * C), jj = r / C, c = r - jj * C;
    const float* d = h ? dlv : dmu;
    float* dw = h ? hb.dw_lv : hb.dw_mu;
    if (!dw) continue;
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += d[n * L + jj] * hb.pooled[(int64_t)n * C + c];
    dw[r] = hb.grad_acc ? dw[r] + s : s;
  }
  for (int e = tid; e < 2 * L; e += 1024) {
    const int h = e / L, jj = e - h * L;
    const float* d = h ? dlv : dmu;
    float* db = h ? hb.db_lv : hb.db_mu;
    if (!db) continue;
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += d[n * L + jj];
    db[jj] = hb.grad_acc ? db[jj] + s : s;
  }
  // dpooled[n][c] = sum_j w_mu[j][c] dmu[n][j] + w_lv[j][c] dlv[n][j]
  for (int e = tid; e < N * C; e += 1024) {
    const int n = e / C, c = e - n * C;
    float s = 0.f;
    for (int jj = 0; jj < L; ++jj)
      s += hb.w_mu[(int64_t)jj * C + c] * dmu[n * L + jj] + hb.w_lv[(int64_t)jj * C + c] * dlv[n * L + jj];
    hb.dpooled[e] = s;
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
  const int rows = 256 / (C / 8);
  const size_t shm = (size_t)(rows + 1) * C * sizeof(float);
  if (shm > 64 * 1024) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((heads_fwd_kernel<T>), dim3(N), dim3(256), shm, st, (const T*)f4, fs, HW, C, w_mu, b_mu, w_lv,
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
  hipLaunchKernelGGL(latent_bwd_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, J, njobs, *heads, N, L,
                     workspace);
  return (int)hipGetLastError();
}
