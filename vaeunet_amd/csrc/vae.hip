// VAE-U-Net pieces (unet/unet_resnet.py): ResNet34 encoder glue, the latent
// bottleneck and its broadcasts.
//
//   encoder maxpool 3x3/s2/p1 ............ timm resnet34 stem (unet_resnet.py:131-137)
//   BasicBlock tail relu(bn2(y) + shortcut)  timm BasicBlock
//   mu/logvar heads: conv1x1 + AdaptiveAvgPool2d(1) == mean over pixels then
//     a [L x C] linear map (unet_resnet.py:140-147, 205-206)
//   reparameterize z = mu + eps*exp(0.5*logvar) (unet_resnet.py:191-194)
//   z_spatial = interpolate(z[...,None,None], size, align_corners=True): an
//     exact broadcast of the per-sample vector (unet_resnet.py:217-221, 93)
//
// NHWC, fixed-channel 8-wide vectors, deterministic reductions.
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

inline unsigned ew_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// ---- max pool 3x3, stride 2, pad 1 (records the window argmax 0..8) ----
template <typename T>
__global__ void maxpool3_fwd_kernel(const T* x, int64_t xs, int N, int H, int W, int C, int Ho, int Wo, T* y,
                                    int64_t ys, uint8_t* idx) {
  const int V = C >> 3;
  int64_t tot = (int64_t)N * Ho * Wo * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t q = e / V;
    int c = (int)(e - q * V) * 8;
    int j = (int)(q % Wo);
    int64_t t = q / Wo;
    int i = (int)(t % Ho);
    int n = (int)(t / Ho);
    float best[8];
    int arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; arg[k] = 0; }
    for (int a = 0; a < 3; ++a) {
      int h = 2 * i - 1 + a;
      if (h < 0 || h >= H) continue;
      for (int b = 0; b < 3; ++b) {
        int w = 2 * j - 1 + b;
        if (w < 0 || w >= W) continue;
        Vec8<T> v;
        v.load(x + (((int64_t)n * H + h) * W + w) * xs + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float f = v.get(k);
          if (f > best[k] || isnan(f)) { best[k] = f; arg[k] = a * 3 + b; }
        }
      }
    }
    Vec8<T> o;
#pragma unroll
    for (int k = 0; k < 8; ++k) { o.set(k, best[k]); idx[q * C + c + k] = (uint8_t)arg[k]; }
    o.store(y + q * ys + c);
  }
}

// gather form: input pixel (h,w) collects dy of every window whose argmax it is
template <typename T>
__global__ void maxpool3_bwd_kernel(const T* dy, int64_t dys, const uint8_t* idx, int N, int H, int W, int C, int Ho,
                                    int Wo, T* dx, int64_t dxs, int accumulate) {
  const int V = C >> 3;
  int64_t tot = (int64_t)N * H * W * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t q = e / V;
    int c = (int)(e - q * V) * 8;
    int w = (int)(q % W);
    int64_t t = q / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    int i0 = h / 2, i1 = (h + 1) / 2;  // windows 2i-1 <= h <= 2i+1
    int j0 = w / 2, j1 = (w + 1) / 2;
    for (int i = i0; i <= i1 && i < Ho; ++i) {
      int a = h - (2 * i - 1);
      if (a < 0 || a > 2) continue;
      for (int j = j0; j <= j1 && j < Wo; ++j) {
        int b = w - (2 * j - 1);
        if (b < 0 || b > 2) continue;
        int64_t oq = ((int64_t)n * Ho + i) * Wo + j;
        Vec8<T> g;
        g.load(dy + oq * dys + c);
        const uint8_t* ip = idx + oq * C + c;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (ip[k] == a * 3 + b) acc[k] += g.get(k);
      }
    }
    T* d = dx + q * dxs + c;
    Vec8<T> o;
    if (accumulate) {
      o.load(d);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += o.get(k);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) o.set(k, acc[k]);
    o.store(d);
  }
}

// ---- BasicBlock tail: out = relu(y*s+t + (r*rs+rt | r)) ----
template <typename T>
__global__ void bn_add_relu_kernel(const T* y, int64_t ys, const float* sc, const float* sh, const T* r, int64_t rs,
                                   const float* rsc, const float* rsh, int64_t P, int C, T* out, int64_t os) {
  const int V = C >> 3;
  int64_t tot = P * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = e / V;
    int c = (int)(e - p * V) * 8;
    Vec8<T> vy, vr, vo;
    vy.load(y + p * ys + c);
    vr.load(r + p * rs + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float s = vy.get(k) * sc[c + k] + sh[c + k];
      float rr = vr.get(k);
      if (rsc) rr = rr * rsc[c + k] + rsh[c + k];
      vo.set(k, fmaxf(s + rr, 0.f));
    }
    vo.store(out + p * os + c);
  }
}

// g = dout * (out > 0)
template <typename T>
__global__ void relu_mask_kernel(const T* dout, int64_t ds, const T* out, int64_t os, int64_t P, int C, T* g,
                                 int64_t gs) {
  const int V = C >> 3;
  int64_t tot = P * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = e / V;
    int c = (int)(e - p * V) * 8;
    Vec8<T> vd, vo, vg;
    vd.load(dout + p * ds + c);
    vo.load(out + p * os + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) vg.set(k, vo.get(k) > 0.f ? vd.get(k) : 0.f);
    vg.store(g + p * gs + c);
  }
}

// out[n][c] (+)= scale * sum_{p of sample n} x[n,p,c]; one block per sample
// stage 1: grid (N, S): block (n, s) sums pixels [s*per, (s+1)*per) of
// sample n into part[n][s][C] (16-byte rows, fixed order)
constexpr int SS_SPLITS = 64;
template <typename T>
__global__ void sample_sum_partial(const T* x, int64_t xs, int HW, int C, int per, float* part) {
  __shared__ float sh[256 * 8];
  const int n = blockIdx.x, sidx = blockIdx.y;
  const int V = C >> 3, R = 256 / V;
  const int cv = threadIdx.x % V, row = threadIdx.x / V;
  const int c = cv * 8;
  const int p0 = sidx * per, p1 = min(HW, p0 + per);
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  if (row < R)
    for (int p = p0 + row; p < p1; p += R) {
      Vec8<T> v;
      v.load(x + ((int64_t)n * HW + p) * xs + c);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v.get(k);
    }
  if (row < R)
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[row * C + c + k] = s[k];
  __syncthreads();
  for (int cc = threadIdx.x; cc < C; cc += 256) {
    float t = 0.f;
    t = lds_sum(sh + cc, R, C);
    part[((int64_t)n * gridDim.y + sidx) * C + cc] = t;
  }
}

// stage 2: out[n][c] (+)= scale * sum_s part[n][s][c] (fixed order)
__global__ void sample_sum_final(const float* part, int N, int S, int C, float scale, float* out, int accumulate) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)N * C) return;
  const int n = (int)(e / C), c = (int)(e - (int64_t)n * C);
  float t = 0.f;
  for (int s = 0; s < S; ++s) t += part[((int64_t)n * S + s) * C + c];
  out[e] = accumulate ? out[e] + scale * t : scale * t;
}

// y[n,p,c] (+)= scale * v[n][c] for every pixel p (exact broadcast)
template <typename T>
__global__ void sample_broadcast_kernel(const float* v, int N, int HW, int C, float scale, T* y, int64_t ys,
                                        int accumulate) {
  int64_t tot = (int64_t)N * HW * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(e % C);
    int64_t q = e / C;
    int n = (int)(q / HW);
    T* d = y + q * ys + c;
    float val = scale * v[(int64_t)n * C + c];
    st1<T>(d, accumulate ? ld1<T>(d) + val : val);
  }
}

// y[b][j] = bias[j] + sum_k x[b][k] w[j][k]
__global__ void linear_small_fwd(const float* x, int B, int K, const float* w, const float* bias, int J, float* y) {
  int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= B * J) return;
  int b = o / J, j = o - b * J;
  double s = bias ? bias[j] : 0.f;
  for (int k = 0; k < K; ++k) s += (double)x[(int64_t)b * K + k] * w[(int64_t)j * K + k];
  y[o] = (float)s;
}

// dx[b][k] (+)= sum_j dy[b][j] w[j][k]; dw[j][k] (+)= sum_b dy[b][j] x[b][k]; db[j] (+)= sum_b dy
__global__ void linear_small_bwd(const float* x, int B, int K, const float* w, int J, const float* dy, float* dx,
                                 int dx_acc, float* dw, float* db, int w_acc) {
  int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (dx && o < B * K) {
    int b = o / K, k = o - b * K;
    float s = 0.f;
    for (int j = 0; j < J; ++j) s += dy[(int64_t)b * J + j] * w[(int64_t)j * K + k];
    dx[o] = dx_acc ? dx[o] + s : s;
  }
  if (dw && o < J * K) {
    int j = o / K, k = o - j * K;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dy[(int64_t)b * J + j] * x[(int64_t)b * K + k];
    dw[o] = w_acc ? dw[o] + s : s;
  }
  if (db && o < J) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dy[(int64_t)b * J + o];
    db[o] = w_acc ? db[o] + s : s;
  }
}

// z = mu + eps * exp(0.5*lv) (eps == null: z = mu)
__global__ void reparam_fwd(const float* mu, const float* lv, const float* eps, int n, float* z) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  z[i] = eps ? mu[i] + eps[i] * expf(0.5f * lv[i]) : mu[i];
}

// dmu (+)= dz ; dlv (+)= dz * eps * 0.5 * exp(0.5*lv)
__global__ void reparam_bwd(const float* lv, const float* eps, const float* dz, int n, float* dmu, float* dlv,
                            int accumulate) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float gm = dz[i];
  float gl = eps ? dz[i] * eps[i] * 0.5f * expf(0.5f * lv[i]) : 0.f;
  dmu[i] = accumulate ? dmu[i] + gm : gm;
  dlv[i] = accumulate ? dlv[i] + gl : gl;
}

inline bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

}  // namespace

#define DISPATCH_T(dtype, ...) \
  if ((dtype) == VU_BF16) { using T = bf16_t; __VA_ARGS__; } else { using T = float; __VA_ARGS__; }

extern "C" int vu_maxpool3s2_fwd(const void* x, int64_t xs, int N, int H, int W, int C, void* y, int64_t ys,
                                 uint8_t* idx, int dtype, void* stream) {
  if (C % 8 || xs % 8 || ys % 8) return (int)hipErrorInvalidValue;
  int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  int64_t work = (int64_t)N * Ho * Wo * C / 8;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((maxpool3_fwd_kernel<T>), dim3(ew_grid(work)), dim3(256), 0, st, (const T*)x, xs, N, H, W, C,
                       Ho, Wo, (T*)y, ys, idx);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_maxpool3s2_bwd(const void* dy, int64_t dys, const uint8_t* idx, int N, int H, int W, int C,
                                 void* dx, int64_t dxs, int accumulate, int dtype, void* stream) {
  if (C % 8 || dys % 8 || dxs % 8) return (int)hipErrorInvalidValue;
  int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  int64_t work = (int64_t)N * H * W * C / 8;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((maxpool3_bwd_kernel<T>), dim3(ew_grid(work)), dim3(256), 0, st, (const T*)dy, dys, idx, N, H,
                       W, C, Ho, Wo, (T*)dx, dxs, accumulate);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_bn_add_relu(const void* y, int64_t ys, const float* sc, const float* sh, const void* r, int64_t rs,
                              const float* rsc, const float* rsh, int64_t P, int C, void* out, int64_t os, int dtype,
                              void* stream) {
  if (C % 8 || ys % 8 || rs % 8 || os % 8) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((bn_add_relu_kernel<T>), dim3(ew_grid(P * C / 8)), dim3(256), 0, st, (const T*)y, ys, sc, sh,
                       (const T*)r, rs, rsc, rsh, P, C, (T*)out, os);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_relu_mask(const void* dout, int64_t ds, const void* out, int64_t os, int64_t P, int C, void* g,
                            int64_t gs, int dtype, void* stream) {
  if (C % 8 || ds % 8 || os % 8 || gs % 8) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((relu_mask_kernel<T>), dim3(ew_grid(P * C / 8)), dim3(256), 0, st, (const T*)dout, ds,
                       (const T*)out, os, P, C, (T*)g, gs);
  })
  return (int)hipGetLastError();
}

extern "C" int64_t vu_sample_sum_workspace_bytes(int N, int C) {
  return (int64_t)N * SS_SPLITS * C * (int64_t)sizeof(float);
}

extern "C" int vu_sample_sum(const void* x, int64_t xs, int N, int HW, int C, float scale, float* out,
                             int accumulate, float* workspace, int dtype, void* stream) {
  if (C % 8 || xs % 8 || !pow2(C / 8) || C / 8 > 256) return (int)hipErrorInvalidValue;
  if (N == 0 || C == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int per = (HW + SS_SPLITS - 1) / SS_SPLITS;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((sample_sum_partial<T>), dim3(N, SS_SPLITS), dim3(256), 0, st, (const T*)x, xs, HW, C, per,
                       workspace);
  })
  hipLaunchKernelGGL(sample_sum_final, dim3((unsigned)(((int64_t)N * C + 255) / 256)), dim3(256), 0, st, workspace,
                     N, SS_SPLITS, C, scale, out, accumulate);
  return (int)hipGetLastError();
}

extern "C" int vu_sample_broadcast(const float* v, int N, int HW, int C, float scale, void* y, int64_t ys,
                                   int accumulate, int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((sample_broadcast_kernel<T>), dim3(ew_grid((int64_t)N * HW * C)), dim3(256), 0, st, v, N, HW,
                       C, scale, (T*)y, ys, accumulate);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_linear_small_fwd(const float* x, int B, int K, const float* w, const float* bias, int J, float* y,
                                   void* stream) {
  hipLaunchKernelGGL(linear_small_fwd, dim3((B * J + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, B, K, w, bias,
                     J, y);
  return (int)hipGetLastError();
}

extern "C" int vu_linear_small_bwd(const float* x, int B, int K, const float* w, int J, const float* dy, float* dx,
                                   int dx_acc, float* dw, float* db, int w_acc, void* stream) {
  int n = B * K > J * K ? B * K : J * K;
  hipLaunchKernelGGL(linear_small_bwd, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, B, K, w, J, dy,
                     dx, dx_acc, dw, db, w_acc);
  return (int)hipGetLastError();
}

extern "C" int vu_reparam_fwd(const float* mu, const float* lv, const float* eps, int n, float* z, void* stream) {
  hipLaunchKernelGGL(reparam_fwd, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, mu, lv, eps, n, z);
  return (int)hipGetLastError();
}

extern "C" int vu_reparam_bwd(const float* lv, const float* eps, const float* dz, int n, float* dmu, float* dlv,
                              int accumulate, void* stream) {
  hipLaunchKernelGGL(reparam_bwd, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, lv, eps, dz, n, dmu, dlv,
                     accumulate);
  return (int)hipGetLastError();
}
