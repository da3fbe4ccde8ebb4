// Inference-side elementwise / blending kernels of the VAE-U-Net sampling
// path:
//   * vu_mean_groups   : torch.stack(predictions).mean(0)   (utils/vae_utils.py:71-72)
//   * vu_sigmoid       : torch.sigmoid                      (visualize_vae.py:83, 345)
//   * vu_patch_blend   : feathered sliding-window accumulation of one patch
//                        prediction (visualize_vae.py:360-384)
//   * vu_blend_finish  : output / (weight + 1e-8)           (visualize_vae.py:409)
//   * vu_uncertainty   : mean / std / entropy / mutual information / coefficient
//                        of variation over the sample axis (visualize_vae.py:90-117)
//   * vu_gather_affine : per-sample integer pixel map (flips / 90-degree
//                        rotations of the patch-cache batches: the geometric
//                        part of utils/data_loading.py:116-120's augmentation)
// All fp32, one thread per output element, fixed summation order (the
// results do not depend on the launch geometry).
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

inline unsigned grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 65535) g = 65535;
  if (g < 1) g = 1;
  return (unsigned)g;
}

__global__ void mean_groups_kernel(const float* x, int groups, int64_t n, float* out) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < groups; ++k) s += x[k * n + e];
    out[e] = s / (float)groups;
  }
}

__global__ void sigmoid_kernel(const float* x, int64_t n, float* y) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    y[e] = 1.f / (1.f + expf(-x[e]));
}

// weight of patch row/column i (length L) along one axis: the reference
// multiplies a ones tensor by ramp on the leading `ov` entries (if `lead`)
// and then by (1 - ramp) on the trailing ones (if `trail`), only when
// L > 2*ov (visualize_vae.py:364-378)
VU_DEV float axis_weight(float w, int i, int L, int ov, int lead, int trail, const float* ramp) {
  if (L > 2 * ov) {
    if (lead && i < ov) w *= ramp[i];
    if (trail && i >= L - ov) w *= 1.f - ramp[i - (L - ov)];
  }
  return w;
}

__global__ void patch_blend_kernel(const float* pred, int64_t pred_img_stride, int B, int ph, int pw, float* out,
                                   float* wsum, int H, int W, int sh, int sw, const float* ramp, int ov, int top,
                                   int bottom, int left, int right) {
  const int64_t n = (int64_t)B * ph * pw;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(e % pw);
    const int64_t t = e / pw;
    const int y = (int)(t % ph);
    const int b = (int)(t / ph);
    float w = axis_weight(1.f, y, ph, ov, top, bottom, ramp);
    w = axis_weight(w, x, pw, ov, left, right, ramp);
    const float p = pred[b * pred_img_stride + (int64_t)y * pw + x];
    const int64_t o = ((int64_t)b * H + sh + y) * W + sw + x;
    out[o] += p * w;
    wsum[o] += w;
  }
}

__global__ void blend_finish_kernel(float* out, const float* wsum, int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
    out[e] = out[e] / (wsum[e] + 1e-8f);
}

__global__ void uncertainty_kernel(const float* seg, int S, int64_t n, float* mean, float* std, float* entropy,
                                   float* mi, float* cv) {
  const float eps = 1e-7f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f, ent = 0.f;
    for (int k = 0; k < S; ++k) {
      const float v = seg[k * n + e];
      s += v;
      ent += -(v * logf(v + eps) + (1.f - v) * logf(1.f - v + eps));
    }
    const float m = s / (float)S;
    float q = 0.f;
    for (int k = 0; k < S; ++k) {
      const float d = seg[k * n + e] - m;
      q += d * d;
    }
    const float sd = S > 1 ? sqrtf(q / (float)(S - 1)) : __builtin_nanf("");  // torch.std: unbiased
    const float h = -(m * logf(m + eps) + (1.f - m) * logf(1.f - m + eps));
    mean[e] = m;
    std[e] = sd;
    entropy[e] = h;
    mi[e] = h - ent / (float)S;
    cv[e] = sd / (m + eps);
  }
}

// y[b, i, j, :] = x[b, m0*i + m1*j + m2, m3*i + m4*j + m5, :] (NHWC, 16-byte
// vectors when C*elem is a multiple of 16, else element-wise)
template <typename T>
__global__ void gather_affine_kernel(const T* x, int B, int H, int W, int C, const int* m, T* y, int Ho, int Wo) {
  const int V = (C % 8 == 0) ? C / 8 : C;
  const bool vec = C % 8 == 0;
  const int64_t n = (int64_t)B * Ho * Wo * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int v = (int)(e % V);
    int64_t t = e / V;
    const int j = (int)(t % Wo);
    t /= Wo;
    const int i = (int)(t % Ho);
    const int b = (int)(t / Ho);
    const int* mb = m + 6 * b;
    const int sy = mb[0] * i + mb[1] * j + mb[2], sx = mb[3] * i + mb[4] * j + mb[5];
    const int64_t src = (((int64_t)b * H + sy) * W + sx) * C, dst = (((int64_t)b * Ho + i) * Wo + j) * C;
    if (vec) {
      Vec8<T> q;
      q.load(x + src + v * 8);
      q.store(y + dst + v * 8);
    } else {
      y[dst + v] = x[src + v];
    }
  }
}

}  // namespace

extern "C" int vu_mean_groups(const float* x, int groups, int64_t n, float* out, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(mean_groups_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, groups, n, out);
  return (int)hipGetLastError();
}

extern "C" int vu_sigmoid(const float* x, int64_t n, float* y, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(sigmoid_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, y);
  return (int)hipGetLastError();
}

extern "C" int vu_patch_blend(const float* pred, int64_t pred_img_stride, int B, int ph, int pw, float* out,
                              float* wsum, int H, int W, int sh, int sw, const float* ramp, int overlap, int top,
                              int bottom, int left, int right, void* stream) {
  if (sh < 0 || sw < 0 || sh + ph > H || sw + pw > W) return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)B * ph * pw;
  if (n == 0) return 0;
  hipLaunchKernelGGL(patch_blend_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, pred, pred_img_stride,
                     B, ph, pw, out, wsum, H, W, sh, sw, ramp, overlap, top, bottom, left, right);
  return (int)hipGetLastError();
}

extern "C" int vu_blend_finish(float* out, const float* wsum, int64_t n, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(blend_finish_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, out, wsum, n);
  return (int)hipGetLastError();
}

extern "C" int vu_uncertainty(const float* seg, int samples, int64_t n, float* mean, float* std, float* entropy,
                              float* mutual_info, float* coeff_var, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(uncertainty_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, seg, samples, n, mean,
                     std, entropy, mutual_info, coeff_var);
  return (int)hipGetLastError();
}

extern "C" int vu_gather_affine(const void* x, int B, int H, int W, int C, const int* map, void* y, int Ho,
                                int Wo, int dtype, void* stream) {
  const int64_t n = (int64_t)B * Ho * Wo * ((C % 8 == 0) ? C / 8 : C);
  if (n == 0) return 0;
  if (dtype == VU_BF16)
    hipLaunchKernelGGL(gather_affine_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, B, H, W, C, map, (bf16_t*)y, Ho, Wo);
  else
    hipLaunchKernelGGL(gather_affine_kernel<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)x, B, H, W, C, map, (float*)y, Ho, Wo);
  return (int)hipGetLastError();
}
