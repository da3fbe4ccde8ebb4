// Optimizer tail of the training step (train.py:406-411): global-norm
// gradient clipping (torch.nn.utils.clip_grad_norm_, norm_type 2) and AdamW
// (torch.optim.AdamW, decoupled weight decay, amsgrad off) as multi-tensor
// launches: one table of tensors, one launch per phase instead of ~15
// foreach launches per parameter group.
//
// Table layout (device memory, VuMtEntry per tensor): the tensors' storage is
// processed linearly (params, grads and moments share strides), cut into
// CHUNK-element chunks; entry.chunk0 is the prefix count of chunks so a block
// finds its tensor by binary search.
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int MT_THREADS = 256;
constexpr int MT_CHUNK = 8192;  // elements per block (32 per thread)

// the table's tensor pointers are generic (flat) pointers; cast to the global
// address space so the element loads and stores issue as global_* (vmcnt
// only) instead of flat_* (vmcnt + lgkmcnt)
typedef __attribute__((address_space(1))) float gfl;
typedef __attribute__((address_space(1))) f32x4 gf32x4;

VU_DEV int find_tensor(const VuMtEntry* t, int n, int64_t chunk) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (t[mid].chunk0 <= chunk) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// per-chunk sum of squares of the grads (fp64, fixed order inside the block)
__global__ void mt_sumsq_kernel(const VuMtEntry* t, int n, double* part) {
  __shared__ double sh[MT_THREADS / 64];
  const int64_t chunk = blockIdx.x;
  const int k = find_tensor(t, n, chunk);
  const int64_t off = (chunk - t[k].chunk0) * MT_CHUNK;
  const int64_t end = min(t[k].numel, off + MT_CHUNK);
  const gfl* g = (const gfl*)(t[k].grad);
  double a = 0;
  if (end - off == MT_CHUNK) {
    // a whole chunk: the thread's 32 loads issued before the first is used
    // (the guarded loop below serialised them behind the fp64 chain: 2.7
    // TB/s); the same elements summed in the same order
    constexpr int U = MT_CHUNK / MT_THREADS;
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = g[off + threadIdx.x + u * MT_THREADS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double d = v[u];
      a += d * d;
    }
  } else {
    for (int64_t i = off + threadIdx.x; i < end; i += MT_THREADS) {
      double v = g[i];
      a += v * v;
    }
  }
  a = warp_sum_d(a);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) part[chunk] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// total norm and clip coefficient: coef = min(1, max_norm / (norm + 1e-6))
__global__ void mt_norm_final(const double* part, int64_t nchunks, float max_norm, float* norm_out,
                              float* coef_out) {
  __shared__ double sh[4];
  double a = 0;
  for (int64_t i = threadIdx.x; i < nchunks; i += 256) a += part[i];
  a = warp_sum_d(a);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x != 0) return;
  const float norm = (float)sqrt((sh[0] + sh[1]) + (sh[2] + sh[3]));
  if (norm_out) *norm_out = norm;
  if (coef_out) {
    float c = max_norm / (norm + 1e-6f);
    *coef_out = c < 1.f ? c : 1.f;
  }
}

__global__ void mt_scale_kernel(const VuMtEntry* t, int n, const float* coef) {
  const int64_t chunk = blockIdx.x;
  const int k = find_tensor(t, n, chunk);
  const int64_t off = (chunk - t[k].chunk0) * MT_CHUNK;
  const int64_t end = min(t[k].numel, off + MT_CHUNK);
  gfl* g = (gfl*)(t[k].grad);
  const float c = *coef;
  for (int64_t i = off + threadIdx.x; i < end; i += MT_THREADS) g[i] *= c;
}

// One AdamW element update, every operation rounded on its own (no fused
// multiply-add contraction): the eager, the capturable scalar and the
// capturable 16-byte paths must produce identical bits whatever the compiler
// vectorises.
VU_DEV void adamw_elem(float gi, float& pi, float& mi, float& vi, float decay, float w1, float beta2, float w2,
                       float eps, float step_size, float bc2s) {
#pragma clang fp contract(off)
  pi = pi * decay;
  mi = mi + w1 * (gi - mi);  // lerp, weight < 0.5 branch
  vi = vi * beta2;
  vi = vi + w2 * gi * gi;
  const float denom = sqrtf(vi) / bc2s + eps;
  pi = pi + (-step_size) * (mi / denom);
}

// AdamW, the element order of torch's _multi_tensor_adamw:
//   p *= 1 - lr*wd; m = lerp(m, g, 1-b1); v = v*b2 + (1-b2) g^2;
//   p += -step_size * m / (sqrt(v) / bc2_sqrt + eps)
// with the per-tensor step_size = lr / (1 - b1^step), bc2_sqrt = sqrt(1 - b2^step)
// taken from the table (tensors may be at different step counts).  The
// scalar factors (1 - lr*wd, 1 - b1, 1 - b2) arrive precomputed in double and
// rounded once, as torch's foreach path passes them.
__global__ void mt_adamw_kernel(const VuMtEntry* t, int n, float decay, float w1, float beta2, float w2,
                                float eps, const float* gscale) {
  const int64_t chunk = blockIdx.x;
  const int k = find_tensor(t, n, chunk);
  const int64_t off = (chunk - t[k].chunk0) * MT_CHUNK;
  const int64_t end = min(t[k].numel, off + MT_CHUNK);
  gfl* p = (gfl*)(t[k].param);
  const gfl* g = (const gfl*)(t[k].grad);
  gfl* m = (gfl*)(t[k].exp_avg);
  gfl* v = (gfl*)(t[k].exp_avg_sq);
  const float step_size = t[k].step_size, bc2s = t[k].bc2_sqrt;
  const float gs = gscale ? *gscale : 1.f;
  for (int64_t i = off + threadIdx.x; i < end; i += MT_THREADS) {
    float gi = g[i];
    if (gscale) gi *= gs;
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(gi, pi, mi, vi, decay, w1, beta2, w2, eps, step_size, bc2s);
    p[i] = pi; m[i] = mi; v[i] = vi;
  }
}

// Capturable AdamW (one HIP graph replays the whole training step): the step
// count lives on the device, the bias corrections are derived from it in
// double exactly as the host path computes them (1 - beta^step, lr / bc1,
// sqrt(bc2)) and rounded to float once; all tensors share the group's step.
// zero_grad: the gradient is cleared after use, so the next backward can
// accumulate into persistent .grad buffers (graph replays need fixed
// addresses).
__global__ void mt_step_incr_kernel(float* step) { *step += 1.f; }

__global__ void mt_adamw_dev_kernel(const VuMtEntry* t, int n, float decay, float w1, float beta2, float w2,
                                    float eps, double lr, double beta1d, double beta2d, const float* step,
                                    int zero_grad, const float* gscale) {
  const int64_t chunk = blockIdx.x;
  const int k = find_tensor(t, n, chunk);
  const int64_t off = (chunk - t[k].chunk0) * MT_CHUNK;
  const int64_t end = min(t[k].numel, off + MT_CHUNK);
  gfl* p = (gfl*)(t[k].param);
  gfl* g = (gfl*)(t[k].grad);
  gfl* m = (gfl*)(t[k].exp_avg);
  gfl* v = (gfl*)(t[k].exp_avg_sq);
  const double sc = (double)*step;
  const float step_size = (float)(lr / (1.0 - pow(beta1d, sc)));
  const float bc2s = (float)sqrt(1.0 - pow(beta2d, sc));
  // gscale (the clip coefficient): g * c rounded once, as vu_mt_scale_grads
  // stores it -- the same bits as scaling first
  const float gc = gscale ? *gscale : 1.f;
  auto upd = [&](float gi, float& pi, float& mi, float& vi) {
    if (gscale) gi = gi * gc;
    adamw_elem(gi, pi, mi, vi, decay, w1, beta2, w2, eps, step_size, bc2s);
  };
  // 16-byte accesses (4 elements per thread and iteration, the four streams'
  // loads in flight together) when the four tensors' chunk starts are
  // 16-byte aligned; the same per-element arithmetic either way
  const bool vec = (((uintptr_t)(p + off) | (uintptr_t)(g + off) | (uintptr_t)(m + off) | (uintptr_t)(v + off)) &
                    15) == 0;
  int64_t i0 = off;
  if (vec) {
    const int64_t nv = (end - off) / 4;
    for (int64_t q = threadIdx.x; q < nv; q += MT_THREADS) {
      const int64_t i = off + 4 * q;
      const f32x4 gv = *reinterpret_cast<const gf32x4*>(g + i);
      f32x4 pv = *reinterpret_cast<const gf32x4*>(p + i);
      f32x4 mv = *reinterpret_cast<const gf32x4*>(m + i);
      f32x4 vv = *reinterpret_cast<const gf32x4*>(v + i);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float pi = pv[u], mi = mv[u], vi = vv[u];
        upd(gv[u], pi, mi, vi);
        pv[u] = pi;
        mv[u] = mi;
        vv[u] = vi;
      }
      *reinterpret_cast<gf32x4*>(p + i) = pv;
      *reinterpret_cast<gf32x4*>(m + i) = mv;
      *reinterpret_cast<gf32x4*>(v + i) = vv;
      if (zero_grad) *reinterpret_cast<gf32x4*>(g + i) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    i0 = off + 4 * nv;
  }
  for (int64_t i = i0 + threadIdx.x; i < end; i += MT_THREADS) {
    float pi = p[i], mi = m[i], vi = v[i];
    upd(g[i], pi, mi, vi);
    p[i] = pi; m[i] = mi; v[i] = vi;
    if (zero_grad) g[i] = 0.f;
  }
}

}  // namespace

extern "C" int vu_mt_adamw_dev_scaled(const VuMtEntry* table, int ntensors, int64_t nchunks, double lr,
                                      double weight_decay, double beta1, double beta2, double eps, float* step,
                                      int zero_grad, const float* grad_scale, void* stream) {
  if (ntensors <= 0 || nchunks <= 0) return 0;
  if (grad_scale && !zero_grad) return (int)hipErrorInvalidValue;  // the scaled gradient is never stored
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(mt_step_incr_kernel, dim3(1), dim3(1), 0, st, step);
  hipLaunchKernelGGL(mt_adamw_dev_kernel, dim3((unsigned)nchunks), dim3(MT_THREADS), 0, st, table, ntensors,
                     (float)(1.0 - lr * weight_decay), (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                     (float)eps, lr, beta1, beta2, step, zero_grad, grad_scale);
  return (int)hipGetLastError();
}

extern "C" int vu_mt_adamw_dev(const VuMtEntry* table, int ntensors, int64_t nchunks, double lr,
                               double weight_decay, double beta1, double beta2, double eps, float* step,
                               int zero_grad, void* stream) {
  return vu_mt_adamw_dev_scaled(table, ntensors, nchunks, lr, weight_decay, beta1, beta2, eps, step, zero_grad,
                                nullptr, stream);
}

extern "C" int64_t vu_mt_chunk_elems() { return MT_CHUNK; }

extern "C" int vu_mt_grad_norm(const VuMtEntry* table, int ntensors, int64_t nchunks, float max_norm,
                               float* total_norm, float* clip_coef, double* workspace, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (ntensors <= 0 || nchunks <= 0) return 0;
  hipLaunchKernelGGL(mt_sumsq_kernel, dim3((unsigned)nchunks), dim3(MT_THREADS), 0, st, table, ntensors,
                     workspace);
  hipLaunchKernelGGL(mt_norm_final, dim3(1), dim3(256), 0, st, workspace, nchunks, max_norm, total_norm,
                     clip_coef);
  return (int)hipGetLastError();
}

extern "C" int vu_mt_scale_grads(const VuMtEntry* table, int ntensors, int64_t nchunks, const float* coef,
                                 void* stream) {
  if (ntensors <= 0 || nchunks <= 0) return 0;
  hipLaunchKernelGGL(mt_scale_kernel, dim3((unsigned)nchunks), dim3(MT_THREADS), 0, (hipStream_t)stream, table,
                     ntensors, coef);
  return (int)hipGetLastError();
}

extern "C" int vu_mt_adamw(const VuMtEntry* table, int ntensors, int64_t nchunks, float decay,
                           float one_minus_beta1, float beta2, float one_minus_beta2, float eps,
                           const float* grad_scale, void* stream) {
  if (ntensors <= 0 || nchunks <= 0) return 0;
  hipLaunchKernelGGL(mt_adamw_kernel, dim3((unsigned)nchunks), dim3(MT_THREADS), 0, (hipStream_t)stream, table,
                     ntensors, decay, one_minus_beta1, beta2, one_minus_beta2, eps, grad_scale);
  return (int)hipGetLastError();
}
