// Training objective (utils/loss.py) and optimizer helpers.
//
//   CombinedLoss (loss.py:44-63) = 0.5*BCEWithLogits(mean) + 0.5*dice_loss
//   dice_loss (loss.py:6-28): p = sigmoid(x) (NaN -> 0, :12-14),
//        dice = (2*sum(p*t) + 1) / (clamp(sum p, .5) + clamp(sum t, .5) + 1)
//   kl_with_free_bits (loss.py:148-170)
//
// One fused pass computes all four global sums (fp64 per block, blocks
// combined in a fixed order), a one-thread epilogue forms the loss on the
// device (no host sync: the reference's isnan().any() sync at loss.py:12 is
// gone), and the backward pass is one elementwise kernel.
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int LBLK = 256;
constexpr int LNB = 1024;  // max blocks for the stage-1 reduction

VU_DEV double block_sum_d(double v, double* sh) {
  v = warp_sum_d(v);
  int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double t = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return t;
}

VU_DEV float bce_logits(float x, float t) {
  // (1 - t) * x + max(-x, 0) + log(exp(-max) + exp(-x - max))  (ATen's form)
  float mx = fmaxf(-x, 0.f);
  return (1.f - t) * x + mx + logf(expf(-mx) + expf(-x - mx));
}

VU_DEV float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void bce_dice_stage1(const float* x, const float* t, int64_t n, double* ws) {
  __shared__ double sh[4];
  double a = 0, b = 0, c = 0, d = 0;
  for (int64_t i = (int64_t)blockIdx.x * LBLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * LBLK) {
    float xv = x[i], tv = t[i];
    float p = sigm(xv);
    if (isnan(p)) p = 0.f;
    a += bce_logits(xv, tv);
    b += (double)p * tv;
    c += p;
    d += tv;
  }
  a = block_sum_d(a, sh);
  b = block_sum_d(b, sh);
  c = block_sum_d(c, sh);
  d = block_sum_d(d, sh);
  if (threadIdx.x == 0) {
    ws[blockIdx.x * 4 + 0] = a; ws[blockIdx.x * 4 + 1] = b;
    ws[blockIdx.x * 4 + 2] = c; ws[blockIdx.x * 4 + 3] = d;
  }
}

__global__ void bce_dice_stage2(const double* ws, int nblk, int64_t n, double* sums, float smooth, float w_bce,
                                float w_dice, float* loss, float* parts) {
  __shared__ double sh[4];
  double s[4] = {0, 0, 0, 0};
  for (int b = threadIdx.x; b < nblk; b += LBLK)
    for (int k = 0; k < 4; ++k) s[k] += ws[b * 4 + k];
  for (int k = 0; k < 4; ++k) s[k] = block_sum_d(s[k], sh);
  if (threadIdx.x != 0) return;
  for (int k = 0; k < 4; ++k) sums[k] = s[k];
  if (loss) {
    float bce = (float)(s[0] / (double)n);
    float I = (float)s[1];
    float sp = fmaxf((float)s[2], smooth * 0.5f), st = fmaxf((float)s[3], smooth * 0.5f);
    float dice = (2.f * I + smooth) / (sp + st + smooth);
    float dl = 1.f - dice;
    loss[0] = w_bce * bce + w_dice * dl;
    if (parts) { parts[0] = bce; parts[1] = dl; }
  }
}

__global__ void bce_dice_bwd_kernel(const float* x, const float* t, int64_t n, const double* sums, float smooth,
                                    float w_bce, float w_dice, const float* gscale, float* grad) {
  const float g = gscale ? gscale[0] : 1.f;
  const float I = (float)sums[1];
  const float spr = (float)sums[2], str = (float)sums[3];
  const float sp = fmaxf(spr, smooth * 0.5f), st = fmaxf(str, smooth * 0.5f);
  const float U = sp + st + smooth;
  const float mp = spr >= smooth * 0.5f ? 1.f : 0.f;
  const float num = 2.f * I + smooth;
  const float inv_n = 1.f / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * LBLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * LBLK) {
    float xv = x[i], tv = t[i];
    float p = sigm(xv);
    float dp = isnan(p) ? 0.f : p * (1.f - p);
    // d dice / dx = dp * (2 t U - num * mp) / U^2
    float ddice = dp * (2.f * tv * U - num * mp) / (U * U);
    grad[i] = g * (w_bce * (p - tv) * inv_n - w_dice * ddice);
  }
}

// kl_with_free_bits: nan_to_num -> 0.5(mu^2+e^lv-lv-1) -> clamp(+-100) ->
// max(., fb) (ties split the gradient 1/2-1/2, like torch.max) -> sum(1).mean()
VU_DEV float nan0(float v) {
  if (isnan(v)) return 0.f;
  if (isinf(v)) return v > 0 ? 3.4028234663852886e38f : -3.4028234663852886e38f;
  return v;
}

__global__ void kl_kernel(const float* mu, const float* lv, int B, int L, float fb, const float* gscale, float* value,
                          float* gmu, float* glv) {
  __shared__ double sh[4];
  double acc = 0;
  const float g = gscale ? gscale[0] : 1.f;
  for (int i = threadIdx.x; i < B * L; i += blockDim.x) {
    float m = nan0(mu[i]), v = nan0(lv[i]);
    float kl = 0.5f * (m * m + expf(v) - v - 1.f);
    float cmask = (kl >= -100.f && kl <= 100.f) ? 1.f : 0.f;
    float klc = fminf(fmaxf(kl, -100.f), 100.f);
    float mmask = 1.f;
    if (fb > 0.f) {
      mmask = klc > fb ? 1.f : (klc == fb ? 0.5f : 0.f);
      klc = fmaxf(klc, fb);
    }
    acc += klc;
    if (gmu) {
      float s = g * cmask * mmask / (float)B;
      bool fm = isfinite(mu[i]), fv = isfinite(lv[i]);
      gmu[i] = fm ? s * m : 0.f;
      glv[i] = fv ? s * 0.5f * (expf(v) - 1.f) : 0.f;
    }
  }
  acc = block_sum_d(acc, sh);
  if (threadIdx.x == 0 && value) {
    float r = (float)(acc / (double)B);
    value[0] = isnan(r) ? 1e-8f : r;
  }
}

__global__ void sumsq_stage1(const float* x, int64_t n, double* ws) {
  __shared__ double sh[4];
  double a = 0;
  for (int64_t i = (int64_t)blockIdx.x * LBLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * LBLK) {
    double v = x[i];
    a += v * v;
  }
  a = block_sum_d(a, sh);
  if (threadIdx.x == 0) ws[blockIdx.x] = a;
}

__global__ void sum_stage2(const double* ws, int nblk, double* out, int accumulate) {
  __shared__ double sh[4];
  double s = 0;
  for (int b = threadIdx.x; b < nblk; b += LBLK) s += ws[b];
  s = block_sum_d(s, sh);
  if (threadIdx.x != 0) return;
  out[0] = accumulate ? out[0] + s : s;
}

// Hard Dice (utils/metrics.py:8-35): a = (x > 0.5), b = (t > 0.5) over the
// whole tensor (reduce_batch_first only changes the view, not the sums);
// exact integer counts, so the result is order-independent.
__global__ void dice_score_stage1(const float* x, const float* t, int64_t n, unsigned long long* ws) {
  __shared__ unsigned long long sh[3][4];
  unsigned long long a = 0, b = 0, ab = 0;
  for (int64_t i = (int64_t)blockIdx.x * LBLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * LBLK) {
    const bool pa = x[i] > 0.5f, pb = t[i] > 0.5f;
    a += pa;
    b += pb;
    ab += pa && pb;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    ab += __shfl_xor(ab, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh[0][w] = a; sh[1][w] = b; sh[2][w] = ab; }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    ws[blockIdx.x * 3 + k] = sh[k][0] + sh[k][1] + sh[k][2] + sh[k][3];
  }
}

__global__ void dice_score_stage2(const unsigned long long* ws, int nblk, float epsilon, float* score,
                                  double* counts) {
  if (threadIdx.x != 0) return;
  unsigned long long a = 0, b = 0, ab = 0;
  for (int i = 0; i < nblk; ++i) { a += ws[i * 3]; b += ws[i * 3 + 1]; ab += ws[i * 3 + 2]; }
  // fp32 arithmetic as the reference: (2*I + eps) / (sum a + sum b + eps)
  const float I = (float)ab, den = (float)a + (float)b;
  score[0] = (a + b == 0) ? 1.f : (2.f * I + epsilon) / (den + epsilon);
  if (counts) { counts[0] = (double)a; counts[1] = (double)b; counts[2] = (double)ab; }
}

int nblocks(int64_t n) {
  int64_t b = (n + LBLK * 4 - 1) / (LBLK * 4);
  if (b > LNB) b = LNB;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" int64_t vu_loss_workspace_bytes() { return (int64_t)LNB * 4 * sizeof(double); }

extern "C" int vu_bce_dice_fwd2(const float* logits, const float* target, int64_t n, double* sums, float smooth,
                                float w_bce, float w_dice, float* loss, float* parts, double* workspace,
                                void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int nb = nblocks(n);
  hipLaunchKernelGGL(bce_dice_stage1, dim3(nb), dim3(LBLK), 0, st, logits, target, n, workspace);
  hipLaunchKernelGGL(bce_dice_stage2, dim3(1), dim3(LBLK), 0, st, workspace, nb, n, sums, smooth, w_bce, w_dice, loss,
                     parts);
  return (int)hipGetLastError();
}

extern "C" int vu_bce_dice_fwd(const float* logits, const float* target, int64_t n, double* sums, double* workspace,
                               void* stream) {
  return vu_bce_dice_fwd2(logits, target, n, sums, 1.f, 0.5f, 0.5f, nullptr, nullptr, workspace, stream);
}

extern "C" int vu_bce_dice_bwd(const float* logits, const float* target, int64_t n, const double* sums, float smooth,
                               float w_bce, float w_dice, const float* gscale, float* grad, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int nb = nblocks(n);
  hipLaunchKernelGGL(bce_dice_bwd_kernel, dim3(nb), dim3(LBLK), 0, st, logits, target, n, sums, smooth, w_bce,
                     w_dice, gscale, grad);
  return (int)hipGetLastError();
}

extern "C" int vu_kl_free_bits2(const float* mu, const float* logvar, int B, int L, float free_bits,
                                const float* gscale, float* value, float* gmu, float* glogvar, void* stream) {
  hipLaunchKernelGGL(kl_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, mu, logvar, B, L, free_bits, gscale, value,
                     gmu, glogvar);
  return (int)hipGetLastError();
}

extern "C" int vu_kl_free_bits(const float* mu, const float* logvar, int B, int L, float free_bits, float* value,
                               float* gmu, float* glogvar, void* stream) {
  return vu_kl_free_bits2(mu, logvar, B, L, free_bits, nullptr, value, gmu, glogvar, stream);
}

extern "C" int vu_sumsq(const float* x, int64_t n, double* out, double* workspace, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int nb = nblocks(n);
  hipLaunchKernelGGL(sumsq_stage1, dim3(nb), dim3(LBLK), 0, st, x, n, workspace);
  hipLaunchKernelGGL(sum_stage2, dim3(1), dim3(LBLK), 0, st, workspace, nb, out, 0);
  return (int)hipGetLastError();
}

extern "C" int vu_dice_score(const float* x, const float* t, int64_t n, float epsilon, float* score,
                             double* counts, double* workspace, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int nb = nblocks(n);
  unsigned long long* ws = reinterpret_cast<unsigned long long*>(workspace);
  hipLaunchKernelGGL(dice_score_stage1, dim3(nb), dim3(LBLK), 0, st, x, t, n, ws);
  hipLaunchKernelGGL(dice_score_stage2, dim3(1), dim3(64), 0, st, ws, nb, epsilon, score, counts);
  return (int)hipGetLastError();
}
