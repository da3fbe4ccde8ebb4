// Patch-cache producer statistics: for every
// stride-spaced P x P window of one scaled image, the two integer counts the
// reference's slicer decides on (utils/data_loading.py:370-397):
//   black  = #pixels whose channel mean is < 0.1    (is_valid_patch, :287-300)
//   lesion = #mask pixels > 0.5                      (has_lesion, :381)
// The host turns them into keep / has_lesion exactly as the reference does
// (black / P^2 <= threshold; lesion > 0).  Integer counts: bit-exact and
// independent of the launch geometry.
//
// Layout: image [C][H][W] fp32 (the reference's CHW float tensor, values in
// [0,1]), mask [H][W] fp32.  One workgroup per window; the P x P window is
// walked row by row with consecutive lanes on consecutive pixels (coalesced).
// The channel mean is formed as torch's CPU mean over dim 0 does: a
// left-to-right fp32 sum, then one correctly rounded division by C.
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int PS_THREADS = 256;

__global__ void __launch_bounds__(PS_THREADS) patch_stats_kernel(const float* __restrict__ img, int C, int H, int W,
                                                                 const float* __restrict__ mask, int P, int stride,
                                                                 int nx, int* __restrict__ black,
                                                                 int* __restrict__ lesion) {
  const int win = blockIdx.x;
  const int y0 = (win / nx) * stride, x0 = (win % nx) * stride;
  const int64_t plane = (int64_t)H * W;
  const float fc = (float)C;
  int nb = 0, nl = 0;
  for (int r = 0; r < P; ++r) {
    const int64_t row = (int64_t)(y0 + r) * W + x0;
    for (int c0 = threadIdx.x; c0 < P; c0 += PS_THREADS) {
      const int64_t o = row + c0;
      float s = img[o];
      for (int k = 1; k < C; ++k) s = s + img[k * plane + o];
      nb += (s / fc < 0.1f) ? 1 : 0;
      nl += (mask[o] > 0.5f) ? 1 : 0;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nb += __shfl_xor(nb, o, 64);
    nl += __shfl_xor(nl, o, 64);
  }
  __shared__ int sb[PS_THREADS / 64], sl[PS_THREADS / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sb[wave] = nb;
    sl[wave] = nl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int tb = 0, tl = 0;
    for (int w = 0; w < PS_THREADS / 64; ++w) {
      tb += sb[w];
      tl += sl[w];
    }
    black[win] = tb;
    lesion[win] = tl;
  }
}

}  // namespace

extern "C" int vu_patch_stats(const float* img, int C, int H, int W, const float* mask, int P, int stride, int ny,
                              int nx, int* black, int* lesion, void* stream) {
  if (C < 1 || P < 1 || stride < 1 || ny < 0 || nx < 0) return (int)hipErrorInvalidValue;
  if (ny == 0 || nx == 0) return 0;
  // every window must lie inside the image
  if ((int64_t)(ny - 1) * stride + P > H || (int64_t)(nx - 1) * stride + P > W) return (int)hipErrorInvalidValue;
  if ((int64_t)ny * nx > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(patch_stats_kernel, dim3((unsigned)(ny * nx)), dim3(PS_THREADS), 0, (hipStream_t)stream, img, C,
                     H, W, mask, P, stride, nx, black, lesion);
  return (int)hipGetLastError();
}
