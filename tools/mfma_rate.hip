// MFMA issue-rate microbenchmark (gfx950): dense TFLOP/s of back-to-back
// independent MFMAs, one or two waves per SIMD, for the bf16 and the
// block-scaled e4m3 (f8f6f4) instructions the conv kernels use.  A tuning
// aid, not product code.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_rate tools/mfma_rate.hip && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int ITERS = 2048;

__global__ __launch_bounds__(256) void k_bf16_16(float* out, int seed) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(float)(threadIdx.x + i + seed); b[i] = (__bf16)(float)(i - seed); }
  f32x4 acc[8] = {};
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[k], 0, 0, 0);
  float s = 0;
  for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_bf16_32(float* out, int seed) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(float)(threadIdx.x + i + seed); b[i] = (__bf16)(float)(i - seed); }
  f32x16 acc[4] = {};
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[k], 0, 0, 0);
  float s = 0;
  for (int k = 0; k < 4; ++k) s += acc[k][0] + acc[k][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fp8_32(float* out, int seed) {
  i32x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = 0x38383838 + (int)threadIdx.x + seed; b[i] = 0x30303030 + i; }
  f32x16 acc[4] = {};
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[k], 0, 0, 0, 0, 0, 0);
  float s = 0;
  for (int k = 0; k < 4; ++k) s += acc[k][0] + acc[k][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fp8_16(float* out, int seed) {
  i32x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = 0x38383838 + (int)threadIdx.x + seed; b[i] = 0x30303030 + i; }
  f32x4 acc[8] = {};
  for (int it = 0; it < ITERS; ++it)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[k], 0, 0, 0, 0, 0, 0);
  float s = 0;
  for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
void run(const char* name, F kern, double flop_per_mfma, int mfma_per_iter, int blocks_per_cu) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int nb = cus * blocks_per_cu;
  float* out;
  hipMalloc(&out, (size_t)nb * 256 * sizeof(float));
  hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, 0, out, 1);
  hipDeviceSynchronize();
  hipEvent_t s, e;
  hipEventCreate(&s);
  hipEventCreate(&e);
  hipEventRecord(s);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(nb), dim3(256), 0, 0, out, r);
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms = 0;
  hipEventElapsedTime(&ms, s, e);
  const double flops = (double)nb * 4 /*waves*/ * ITERS * mfma_per_iter * flop_per_mfma * reps;
  printf("%-34s %d wave(s)/SIMD: %8.1f TFLOP/s\n", name, blocks_per_cu, flops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  for (int w = 1; w <= 2; ++w) {
    run("bf16 16x16x32", k_bf16_16, 2.0 * 16 * 16 * 32, 8, w);
    run("bf16 32x32x16", k_bf16_32, 2.0 * 32 * 32 * 16, 4, w);
    run("e4m3 scaled 32x32x64 (f8f6f4)", k_fp8_32, 2.0 * 32 * 32 * 64, 4, w);
    run("e4m3 scaled 16x16x128 (f8f6f4)", k_fp8_16, 2.0 * 16 * 16 * 128, 8, w);
  }
  return 0;
}
