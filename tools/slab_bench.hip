// Microbenchmark: variants of the split-K slab reduction (sum over `splits`
// fp32 slabs of `tot` values) on a freshly written slab.
//   hipcc --offload-arch=gfx950 -O3 -o build/slab_bench tools/slab_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void fill(float* s, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s[i] = v + (float)(i & 7);
}

// V0: 64 outputs x 4 split lanes, scalar
__global__ void v0(const float* slab, int splits, int64_t tot, float* out) {
  __shared__ float sh[4][64];
  const int l = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t idx = (int64_t)blockIdx.x * 64 + l;
  float a[4] = {0, 0, 0, 0};
  if (idx < tot) {
    int k = q;
    for (; k + 12 < splits; k += 16)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += slab[(int64_t)(k + 4 * u) * tot + idx];
    for (; k < splits; k += 4) a[0] += slab[(int64_t)k * tot + idx];
  }
  sh[q][l] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (q == 0 && idx < tot) out[idx] = (sh[0][l] + sh[1][l]) + (sh[2][l] + sh[3][l]);
}

// V1: 16 quads x 16 split lanes, float4
__global__ void v1(const float* slab, int splits, int64_t tot, float* out) {
  __shared__ f32x4 sh[16][16];
  const int ql = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int64_t idx = (int64_t)blockIdx.x * 64 + ql * 4;
  f32x4 a[4];
  for (int u = 0; u < 4; ++u) a[u] = f32x4{0, 0, 0, 0};
  if (idx < tot) {
    int k = sl;
    for (; k + 48 < splits; k += 64)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += *(const f32x4*)(slab + (int64_t)(k + 16 * u) * tot + idx);
    for (; k < splits; k += 16) a[0] += *(const f32x4*)(slab + (int64_t)k * tot + idx);
  }
  sh[sl][ql] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (sl == 0 && idx < tot) {
    f32x4 s = sh[0][ql];
    for (int q = 1; q < 16; ++q) s += sh[q][ql];
    *(f32x4*)(out + idx) = s;
  }
}

// V2<QW, SL, U>: QW quads (4*QW outputs) x SL split lanes per block
// (QW*SL = 256), U float4 loads in flight per lane
template <int QW, int SL, int U>
__global__ void v2(const float* slab, int splits, int64_t tot, float* out) {
  __shared__ f32x4 sh[SL][QW];
  const int ql = threadIdx.x % QW, sl = threadIdx.x / QW;
  const int64_t idx = (int64_t)blockIdx.x * (4 * QW) + ql * 4;
  f32x4 a[U];
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = f32x4{0, 0, 0, 0};
  if (idx < tot) {
    int k = sl;
    for (; k + SL * (U - 1) < splits; k += SL * U)
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] += *(const f32x4*)(slab + (int64_t)(k + SL * u) * tot + idx);
    for (; k < splits; k += SL) a[0] += *(const f32x4*)(slab + (int64_t)k * tot + idx);
  }
#pragma unroll
  for (int u = 1; u < U; ++u) a[0] += a[u];
  sh[sl][ql] = a[0];
  __syncthreads();
  if (sl == 0 && idx < tot) {
    f32x4 s = sh[0][ql];
    for (int q = 1; q < SL; ++q) s += sh[q][ql];
    *(f32x4*)(out + idx) = s;
  }
}

// V3: contiguous-split mapping: lane sl handles splits [sl*per, (sl+1)*per)
template <int QW, int SL, int U>
__global__ void v3(const float* slab, int splits, int64_t tot, float* out) {
  __shared__ f32x4 sh[SL][QW];
  const int ql = threadIdx.x % QW, sl = threadIdx.x / QW;
  const int64_t idx = (int64_t)blockIdx.x * (4 * QW) + ql * 4;
  const int per = (splits + SL - 1) / SL;
  const int kb = sl * per, ke = min(splits, kb + per);
  f32x4 a[U];
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = f32x4{0, 0, 0, 0};
  if (idx < tot) {
    int k = kb;
    for (; k + U <= ke; k += U)
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] += *(const f32x4*)(slab + (int64_t)(k + u) * tot + idx);
    for (; k < ke; ++k) a[0] += *(const f32x4*)(slab + (int64_t)k * tot + idx);
  }
#pragma unroll
  for (int u = 1; u < U; ++u) a[0] += a[u];
  sh[sl][ql] = a[0];
  __syncthreads();
  if (sl == 0 && idx < tot) {
    f32x4 s = sh[0][ql];
    for (int q = 1; q < SL; ++q) s += sh[q][ql];
    *(f32x4*)(out + idx) = s;
  }
}

typedef void (*Kern)(const float*, int, int64_t, float*);

int main() {
  struct Case { int64_t tot; int splits; } cases[] = {
      {64 * 576, 256}, {128 * 1152, 64}, {64 * 1152, 128}, {256 * 2304, 16}, {64 * 64, 256}, {128 * 256, 128}};
  struct V { const char* name; Kern k; int per_block; } vs[] = {
      {"v0 s64x4", v0, 64},
      {"v1 q16x16 U4", v1, 64},
      {"v2 q64x4 U4", v2<64, 4, 4>, 256},
      {"v2 q64x4 U8", v2<64, 4, 8>, 256},
      {"v2 q32x8 U4", v2<32, 8, 4>, 128},
      {"v2 q32x8 U8", v2<32, 8, 8>, 128},
      {"v2 q16x16 U8", v2<16, 16, 8>, 64},
      {"v3 q64x4 U8", v3<64, 4, 8>, 256},
      {"v3 q32x8 U8", v3<32, 8, 8>, 128},
      {"v3 q16x16 U8", v3<16, 16, 8>, 64},
      {"v3 q16x16 U4", v3<16, 16, 4>, 64},
  };
  float *slab, *out, *big;
  hipMalloc(&slab, (size_t)400 << 20);
  hipMalloc(&big, (size_t)512 << 20);
  hipMalloc(&out, (size_t)64 << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& c : cases) {
    int64_t n = c.tot * c.splits;
    printf("tot %lld splits %d  (%.1f MB)\n", (long long)c.tot, c.splits, n * 4 / 1e6);
    std::vector<float> ref;
    for (auto& v : vs) {
      float best = 1e9, sum = 0;
      const int R = 20;
      for (int r = 0; r < R + 2; ++r) {
        fill<<<1024, 256>>>(big, (int64_t)128 << 20, 0.f);   // evict
        fill<<<2048, 256>>>(slab, n, 1.f);                   // freshly written slab
        hipEventRecord(e0);
        hipLaunchKernelGGL(v.k, dim3((unsigned)((c.tot + v.per_block - 1) / v.per_block)), dim3(256), 0, 0,
                           slab, c.splits, c.tot, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2) { sum += ms; if (ms < best) best = ms; }
      }
      std::vector<float> h(c.tot);
      hipMemcpy(h.data(), out, c.tot * 4, hipMemcpyDeviceToHost);
      double err = 0;
      if (ref.empty()) ref = h;
      for (int64_t i = 0; i < c.tot; ++i) err = std::max(err, (double)std::abs(h[i] - ref[i]));
      printf("  %-14s avg %7.2f us  min %7.2f us  %6.2f TB/s  err %g\n", v.name, sum / R * 1e3, best * 1e3,
             n * 4 / (sum / R * 1e-3) / 1e12, err);
    }
  }
  return 0;
}
