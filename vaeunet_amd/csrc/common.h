// Shared device helpers for the VAE-U-Net HIP kernels (gfx950 / CDNA4 only).
//
// Storage types: activations are NHWC ("channels_last"), either bf16 (speed
// mode, the autocast path of train.py:385) or fp32 (parity mode).  Every
// kernel is templated on the storage type T in {float, bf16_t}; arithmetic
// and all reductions are fp32 (partials combined in fp64 where counts reach
// millions of pixels).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

enum VuDType { VU_F32 = 0, VU_BF16 = 1 };

#define VU_DEV __device__ __forceinline__

VU_DEV float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
VU_DEV uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// Scalar load/store of one element as fp32.
template <typename T> VU_DEV float ld1(const T* p);
template <> VU_DEV float ld1<float>(const float* p) { return *p; }
template <> VU_DEV float ld1<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> VU_DEV void st1(T* p, float v);
template <> VU_DEV void st1<float>(float* p, float v) { *p = v; }
template <> VU_DEV void st1<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// Epilogue activation of the GEMM kernels (VuGemmFwd.relu): applied to
// accumulator + bias before the storage rounding (per element: the
// LDS-staged kernels).  The register-epilogue kernels instead clamp their
// rounded accumulators in one block behind a uniform branch (relu commutes
// with the rounding), so the training instantiations pay one scalar branch.
VU_DEV float epi_act(float v, int relu) { return relu ? fmaxf(v, 0.f) : v; }
template <int N>
VU_DEV void epi_relu(f32x4 (&a)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) a[i][r] = fmaxf(a[i][r], 0.f);
}

// Division by a divisor fixed for the whole launch (image width, pixels per
// image, ConvT output channels), for dividends n < 2^31: q = (umulhi(n, m) +
// n) >> l with l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1 (Granlund
// & Montgomery; exact for every n < 2^31).  Built once per thread (uniform
// arguments: scalar code); each division is then 3 VALU ops instead of the
// ~20 of a runtime 32-bit integer division.
struct FastDiv {
  uint32_t m, l, d;
  VU_DEV explicit FastDiv(uint32_t dd) : d(dd) {
    l = 0;
    while ((1u << l) < dd && l < 31) ++l;
    m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - dd)) / dd) + 1u;
  }
  VU_DEV uint32_t div(uint32_t n) const { return (__umulhi(n, m) + n) >> l; }
};

// Kahan-compensated acc += part (fp32 parity-mode GEMMs: the per-K-step MFMA
// partials summed with an error that does not grow with K).  c carries the
// negative of the low-order bits lost so far; the caller finishes with
// acc -= c.  (No fast-math in this library: the compiler keeps the order.)
VU_DEV void kahan_add(f32x4& acc, f32x4& c, const f32x4& part) {
  const f32x4 y = part - c;
  const f32x4 t = acc + y;
  c = (t - acc) - y;
  acc = t;
}

// border class of a row / column index (VuGemmFwd.zbias): 0 first, 2 last, 1 inside
VU_DEV int zb_class(int v, int L) { return v == 0 ? 0 : (v == L - 1 ? 2 : 1); }

// Round a float to the storage precision (identity for fp32).
template <typename T> VU_DEV float rnd(float v);
template <> VU_DEV float rnd<float>(float v) { return v; }
template <> VU_DEV float rnd<bf16_t>(float v) { return bf2f(f2bf(v)); }

// 8-element vector helpers (16 B for bf16, 32 B for fp32).
template <typename T> struct Vec8;
template <> struct Vec8<bf16_t> {
  u32x4 v;
  VU_DEV void load(const bf16_t* p) { v = *reinterpret_cast<const u32x4*>(p); }
  // streaming (last-use) load: non-temporal cache policy
  VU_DEV void load_nt(const bf16_t* p) { v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)); }
  VU_DEV void store(bf16_t* p) const { *reinterpret_cast<u32x4*>(p) = v; }
  VU_DEV float get(int i) const {
    uint32_t w = v[i >> 1];
    return __uint_as_float((i & 1) ? (w & 0xffff0000u) : (w << 16));
  }
  VU_DEV void set(int i, float f) {
    uint32_t h = f2bf(f);
    uint32_t w = v[i >> 1];
    v[i >> 1] = (i & 1) ? ((w & 0xffffu) | (h << 16)) : ((w & 0xffff0000u) | h);
  }
  VU_DEV void zero() { v = u32x4{0, 0, 0, 0}; }
};
template <> struct Vec8<float> {
  f32x4 a, b;
  VU_DEV void load(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  VU_DEV void load_nt(const float* p) {
    a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
  }
  VU_DEV void store(float* p) const {
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
  VU_DEV float get(int i) const { return i < 4 ? a[i & 3] : b[i & 3]; }
  VU_DEV void set(int i, float f) {
    if (i < 4) a[i & 3] = f; else b[i & 3] = f;
  }
  VU_DEV void zero() { a = f32x4{0, 0, 0, 0}; b = a; }
};

VU_DEV float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
VU_DEV double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap of a linear block id (cdna_hip_programming T1):
// consecutive logical ids land on the same XCD (blocks b, b+8 share one).
VU_DEV int xcd_remap(int bid, int nblk) {
  if (nblk < 16) return bid;
  int q = nblk >> 3, r = nblk & 7, xcd = bid & 7, pos = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

// Deterministic fp64 column sums of a partial matrix written by a stage-1
// reduction: element (row r, quantity k, column c) lives at
// part[r * row_stride + k * q_stride + c].  A 1024-thread block covers 32
// columns x 32 row lanes; a lane loads its rows COLSUM_U at a time from
// clamped addresses, unconditionally (a guarded or loop-carried load per row
// serialises the memory round trips: the stage-2 pass is latency-, not
// bandwidth-bound), then a fixed-shape LDS tree folds the 32 lanes.  Every
// thread of the block must call it; out[k] is valid for threads with lane 0
// (threadIdx.x < 32).  Summation order is fixed: results are reproducible.
constexpr int COLSUM_THREADS = 1024, COLSUM_U = 8;
template <int NQ>
VU_DEV void colsum32(const float* part, int rows, int64_t row_stride, int64_t q_stride, int col, bool valid,
                     double* out) {
  __shared__ double sh[NQ][32][32];
  const int cl = threadIdx.x & 31, q = threadIdx.x >> 5;
  const int cc = valid ? col : 0;
  double s[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) s[k] = 0.0;
  for (int r0 = 0; r0 < rows; r0 += 32 * COLSUM_U) {
    float v[COLSUM_U][NQ];
#pragma unroll
    for (int u = 0; u < COLSUM_U; ++u) {
      const int r = min(r0 + q + 32 * u, rows - 1);
#pragma unroll
      for (int k = 0; k < NQ; ++k) v[u][k] = part[(int64_t)r * row_stride + k * q_stride + cc];
    }
#pragma unroll
    for (int u = 0; u < COLSUM_U; ++u)
#pragma unroll
      for (int k = 0; k < NQ; ++k) s[k] += (valid && r0 + q + 32 * u < rows) ? (double)v[u][k] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) sh[k][q][cl] = s[k];
  __syncthreads();
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1) {
    if (q < w)
#pragma unroll
      for (int k = 0; k < NQ; ++k) sh[k][q][cl] += sh[k][q + w][cl];
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < NQ; ++k) out[k] = sh[k][0][cl];
}

// sum_{q < n} p[q * stride] accumulated from 0.f in the order q = 0, 1, ...
// (bit-identical to the plain loop) with 8 LDS reads in flight: the block-
// reduction tails of the streaming kernels read one term per LDS round trip
// as a loop-carried chain (round 6: up to 256 serial reads by one thread).
VU_DEV float lds_sum(const float* p, int n, int stride) {
  float s = 0.f;
  int q = 0;
  for (; q + 8 <= n; q += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(q + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; q < n; ++q) s += p[q * stride];
  return s;
}

#define VU_CHECK_LAUNCH() return (int)hipGetLastError()
