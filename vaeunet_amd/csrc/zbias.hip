// The latent-broadcast shortcut of a DecoderBlock's conv1 (round 5;
// unet/unet_resnet.py:37-41, 92-99).
//
// conv1 contracts over the channel concat [x, skip, z_proj(z)]; the z_proj
// source is interpolate(z[..., None, None]) through a 1x1 conv + BatchNorm +
// ReLU -- a per-sample CONSTANT map c_n (latent.hip computes c_n on the
// sample vectors).  A 3x3 convolution of a constant map is, at output pixel
// (h, w), W_z c_n summed over the taps that read inside the image: one of 9
// vectors per sample, by the pixel's border class (corner, edge, interior).
// So the z channels leave conv1's K loop (and the 64-channel-padded map is
// never written nor read):
//
//   vu_zbias_fwd  table[n][cls][c] = sum over the taps valid for cls of
//                 S[n][c][tap],  S = sum_l W[c][cz0 + l][tap] c_n[l]
//                 -> VuGemmFwd.zbias of conv1's GEMM (added in its epilogue);
//   vu_zbias_bwd  the backward: with dy = conv1's pre-BN output gradient and
//                 R[n][c][tap] = the sum of dy over the output pixels whose tap
//                 reads inside the image (the total minus the excluded border
//                 row / column sums plus the corner they both excluded),
//                   dW[c][cz0 + l][tap] (+)= sum_n c_n[l] R[n][c][tap]
//                   dc[n][l]              = sum_c sum_tap W[c][cz0+l][tap] R[n][c][tap]
//                 -- dc is the pixel sum of d(map) the latent backward needs
//                 (vu_latent_bwd_sums produced it from the map gradient).
//                 Three launches: region partials per (sample, pixel chunk
//                 of ~64 KB of dy); per (sample, 64 statistics) the sum of those
//                 partials; per 32 output channels, R from the sums and the
//                 corner pixels, the z columns of dW and the dc partial of those
//                 channels into split `chunk` of the consumer's part array
//                 (vu_latent_bwd sums the splits).
// Every sum runs in a fixed order (reproducible run to run).
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int ZB_MAXJ = 8;
constexpr int ZB_SPLITS = 32;  // == latent.hip LAT_SPLITS: the part array is [N][32][L]
constexpr int ZB_CHUNK_ELEMS = 32768;  // dy elements per region-pass block (64 KB in bf16)
constexpr int ZB_CW = 32;      // output channels per finish block
constexpr int ZB_NS = 5;       // region partials: total, col 0, col W-1, row 0, row H-1
constexpr int ZB_MAXN = 64;

struct ZbJobs {
  VuZbJob j[ZB_MAXJ];
};

VU_DEV int find_job(const ZbJobs& jobs, int njobs) {
  int j = 0;
  while (j + 1 < njobs && (int64_t)blockIdx.x >= jobs.j[j + 1].block0) ++j;
  return j;
}

// tap k (0..2) of a row / column is inside the image for border class cr
VU_DEV bool tap_in(int cr, int k) { return !((cr == 0 && k == 0) || (cr == 2 && k == 2)); }

// pixels per region-pass block: ~ZB_CHUNK_ELEMS elements of dy whatever co is
// (a fixed pixel count left the wide-channel jobs with a handful of 1 MB blocks)
__host__ __device__ inline int pix_chunk(int co) { return co >= ZB_CHUNK_ELEMS / 16 ? 16 : ZB_CHUNK_ELEMS / co; }
__host__ __device__ inline int n_chunks(int co, int H, int W) { return (H * W + pix_chunk(co) - 1) / pix_chunk(co); }

// dst[0, n) = src(e) staged into LDS by the block, 8 independent loads in
// flight per thread (a load -> store loop waits out one latency per element)
template <typename F>
VU_DEV void stage(float* dst, int n, F src) {
  for (int b = threadIdx.x; b < n; b += 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = b + u * 256;
      v[u] = src(e < n ? e : n - 1);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (b + u * 256 < n) dst[b + u * 256] = v[u];
  }
}

// the block's z weights [ZB_CW][L][9] (zero past co)
VU_DEV void stage_w(float* Wl, const VuZbJob& J, int c0, int cw) {
  const int L = J.L;
  stage(Wl, ZB_CW * L * 9, [&](int e) {
    const int c = e / (L * 9), rem = e - c * (L * 9), l = rem / 9, t = rem - l * 9;
    const int cc = c < cw ? c0 + c : c0;
    const float v = J.w[(int64_t)cc * J.ws_co + (int64_t)(J.cz0 + l) * J.ws_ci + (t / 3) * J.ws_ky + (t % 3) * J.ws_kx];
    return c < cw ? v : 0.f;
  });
}

// ---- forward: the bias tables -------------------------------------------
// one block per (job, 32 output channels): that chunk's z weights [32][L][9]
// and the vectors [N][L] staged in LDS (every global load issued up front),
// then thread (n, c) forms its 9 tap sums and the 9 border-class rows
__global__ __launch_bounds__(256) void zbias_fwd_kernel(const ZbJobs jobs, int njobs, int N) {
  extern __shared__ float zsm[];
  const VuZbJob& J = jobs.j[find_job(jobs, njobs)];
  const int chunk = (int)((int64_t)blockIdx.x - J.block0);
  const int c0 = chunk * ZB_CW, cw = J.co - c0 < ZB_CW ? J.co - c0 : ZB_CW;
  const int L = J.L, tid = threadIdx.x;
  float* Wl = zsm;                 // [ZB_CW][L][9]
  float* A = Wl + ZB_CW * L * 9;   // [N][L]
  stage(A, N * L, [&](int e) { return J.act[e]; });
  stage_w(Wl, J, c0, cw);
  __syncthreads();
  for (int e = tid; e < N * cw; e += 256) {
    const int n = e / cw, c = e - n * cw;
    float S[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) S[t] = 0.f;
    const float* wr = Wl + c * L * 9;
    for (int l = 0; l < L; ++l) {
      const float av = A[n * L + l];
#pragma unroll
      for (int t = 0; t < 9; ++t) S[t] += wr[l * 9 + t] * av;
    }
    const float sc = J.row_scale ? J.row_scale[c0 + c] : 1.f;
#pragma unroll
    for (int cr = 0; cr < 3; ++cr)
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        float t = 0.f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
            if (tap_in(cr, ky) && tap_in(cc, kx)) t += S[ky * 3 + kx];
        J.table[((int64_t)n * 9 + cr * 3 + cc) * J.co + c0 + c] = t * sc;
      }
  }
}

// ---- backward 1: region partials per (sample, pixel chunk) ---------------
// rs[((n * nch + chunk) * ZB_NS + k) * co + c], nch = n_chunks(co, H, W); a
// chunk is pix_chunk(co) consecutive pixels of one sample, 8 loads in flight
// per thread
template <typename T>
__global__ __launch_bounds__(256) void zbias_rs_kernel(const ZbJobs jobs, int njobs, int N) {
  __shared__ float sh[ZB_NS * 2048];
  const VuZbJob& J = jobs.j[find_job(jobs, njobs)];
  const int H = J.H, W = J.W, C = J.co;
  const int HW = H * W, pch = pix_chunk(C), nch = (HW + pch - 1) / pch;
  const int lb = (int)((int64_t)blockIdx.x - J.block0);
  const int n = lb / nch, chunk = lb - (lb / nch) * nch;
  const int V = C >> 3, slots = 256 / V;
  const int tid = threadIdx.x, cv = tid % V, slot = tid / V;
  const int p0 = chunk * pch, p1 = min(HW, p0 + pch);
  constexpr int U = 8;
  float s[ZB_NS][8];
#pragma unroll
  for (int k = 0; k < ZB_NS; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) s[k][e] = 0.f;
  if (slot < slots) {
    const T* base = reinterpret_cast<const T*>(J.dy) + (int64_t)n * HW * J.dy_stride + cv * 8;
    const FastDiv dw((uint32_t)W);
    for (int p = p0 + slot; p < p1; p += U * slots) {
      Vec8<T> v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // clamped loads, summed only when inside
        const int q = p + u * slots;
        v[u].load(base + (int64_t)(q < p1 ? q : p1 - 1) * J.dy_stride);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = p + u * slots;
        if (q >= p1) break;
        const int y = (int)dw.div((uint32_t)q), x = q - y * W;
        const float m1 = x == 0 ? 1.f : 0.f, m2 = x == W - 1 ? 1.f : 0.f;
        const float m3 = y == 0 ? 1.f : 0.f, m4 = y == H - 1 ? 1.f : 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[u].get(e);
          s[0][e] += d;
          s[1][e] = fmaf(m1, d, s[1][e]);
          s[2][e] = fmaf(m2, d, s[2][e]);
          s[3][e] = fmaf(m3, d, s[3][e]);
          s[4][e] = fmaf(m4, d, s[4][e]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < ZB_NS; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) sh[(k * slots + slot) * C + cv * 8 + e] = s[k][e];
  }
  __syncthreads();
  for (int q = tid; q < ZB_NS * C; q += 256) {
    const int k = q / C, c = q - (q / C) * C;
    float t = 0.f;
    for (int r = 0; r < slots; ++r) t += sh[(k * slots + r) * C + c];
    J.rs[(((int64_t)n * nch + chunk) * ZB_NS + k) * C + c] = t;
  }
}

// ---- backward 2: per (sample, 64 statistics): the sum of the chunk
// partials -> S[n][k][c] (after the partials in rs); 4 lanes per statistic,
// 8 loads in flight each, then a fixed-order LDS reduction
__global__ __launch_bounds__(256) void zbias_sum_kernel(const ZbJobs jobs, int njobs, int N) {
  __shared__ float red[4][64];
  const VuZbJob& J = jobs.j[find_job(jobs, njobs)];
  const int C = J.co, nv = ZB_NS * C, ngrp = (nv + 63) / 64;
  const int lb = (int)((int64_t)blockIdx.x - J.block0);
  const int n = lb / ngrp, grp = lb - (lb / ngrp) * ngrp;
  const int nch = n_chunks(C, J.H, J.W);
  const int v = threadIdx.x & 63, lane = threadIdx.x >> 6, q = grp * 64 + v;
  float t = 0.f;
  if (q < nv) {
    const float* rp = J.rs + (int64_t)n * nch * nv + q;
    for (int b0 = lane; b0 < nch; b0 += 4 * 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int b = b0 + u * 4;
        x[u] = rp[(int64_t)(b < nch ? b : lane) * nv];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b0 + u * 4 < nch) t += x[u];
    }
  }
  red[lane][v] = t;
  __syncthreads();
  if (lane == 0 && q < nv)
    J.rs[(int64_t)N * nch * nv + (int64_t)n * nv + q] = ((red[0][v] + red[1][v]) + red[2][v]) + red[3][v];
}

// ---- backward 3: per 32 output channels: R[n][c][tap] from the sums and the
// four corner pixels of dy, then the z columns of dW and the dc partial of
// these channels (into split `chunk` of part; chunk 0 also zeroes the splits
// no chunk uses), from R, the z weights and the vectors in LDS
//   dW[c0 + c][cz0 + l][tap] (+)= sum_n act[n][l] R[n][c][tap]
//   dc_chunk[n][l]              = sum_{c, tap} W[c0 + c][cz0 + l][tap] R[n][c][tap]
template <typename T>
__global__ __launch_bounds__(256) void zbias_dw_kernel(const ZbJobs jobs, int njobs, int N) {
  extern __shared__ float zsm[];
  const VuZbJob& J = jobs.j[find_job(jobs, njobs)];
  const int chunk = (int)((int64_t)blockIdx.x - J.block0);
  const int c0 = chunk * ZB_CW, cw = J.co - c0 < ZB_CW ? J.co - c0 : ZB_CW;
  const int L = J.L, C = J.co, H = J.H, W = J.W, tid = threadIdx.x;
  const int nch = n_chunks(C, H, W);
  const int nchunks = (C + ZB_CW - 1) / ZB_CW;
  float* R = zsm;                  // [N][ZB_CW][9]
  float* A = R + N * ZB_CW * 9;    // [N][L]
  float* Wl = A + N * L;           // [ZB_CW][L][9]
  const float* S = J.rs + (int64_t)N * nch * ZB_NS * C;
  const T* dy = reinterpret_cast<const T*>(J.dy);
  stage(A, N * L, [&](int e) { return J.act[e]; });
  stage_w(Wl, J, c0, cw);
  for (int e = tid; e < N * ZB_CW; e += 256) {
    const int n = e / ZB_CW, c = e - n * ZB_CW;
    const int cc = c0 + (c < cw ? c : 0);
    const float* sp = S + (int64_t)n * ZB_NS * C + cc;
    const T* dn = dy + (int64_t)n * H * W * J.dy_stride + cc;
    const float tot = sp[0], col0 = sp[C], colL = sp[2 * C], row0 = sp[3 * C], rowL = sp[4 * C];
    const float k00 = ld1<T>(dn), k0L = ld1<T>(dn + (int64_t)(W - 1) * J.dy_stride);
    const float kL0 = ld1<T>(dn + (int64_t)(H - 1) * W * J.dy_stride);
    const float kLL = ld1<T>(dn + ((int64_t)(H - 1) * W + W - 1) * J.dy_stride);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float r = tot;
        if (ky == 0) r -= row0;
        if (ky == 2) r -= rowL;
        if (kx == 0) r -= col0;
        if (kx == 2) r -= colL;
        if (ky == 0 && kx == 0) r += k00;
        if (ky == 0 && kx == 2) r += k0L;
        if (ky == 2 && kx == 0) r += kL0;
        if (ky == 2 && kx == 2) r += kLL;
        R[e * 9 + ky * 3 + kx] = c < cw ? r : 0.f;
      }
  }
  __syncthreads();
  for (int e = tid; J.dw && e < cw * L; e += 256) {
    const int c = e / L, l = e - (e / L) * L;
    float s[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) s[t] = 0.f;
    for (int n = 0; n < N; ++n) {
      const float a = A[n * L + l];
#pragma unroll
      for (int t = 0; t < 9; ++t) s[t] += a * R[(n * ZB_CW + c) * 9 + t];
    }
    float* d = J.dw + (int64_t)(c0 + c) * J.ws_co + (int64_t)(J.cz0 + l) * J.ws_ci;
    float old[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) old[t] = J.grad_acc ? d[(t / 3) * J.ws_ky + (t % 3) * J.ws_kx] : 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) d[(t / 3) * J.ws_ky + (t % 3) * J.ws_kx] = J.grad_acc ? old[t] + s[t] : s[t];
  }
  for (int e = tid; e < N * L; e += 256) {
    const int n = e / L, l = e - (e / L) * L;
    float s = 0.f;
    for (int c = 0; c < cw; ++c) {
      const float* w = Wl + (c * L + l) * 9;
      const float* r = R + (n * ZB_CW + c) * 9;
#pragma unroll
      for (int t = 0; t < 9; ++t) s += w[t] * r[t];
    }
    J.part[((int64_t)n * ZB_SPLITS + chunk) * L + l] = s;
    if (chunk == 0)
      for (int sp = nchunks; sp < ZB_SPLITS; ++sp) J.part[((int64_t)n * ZB_SPLITS + sp) * L + l] = 0.f;
  }
}

#define DISPATCH_T(dtype, ...) \
  if ((dtype) == VU_BF16) { using T = bf16_t; __VA_ARGS__; } else { using T = float; __VA_ARGS__; }

size_t fwd_lds_bytes(int N, int L) { return (size_t)(ZB_CW * L * 9 + N * L) * sizeof(float); }
size_t dw_lds_bytes(int N, int L) { return (size_t)(N * ZB_CW * 9 + N * L + ZB_CW * L * 9) * sizeof(float); }

int pack(const VuZbJob* jobs, int njobs, ZbJobs& J) {
  if (njobs < 1 || njobs > ZB_MAXJ) return (int)hipErrorInvalidValue;
  for (int j = 0; j < njobs; ++j) J.j[j] = jobs[j];
  return 0;
}

}  // namespace

extern "C" int vu_zbias_supported(int N, int L, int co) {
  if (N < 1 || N > ZB_MAXN || L < 1 || L > 64 || co < 8 || co % 8 || co / 8 > 256) return 0;
  const size_t cap = 160 * 1024;
  if ((co + ZB_CW - 1) / ZB_CW > ZB_SPLITS) return 0;  // dc partials: one split per 32 channels
  return fwd_lds_bytes(N, L) <= cap && dw_lds_bytes(N, L) <= cap ? 1 : 0;
}

// region partials [N][nch][5][co], then their sums [N][5][co]
extern "C" int64_t vu_zbias_rs_floats(int N, int co, int H, int W) {
  if (co < 8) return 0;
  return (int64_t)N * ((int64_t)n_chunks(co, H, W) + 1) * ZB_NS * co;
}

extern "C" int vu_zbias_fwd(const VuZbJob* jobs, int njobs, int N, void* stream) {
  ZbJobs J;
  if (int rc = pack(jobs, njobs, J)) return rc;
  int64_t blocks = 0;
  int maxL = 1;
  for (int j = 0; j < njobs; ++j) {
    VuZbJob& q = J.j[j];
    if (!vu_zbias_supported(N, q.L, q.co) || !q.w || !q.act || !q.table) return (int)hipErrorInvalidValue;
    q.block0 = blocks;
    blocks += (q.co + ZB_CW - 1) / ZB_CW;
    maxL = q.L > maxL ? q.L : maxL;
  }
  hipLaunchKernelGGL(zbias_fwd_kernel, dim3((unsigned)blocks), dim3(256), fwd_lds_bytes(N, maxL),
                     (hipStream_t)stream, J, njobs, N);
  return (int)hipGetLastError();
}

extern "C" int vu_zbias_bwd(const VuZbJob* jobs, int njobs, int N, int dtype, void* stream) {
  ZbJobs J;
  if (int rc = pack(jobs, njobs, J)) return rc;
  int64_t rblocks = 0;
  int maxL = 1;
  for (int j = 0; j < njobs; ++j) {
    VuZbJob& q = J.j[j];
    if (!vu_zbias_supported(N, q.L, q.co) || !q.w || !q.act || !q.dy || !q.rs || !q.part ||
        q.H < 2 || q.W < 2 || q.dy_stride % 8)
      return (int)hipErrorInvalidValue;
    if ((int64_t)q.H * q.W > (1 << 30) / q.co) return (int)hipErrorInvalidValue;
    q.block0 = rblocks;
    rblocks += (int64_t)N * n_chunks(q.co, q.H, q.W);
    maxL = q.L > maxL ? q.L : maxL;
  }
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((zbias_rs_kernel<T>), dim3((unsigned)rblocks), dim3(256), 0, st, J, njobs, N);
  })
  int64_t sblocks = 0;
  for (int j = 0; j < njobs; ++j) {
    J.j[j].block0 = sblocks;
    sblocks += (int64_t)N * ((ZB_NS * J.j[j].co + 63) / 64);
  }
  hipLaunchKernelGGL(zbias_sum_kernel, dim3((unsigned)sblocks), dim3(256), 0, st, J, njobs, N);
  int64_t dblocks = 0;
  for (int j = 0; j < njobs; ++j) {
    J.j[j].block0 = dblocks;
    dblocks += (J.j[j].co + ZB_CW - 1) / ZB_CW;
  }
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((zbias_dw_kernel<T>), dim3((unsigned)dblocks), dim3(256), dw_lds_bytes(N, maxL), st, J,
                       njobs, N);
  })
  return (int)hipGetLastError();
}
