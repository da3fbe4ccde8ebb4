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

// the block's z weights, Wl[(l * 9 + tap) * ZB_WP + c] (zero past co): channel
// fastest and padded, so lanes over channels (forward) and over l (dc) read
// distinct banks -- a [c][l][tap] layout put the 32 channels of a wave at a
// 288-float stride, 2 banks, 16-way conflicts on every read
constexpr int ZB_WP = ZB_CW + 1;
// every load is issued before the first LDS write: 16-byte loads when the
// weight's z part is made of aligned contiguous runs -- one round trip at
// L = 32 -- else 16 scalar loads per batch.  Two run layouts:
//   1: contiguous [co][ci][3][3]: per channel, (l, tap) = L * 9 floats;
//   2: channels_last [co][3][3][ci] (the model after .to(channels_last)):
//      per (channel, tap), l = L floats
constexpr int ZB_WU = 12;
VU_DEV int w_runs16(const VuZbJob& J) {
  if (((uintptr_t)J.w & 15) || (J.L & 3) || (J.ws_co & 3)) return 0;
  if (J.ws_kx == 1 && J.ws_ky == 3 && J.ws_ci == 9 && ((J.cz0 * 9) & 3) == 0) return 1;
  if (J.ws_ci == 1 && (J.ws_kx & 3) == 0 && (J.ws_ky & 3) == 0 && (J.cz0 & 3) == 0) return 2;
  return 0;
}
struct WStage {
  f32x4 v[ZB_WU];
};
// float4 e of the block's weights: channel c and its first (l, tap) index pair
VU_DEV void w_run_pos(const VuZbJob& J, int mode, int e, int& c, int& l, int& t, int64_t& off) {
  const int L = J.L, r4 = L * 9 / 4;
  c = e / r4;
  const int q = e - c * r4;
  if (mode == 1) {   // q-th float4 of the (l, tap) row
    l = q * 4 / 9;
    t = q * 4 - l * 9;
    off = (int64_t)J.cz0 * 9 + q * 4;
  } else {           // tap q / (L / 4), l from 4 * (q % (L / 4))
    const int l4 = L / 4;
    t = q / l4;
    l = (q - t * l4) * 4;
    off = (int64_t)(t / 3) * J.ws_ky + (t % 3) * J.ws_kx + J.cz0 + l;
  }
}
VU_DEV void stage_w_load(WStage& S, const VuZbJob& J, int mode, int c0, int cw, int b) {
  const int n4 = ZB_CW * J.L * 9 / 4;
#pragma unroll
  for (int u = 0; u < ZB_WU; ++u) {
    const int e = b + u * 256 < n4 ? b + u * 256 : n4 - 1;
    int c, l, t;
    int64_t off;
    w_run_pos(J, mode, e, c, l, t, off);
    const int cc = c < cw ? c0 + c : c0;
    S.v[u] = *reinterpret_cast<const f32x4*>(J.w + (int64_t)cc * J.ws_co + off);
  }
}
VU_DEV void stage_w_store(float* Wl, const WStage& S, const VuZbJob& J, int mode, int cw, int b) {
  const int n4 = ZB_CW * J.L * 9 / 4;
#pragma unroll
  for (int u = 0; u < ZB_WU; ++u) {
    const int e = b + u * 256;
    if (e < n4) {
      int c, l, t;
      int64_t off;
      w_run_pos(J, mode, e, c, l, t, off);
      if (mode == 1) {   // (l, tap) index rem = l * 9 + t, consecutive
        const int rem = l * 9 + t;
#pragma unroll
        for (int k = 0; k < 4; ++k) Wl[(rem + k) * ZB_WP + c] = c < cw ? S.v[u][k] : 0.f;
      } else {           // l .. l + 3 at tap t
#pragma unroll
        for (int k = 0; k < 4; ++k) Wl[((l + k) * 9 + t) * ZB_WP + c] = c < cw ? S.v[u][k] : 0.f;
      }
    }
  }
}
VU_DEV void stage_w_slow(float* Wl, const VuZbJob& J, int c0, int cw) {
  const int L = J.L, n = ZB_CW * L * 9;
  for (int b = threadIdx.x; b < n; b += 256 * 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {   // e = (c, l, tap)
      const int e = b + u * 256 < n ? b + u * 256 : n - 1;
      const int c = e / (L * 9), rem = e - c * (L * 9), l = rem / 9, t = rem - l * 9;
      const int cc = c < cw ? c0 + c : c0;
      v[u] = J.w[(int64_t)cc * J.ws_co + (int64_t)(J.cz0 + l) * J.ws_ci + (t / 3) * J.ws_ky + (t % 3) * J.ws_kx];
      v[u] = c < cw ? v[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = b + u * 256;
      if (e < n) {
        const int c = e / (L * 9), rem = e - c * (L * 9);
        Wl[rem * ZB_WP + c] = v[u];
      }
    }
  }
}
// `pre` runs between the first batch's loads and its LDS writes (the caller's
// own loads then share the round trip)
template <typename F>
VU_DEV void stage_w(float* Wl, const VuZbJob& J, int c0, int cw, F pre) {
  const int mode = w_runs16(J);
  if (!mode) {
    pre();
    stage_w_slow(Wl, J, c0, cw);
    return;
  }
  const int n4 = ZB_CW * J.L * 9 / 4;
  WStage S;
  stage_w_load(S, J, mode, c0, cw, threadIdx.x);
  pre();
  stage_w_store(Wl, S, J, mode, cw, threadIdx.x);
  for (int b = threadIdx.x + 256 * ZB_WU; b < n4; b += 256 * ZB_WU) {
    stage_w_load(S, J, mode, c0, cw, b);
    stage_w_store(Wl, S, J, mode, cw, b);
  }
}

// ---- forward: the bias tables -------------------------------------------
// one block per (job, 32 output channels): that chunk's z weights [32][L][9]
// and the vectors [N][L] staged in LDS (every global load issued up front),
// then thread (n, c) forms its 9 tap sums and the 9 border-class rows
__global__ __launch_bounds__(256) void zbias_fwd_kernel(const ZbJobs jobs, int njobs, int N, int dbg) {
  extern __shared__ float zsm[];
  const VuZbJob& J = jobs.j[find_job(jobs, njobs)];
  const int chunk = (int)((int64_t)blockIdx.x - J.block0);
  const int c0 = chunk * ZB_CW, cw = J.co - c0 < ZB_CW ? J.co - c0 : ZB_CW;
  const int L = J.L, tid = threadIdx.x;
  float* Wl = zsm;                 // [L * 9][ZB_WP]
  float* A = Wl + ZB_WP * L * 9;   // [N][L]
  if (!(dbg & 1)) stage_w(Wl, J, c0, cw, [&] { stage(A, N * L, [&](int e) { return J.act[e]; }); });
  __syncthreads();
  for (int e = tid; e < N * cw && !(dbg & 2); e += 256) {
    const int n = e / cw, c = e - n * cw;
    float S[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) S[t] = 0.f;
    const float* wr = Wl + c;
    for (int l = 0; l < L; ++l) {
      const float av = A[n * L + l];
#pragma unroll
      for (int t = 0; t < 9; ++t) S[t] += wr[(l * 9 + t) * ZB_WP] * av;
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
  __shared__ __attribute__((aligned(16))) float sh[ZB_NS * 2048];
  const VuZbJob& J = jobs.j[find_job(jobs, njobs)];
  if (J.rs_ready) return;   // partials already written by vu_bn_bwd_apply_zrs (block-uniform)
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
#pragma unroll
        for (int e = 0; e < 8; ++e) s[0][e] += v[u].get(e);
        if (x == 0 || x == W - 1 || y == 0 || y == H - 1) {   // border pixels only (2/W of a row band)
          const float m1 = x == 0 ? 1.f : 0.f, m2 = x == W - 1 ? 1.f : 0.f;
          const float m3 = y == 0 ? 1.f : 0.f, m4 = y == H - 1 ? 1.f : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = v[u].get(e);
            s[1][e] = fmaf(m1, d, s[1][e]);
            s[2][e] = fmaf(m2, d, s[2][e]);
            s[3][e] = fmaf(m3, d, s[3][e]);
            s[4][e] = fmaf(m4, d, s[4][e]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < ZB_NS; ++k) {
      f32x4* d = reinterpret_cast<f32x4*>(sh + (k * slots + slot) * C + cv * 8);
      d[0] = f32x4{s[k][0], s[k][1], s[k][2], s[k][3]};
      d[1] = f32x4{s[k][4], s[k][5], s[k][6], s[k][7]};
    }
  }
  __syncthreads();
  for (int q = tid; q < ZB_NS * C; q += 256) {
    const int k = q / C, c = q - (q / C) * C;
    float t = 0.f;
    t = lds_sum(sh + (k * slots) * C + c, slots, C);
    J.rs[(((int64_t)n * nch + chunk) * ZB_NS + k) * C + c] = t;
  }
}

// ---- backward 1, fused (round 6): the BatchNorm(+ReLU) backward apply of
// conv1's BatchNorm -- the pass that WRITES dy -- taking the region partials
// of the values it stores.  Same blocks (sample, pixel chunk), the same lane
// -> (pixel, 8 channels) map and summation order as zbias_rs_kernel, and the
// per-element arithmetic of vu_bn_bwd_apply (bn.hip bn_bwd_apply_kernel):
// dy and rs come out bit-identical to the two separate passes, without the
// re-read of dy.
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_zrs_kernel(const T* dz_in, int64_t dzs, const T* x, int64_t xs,
                                                               int H, int W, int C, const float* scale,
                                                               const float* shift, const float* mean,
                                                               const float* coef, int relu, T* dy, int64_t dys,
                                                               float* rs) {
  __shared__ __attribute__((aligned(16))) float sh[ZB_NS * 2048];
  const int HW = H * W, pch = pix_chunk(C), nch = (HW + pch - 1) / pch;
  const int n = (int)blockIdx.x / nch, chunk = (int)blockIdx.x - n * nch;
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
    const int c = cv * 8;
    float sc[8], sf[8], mu[8], k1[8], k2[8], k3[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = scale[c + i]; sf[i] = shift[c + i]; mu[i] = mean[c + i];
      k1[i] = coef[c + i]; k2[i] = coef[C + c + i]; k3[i] = coef[2 * C + c + i];
    }
    const int64_t nb = (int64_t)n * HW;
    const FastDiv dw((uint32_t)W);
    for (int p = p0 + slot; p < p1; p += U * slots) {
      Vec8<T> vd[U], vx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // clamped loads, used only when inside
        const int q = p + u * slots;
        const int64_t qc = nb + (q < p1 ? q : p1 - 1);
        vd[u].load(dz_in + qc * dzs + c);
        vx[u].load(x + qc * xs + c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = p + u * slots;
        if (q >= p1) break;
        Vec8<T> vo;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float xv = vx[u].get(i), d = vd[u].get(i);
          if (relu && !(fmaf(xv, sc[i], sf[i]) > 0.f)) d = 0.f;
          vo.set(i, fmaf(k1[i], d, k2[i] * (xv - mu[i])) + k3[i]);
        }
        vo.store(dy + (nb + q) * dys + c);
        const int y = (int)dw.div((uint32_t)q), xq = q - y * W;
#pragma unroll
        for (int e = 0; e < 8; ++e) s[0][e] += vo.get(e);
        if (xq == 0 || xq == W - 1 || y == 0 || y == H - 1) {
          const float m1 = xq == 0 ? 1.f : 0.f, m2 = xq == W - 1 ? 1.f : 0.f;
          const float m3 = y == 0 ? 1.f : 0.f, m4 = y == H - 1 ? 1.f : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = vo.get(e);
            s[1][e] = fmaf(m1, d, s[1][e]);
            s[2][e] = fmaf(m2, d, s[2][e]);
            s[3][e] = fmaf(m3, d, s[3][e]);
            s[4][e] = fmaf(m4, d, s[4][e]);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < ZB_NS; ++k) {
      f32x4* d = reinterpret_cast<f32x4*>(sh + (k * slots + slot) * C + cv * 8);
      d[0] = f32x4{s[k][0], s[k][1], s[k][2], s[k][3]};
      d[1] = f32x4{s[k][4], s[k][5], s[k][6], s[k][7]};
    }
  }
  __syncthreads();
  for (int q = tid; q < ZB_NS * C; q += 256) {
    const int k = q / C, c = q - (q / C) * C;
    float t = 0.f;
    t = lds_sum(sh + (k * slots) * C + c, slots, C);
    rs[(((int64_t)n * nch + chunk) * ZB_NS + k) * C + c] = t;
  }
}

// ---- backward 2: per (sample, 16 statistics): the sum of the chunk
// partials -> S[n][k][c] (after the partials in rs); 16 lanes per statistic
// (<= 8 loads each at 128 chunks: one round trip), then a fixed-order LDS
// reduction
constexpr int ZB_SV = 16, ZB_SL = 256 / ZB_SV;
__global__ __launch_bounds__(256) void zbias_sum_kernel(const ZbJobs jobs, int njobs, int N) {
  __shared__ float red[ZB_SL][ZB_SV];
  const VuZbJob& J = jobs.j[find_job(jobs, njobs)];
  const int C = J.co, nv = ZB_NS * C, ngrp = (nv + ZB_SV - 1) / ZB_SV;
  const int lb = (int)((int64_t)blockIdx.x - J.block0);
  const int n = lb / ngrp, grp = lb - (lb / ngrp) * ngrp;
  const int nch = n_chunks(C, J.H, J.W);
  const int v = threadIdx.x % ZB_SV, lane = threadIdx.x / ZB_SV, q = grp * ZB_SV + v;
  float t = 0.f;
  if (q < nv) {
    const float* rp = J.rs + (int64_t)n * nch * nv + q;
    for (int b0 = lane; b0 < nch; b0 += ZB_SL * 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int b = b0 + u * ZB_SL;
        x[u] = rp[(int64_t)(b < nch ? b : lane) * nv];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b0 + u * ZB_SL < nch) t += x[u];
    }
  }
  red[lane][v] = t;
  __syncthreads();
  if (lane == 0 && q < nv) {
    float r = 0.f;
#pragma unroll
    for (int k = 0; k < ZB_SL; ++k) r += red[k][v];
    J.rs[(int64_t)N * nch * nv + (int64_t)n * nv + q] = r;
  }
}

// ---- backward 3: per 32 output channels: R[n][c][tap] from the sums and the
// four corner pixels of dy, then the z columns of dW and the dc partial of
// these channels (into split `chunk` of part; chunk 0 also zeroes the splits
// no chunk uses), from R, the z weights and the vectors in LDS
//   dW[c0 + c][cz0 + l][tap] (+)= sum_n act[n][l] R[n][c][tap]
//   dc_chunk[n][l]              = sum_{c, tap} W[c0 + c][cz0 + l][tap] R[n][c][tap]
template <typename T>
__global__ __launch_bounds__(256) void zbias_dw_kernel(const ZbJobs jobs, int njobs, int N, int dbg) {
  extern __shared__ float zsm[];
  const VuZbJob& J = jobs.j[find_job(jobs, njobs)];
  const int chunk = (int)((int64_t)blockIdx.x - J.block0);
  const int c0 = chunk * ZB_CW, cw = J.co - c0 < ZB_CW ? J.co - c0 : ZB_CW;
  const int L = J.L, C = J.co, H = J.H, W = J.W, tid = threadIdx.x;
  const int nch = n_chunks(C, H, W);
  const int nchunks = (C + ZB_CW - 1) / ZB_CW;
  float* R = zsm;                  // [N][ZB_CW][9]
  float* A = R + N * ZB_CW * 9;    // [N][L]
  float* Wl = A + N * L;           // [L * 9][ZB_WP]
  const float* S = J.rs + (int64_t)N * nch * ZB_NS * C;
  const T* dy = reinterpret_cast<const T*>(J.dy);
  // R from the sums and the corners; its loads share the weight staging's round trip
  auto rloop = [&] {
    stage(A, N * L, [&](int e) { return J.act[e]; });
    for (int e = tid; e < N * ZB_CW && !(dbg & 4); e += 256) {
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
  };
  if (!(dbg & 1))
    stage_w(Wl, J, c0, cw, rloop);
  else
    rloop();
  __syncthreads();
  for (int e = tid; J.dw && e < cw * L && !(dbg & 2); e += 256) {
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
  for (int e = tid; e < N * L && !(dbg & 8); e += 256) {
    const int n = e / L, l = e - (e / L) * L;
    float s = 0.f;
    for (int c = 0; c < cw; ++c) {
      const float* w = Wl + l * 9 * ZB_WP + c;
      const float* r = R + (n * ZB_CW + c) * 9;
#pragma unroll
      for (int t = 0; t < 9; ++t) s += w[t * ZB_WP] * r[t];
    }
    J.part[((int64_t)n * ZB_SPLITS + chunk) * L + l] = s;
    if (chunk == 0)
      for (int sp = nchunks; sp < ZB_SPLITS; ++sp) J.part[((int64_t)n * ZB_SPLITS + sp) * L + l] = 0.f;
  }
}

#define DISPATCH_T(dtype, ...) \
  if ((dtype) == VU_BF16) { using T = bf16_t; __VA_ARGS__; } else { using T = float; __VA_ARGS__; }

size_t fwd_lds_bytes(int N, int L) { return (size_t)(ZB_WP * L * 9 + N * L) * sizeof(float); }
size_t dw_lds_bytes(int N, int L) { return (size_t)(N * ZB_CW * 9 + N * L + ZB_WP * L * 9) * sizeof(float); }

int pack(const VuZbJob* jobs, int njobs, ZbJobs& J) {
  if (njobs < 1 || njobs > ZB_MAXJ) return (int)hipErrorInvalidValue;
  for (int j = 0; j < njobs; ++j) J.j[j] = jobs[j];
  return 0;
}

int g_zb_dbg = 0;   // timing experiments only (tools/zbias_bench.py): phases skipped, results wrong

}  // namespace

extern "C" void vu_zbias_set_debug(int mode) { g_zb_dbg = mode; }

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
                     (hipStream_t)stream, J, njobs, N, g_zb_dbg);
  return (int)hipGetLastError();
}

extern "C" int vu_bn_bwd_apply_zrs_ok(int H, int W, int C, int64_t dzs, int64_t xs, int64_t dys) {
  return H >= 2 && W >= 2 && C >= 8 && C % 8 == 0 && C / 8 <= 256 && dzs % 8 == 0 && xs % 8 == 0 &&
         dys % 8 == 0 && (int64_t)H * W <= (1 << 30) / C;
}

extern "C" int vu_bn_bwd_apply_zrs(const void* dz, int64_t dzs, const void* x, int64_t xs, int N, int H, int W, int C,
                                   const float* scale, const float* shift, const float* mean, const float* coef,
                                   int relu, void* dy, int64_t dys, float* rs, int dtype, void* stream) {
  if (!vu_bn_bwd_apply_zrs_ok(H, W, C, dzs, xs, dys) || N < 1 || !rs) return (int)hipErrorInvalidValue;
  const int64_t blocks = (int64_t)N * n_chunks(C, H, W);
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((bn_bwd_apply_zrs_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       (const T*)dz, dzs, (const T*)x, xs, H, W, C, scale, shift, mean, coef, relu, (T*)dy, dys, rs);
  })
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
  bool all_ready = true;
  for (int j = 0; j < njobs; ++j) all_ready = all_ready && J.j[j].rs_ready;
  if (!all_ready) {
    DISPATCH_T(dtype, {
      hipLaunchKernelGGL((zbias_rs_kernel<T>), dim3((unsigned)rblocks), dim3(256), 0, st, J, njobs, N);
    })
  }
  int64_t sblocks = 0;
  for (int j = 0; j < njobs; ++j) {
    J.j[j].block0 = sblocks;
    sblocks += (int64_t)N * ((ZB_NS * J.j[j].co + ZB_SV - 1) / ZB_SV);
  }
  hipLaunchKernelGGL(zbias_sum_kernel, dim3((unsigned)sblocks), dim3(256), 0, st, J, njobs, N);
  int64_t dblocks = 0;
  for (int j = 0; j < njobs; ++j) {
    J.j[j].block0 = dblocks;
    dblocks += (J.j[j].co + ZB_CW - 1) / ZB_CW;
  }
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((zbias_dw_kernel<T>), dim3((unsigned)dblocks), dim3(256), dw_lds_bytes(N, maxL), st, J,
                       njobs, N, g_zb_dbg);
  })
  return (int)hipGetLastError();
}
