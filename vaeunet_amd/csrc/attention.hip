// AttentionGate (unet_parts.py:7-30 / unet_resnet.py:6-29) memory-bound parts
// and the tiny-output 1x1 convolutions (OutConv unet_parts.py:97-103,
// final_conv unet_resnet.py:189).
//
//   g1 = BN(W_g g + b_g), x1 = BN(W_x x + b_x)      (GEMMs: gemm_fwd.hip)
//   s  = relu(g1 + x1)                              \
//   q  = W_psi s + b_psi   (F_int -> 1)              } vu_attn_psi_fwd (one pass)
//   p  = sigmoid(BN(q));  out = x * p               vu_attn_gate_fwd
//
// A pixel's F_int channels are spread over LPP = F_int/8 lanes (8 channels
// per lane, 16-byte loads), the dot product reduced with cross-lane shuffles;
// a 256-thread block owns a 256-pixel tile and emits that tile's BatchNorm(1)
// partial (sum, centered M2).  Weight-gradient sums use per-block partial
// slabs reduced in a fixed order (deterministic, no float atomics).
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

constexpr int TILE = 256;  // pixels per block

inline unsigned ew_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Sum over aligned groups of lpp lanes (lpp a power of two, uniform): DPP
// lane permutations within 16-lane rows (xor 1, xor 2, half-row mirror,
// row mirror: each step pairs every lane with one holding the other half of
// its group), LDS-crossbar shuffles only across rows.  A ds_bpermute chain
// costs one LDS round trip per step, and these per-pixel dot products run
// one chain per pixel.
template <int CTRL>
VU_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

// opaque register tie of a Vec8 (keeps its computation above a guarded store)
VU_DEV void vec8_tie(Vec8<bf16_t>& v) { asm volatile("" : "+v"(v.v)); }
VU_DEV void vec8_tie(Vec8<float>& v) { asm volatile("" : "+v"(v.a), "+v"(v.b)); }

VU_DEV float group_sum(float v, int lpp) {
  if (lpp >= 2) v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  if (lpp >= 4) v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  if (lpp >= 8) v += dpp_f<0x141>(v);  // row_half_mirror
  if (lpp >= 16) v += dpp_f<0x140>(v); // row_mirror
  if (lpp >= 32) v += __shfl_xor(v, 16, 64);
  if (lpp >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}

// psi = sigmoid(BN(q)).  fp32 (parity mode): the correctly rounded-ish libm
// exp -- the fast __expf carries a small SYSTEMATIC error, and the psi
// BatchNorm(1) affine gradients are sums over every pixel of terms that
// cancel to 1e-3 of their magnitude, where a bias adds up coherently (the
// HIP path had 2-3x the fp32 oracle's error on psi.1.weight, round 6).
// bf16 (speed mode): __expf.
template <typename T>
VU_DEV float gate_sigmoid(float z) {
  if constexpr (sizeof(T) == 4) return 1.f / (1.f + expf(-z));
  else return 1.f / (1.f + __expf(-z));
}

template <typename T>
VU_DEV void load8(const T* p, float* f) {
  Vec8<T> v; v.load(p);
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = v.get(k);
}

// block reduction of one float over 256 threads, result broadcast
VU_DEV float block_sum(float v, float* sh) {
  v = warp_sum(v);
  int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  float t = sh[0] + sh[1] + sh[2] + sh[3];
  return t;
}

template <typename T>
__global__ void psi_fwd_kernel(const T* ug, const T* ux, int64_t P, int F, const float* sg, const float* tg,
                               const float* sx, const float* tx, const float* wpsi, const float* bpsi, float* q,
                               float* psum, float* pm2) {
  __shared__ float sq[TILE];
  __shared__ float red[4];
  const int lpp = F >> 3;              // lanes per pixel (power of two <= 64)
  const int ppw = 64 / lpp;            // pixels per wave-pass
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane % lpp, slot = lane / lpp;
  const int64_t p0 = (int64_t)blockIdx.x * TILE;
  const int c = sub * 8;
  float wsg[8], wtg[8], wsx[8], wtx[8], wp[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wsg[k] = sg[c + k]; wtg[k] = tg[c + k]; wsx[k] = sx[c + k]; wtx[k] = tx[c + k]; wp[k] = wpsi[c + k];
  }
  const float b = bpsi[0];
  for (int i = w * ppw + slot; i < TILE; i += 4 * ppw) {
    int64_t p = p0 + i;
    float acc = 0.f;
    if (p < P) {
      float a[8], bb[8];
      load8<T>(ug + p * F + c, a);
      load8<T>(ux + p * F + c, bb);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s = fmaxf(a[k] * wsg[k] + wtg[k] + bb[k] * wsx[k] + wtx[k], 0.f);
        acc += wp[k] * s;
      }
    }
    acc = group_sum(acc, lpp) + b;
    if (sub == 0) {
      sq[i] = p < P ? acc : 0.f;
      if (p < P) q[p] = acc;
    }
  }
  __syncthreads();
  int64_t nvalid = P - p0 < TILE ? P - p0 : TILE;
  float v = threadIdx.x < nvalid ? sq[threadIdx.x] : 0.f;
  float tot = block_sum(v, red);
  float mean = tot / (float)nvalid;
  float d = threadIdx.x < nvalid ? sq[threadIdx.x] - mean : 0.f;
  float m2 = block_sum(d * d, red);
  if (threadIdx.x == 0) { psum[blockIdx.x] = tot; pm2[blockIdx.x] = m2; }
}

// Batched variants (default, VU_TUNE_ATTN = 1): each lane issues the loads of
// U pixel rows (or U 16-byte vectors) before it uses any of them, so a wave
// keeps U times the bytes in flight; the loads of out-of-range rows are
// clamped to the last valid row and their results dropped.  Same pixel -> lane
// assignment and summation order as the one-row kernels (equal up to the
// compiler's fma contraction of the per-lane sums).
int g_attn = 1;

template <typename T, int U>
__global__ __launch_bounds__(256) void psi_fwd_u_kernel(const T* ug, const T* ux, int64_t P, int F, const float* sg,
                                                        const float* tg, const float* sx, const float* tx,
                                                        const float* wpsi, const float* bpsi, float* q, float* psum,
                                                        float* pm2) {
  __shared__ float sq[TILE];
  __shared__ float red[4];
  const int lpp = F >> 3, ppw = 64 / lpp;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane % lpp, slot = lane / lpp;
  const int64_t p0 = (int64_t)blockIdx.x * TILE;
  const int c = sub * 8;
  float wsg[8], wtg[8], wsx[8], wtx[8], wp[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wsg[k] = sg[c + k]; wtg[k] = tg[c + k]; wsx[k] = sx[c + k]; wtx[k] = tx[c + k]; wp[k] = wpsi[c + k];
  }
  const float b = bpsi[0];
  const int niter = lpp;  // TILE / (4 * ppw)
  for (int it = 0; it < niter; it += U) {
    Vec8<T> va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (it + u < niter) {  // uniform
        int64_t p = p0 + w * ppw + slot + (it + u) * 4 * ppw;
        p = p < P ? p : P - 1;
        va[u].load(ug + p * F + c);
        vb[u].load(ux + p * F + c);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (it + u >= niter) break;
      const int i = w * ppw + slot + (it + u) * 4 * ppw;
      const int64_t p = p0 + i;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s = fmaxf(va[u].get(k) * wsg[k] + wtg[k] + vb[u].get(k) * wsx[k] + wtx[k], 0.f);
        acc += wp[k] * s;
      }
      if (p >= P) acc = 0.f;
      acc = group_sum(acc, lpp) + b;
      if (sub == 0) {
        sq[i] = p < P ? acc : 0.f;
        if (p < P) q[p] = acc;
      }
    }
  }
  __syncthreads();
  int64_t nvalid = P - p0 < TILE ? P - p0 : TILE;
  float v = threadIdx.x < nvalid ? sq[threadIdx.x] : 0.f;
  float tot = block_sum(v, red);
  float mean = tot / (float)nvalid;
  float d = threadIdx.x < nvalid ? sq[threadIdx.x] - mean : 0.f;
  float m2 = block_sum(d * d, red);
  if (threadIdx.x == 0) { psum[blockIdx.x] = tot; pm2[blockIdx.x] = m2; }
}

// out = x * sigmoid(q*s + t): U independent 16-byte vectors per thread and
// iteration; V = C/8 vectors per pixel, a power of two (shift, no division)
template <typename T, int U>
__global__ __launch_bounds__(256) void gate_fwd_u_kernel(const float* q, const float* st, const T* x, int64_t xs,
                                                         int64_t P, int vsh, float* pmap, T* out, int64_t os) {
  const int64_t tot = P << vsh;
  const int vm = (1 << vsh) - 1;
  const float s = st[0], t = st[1];
  const int64_t step = (int64_t)gridDim.x * 256 * U;
  for (int64_t e0 = (int64_t)blockIdx.x * 256 * U + threadIdx.x; e0 < tot; e0 += step) {
    Vec8<T> v[U];
    float qv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t e = e0 + u * 256;
      e = e < tot ? e : tot - 1;
      const int64_t p = e >> vsh;
      const int c = (int)(e & vm) * 8;
      qv[u] = q[p];
      v[u].load(x + p * xs + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = e0 + u * 256;
      if (e >= tot) break;
      const int64_t p = e >> vsh;
      const int c = (int)(e & vm) * 8;
      const float pv = gate_sigmoid<T>(qv[u] * s + t);
      if (c == 0 && pmap) pmap[p] = pv;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[u].set(k, v[u].get(k) * pv);
      v[u].store(out + p * os + c);
    }
  }
}

template <typename T>
__global__ void gate_fwd_kernel(const float* q, const float* st, const T* x, int64_t xs, int64_t P, int C,
                                float* pmap, T* out, int64_t os) {
  int V = C >> 3;
  int64_t tot = P * V;
  const float s = st[0], t = st[1];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = e / V;
    int c = (int)(e - p * V) * 8;
    float z = q[p] * s + t;
    float pv = gate_sigmoid<T>(z);
    if (c == 0 && pmap) pmap[p] = pv;
    Vec8<T> v; v.load(x + p * xs + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) v.set(k, v.get(k) * pv);
    v.store(out + p * os + c);
  }
}

// dx = dout * p ; dbnq[p] = (sum_c dout*x) * p*(1-p)
template <typename T>
__global__ void gate_bwd_kernel(const T* dout, int64_t dos, const T* x, int64_t xs, const float* pmap, int64_t P,
                                int C, T* dx, int64_t dxs, float* dbnq) {
  const int lpp = C >> 3 > 64 ? 64 : C >> 3;   // lanes per pixel
  const int ppw = 64 / lpp;
  const int lane = threadIdx.x & 63;
  const int sub = lane % lpp, slot = lane / lpp;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t pb = wave * ppw; pb < P; pb += nwaves * ppw) {
    int64_t p = pb + slot;
    float acc = 0.f;
    if (p < P) {
      float pv = pmap[p];
      for (int c = sub * 8; c < C; c += lpp * 8) {
        Vec8<T> vd, vx, vo;
        vd.load(dout + p * dos + c);
        vx.load(x + p * xs + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          acc += vd.get(k) * vx.get(k);
          vo.set(k, vd.get(k) * pv);
        }
        vo.store(dx + p * dxs + c);
      }
    }
    acc = group_sum(acc, lpp);
    if (sub == 0 && p < P) { float pv = pmap[p]; dbnq[p] = acc * pv * (1.f - pv); }
  }
}

// gate backward for C <= 512 (one 8-channel chunk per lane), U pixel rows of
// loads in flight per lane
template <typename T, int U>
__global__ __launch_bounds__(256) void gate_bwd_u_kernel(const T* dout, int64_t dos, const T* x, int64_t xs,
                                                         const float* pmap, int64_t P, int C, T* dx, int64_t dxs,
                                                         float* dbnq) {
  const int lpp = C >> 3;
  const int ppw = 64 / lpp;
  const int lane = threadIdx.x & 63;
  const int sub = lane % lpp, slot = lane / lpp;
  const int c = sub * 8;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t pb = wave * ppw * U; pb < P; pb += nwaves * ppw * U) {
    Vec8<T> vd[U], vx[U];
    float pv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t p = pb + u * ppw + slot;
      p = p < P ? p : P - 1;
      pv[u] = pmap[p];
      vd[u].load(dout + p * dos + c);
      vx[u].load(x + p * xs + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t p = pb + u * ppw + slot;
      float acc = 0.f;
      Vec8<T> vo;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc += vd[u].get(k) * vx[u].get(k);
        vo.set(k, vd[u].get(k) * pv[u]);
      }
      if (p < P) vo.store(dx + p * dxs + c);
      acc = group_sum(acc, lpp);
      if (sub == 0 && p < P) dbnq[p] = acc * pv[u] * (1.f - pv[u]);
    }
  }
}

// ds[p,c] = dq[p]*wpsi[c]*(s>0); per-block partials of dwpsi[c] and dbpsi
// (grid-stride over 256-pixel tiles, so at most MAXB partial rows)
constexpr int MAXB = 1024;

// BNB (round 6): the kernel also emits the first stage of the backward
// reduction of BOTH BatchNorms in front of the sum (W_g's over ug, W_x's over
// ux; unet_parts.py:11-20), whose output gradient is ds itself (no ReLU
// between: the ReLU is after the sum): sum dz and sum dz (u - mean) invstd
// with dz = the stored ds -- vu_bn_bwd_reduce's arithmetic -- as bnb_g / bnb_x
// [block][2][F] (VuGemmFwd.bnb_part's layout), from the ug, ux and ds values
// already in registers: the two separate reduction passes over ds, ug and
// ds, ux are not run.
template <typename T, int U, bool BNB = false>
__global__ __launch_bounds__(256) void psi_bwd_u_kernel(const T* ug, const T* ux, int64_t P, int F, const float* sg,
                                                        const float* tg, const float* sx, const float* tx,
                                                        const float* wpsi, const float* dq, T* ds, float* part,
                                                        const float* mg = nullptr, const float* ig = nullptr,
                                                        const float* mx = nullptr, const float* ix = nullptr,
                                                        float* bnb_g = nullptr, float* bnb_x = nullptr) {
  __shared__ float sh[256 * 8];
  __shared__ float sb[256];
  const int lpp = F >> 3, ppw = 64 / lpp;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane % lpp, slot = lane / lpp;
  const int c = sub * 8;
  float wsg[8], wtg[8], wsx[8], wtx[8], wp[8], dw[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wsg[k] = sg[c + k]; wtg[k] = tg[c + k]; wsx[k] = sx[c + k]; wtx[k] = tx[c + k]; wp[k] = wpsi[c + k];
    dw[k] = 0.f;
  }
  float bmg[8], big[8], bmx[8], bix[8], z0[8], zg[8], zx[8];
  if constexpr (BNB)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bmg[k] = mg[c + k]; big[k] = ig[c + k]; bmx[k] = mx[c + k]; bix[k] = ix[c + k];
      z0[k] = 0.f; zg[k] = 0.f; zx[k] = 0.f;
    }
  float db = 0.f;
  const int niter = lpp;  // TILE / (4 * ppw)
  for (int64_t p0 = (int64_t)blockIdx.x * TILE; p0 < P; p0 += (int64_t)gridDim.x * TILE) {
    for (int it = 0; it < niter; it += U) {
      Vec8<T> va[U], vb[U];
      float g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (it + u < niter) {
          int64_t p = p0 + w * ppw + slot + (it + u) * 4 * ppw;
          p = p < P ? p : P - 1;
          g[u] = dq[p];
          va[u].load(ug + p * F + c);
          vb[u].load(ux + p * F + c);
        }
      }
      // every row's output formed (and tied) before the guarded stores: with
      // the work inside the branches each store waited vmcnt(0) -- i.e. for
      // the previous row's store (4 serial write round trips per round)
      Vec8<T> o[U];
      bool okp[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t p = p0 + w * ppw + slot + (it + u) * 4 * ppw;
        okp[u] = it + u < niter && p < P;
        if (okp[u] && sub == 0) db += g[u];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float s = va[u].get(k) * wsg[k] + wtg[k] + vb[u].get(k) * wsx[k] + wtx[k];
          bool on = s > 0.f;
          if (okp[u]) dw[k] += on ? g[u] * s : 0.f;
          o[u].set(k, on ? g[u] * wp[k] : 0.f);
          if constexpr (BNB) {
            if (okp[u]) {
              const float dz = o[u].get(k);  // the stored (rounded) ds
              z0[k] += dz;
              zg[k] += dz * ((va[u].get(k) - bmg[k]) * big[k]);
              zx[k] += dz * ((vb[u].get(k) - bmx[k]) * bix[k]);
            }
          }
        }
        vec8_tie(o[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (okp[u]) o[u].store(ds + (p0 + w * ppw + slot + (it + u) * 4 * ppw) * F + c);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) sh[threadIdx.x * 8 + k] = dw[k];
  sb[threadIdx.x] = db;
  __syncthreads();
  for (int cc = threadIdx.x; cc < F; cc += 256) {
    int sb_ = cc >> 3, k = cc & 7;
    float s = 0.f;
    s = lds_sum(sh + sb_ * 8 + k, (256 - sb_ + lpp - 1) / lpp, lpp * 8);
    part[(int64_t)blockIdx.x * (F + 1) + cc] = s;
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    s = lds_sum(sb, 256, 1);
    part[(int64_t)blockIdx.x * (F + 1) + F] = s;
  }
  if constexpr (BNB) {
    // threads with equal `sub` hold the same channels: fixed-order sums, as
    // the dwpsi partials above; sum dz goes to both BatchNorms' rows
    for (int q = 0; q < 3; ++q) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) sh[threadIdx.x * 8 + k] = q == 0 ? z0[k] : (q == 1 ? zg[k] : zx[k]);
      __syncthreads();
      for (int cc = threadIdx.x; cc < F; cc += 256) {
        int sb_ = cc >> 3, k = cc & 7;
        float v = 0.f;
        v = lds_sum(sh + sb_ * 8 + k, (256 - sb_ + lpp - 1) / lpp, lpp * 8);
        if (q == 0) {
          bnb_g[((int64_t)blockIdx.x * 2 + 0) * F + cc] = v;
          bnb_x[((int64_t)blockIdx.x * 2 + 0) * F + cc] = v;
        } else {
          (q == 1 ? bnb_g : bnb_x)[((int64_t)blockIdx.x * 2 + 1) * F + cc] = v;
        }
      }
    }
  }
}

template <typename T>
__global__ void psi_bwd_kernel(const T* ug, const T* ux, int64_t P, int F, const float* sg, const float* tg,
                               const float* sx, const float* tx, const float* wpsi, const float* dq, T* ds,
                               float* part) {
  __shared__ float sh[256 * 8];
  __shared__ float sb[256];
  const int lpp = F >> 3, ppw = 64 / lpp;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sub = lane % lpp, slot = lane / lpp;
  const int c = sub * 8;
  float wsg[8], wtg[8], wsx[8], wtx[8], wp[8], dw[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wsg[k] = sg[c + k]; wtg[k] = tg[c + k]; wsx[k] = sx[c + k]; wtx[k] = tx[c + k]; wp[k] = wpsi[c + k];
    dw[k] = 0.f;
  }
  float db = 0.f;
  for (int64_t p0 = (int64_t)blockIdx.x * TILE; p0 < P; p0 += (int64_t)gridDim.x * TILE) {
    for (int i = w * ppw + slot; i < TILE; i += 4 * ppw) {
      int64_t p = p0 + i;
      if (p >= P) continue;
      float g = dq[p];
      if (sub == 0) db += g;
      float a[8], bb[8];
      load8<T>(ug + p * F + c, a);
      load8<T>(ux + p * F + c, bb);
      Vec8<T> o;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float s = a[k] * wsg[k] + wtg[k] + bb[k] * wsx[k] + wtx[k];
        bool on = s > 0.f;
        dw[k] += on ? g * s : 0.f;
        o.set(k, on ? g * wp[k] : 0.f);
      }
      o.store(ds + p * F + c);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) sh[threadIdx.x * 8 + k] = dw[k];
  sb[threadIdx.x] = db;
  __syncthreads();
  // threads with equal `sub` hold the same channels: sum them in fixed order
  for (int cc = threadIdx.x; cc < F; cc += 256) {
    int sb_ = cc >> 3, k = cc & 7;
    float s = 0.f;
    s = lds_sum(sh + sb_ * 8 + k, (256 - sb_ + lpp - 1) / lpp, lpp * 8);
    part[(int64_t)blockIdx.x * (F + 1) + cc] = s;
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    s = lds_sum(sb, 256, 1);
    part[(int64_t)blockIdx.x * (F + 1) + F] = s;
  }
}

// column sums of [nblk][width] partials (colsum32: fp64, fixed order)
__global__ void part_final(const float* part, int nblk, int width, float* out, int n_out, float* out2,
                           int accumulate) {
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const int cl = c < width ? c : width - 1;
  float* o = cl < n_out ? (out ? out + cl : nullptr) : (out2 ? out2 + (cl - n_out) : nullptr);
  const float o0 = (accumulate && o) ? *o : 0.f;   // loaded before the sums (bn_bwd_final)
  double s[1];
  colsum32<1>(part, nblk, width, 0, c, c < width, s);
  if (threadIdx.x >= 32 || c >= width || o == nullptr) return;
  *o = accumulate ? o0 + (float)s[0] : (float)s[0];
}

// ---- tiny-output pointwise conv ----
// BNA (round 6): x is the PRE-BatchNorm tensor of the producing DoubleConv and
// the operand is a = relu(x * bn_scale + bn_shift) rounded to the storage
// type -- exactly the bytes vu_bn_apply would have stored -- formed in
// registers, so the UNet's last BatchNorm + ReLU is never materialised
// (unet_parts.py:44-45 feeding OutConv :100).
template <typename T, bool BNA = false, int JM = 4>
__global__ void pw_fwd_kernel(const T* x, int64_t xs, int64_t P, int C, int J, const float* w, const float* b,
                              float* y, int64_t ys, const float* bn_scale = nullptr, const float* bn_shift = nullptr) {
  const int lpp = C >> 3 > 64 ? 64 : C >> 3;
  const int ppw = 64 / lpp;
  const int lane = threadIdx.x & 63;
  const int sub = lane % lpp, slot = lane / lpp;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  if (C <= 512) {
    // one 8-channel chunk per lane: its weights and the bias live in
    // registers (the compiler cannot hoist per-pixel weight loads that may
    // alias y), and PU pixel rows per lane are loaded before any is used
    // (cold-cache 512^2 x 64 -> 2: 135 -> 107 us with the DPP group sums)
    constexpr int PU = 4;   // (8 rows in flight: 144 VGPRs, 3 waves per SIMD, measured 71 -> 91 us)
    const int c = sub * 8;
    // JM: the largest J this instantiation serves (outputs j >= J carry zero
    // weights); JM = 2 halves the FMAs and group sums of the UNet's 2-class head
    float wr[JM][8], bj[JM], bsc[8], bsh[8];
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      bj[j] = (j < J && b) ? b[j] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) wr[j][k] = j < J ? w[j * C + c + k] : 0.f;
    }
    if constexpr (BNA)
#pragma unroll
      for (int k = 0; k < 8; ++k) { bsc[k] = bn_scale[c + k]; bsh[k] = bn_shift[c + k]; }
    for (int64_t pb = wave * ppw * PU; pb < P; pb += nwaves * ppw * PU) {
      // the PU loads from clamped pixel addresses, unconditionally: a guarded
      // load per pixel sat in its own basic block with a vmcnt(0) wait after
      // it, serialising the round trips (512^2 x 64 -> 2 at ~3 TB/s); rows
      // past P are zeroed after the loads
      float f[PU][8];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int64_t p = pb + u * ppw + slot;
        load8<T>(x + (p < P ? p : P - 1) * xs + c, f[u]);
      }
      if constexpr (BNA)
#pragma unroll
        for (int u = 0; u < PU; ++u)
#pragma unroll
          for (int k = 0; k < 8; ++k) f[u][k] = rnd<T>(fmaxf(fmaf(f[u][k], bsc[k], bsh[k]), 0.f));
#pragma unroll
      for (int u = 0; u < PU; ++u)
        if (pb + u * ppw + slot >= P)
#pragma unroll
          for (int k = 0; k < 8; ++k) f[u][k] = 0.f;
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int64_t p = pb + u * ppw + slot;
        float acc[JM];
#pragma unroll
        for (int j = 0; j < JM; ++j) {
          acc[j] = 0.f;
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[j] += f[u][k] * wr[j][k];
          acc[j] = group_sum(acc[j], lpp);
        }
        if (sub == 0 && p < P)
          for (int j = 0; j < J; ++j) y[p * ys + j] = acc[j] + bj[j];
      }
    }
    return;
  }
  if constexpr (BNA) return;  // (host: C <= 512 only)
  for (int64_t pb = wave * ppw; pb < P; pb += nwaves * ppw) {
    int64_t p = pb + slot;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (p < P) {
      for (int c = sub * 8; c < C; c += lpp * 8) {
        float f[8];
        load8<T>(x + p * xs + c, f);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < J)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[j] += f[k] * w[j * C + c + k];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = group_sum(acc[j], lpp);
    if (sub == 0 && p < P)
      for (int j = 0; j < J; ++j) y[p * ys + j] = acc[j] + (b ? b[j] : 0.f);
  }
}

// dx = dy w ; per-block partials of dw[j][c] = sum dy[p,j] x[p,c] and db[j]
// BNA (round 6): x is the pre-BatchNorm tensor (the operand a = relu(x * sc +
// sh) rounded to T is re-formed in registers, as pw_fwd_kernel<BNA>), and the
// block also emits the first stage of that BatchNorm's backward reduction over
// its pixels -- sum dz, sum dz * (x - mean) * invstd with dz = the stored
// (rounded) dx masked by the ReLU, vu_bn_bwd_reduce's arithmetic -- as
// bnb[blk][2][C] (VuGemmFwd.bnb_part's layout), so the separate reduction
// pass over dx and x is not run.
template <typename T, bool BNA = false, int JM = 4>
__global__ __launch_bounds__(256) void pw_bwd_kernel(const T* x, int64_t xs, const float* dy, int64_t dys, int64_t P, int C, int J,
                              const float* w, T* dx, int64_t dxs, float* part, const float* bn_scale = nullptr,
                              const float* bn_shift = nullptr, const float* bn_mean = nullptr,
                              const float* bn_invstd = nullptr, float* bnb = nullptr) {
  __shared__ float sh[256 * 8];
  const int lpp = C >> 3;   // <= 32 enforced on host (C <= 256)
  const int ppw = 64 / lpp;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sub = lane % lpp, slot = lane / lpp;
  const int c = sub * 8;
  const int width = J * C + J;
  // JM as in pw_fwd_kernel: dy columns j >= J are read as zero
  float dw[JM][8], db[JM], wr[JM][8];
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    db[j] = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) { dw[j][k] = 0.f; wr[j][k] = j < J ? w[j * C + c + k] : 0.f; }
  }
  float bsc[8], bsh[8], bmu[8], bis[8], z0[8], z1[8];
  if constexpr (BNA)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bsc[k] = bn_scale[c + k]; bsh[k] = bn_shift[c + k]; bmu[k] = bn_mean[c + k]; bis[k] = bn_invstd[c + k];
      z0[k] = 0.f; z1[k] = 0.f;
    }
  // PU pixel rows per lane are loaded (from clamped addresses, unconditionally)
  // before any is used: a guarded load per pixel serialised the round trips
  // (as pw_fwd_kernel); rows past the tile or P get a zero dy, so they add
  // nothing to dw, db or the BatchNorm sums, and are not stored.
  constexpr int PU = 2;
  const int step = 4 * ppw;
  for (int64_t p0 = (int64_t)blockIdx.x * TILE; p0 < P; p0 += (int64_t)gridDim.x * TILE) {
    for (int i0 = wv * ppw + slot; i0 < TILE; i0 += step * PU) {
      float g[PU][JM], f[PU][8], xr[PU][8];
      bool ok[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int64_t p = p0 + i0 + u * step;
        ok[u] = i0 + u * step < TILE && p < P;
        const int64_t pc = p < P ? p : P - 1;
#pragma unroll
        for (int j = 0; j < JM; ++j) g[u][j] = j < J ? dy[pc * dys + j] : 0.f;
        load8<T>(x + pc * xs + c, f[u]);
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        if (!ok[u])
#pragma unroll
          for (int j = 0; j < JM; ++j) g[u][j] = 0.f;
        if constexpr (BNA)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            xr[u][k] = f[u][k];
            f[u][k] = rnd<T>(fmaxf(fmaf(xr[u][k], bsc[k], bsh[k]), 0.f));
          }
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        Vec8<T> o;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < JM; ++j) { dw[j][k] += g[u][j] * f[u][k]; s += g[u][j] * wr[j][k]; }
          o.set(k, s);
          if constexpr (BNA) {
            float dz = o.get(k);  // the stored (rounded) value, as the reduction pass would read it
            if (!(xr[u][k] * bsc[k] + bsh[k] > 0.f)) dz = 0.f;
            z0[k] += dz;
            z1[k] += dz * ((xr[u][k] - bmu[k]) * bis[k]);
          }
        }
        if (ok[u]) o.store(dx + (p0 + i0 + u * step) * dxs + c);
        if (sub == 0)
#pragma unroll
          for (int j = 0; j < JM; ++j) db[j] += g[u][j];
      }
    }
  }
  for (int j = 0; j < J; ++j) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[threadIdx.x * 8 + k] = dw[j][k];
    __syncthreads();
    for (int cc = threadIdx.x; cc < C; cc += 256) {
      int sb_ = cc >> 3, k = cc & 7;
      float s = 0.f;
      s = lds_sum(sh + sb_ * 8 + k, (256 - sb_ + lpp - 1) / lpp, lpp * 8);
      part[(int64_t)blockIdx.x * width + j * C + cc] = s;
    }
    __syncthreads();
    sh[threadIdx.x] = db[j];
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
      s = lds_sum(sh, 256, 1);
      part[(int64_t)blockIdx.x * width + J * C + j] = s;
    }
  }
  if constexpr (BNA) {
    // threads with equal `sub` hold the same channels: fixed-order sums
    for (int q = 0; q < 2; ++q) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; ++k) sh[threadIdx.x * 8 + k] = q ? z1[k] : z0[k];
      __syncthreads();
      for (int cc = threadIdx.x; cc < C; cc += 256) {
        int sb_ = cc >> 3, k = cc & 7;
        float s = 0.f;
        s = lds_sum(sh + sb_ * 8 + k, (256 - sb_ + lpp - 1) / lpp, lpp * 8);
        bnb[((int64_t)blockIdx.x * 2 + q) * C + cc] = s;
      }
    }
  }
}

inline bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

}  // namespace

int attn_tune(int key, int value) {
  if (key == VU_TUNE_ATTN) {
    g_attn = value;
    return 0;
  }
  return -1;
}

#define DISPATCH_T(dtype, ...) \
  if ((dtype) == VU_BF16) { using T = bf16_t; __VA_ARGS__; } else { using T = float; __VA_ARGS__; }

extern "C" int64_t vu_attn_tile_rows() { return TILE; }

extern "C" int vu_attn_psi_fwd(const void* ug, const void* ux, int64_t P, int F, const float* sg, const float* tg,
                               const float* sx, const float* tx, const float* wpsi, const float* bpsi, float* q,
                               float* psum, float* pm2, int64_t tile_rows, int dtype, void* stream) {
  if (F % 8 != 0 || !pow2(F / 8) || F / 8 > 64 || tile_rows != TILE) return (int)hipErrorInvalidValue;
  int nblk = (int)((P + TILE - 1) / TILE);
  if (nblk == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (g_attn)
      hipLaunchKernelGGL((psi_fwd_u_kernel<T, 4>), dim3(nblk), dim3(256), 0, st, (const T*)ug, (const T*)ux, P, F, sg,
                         tg, sx, tx, wpsi, bpsi, q, psum, pm2);
    else
      hipLaunchKernelGGL((psi_fwd_kernel<T>), dim3(nblk), dim3(256), 0, st, (const T*)ug, (const T*)ux, P, F, sg, tg,
                         sx, tx, wpsi, bpsi, q, psum, pm2);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_attn_gate_fwd(const float* q, const float* st_, const void* x, int64_t xs, int64_t P, int C,
                                float* pmap, void* out, int64_t os, int dtype, void* stream) {
  if (C % 8 != 0 || xs % 8 != 0 || os % 8 != 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (P == 0) return 0;
  const int V = C / 8;
  DISPATCH_T(dtype, {
    if (g_attn && pow2(V))
      hipLaunchKernelGGL((gate_fwd_u_kernel<T, 4>), dim3(ew_grid(P * V / 4)), dim3(256), 0, st, q, st_, (const T*)x,
                         xs, P, __builtin_ctz(V), pmap, (T*)out, os);
    else
      hipLaunchKernelGGL((gate_fwd_kernel<T>), dim3(ew_grid(P * C / 8)), dim3(256), 0, st, q, st_, (const T*)x, xs, P,
                         C, pmap, (T*)out, os);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_attn_gate_bwd(const void* dout, int64_t dos, const void* x, int64_t xs, const float* pmap,
                                int64_t P, int C, void* dx, int64_t dxs, float* dqpre, int dtype, void* stream) {
  if (C % 8 != 0 || !pow2(C / 8 > 64 ? 64 : C / 8) || dos % 8 || xs % 8 || dxs % 8) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (P == 0) return 0;
  DISPATCH_T(dtype, {
    if (g_attn && C <= 512)
      hipLaunchKernelGGL((gate_bwd_u_kernel<T, 2>), dim3(ew_grid(P * 8)), dim3(256), 0, st, (const T*)dout, dos,
                         (const T*)x, xs, pmap, P, C, (T*)dx, dxs, dqpre);
    else
      hipLaunchKernelGGL((gate_bwd_kernel<T>), dim3(ew_grid(P * 8)), dim3(256), 0, st, (const T*)dout, dos,
                         (const T*)x, xs, pmap, P, C, (T*)dx, dxs, dqpre);
  })
  return (int)hipGetLastError();
}

extern "C" int64_t vu_attn_psi_bwd_blocks(int64_t P) {
  const int64_t nb = (P + TILE - 1) / TILE;
  return nb < MAXB ? nb : MAXB;
}

extern "C" int vu_attn_psi_bwd_bnb_ok(int F) {
  return F % 8 == 0 && pow2(F / 8) && F / 8 <= 64 && F <= 2048 && g_attn ? 1 : 0;
}

extern "C" int vu_attn_psi_bwd_bnb(const void* ug, const void* ux, int64_t P, int F, const float* sg, const float* tg,
                                   const float* sx, const float* tx, const float* wpsi, const float* dq, void* ds,
                                   float* dwpsi, float* dbpsi, int accumulate, float* workspace,
                                   const float* mean_g, const float* invstd_g, const float* mean_x,
                                   const float* invstd_x, float* bnb_g, float* bnb_x, int dtype, void* stream) {
  if (F % 8 != 0 || !pow2(F / 8) || F / 8 > 64 || F > 2048 || !g_attn || !mean_g || !invstd_g || !mean_x ||
      !invstd_x || !bnb_g || !bnb_x)
    return (int)hipErrorInvalidValue;
  const int nblk = (int)vu_attn_psi_bwd_blocks(P);
  if (nblk == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  // VU_TUNE_ATTN 2: two pixel rows per lane in flight instead of four (209 -> 162 VGPRs, occupancy 2 -> 3)
  DISPATCH_T(dtype, {
    if (g_attn == 2)
      hipLaunchKernelGGL((psi_bwd_u_kernel<T, 2, true>), dim3(nblk), dim3(256), 0, st, (const T*)ug, (const T*)ux,
                         P, F, sg, tg, sx, tx, wpsi, dq, (T*)ds, workspace, mean_g, invstd_g, mean_x, invstd_x,
                         bnb_g, bnb_x);
    else
      hipLaunchKernelGGL((psi_bwd_u_kernel<T, 4, true>), dim3(nblk), dim3(256), 0, st, (const T*)ug, (const T*)ux,
                         P, F, sg, tg, sx, tx, wpsi, dq, (T*)ds, workspace, mean_g, invstd_g, mean_x, invstd_x,
                         bnb_g, bnb_x);
  })
  hipLaunchKernelGGL(part_final, dim3((F + 1 + 31) / 32), dim3(COLSUM_THREADS), 0, st, workspace, nblk, F + 1, dwpsi,
                     F, dbpsi, accumulate);
  return (int)hipGetLastError();
}

extern "C" int64_t vu_attn_psi_bwd_workspace_bytes(int64_t P, int F) {
  int64_t nb = (P + TILE - 1) / TILE;
  return (nb < MAXB ? nb : MAXB) * (F + 1) * (int64_t)sizeof(float);
}

extern "C" int vu_attn_psi_bwd(const void* ug, const void* ux, int64_t P, int F, const float* sg, const float* tg,
                               const float* sx, const float* tx, const float* wpsi, const float* dq, void* ds,
                               float* dwpsi, float* dbpsi, int accumulate, float* workspace, int dtype,
                               void* stream) {
  if (F % 8 != 0 || !pow2(F / 8) || F / 8 > 64 || F > 2048) return (int)hipErrorInvalidValue;
  int nblk = (int)((P + TILE - 1) / TILE);
  if (nblk == 0) return 0;
  if (nblk > MAXB) nblk = MAXB;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (g_attn)
      hipLaunchKernelGGL((psi_bwd_u_kernel<T, 4>), dim3(nblk), dim3(256), 0, st, (const T*)ug, (const T*)ux, P, F, sg,
                         tg, sx, tx, wpsi, dq, (T*)ds, workspace);
    else
      hipLaunchKernelGGL((psi_bwd_kernel<T>), dim3(nblk), dim3(256), 0, st, (const T*)ug, (const T*)ux, P, F, sg, tg,
                         sx, tx, wpsi, dq, (T*)ds, workspace);
  })
  hipLaunchKernelGGL(part_final, dim3((F + 1 + 31) / 32), dim3(COLSUM_THREADS), 0, st, workspace, nblk, F + 1, dwpsi, F, dbpsi,
                     accumulate);
  return (int)hipGetLastError();
}

extern "C" int vu_pointwise_fwd(const void* x, int64_t xs, int64_t P, int C, int J, const float* w, const float* b,
                                float* y, int64_t ys, int dtype, void* stream) {
  if (C % 8 != 0 || xs % 8 != 0 || J < 1 || J > 4 || !pow2(C / 8 > 64 ? 64 : C / 8)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (P == 0) return 0;
  DISPATCH_T(dtype, {
    if (J <= 2 && C <= 512)
      hipLaunchKernelGGL((pw_fwd_kernel<T, false, 2>), dim3(ew_grid(P * 8)), dim3(256), 0, st, (const T*)x, xs, P, C, J,
                         w, b, y, ys);
    else
      hipLaunchKernelGGL((pw_fwd_kernel<T>), dim3(ew_grid(P * 8)), dim3(256), 0, st, (const T*)x, xs, P, C, J, w, b, y,
                         ys);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_pointwise_bn_fwd(const void* x, int64_t xs, int64_t P, int C, int J, const float* bn_scale,
                                   const float* bn_shift, const float* w, const float* b, float* y, int64_t ys,
                                   int dtype, void* stream) {
  if (C % 8 != 0 || xs % 8 != 0 || J < 1 || J > 4 || C > 512 || !pow2(C / 8) || !bn_scale || !bn_shift)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (P == 0) return 0;
  DISPATCH_T(dtype, {
    if (J <= 2)
      hipLaunchKernelGGL((pw_fwd_kernel<T, true, 2>), dim3(ew_grid(P * 8)), dim3(256), 0, st, (const T*)x, xs, P, C, J,
                         w, b, y, ys, bn_scale, bn_shift);
    else
      hipLaunchKernelGGL((pw_fwd_kernel<T, true>), dim3(ew_grid(P * 8)), dim3(256), 0, st, (const T*)x, xs, P, C, J, w,
                         b, y, ys, bn_scale, bn_shift);
  })
  return (int)hipGetLastError();
}

extern "C" int64_t vu_pointwise_bn_bwd_blocks(int64_t P) {
  const int64_t nb = (P + TILE - 1) / TILE;
  return nb < MAXB ? nb : MAXB;
}

extern "C" int vu_pointwise_bn_bwd(const void* x, int64_t xs, const float* bn_coef, int64_t coef_stride,
                                   const float* dy, int64_t dys, int64_t P, int C, int J, const float* w, void* dx,
                                   int64_t dxs, float* dw, float* db, int accumulate, float* workspace, float* bnb,
                                   int dtype, void* stream) {
  if (C % 8 != 0 || xs % 8 || dxs % 8 || J < 1 || J > 4 || !pow2(C / 8) || C / 8 > 32 || !bn_coef || !bnb ||
      coef_stride < C)
    return (int)hipErrorInvalidValue;
  int nblk = (int)vu_pointwise_bn_bwd_blocks(P);
  if (nblk == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (J <= 2)
      hipLaunchKernelGGL((pw_bwd_kernel<T, true, 2>), dim3(nblk), dim3(256), 0, st, (const T*)x, xs, dy, dys, P, C, J,
                         w, (T*)dx, dxs, workspace, bn_coef, bn_coef + coef_stride, bn_coef + 2 * coef_stride,
                         bn_coef + 3 * coef_stride, bnb);
    else
      hipLaunchKernelGGL((pw_bwd_kernel<T, true>), dim3(nblk), dim3(256), 0, st, (const T*)x, xs, dy, dys, P, C, J, w,
                         (T*)dx, dxs, workspace, bn_coef, bn_coef + coef_stride, bn_coef + 2 * coef_stride,
                         bn_coef + 3 * coef_stride, bnb);
  })
  hipLaunchKernelGGL(part_final, dim3((J * C + J + 31) / 32), dim3(COLSUM_THREADS), 0, st, workspace, nblk, J * C + J, dw,
                     J * C, db, accumulate);
  return (int)hipGetLastError();
}

extern "C" int64_t vu_pointwise_bwd_workspace_bytes(int64_t P, int C, int J) {
  int64_t nb = (P + TILE - 1) / TILE;
  return (nb < MAXB ? nb : MAXB) * (int64_t)(J * C + J) * (int64_t)sizeof(float);
}

extern "C" int vu_pointwise_bwd(const void* x, int64_t xs, const float* dy, int64_t dys, int64_t P, int C, int J,
                                const float* w, void* dx, int64_t dxs, float* dw, float* db, int accumulate,
                                float* workspace, int dtype, void* stream) {
  if (C % 8 != 0 || xs % 8 || dxs % 8 || J < 1 || J > 4 || !pow2(C / 8) || C / 8 > 32)
    return (int)hipErrorInvalidValue;
  int nblk = (int)((P + TILE - 1) / TILE);
  if (nblk == 0) return 0;
  if (nblk > MAXB) nblk = MAXB;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (J <= 2)
      hipLaunchKernelGGL((pw_bwd_kernel<T, false, 2>), dim3(nblk), dim3(256), 0, st, (const T*)x, xs, dy, dys, P, C, J,
                         w, (T*)dx, dxs, workspace);
    else
      hipLaunchKernelGGL((pw_bwd_kernel<T>), dim3(nblk), dim3(256), 0, st, (const T*)x, xs, dy, dys, P, C, J, w,
                         (T*)dx, dxs, workspace);
  })
  hipLaunchKernelGGL(part_final, dim3((J * C + J + 31) / 32), dim3(COLSUM_THREADS), 0, st, workspace, nblk, J * C + J, dw, J * C,
                     db, accumulate);
  return (int)hipGetLastError();
}
