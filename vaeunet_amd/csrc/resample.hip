// Max-pool 2x2 (Down, unet_parts.py:57), bilinear align_corners=True
// upsampling (Up bilinear :73, DecoderBlock :79/93, UNetResNet :238) with the
// F.pad of unet_parts.py:85-89 folded into the output placement, and the
// layout / cast helpers (input packing, weight permutes, strided copies).
//
// All NHWC, 8 channels (16 B bf16 / 32 B fp32) per thread where the channel
// count allows, grid-stride loops.  Backward passes are gathers (each output
// element written exactly once, no atomics) so results are deterministic.
#include "common.h"
#include "../../include/vaeunet.h"

namespace {

inline unsigned ew_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// ------------------------------ max pool --------------------------------
// PyTorch CPU/GPU max_pool2d scan: window row-major, update when
// (v > best || isnan(v)): ties keep the FIRST max.
template <typename T, int VW>
__global__ void maxpool_fwd_kernel(const T* x, int64_t xs, int N, int H, int W, int C, T* y, int64_t ys) {
  int Ho = H >> 1, Wo = W >> 1, V = C / VW;
  int64_t tot = (int64_t)N * Ho * Wo * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t q = e / V;
    int c = (int)(e - q * V) * VW;
    int j = (int)(q % Wo);
    int64_t t = q / Wo;
    int i = (int)(t % Ho);
    int n = (int)(t / Ho);
    float best[VW];
#pragma unroll
    for (int k = 0; k < VW; ++k) best[k] = -INFINITY;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const T* src = x + (((int64_t)n * H + 2 * i + a) * W + 2 * j + b) * xs + c;
        if (VW == 8) {
          Vec8<T> v; v.load(src);
#pragma unroll
          for (int k = 0; k < VW; ++k) { float f = v.get(k); if (f > best[k] || isnan(f)) best[k] = f; }
        } else {
          float f = ld1<T>(src); if (f > best[0] || isnan(f)) best[0] = f;
        }
      }
    T* dst = y + q * ys + c;
    if (VW == 8) { Vec8<T> v; for (int k = 0; k < 8; ++k) v.set(k, best[k]); v.store(dst); }
    else st1<T>(dst, best[0]);
  }
}

template <typename T, int VW, bool NT>
__global__ void maxpool_bwd_kernel(const T* x, int64_t xs, const T* dy, int64_t dys, int N, int H, int W, int C,
                                   T* dx, int64_t dxs, const T* add, int64_t adds) {
  int Ho = H >> 1, Wo = W >> 1, V = C / VW;
  int64_t tot = (int64_t)N * Ho * Wo * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t q = e / V;
    int c = (int)(e - q * V) * VW;
    int j = (int)(q % Wo);
    int64_t t = q / Wo;
    int i = (int)(t % Ho);
    int n = (int)(t / Ho);
    float best[VW];
    int arg[VW];
    float vals[4][VW], g[VW], o[4][VW];
    // every load of the window (4 x, dy, 4 skip-gradient rows) is issued
    // before any is used; all of them are last uses (NT: non-temporal)
    if (VW == 8) {
      Vec8<T> vx[4], vg, va[4];
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        const int64_t pix = ((int64_t)n * H + 2 * i + (ab >> 1)) * W + 2 * j + (ab & 1);
        if (NT) vx[ab].load_nt(x + pix * xs + c); else vx[ab].load(x + pix * xs + c);
        if (add) { if (NT) va[ab].load_nt(add + pix * adds + c); else va[ab].load(add + pix * adds + c); }
      }
      if (NT) vg.load_nt(dy + q * dys + c); else vg.load(dy + q * dys + c);
#pragma unroll
      for (int ab = 0; ab < 4; ++ab)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          vals[ab][k] = vx[ab].get(k);
          o[ab][k] = add ? va[ab].get(k) : 0.f;
        }
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = vg.get(k);
    } else {
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        const int64_t pix = ((int64_t)n * H + 2 * i + (ab >> 1)) * W + 2 * j + (ab & 1);
        vals[ab][0] = ld1<T>(x + pix * xs + c);
        o[ab][0] = add ? ld1<T>(add + pix * adds + c) : 0.f;
      }
      g[0] = ld1<T>(dy + q * dys + c);
    }
#pragma unroll
    for (int k = 0; k < VW; ++k) { best[k] = -INFINITY; arg[k] = 0; }
#pragma unroll
    for (int ab = 0; ab < 4; ++ab)
#pragma unroll
      for (int k = 0; k < VW; ++k) {
        float f = vals[ab][k];
        if (f > best[k] || isnan(f)) { best[k] = f; arg[k] = ab; }
      }
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) {
      const int64_t pix = ((int64_t)n * H + 2 * i + (ab >> 1)) * W + 2 * j + (ab & 1);
#pragma unroll
      for (int k = 0; k < VW; ++k) if (arg[k] == ab) o[ab][k] += g[k];
      if (VW == 8) { Vec8<T> v; for (int k = 0; k < 8; ++k) v.set(k, o[ab][k]); v.store(dx + pix * dxs + c); }
      else st1<T>(dx + pix * dxs + c, o[ab][0]);
    }
  }
}

// rows/cols of an odd-sized input that no window covers: dx = add (or 0)
template <typename T>
__global__ void maxpool_bwd_border(int N, int H, int W, int C, T* dx, int64_t dxs, const T* add, int64_t adds) {
  int Ho = H >> 1, Wo = W >> 1;
  int64_t tot = (int64_t)N * H * W * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(e % C);
    int64_t pix = e / C;
    int w = (int)(pix % W), h = (int)((pix / W) % H);
    if (h < 2 * Ho && w < 2 * Wo) continue;
    st1<T>(dx + pix * dxs + c, add ? ld1<T>(add + pix * adds + c) : 0.f);
  }
}

// ---------------------------- bilinear (align_corners) ------------------
VU_DEV float ac_scale(int in, int out) { return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f; }

VU_DEV void ac_src(int o, float scale, int in, int& i0, int& i1, float& l1) {
  float src = scale * (float)o;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

template <typename T, int VW>
__global__ void upsample_fwd_kernel(const T* x, int64_t xs, int N, int Hi, int Wi, int C, T* y, int64_t ys,
                                    int Ho, int Wo, int Hp, int Wp, int py, int px) {
  float sh = ac_scale(Hi, Ho), sw = ac_scale(Wi, Wo);
  int V = C / VW;
  int64_t tot = (int64_t)N * Hp * Wp * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t q = e / V;
    int c = (int)(e - q * V) * VW;
    int X = (int)(q % Wp);
    int64_t t = q / Wp;
    int Y = (int)(t % Hp);
    int n = (int)(t / Hp);
    int oy = Y - py, ox = X - px;
    float o[VW];
#pragma unroll
    for (int k = 0; k < VW; ++k) o[k] = 0.f;
    if (oy >= 0 && oy < Ho && ox >= 0 && ox < Wo) {
      int y0, y1, x0, x1; float ly, lx;
      ac_src(oy, sh, Hi, y0, y1, ly);
      ac_src(ox, sw, Wi, x0, x1, lx);
      float hy = 1.f - ly, hx = 1.f - lx;
      const T* b = x + (int64_t)n * Hi * Wi * xs + c;
      const T* p00 = b + ((int64_t)y0 * Wi + x0) * xs;
      const T* p01 = b + ((int64_t)y0 * Wi + x1) * xs;
      const T* p10 = b + ((int64_t)y1 * Wi + x0) * xs;
      const T* p11 = b + ((int64_t)y1 * Wi + x1) * xs;
      if (VW == 8) {
        Vec8<T> a, bb, cc, d;
        a.load(p00); bb.load(p01); cc.load(p10); d.load(p11);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          o[k] = hy * (hx * a.get(k) + lx * bb.get(k)) + ly * (hx * cc.get(k) + lx * d.get(k));
      } else {
        o[0] = hy * (hx * ld1<T>(p00) + lx * ld1<T>(p01)) + ly * (hx * ld1<T>(p10) + lx * ld1<T>(p11));
      }
    }
    T* dst = y + q * ys + c;
    if (VW == 8) { Vec8<T> v; for (int k = 0; k < 8; ++k) v.set(k, o[k]); v.store(dst); }
    else st1<T>(dst, o[0]);
  }
}

// weight of input index i in output index o (both terms of the stencil)
VU_DEV float ac_w(int o, int i, float scale, int in) {
  int i0, i1; float l1;
  ac_src(o, scale, in, i0, i1, l1);
  float w = 0.f;
  if (i0 == i) w += 1.f - l1;
  if (i1 == i) w += l1;
  return w;
}

VU_DEV void ac_range(int i, float scale, int in, int out, int& lo, int& hi) {
  if (scale == 0.f) { lo = 0; hi = (i == 0) ? out - 1 : -1; return; }
  float a = (float)(i - 1) / scale, b = (float)(i + 1) / scale;
  lo = (int)floorf(a) - 1; hi = (int)ceilf(b) + 1;
  if (lo < 0) lo = 0;
  if (hi > out - 1) hi = out - 1;
}

template <typename T, int VW>
__global__ void upsample_bwd_kernel(const T* dy, int64_t dys, int N, int Hi, int Wi, int C, T* dx, int64_t dxs,
                                    int Ho, int Wo, int Hp, int Wp, int py, int px, int accumulate) {
  float sh = ac_scale(Hi, Ho), sw = ac_scale(Wi, Wo);
  int V = C / VW;
  int64_t tot = (int64_t)N * Hi * Wi * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t q = e / V;
    int c = (int)(e - q * V) * VW;
    int j = (int)(q % Wi);
    int64_t t = q / Wi;
    int i = (int)(t % Hi);
    int n = (int)(t / Hi);
    int ylo, yhi, xlo, xhi;
    ac_range(i, sh, Hi, Ho, ylo, yhi);
    ac_range(j, sw, Wi, Wo, xlo, xhi);
    float o[VW];
#pragma unroll
    for (int k = 0; k < VW; ++k) o[k] = 0.f;
    if constexpr (VW == 8) {
      // the contributing output rows / columns (<= 4 each for the 2x
      // upsampling) collected first, then all their loads issued together and
      // summed in the same (row, column) order as the loop below, which
      // issued one load per memory round trip
      // (static slots filled by selects: a dynamically indexed array was
      // placed in LDS by the compiler)
      int yv[4] = {0, 0, 0, 0}, xv[4] = {0, 0, 0, 0};
      float wyv[4] = {0.f, 0.f, 0.f, 0.f}, wxv[4] = {0.f, 0.f, 0.f, 0.f};
      int ny = 0, nx = 0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int yy = ylo + r;
        const float wy = yy <= yhi ? ac_w(yy, i, sh, Hi) : 0.f;
        const bool ok = wy != 0.f && yy + py >= 0 && yy + py < Hp;
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (ok && ny == t) { yv[t] = yy; wyv[t] = wy; }
        ny += ok ? 1 : 0;
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int xx = xlo + r;
        const float wx = xx <= xhi ? ac_w(xx, j, sw, Wi) : 0.f;
        const bool ok = wx != 0.f && xx + px >= 0 && xx + px < Wp;
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (ok && nx == t) { xv[t] = xx; wxv[t] = wx; }
        nx += ok ? 1 : 0;
      }
      if (ny <= 4 && nx <= 4 && yhi - ylo < 8 && xhi - xlo < 8) {
        Vec8<T> v[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            // slots past the counts re-load slot 0's pixel (in range: clamped
            // to row / column py, px when there is no contributor at all)
            const int yy = a < ny ? yv[a] : (ny > 0 ? yv[0] : -py);
            const int xx = b < nx ? xv[b] : (nx > 0 ? xv[0] : -px);
            v[a][b].load(dy + (((int64_t)n * Hp + yy + py) * Wp + xx + px) * dys + c);
          }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            if (a >= ny || b >= nx) continue;
            const float wgt = wyv[a] * wxv[b];
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] += wgt * v[a][b].get(k);
          }
        T* dst = dx + q * dxs + c;
        Vec8<T> w8;
        if (accumulate) { w8.load(dst); for (int k = 0; k < 8; ++k) o[k] += w8.get(k); }
        for (int k = 0; k < 8; ++k) w8.set(k, o[k]);
        w8.store(dst);
        continue;
      }
    }
    for (int yy = ylo; yy <= yhi; ++yy) {
      float wy = ac_w(yy, i, sh, Hi);
      if (wy == 0.f) continue;
      if (yy + py < 0 || yy + py >= Hp) continue;  // cropped by a negative F.pad
      for (int xx = xlo; xx <= xhi; ++xx) {
        float wx = ac_w(xx, j, sw, Wi);
        if (wx == 0.f || xx + px < 0 || xx + px >= Wp) continue;
        const T* src = dy + (((int64_t)n * Hp + yy + py) * Wp + xx + px) * dys + c;
        float wgt = wy * wx;
        if (VW == 8) {
          Vec8<T> v; v.load(src);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += wgt * v.get(k);
        } else o[0] += wgt * ld1<T>(src);
      }
    }
    T* dst = dx + q * dxs + c;
    if (VW == 8) {
      Vec8<T> v;
      if (accumulate) { v.load(dst); for (int k = 0; k < 8; ++k) o[k] += v.get(k); }
      for (int k = 0; k < 8; ++k) v.set(k, o[k]);
      v.store(dst);
    } else {
      if (accumulate) o[0] += ld1<T>(dst);
      st1<T>(dst, o[0]);
    }
  }
}

// ------------------------------ layout helpers ---------------------------
template <typename TO>
__global__ void permute4_kernel(const float* in, int64_t base, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                                int d0, int d1, int d2, int d3, int d3v, TO* out) {
  int64_t tot = (int64_t)d0 * d1 * d2 * d3;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = e;
    int i3 = (int)(r % d3); r /= d3;
    int i2 = (int)(r % d2); r /= d2;
    int i1 = (int)(r % d1);
    int i0 = (int)(r / d1);
    st1<TO>(out + e, i3 < d3v ? in[base + i0 * s0 + i1 * s1 + i2 * s2 + i3 * s3] : 0.f);
  }
}

template <typename TI, typename TO>
__global__ void copy_kernel(const TI* x, int64_t xs, TO* y, int64_t ys, int64_t P, int C, int accumulate) {
  int64_t tot = P * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = e / C;
    int c = (int)(e - p * C);
    float v = ld1<TI>(x + p * xs + c);
    TO* d = y + p * ys + c;
    st1<TO>(d, accumulate ? v + ld1<TO>(d) : v);
  }
}

template <typename T>
__global__ void copy8_kernel(const T* x, int64_t xs, T* y, int64_t ys, int64_t P, int C, int accumulate) {
  int V = C >> 3;
  int64_t tot = P * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = e / V;
    int c = (int)(e - p * V) * 8;
    Vec8<T> v;
    v.load(x + p * xs + c);
    if (accumulate) {
      Vec8<T> w; w.load(y + p * ys + c);
      for (int k = 0; k < 8; ++k) v.set(k, v.get(k) + w.get(k));
    }
    v.store(y + p * ys + c);
  }
}

template <typename TO>
__global__ void input_pack_kernel(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int N, int C,
                                  int H, int W, int Cp, TO* y) {
  int64_t tot = (int64_t)N * H * W * Cp;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(e % Cp);
    int64_t pix = e / Cp;
    int w = (int)(pix % W);
    int64_t t = pix / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    float v = c < C ? x[n * sn + c * sc + h * sh + w * sw] : 0.f;
    st1<TO>(y + e, v);
  }
}

// The 8-channel packing of the image (Cp == 8, C <= 8, N*H*W < 2^31): one
// thread per pixel, the pixel decoded by multiply-shift, its C source values
// loaded together and the 8 output channels written as ONE 16-byte (bf16) /
// 32-byte (fp32) store.  The element-per-thread form above spent two 64-bit
// divisions per output element: 52 us for the 512^2 batch-8 image (1.1 TB/s).
template <typename TO>
__global__ __launch_bounds__(256) void input_pack8_kernel(const float* x, int64_t sn, int64_t sc, int64_t sh,
                                                          int64_t sw, int P, int C, int H, int W, TO* y) {
  const FastDiv div_hw((uint32_t)(H * W)), div_w((uint32_t)W);
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    const int n = (int)div_hw.div((uint32_t)p);
    const int rem = p - n * H * W;
    const int h = (int)div_w.div((uint32_t)rem), w = rem - h * W;
    const float* px = x + n * sn + h * sh + w * sw;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = px[(c < C ? c : C - 1) * sc];  // unguarded: loads issue together
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = c < C ? v[c] : 0.f;
    Vec8<TO> o;
#pragma unroll
    for (int c = 0; c < 8; ++c) o.set(c, v[c]);
    o.store(y + (int64_t)p * 8);
  }
}

// The common case of the packing: a dense NHWC 3-channel fp32 image (the
// channels_last input batch).  A lane takes 4 pixels = 48 contiguous bytes
// (three 16-byte loads) and writes their 4 x 8 channels contiguously: no
// pixel decode, no 12-byte-strided scalar loads.
template <typename TO>
__global__ __launch_bounds__(256) void input_pack3x4_kernel(const float* x, int64_t Q, TO* y) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < Q; q += (int64_t)gridDim.x * blockDim.x) {
    const f32x4* s = reinterpret_cast<const f32x4*>(x + q * 12);
    const f32x4 a = s[0], b = s[1], c = s[2];
    const float v[12] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3], c[0], c[1], c[2], c[3]};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      Vec8<TO> o;
      o.zero();
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) o.set(ch, v[3 * k + ch]);
      o.store(y + (q * 4 + k) * 8);
    }
  }
}

}  // namespace

#define DISPATCH_T(dtype, ...) \
  if ((dtype) == VU_BF16) { using T = bf16_t; __VA_ARGS__; } else { using T = float; __VA_ARGS__; }

extern "C" int vu_maxpool2_fwd(const void* x, int64_t xs, int N, int H, int W, int C, void* y, int64_t ys,
                               int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int64_t work = (int64_t)N * (H / 2) * (W / 2) * C;
  if (work == 0) return 0;
  bool vec = C % 8 == 0 && xs % 8 == 0 && ys % 8 == 0;
  DISPATCH_T(dtype, {
    if (vec) hipLaunchKernelGGL((maxpool_fwd_kernel<T, 8>), dim3(ew_grid(work / 8)), dim3(256), 0, st,
                                (const T*)x, xs, N, H, W, C, (T*)y, ys);
    else hipLaunchKernelGGL((maxpool_fwd_kernel<T, 1>), dim3(ew_grid(work)), dim3(256), 0, st,
                            (const T*)x, xs, N, H, W, C, (T*)y, ys);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_maxpool2_bwd(const void* x, int64_t xs, const void* dy, int64_t dys, int N, int H, int W, int C,
                               void* dx, int64_t dxs, const void* add, int64_t adds, int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int64_t work = (int64_t)N * (H / 2) * (W / 2) * C;
  bool vec = C % 8 == 0 && xs % 8 == 0 && dys % 8 == 0 && dxs % 8 == 0 && (!add || adds % 8 == 0);
  DISPATCH_T(dtype, {
    if (work > 0) {
      // non-temporal loads once the input no longer fits beside the stream
      // in the Infinity Cache (the BN streams' 32 MB rule, bn.hip)
      const bool nt = (int64_t)N * H * W * C * (int64_t)sizeof(T) >= 32000000;
      if (vec && nt)
        hipLaunchKernelGGL((maxpool_bwd_kernel<T, 8, true>), dim3(ew_grid(work / 8)), dim3(256), 0, st,
                           (const T*)x, xs, (const T*)dy, dys, N, H, W, C, (T*)dx, dxs, (const T*)add, adds);
      else if (vec)
        hipLaunchKernelGGL((maxpool_bwd_kernel<T, 8, false>), dim3(ew_grid(work / 8)), dim3(256), 0, st,
                           (const T*)x, xs, (const T*)dy, dys, N, H, W, C, (T*)dx, dxs, (const T*)add, adds);
      else hipLaunchKernelGGL((maxpool_bwd_kernel<T, 1, false>), dim3(ew_grid(work)), dim3(256), 0, st,
                              (const T*)x, xs, (const T*)dy, dys, N, H, W, C, (T*)dx, dxs, (const T*)add, adds);
    }
    if ((H & 1) || (W & 1))
      hipLaunchKernelGGL((maxpool_bwd_border<T>), dim3(ew_grid((int64_t)N * H * W * C)), dim3(256), 0, st,
                         N, H, W, C, (T*)dx, dxs, (const T*)add, adds);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_upsample_fwd(const void* x, int64_t xs, int N, int Hi, int Wi, int C, void* y, int64_t ys,
                               int Ho, int Wo, int Hp, int Wp, int py, int px, int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int64_t work = (int64_t)N * Hp * Wp * C;
  if (work == 0) return 0;
  bool vec = C % 8 == 0 && xs % 8 == 0 && ys % 8 == 0;
  DISPATCH_T(dtype, {
    if (vec) hipLaunchKernelGGL((upsample_fwd_kernel<T, 8>), dim3(ew_grid(work / 8)), dim3(256), 0, st,
                                (const T*)x, xs, N, Hi, Wi, C, (T*)y, ys, Ho, Wo, Hp, Wp, py, px);
    else hipLaunchKernelGGL((upsample_fwd_kernel<T, 1>), dim3(ew_grid(work)), dim3(256), 0, st,
                            (const T*)x, xs, N, Hi, Wi, C, (T*)y, ys, Ho, Wo, Hp, Wp, py, px);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_upsample_bwd(const void* dy, int64_t dys, int N, int Hi, int Wi, int C, void* dx, int64_t dxs,
                               int Ho, int Wo, int Hp, int Wp, int py, int px, int accumulate, int dtype,
                               void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int64_t work = (int64_t)N * Hi * Wi * C;
  if (work == 0) return 0;
  bool vec = C % 8 == 0 && dys % 8 == 0 && dxs % 8 == 0;
  DISPATCH_T(dtype, {
    if (vec) hipLaunchKernelGGL((upsample_bwd_kernel<T, 8>), dim3(ew_grid(work / 8)), dim3(256), 0, st,
                                (const T*)dy, dys, N, Hi, Wi, C, (T*)dx, dxs, Ho, Wo, Hp, Wp, py, px, accumulate);
    else hipLaunchKernelGGL((upsample_bwd_kernel<T, 1>), dim3(ew_grid(work)), dim3(256), 0, st,
                            (const T*)dy, dys, N, Hi, Wi, C, (T*)dx, dxs, Ho, Wo, Hp, Wp, py, px, accumulate);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_permute4(const float* in, int64_t base, int64_t s0, int64_t s1, int64_t s2, int64_t s3, int d0,
                           int d1, int d2, int d3, int d3v, void* out, int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int64_t tot = (int64_t)d0 * d1 * d2 * d3;
  if (tot == 0) return 0;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((permute4_kernel<T>), dim3(ew_grid(tot)), dim3(256), 0, st, in, base, s0, s1, s2, s3, d0, d1,
                       d2, d3, d3v, (T*)out);
  })
  return (int)hipGetLastError();
}

// Batched vu_permute4: every derived weight layout of a training step in one
// launch (the per-step rebuild of the bf16 GEMM weight images after the
// optimizer step, engine.py weight caches).  A job whose output-fastest dim
// (3) is not the input-fastest one (e.g. the flipped [ci][tap][co] input-
// gradient images: co is the slowest input dim) is a batched 2-D transpose:
// 32x32 tiles through LDS, coalesced reads along the input-fast dim q and
// coalesced writes along dim 3 (PERM_TILE x PERM_TILE tiles).  Other jobs are streamed PERM_CHUNK elements
// per block.  chunk0 is the prefix block count (binary search per block).
namespace {
constexpr int PERM_CHUNK = 4096, PERM_TILE = 64;
// global-address-space views of the job pointers (read from a device table:
// through generic pointers the loads are flat instructions, which count in
// lgkmcnt and so wait behind / hold up the tile transposes' LDS traffic)
typedef __attribute__((address_space(1))) float gfl;
typedef __attribute__((address_space(1))) bf16_t gbf;
typedef __attribute__((address_space(1))) u32x2 gu32x2;
typedef __attribute__((address_space(1))) f32x4 gf32x4;

template <int T, typename Put>
__device__ __forceinline__ void tap_tile(const VuPermJob& j, const gfl* in, const int* d, const int* st,
                                         uint32_t blk, float* big, Put put) {
  const int sT = st[2];
  const bool run0 = j.s0 == (int64_t)T * (sT < 0 ? -sT : sT);   // dim 0 pairs with the taps
  const uint32_t t3n = (d[3] + 31) / 32;
  const int a0 = (int)(blk / t3n) * 32, b0 = (int)(blk - (blk / t3n) * t3n) * 32;
  constexpr int n = 32 * T * 32;
  for (int e = threadIdx.x; e < n; e += 256) {
    const int t = e % T, r = e / T;
    const int x = r & 31, y = r >> 5;                 // x: the run dim, y: the other
    const int a = run0 ? x : y, bb = run0 ? y : x;    // (dim 0, dim 3) offsets in the tile
    float v = 0.f;
    if (a0 + a < d[0] && b0 + bb < d[3] && b0 + bb < j.d3v) v = in[(a0 + a) * st[0] + t * sT + (b0 + bb) * st[3]];
    big[(a * T + t) * 33 + bb] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += 256) {
    const int bb = e & 31, r = e >> 5;                // r = a * T + t
    const int a = r / T;
    if (a0 + a >= d[0] || b0 + bb >= d[3]) continue;
    put(((uint32_t)(a0 + a) * T + (r - a * T)) * d[3] + b0 + bb, big[r * 33 + bb]);
  }
}

__global__ __launch_bounds__(256) void permute4_batch_kernel(const VuPermJob* jobs, int n) {
  __shared__ float tile[PERM_TILE][PERM_TILE + 1];
  const int64_t chunk = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].chunk0 <= chunk) lo = mid; else hi = mid - 1;
  }
  const VuPermJob& j = jobs[lo];
  // 32-bit index math (every weight image has < 2^31 elements)
  const int d[4] = {j.d0, j.d1, j.d2, j.d3};
  const int st[4] = {(int)j.s0, (int)j.s1, (int)j.s2, (int)j.s3};
  const gfl* in = (const gfl*)(j.in + j.base);
  const uint32_t blk = (uint32_t)(chunk - j.chunk0);
  auto put = [&](uint32_t e, float v) {
    if (j.dtype == VU_BF16) ((gbf*)j.out)[e] = f2bf(v);
    else ((gfl*)j.out)[e] = v;
  };
  if (j.q == 5) {
    // the input is row-major in the output's dim order (the forward image of a
    // channels_last weight: [co][kh][kw][ci] on both sides): a converting
    // copy, 4 elements per thread, no index arithmetic
    const uint32_t tot = (uint32_t)d[0] * d[1] * d[2] * d[3];
    const uint32_t e0 = blk * PERM_CHUNK;
    const uint32_t e1 = e0 + PERM_CHUNK < tot ? e0 + PERM_CHUNK : tot;
    for (uint32_t e = e0 + 4 * threadIdx.x; e < e1; e += 4 * blockDim.x) {
      if (e + 4 <= e1 && ((uintptr_t)(in + e) & 15) == 0) {
        const f32x4 v = *(const gf32x4*)(in + e);
        if (j.dtype == VU_BF16) {
          u32x2 o;
          o[0] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          o[1] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          *(gu32x2*)((gbf*)j.out + e) = o;
        } else {
          *(gf32x4*)((gfl*)j.out + e) = v;
        }
      } else {
        for (uint32_t k = e; k < e + 4 && k < e1; ++k) put(k, in[k]);
      }
    }
    return;
  }
  if (j.q >= 3) {
    const uint32_t d1 = d[1], d2 = d[2], d3 = d[3];
    const uint32_t tot = (uint32_t)d[0] * d1 * d2 * d3;
    const uint32_t e0 = blk * PERM_CHUNK;
    const uint32_t e1 = e0 + PERM_CHUNK < tot ? e0 + PERM_CHUNK : tot;
    for (uint32_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
      const uint32_t r = e / d3, i3 = e - r * d3;
      const uint32_t r2 = r / d2, i2 = r - r2 * d2;
      const uint32_t i0 = r2 / d1, i1 = r2 - i0 * d1;
      put(e, (int)i3 < j.d3v ? in[(int)i0 * st[0] + (int)i1 * st[1] + (int)i2 * st[2] + (int)i3 * st[3]] : 0.f);
    }
    return;
  }
  // tiled transpose between dim q (input-fast) and dim 3 (output-fast), 64 x
  // 64 tiles: 256-byte fp32 reads and 128-byte bf16 writes per wave row (the
  // 32 x 32 tiles of round 3 wrote half lines and moved 4 KB per block: the
  // step's weight refresh ran at ~2 TB/s)
  constexpr int TT = PERM_TILE;
  const int q = j.q;
  const int a = q == 0 ? 1 : 0, c = q == 2 ? 1 : 2;  // the two batch dims, in order
  const uint32_t tq = (d[q] + TT - 1) / TT, t3 = (d[3] + TT - 1) / TT;
  const uint32_t b = blk / (tq * t3), rem = blk - b * (tq * t3);
  // a caller that sized the job's block range for another tile size: blocks
  // past the job's real tile count do nothing (block-uniform, before the barrier)
  if (b >= (uint32_t)d[a] * (uint32_t)d[c]) return;
  const int iq0 = (int)(rem / t3) * TT, i30 = (int)(rem - (rem / t3) * t3) * TT;
  const int ia = (int)(b / d[c]), ic = (int)(b - (b / d[c]) * d[c]);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const gfl* ib = in + ia * st[a] + ic * st[c];
  float v[TT / 4];
#pragma unroll
  for (int k = 0; k < TT / 4; ++k) {
    const int iq = iq0 + tx, i3 = i30 + ty + 4 * k;
    v[k] = (iq < d[q] && i3 < d[3] && i3 < j.d3v) ? ib[iq * st[q] + i3 * st[3]] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < TT / 4; ++k) tile[ty + 4 * k][tx] = v[k];
  __syncthreads();
  int idx[4];
  idx[a] = ia;
  idx[c] = ic;
#pragma unroll
  for (int k = 0; k < TT / 4; ++k) {
    const int i3 = i30 + tx, iq = iq0 + ty + 4 * k;
    if (iq >= d[q] || i3 >= d[3]) continue;
    idx[q] = iq;
    const uint32_t e = (((uint32_t)idx[0] * d[1] + idx[1]) * d[2] + idx[2]) * d[3] + i3;
    put(e, tile[tx][ty + 4 * k]);
  }
}
// The 3x3 / 2x2 weight images (q = 4, see tap_tile) in a launch of their own:
// the 38 KB tile would cap every block of the generic kernel at 4 per CU
// (the first round-4 version, one kernel for all jobs, ran the refresh in
// 287 us instead of 156).
__global__ __launch_bounds__(256) void permute4_tap_kernel(const VuPermJob* jobs, int n) {
  __shared__ float big[32 * 9 * 33];
  const int64_t chunk = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].chunk0 <= chunk) lo = mid; else hi = mid - 1;
  }
  const VuPermJob& j = jobs[lo];
  const int d[4] = {j.d0, j.d1, j.d2, j.d3};
  const int st[4] = {(int)j.s0, (int)j.s1, (int)j.s2, (int)j.s3};
  const gfl* in = (const gfl*)(j.in + j.base);
  const uint32_t blk = (uint32_t)(chunk - j.chunk0);
  auto put = [&](uint32_t e, float v) {
    if (j.dtype == VU_BF16) ((gbf*)j.out)[e] = f2bf(v);
    else ((gfl*)j.out)[e] = v;
  };
  if (d[1] * d[2] == 9) tap_tile<9>(j, in, d, st, blk, big, put);
  else tap_tile<4>(j, in, d, st, blk, big, put);
}
}  // namespace

extern "C" int64_t vu_permute4_chunk(void) { return PERM_CHUNK; }
extern "C" int64_t vu_permute4_tile(void) { return PERM_TILE; }

extern "C" int vu_permute4_batch2(const VuPermJob* jobs, int njobs, int ntap, int64_t tap_blocks,
                                  int64_t rest_blocks, void* stream) {
  if (njobs < 0 || ntap < 0 || ntap > njobs) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (ntap > 0 && tap_blocks > 0)
    hipLaunchKernelGGL(permute4_tap_kernel, dim3((unsigned)tap_blocks), dim3(256), 0, st, jobs, ntap);
  if (njobs > ntap && rest_blocks > 0)
    hipLaunchKernelGGL(permute4_batch_kernel, dim3((unsigned)rest_blocks), dim3(256), 0, st, jobs + ntap,
                       njobs - ntap);
  return (int)hipGetLastError();
}

extern "C" int vu_permute4_batch(const VuPermJob* jobs, int njobs, int64_t nchunks, void* stream) {
  if (njobs <= 0 || nchunks <= 0) return 0;
  hipLaunchKernelGGL(permute4_batch_kernel, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, jobs, njobs);
  return (int)hipGetLastError();
}

namespace {
__global__ void zero_kernel(char* y, int64_t ys_bytes, int64_t P, int row_bytes) {
  // 4-byte words of each pixel's channel run (row_bytes % 4 == 0)
  const int wpr = row_bytes >> 2;
  const int64_t tot = P * wpr;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = e / wpr;
    reinterpret_cast<uint32_t*>(y + p * ys_bytes)[e - p * wpr] = 0u;
  }
}
}  // namespace

// y[p][0..C) = 0 for P pixels at pixel stride ys (a channel slice of an NHWC
// tensor: the zero channels a 64-aligned concat source is padded with)
// one wave sleeping ~rounds x 3.4 us (s_sleep 127 = 127 x 64 clocks): put
// in front of a timed launch (bench.py's roofline leg), it keeps the queue
// busy while the host enqueues the start event, the launch and the end
// event, so the event pair brackets the kernel and not the host's enqueue
// time.  No memory access.
namespace {
__global__ void delay_kernel(int rounds) {
  for (int i = 0; i < rounds; ++i) __builtin_amdgcn_s_sleep(127);
}
}  // namespace

extern "C" int vu_gpu_delay(int rounds, void* stream) {
  if (rounds < 0 || rounds > 1000) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, rounds);
  return (int)hipGetLastError();
}

extern "C" int vu_zero(void* y, int64_t ys, int64_t P, int C, int dtype, void* stream) {
  const int eb = dtype == VU_BF16 ? 2 : 4;
  if ((C * eb) % 4 != 0) return (int)hipErrorInvalidValue;
  const int64_t tot = P * (C * eb / 4);
  if (tot == 0) return 0;
  hipLaunchKernelGGL(zero_kernel, dim3(ew_grid(tot)), dim3(256), 0, (hipStream_t)stream, (char*)y, ys * eb, P,
                     C * eb);
  return (int)hipGetLastError();
}

namespace {
// up[n][y][x][c] = (y, x even and (y/2, x/2) inside dy) ? dy[n][y/2][x/2][c] : 0,
// 16-byte vectors, one pixel row of 8-channel groups per lane group
template <typename T>
__global__ void zero_insert2_kernel(const T* dy, int64_t dys, int h, int w, T* up, int64_t ups, int H, int W,
                                    int C, int64_t P) {
  const int V = C >> 3;
  const int64_t tot = P * V;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = e / V;
    const int c = (int)(e - p * V) * 8;
    const int x = (int)(p % W);
    const int64_t t = p / W;
    const int y = (int)(t % H);
    const int64_t n = t / H;
    Vec8<T> v;
    if (((x | y) & 1) == 0 && (y >> 1) < h && (x >> 1) < w)
      v.load(dy + ((n * h + (y >> 1)) * w + (x >> 1)) * dys + c);
    else
      v.zero();
    v.store(up + p * ups + c);
  }
}
}  // namespace

// Zero insertion for the input gradient of a stride-2 convolution (the VAE
// encoder's 3x3/s2 convs, unet_resnet.py:131-137 via timm BasicBlock): the
// (H, W) map holding dy (h, w) at the even pixels and zeros elsewhere, so the
// input gradient runs as ONE stride-1 3x3 convolution on the halo kernels
// instead of four small parity-class GEMMs.  C % 8 == 0, strides % 8 == 0.
extern "C" int vu_zero_insert2(const void* dy, int64_t dys, int N, int h, int w, int C, void* up, int64_t ups,
                               int H, int W, int dtype, void* stream) {
  if (C % 8 != 0 || dys % 8 != 0 || ups % 8 != 0 || N < 0 || H < 0 || W < 0) return (int)hipErrorInvalidValue;
  const int64_t P = (int64_t)N * H * W;
  if (P == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((zero_insert2_kernel<T>), dim3(ew_grid(P * (C / 8))), dim3(256), 0, st, (const T*)dy, dys, h,
                       w, (T*)up, ups, H, W, C, P);
  })
  return (int)hipGetLastError();
}

extern "C" int vu_copy(const void* x, int64_t xs, int xdtype, void* y, int64_t ys, int ydtype, int64_t P, int C,
                       int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int64_t tot = P * C;
  if (tot == 0) return 0;
  if (xdtype == ydtype && C % 8 == 0 && xs % 8 == 0 && ys % 8 == 0) {
    DISPATCH_T(xdtype, {
      hipLaunchKernelGGL((copy8_kernel<T>), dim3(ew_grid(tot / 8)), dim3(256), 0, st, (const T*)x, xs, (T*)y, ys, P,
                         C, accumulate);
    })
  } else if (xdtype == VU_BF16) {
    if (ydtype == VU_BF16)
      hipLaunchKernelGGL((copy_kernel<bf16_t, bf16_t>), dim3(ew_grid(tot)), dim3(256), 0, st, (const bf16_t*)x, xs,
                         (bf16_t*)y, ys, P, C, accumulate);
    else
      hipLaunchKernelGGL((copy_kernel<bf16_t, float>), dim3(ew_grid(tot)), dim3(256), 0, st, (const bf16_t*)x, xs,
                         (float*)y, ys, P, C, accumulate);
  } else {
    if (ydtype == VU_BF16)
      hipLaunchKernelGGL((copy_kernel<float, bf16_t>), dim3(ew_grid(tot)), dim3(256), 0, st, (const float*)x, xs,
                         (bf16_t*)y, ys, P, C, accumulate);
    else
      hipLaunchKernelGGL((copy_kernel<float, float>), dim3(ew_grid(tot)), dim3(256), 0, st, (const float*)x, xs,
                         (float*)y, ys, P, C, accumulate);
  }
  return (int)hipGetLastError();
}

extern "C" int vu_input_pack(const float* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int N, int C, int H,
                             int W, int Cp, void* y, int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int64_t tot = (int64_t)N * H * W * Cp;
  if (tot == 0) return 0;
  const int64_t P = (int64_t)N * H * W;
  if (Cp == 8 && C == 3 && sc == 1 && sw == 3 && sh == 3 * (int64_t)W && sn == 3 * (int64_t)H * W && P % 4 == 0 &&
      ((uintptr_t)x & 15) == 0) {
    DISPATCH_T(dtype, {
      hipLaunchKernelGGL((input_pack3x4_kernel<T>), dim3(ew_grid(P / 4)), dim3(256), 0, st, x, P / 4, (T*)y);
    })
    return (int)hipGetLastError();
  }
  if (Cp == 8 && C >= 1 && C <= 8 && P < ((int64_t)1 << 31) && (int64_t)H * W < ((int64_t)1 << 31)) {
    DISPATCH_T(dtype, {
      hipLaunchKernelGGL((input_pack8_kernel<T>), dim3(ew_grid(P)), dim3(256), 0, st, x, sn, sc, sh, sw, (int)P, C,
                         H, W, (T*)y);
    })
    return (int)hipGetLastError();
  }
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((input_pack_kernel<T>), dim3(ew_grid(tot)), dim3(256), 0, st, x, sn, sc, sh, sw, N, C, H, W,
                       Cp, (T*)y);
  })
  return (int)hipGetLastError();
}
