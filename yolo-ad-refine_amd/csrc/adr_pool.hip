// Pooling / resampling kernels on NHWC views, forward and backward (gather form, deterministic).
//   * max pool k x k, stride 1, pad k/2 (SPPF, block.py:177-196): first maximum in row-major window order,
//     as PyTorch's CPU kernel picks it, so gradients route to the same element.
//   * axis means (row means over W, column means over H) and the separable gate
//     out = x * a_h[n,h,c] * a_w[n,w,c]  (ELA_HSFPN block.py:1418-1424; CoordAtt head.py:689-707).
//   * adaptive average pooling, any in/out size (MLCA block.py:1558-1581; CrossScaleAttentionTSSA :2455).
//   * bilinear resize, align_corners=False (CrossScaleAttentionTSSA block.py:2459-2462).
//   * nearest upsample by an integer factor (nn.Upsample(None, 2, 'nearest') rows of yolo11.yaml).
#include "adr_common.h"
#include <initializer_list>

namespace adr {

__device__ __forceinline__ int ad_start(int o, int in, int out) { return (int)(((long)o * in) / out); }
__device__ __forceinline__ int ad_end(int o, int in, int out) { return (int)(((long)(o + 1) * in + out - 1) / out); }

// ---- max pool (stride 1) ----
template <typename T, int VW>
__global__ void __launch_bounds__(256) maxpool_kernel(const T* x, int xcs, T* y, int ycs, uint8_t* arg, int N, int H,
                                                      int W, int C, int k) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  const int p = k / 2;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    float best[VW];
    int bi[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      best[e] = -INFINITY;
      bi[e] = 0;
    }
    for (int dy = 0; dy < k; ++dy) {
      const int ih = h - p + dy;
      if (ih < 0 || ih >= H) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int iw = w - p + dx;
        if (iw < 0 || iw >= W) continue;
        float v[VW];
        vload<T, VW>(x + (((long)n * H + ih) * W + iw) * xcs + c0, v);
#pragma unroll
        for (int e = 0; e < VW; ++e)
          if (v[e] > best[e] || isnan(v[e])) {
            best[e] = v[e];
            bi[e] = dy * k + dx;
          }
      }
    }
    vstore<T, VW>(y + pix * ycs + c0, best);
#pragma unroll
    for (int e = 0; e < VW; ++e) arg[pix * C + c0 + e] = (uint8_t)bi[e];
  }
}

template <typename T, int VW>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const T* dy, int dcs, const uint8_t* arg, T* dx, int ocs,
                                                          int N, int H, int W, int C, int k, int accumulate) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  const int p = k / 2;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    // outputs (oh, ow) whose window contains (h, w): oh in [h-p, h+p]
    for (int oh = h - p; oh <= h + p; ++oh) {
      if (oh < 0 || oh >= H) continue;
      const int dyy = h - (oh - p);
      for (int ow = w - p; ow <= w + p; ++ow) {
        if (ow < 0 || ow >= W) continue;
        const int want = dyy * k + (w - (ow - p));
        const long o = ((long)n * H + oh) * W + ow;
        float g[VW];
        vload<T, VW>(dy + o * dcs + c0, g);
#pragma unroll
        for (int e = 0; e < VW; ++e)
          if (arg[o * C + c0 + e] == want) s[e] += g[e];
      }
    }
    vstore_acc<T, VW>(dx + pix * ocs + c0, s, accumulate);
  }
}

// ---- axis means: blocks [0, H) -> row means, [H, H+W) -> column means; threads = channel groups x line splits,
// fixed-order LDS combine ----
template <typename T, int VW>
__global__ void __launch_bounds__(256) axis_mean_kernel(const T* x, int xcs, int N, int H, int W, int C, T* oh,
                                                        long ohn, T* ow, long own) {
  __shared__ float red[256 * VW];
  const int n = blockIdx.y, b = blockIdx.x;
  const bool row = b < H;
  const int idx = row ? b : b - H;
  const int L = row ? W : H;
  const int G = C / VW;
  for (int cb = 0; cb < G; cb += 256) {
    const int gn = min(256, G - cb), S = 256 / gn;
    const int cg = cb + threadIdx.x % gn, sp = threadIdx.x / gn;
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    if (sp < S)
      for (int j = sp; j < L; j += S) {
        const int hh = row ? idx : j, ww = row ? j : idx;
        float v[VW];
        vload<T, VW>(x + (((long)n * H + hh) * W + ww) * xcs + cg * VW, v);
#pragma unroll
        for (int e = 0; e < VW; ++e) s[e] += v[e];
      }
#pragma unroll
    for (int e = 0; e < VW; ++e) red[threadIdx.x * VW + e] = s[e];
    __syncthreads();
    if (threadIdx.x < gn) {
      float t[VW];
#pragma unroll
      for (int e = 0; e < VW; ++e) t[e] = 0.f;
      for (int q = 0; q < S; ++q)
#pragma unroll
        for (int e = 0; e < VW; ++e) t[e] += red[(q * gn + threadIdx.x) * VW + e];
#pragma unroll
      for (int e = 0; e < VW; ++e) t[e] /= (float)L;
      T* dst = row ? oh + n * ohn + (long)idx * C : ow + n * own + (long)idx * C;
      vstore<T, VW>(dst + cg * VW, t);
    }
    __syncthreads();
  }
}

template <typename T, int VW>
__global__ void __launch_bounds__(256) axis_mean_bwd_kernel(const T* dh, long dhn, const T* dw, long dwn, T* dx,
                                                            int ocs, int N, int H, int W, int C, int accumulate) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  const float iw = 1.f / (float)W, ih = 1.f / (float)H;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    float a[VW], b[VW];
    vload<T, VW>(dh + n * dhn + (long)h * C + c0, a);
    vload<T, VW>(dw + n * dwn + (long)w * C + c0, b);
#pragma unroll
    for (int e = 0; e < VW; ++e) a[e] = a[e] * iw + b[e] * ih;
    vstore_acc<T, VW>(dx + pix * ocs + c0, a, accumulate);
  }
}

// ---- separable gate: out = (x ? x : 1) * ah[n,h,c] * aw[n,w,c] ----
template <typename T, int VW>
__global__ void __launch_bounds__(256) gate_kernel(const T* x, int xcs, const T* ah, long ahn, const T* aw, long awn,
                                                   T* o, int ocs, int N, int H, int W, int C) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    float a[VW], b[VW];
    vload<T, VW>(ah + n * ahn + (long)h * C + c0, a);
    vload<T, VW>(aw + n * awn + (long)w * C + c0, b);
#pragma unroll
    for (int e = 0; e < VW; ++e) a[e] *= b[e];
    if (x) {
      float v[VW];
      vload<T, VW>(x + pix * xcs + c0, v);
#pragma unroll
      for (int e = 0; e < VW; ++e) a[e] *= v[e];
    }
    vstore<T, VW>(o + pix * ocs + c0, a);
  }
}

// gate backward: blocks [0,H): dah[n,h,c] = sum_w dout*x*aw ; [H,H+W): daw[n,w,c] = sum_h dout*x*ah
template <typename T, int VW>
__global__ void __launch_bounds__(256) gate_bwd_reduce_kernel(const T* x, int xcs, const T* ah, long ahn, const T* aw,
                                                              long awn, const T* dout, int dcs, T* dah, long dahn,
                                                              T* daw, long dawn, int N, int H, int W, int C,
                                                              int zero_other) {
  __shared__ float red[256 * VW];
  const int n = blockIdx.y, b = blockIdx.x;
  const bool row = b < H;
  const int idx = row ? b : b - H;
  const int L = row ? W : H;
  const int G = C / VW;
  for (int cb = 0; cb < G; cb += 256) {
    const int gn = min(256, G - cb), S = 256 / gn;
    const int cg = cb + threadIdx.x % gn, sp = threadIdx.x / gn, c0 = cg * VW;
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    if (sp < S)
      for (int j = sp; j < L; j += S) {
        const int hh = row ? idx : j, ww = row ? j : idx;
        const long pix = ((long)n * H + hh) * W + ww;
        float d[VW], o[VW];
        vload<T, VW>(dout + pix * dcs + c0, d);
        if (row) vload<T, VW>(aw + n * awn + (long)ww * C + c0, o);
        else vload<T, VW>(ah + n * ahn + (long)hh * C + c0, o);
        if (x) {
          float v[VW];
          vload<T, VW>(x + pix * xcs + c0, v);
#pragma unroll
          for (int e = 0; e < VW; ++e) o[e] *= v[e];
        }
#pragma unroll
        for (int e = 0; e < VW; ++e) s[e] += d[e] * o[e];
      }
#pragma unroll
    for (int e = 0; e < VW; ++e) red[threadIdx.x * VW + e] = s[e];
    __syncthreads();
    if (threadIdx.x < gn) {
      float t[VW];
#pragma unroll
      for (int e = 0; e < VW; ++e) t[e] = 0.f;
      for (int q = 0; q < S; ++q)
#pragma unroll
        for (int e = 0; e < VW; ++e) t[e] += red[(q * gn + threadIdx.x) * VW + e];
      T* dst = row ? dah + n * dahn + (long)idx * C : daw + n * dawn + (long)idx * C;
      vstore<T, VW>(dst + c0, t);
      if (zero_other) {  // coord layout: row b of the other (H + W)-row gradient is unused by the gate: zero it
        float z[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) z[e] = 0.f;
        T* oth = row ? daw + n * dawn + (long)(idx - H) * C : dah + n * dahn + (long)(idx + H) * C;
        vstore<T, VW>(oth + c0, z);
      }
    }
    __syncthreads();
  }
}

template <typename T, int VW>
__global__ void __launch_bounds__(256) gate_bwd_x_kernel(const T* ah, long ahn, const T* aw, long awn, const T* dout,
                                                         int dcs, T* dx, int ocs, int N, int H, int W, int C,
                                                         int accumulate) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    float a[VW], b[VW], d[VW];
    vload<T, VW>(ah + n * ahn + (long)h * C + c0, a);
    vload<T, VW>(aw + n * awn + (long)w * C + c0, b);
    vload<T, VW>(dout + pix * dcs + c0, d);
#pragma unroll
    for (int e = 0; e < VW; ++e) d[e] *= a[e] * b[e];
    vstore_acc<T, VW>(dx + pix * ocs + c0, d, accumulate);
  }
}

// ---- adaptive average pool ----
template <typename T, int VW>
__global__ void __launch_bounds__(256) adapool_kernel(const T* x, int xcs, int N, int H, int W, int C, T* y, int ycs,
                                                      int OH, int OW) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * OH * OW;
  POOL_LOOP(L, npix, G) {
    int n, oh, ow;
    pix_nhw(pix, OH, OW, n, oh, ow);
    const int c0 = cg * VW;
    const int hs = ad_start(oh, H, OH), he = ad_end(oh, H, OH), ws = ad_start(ow, W, OW), we = ad_end(ow, W, OW);
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) {
        float v[VW];
        vload<T, VW>(x + (((long)n * H + h) * W + w) * xcs + c0, v);
#pragma unroll
        for (int e = 0; e < VW; ++e) s[e] += v[e];
      }
    const float inv = 1.f / (float)((he - hs) * (we - ws));
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] *= inv;
    vstore<T, VW>(y + pix * ycs + c0, s);
  }
}

template <typename T, int VW>
__global__ void __launch_bounds__(256) adapool_bwd_kernel(const T* dy, int dcs, int N, int H, int W, int C, T* dx,
                                                          int ocs, int OH, int OW, int accumulate) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    // candidate output rows: those whose [start, end) contains h
    int oh0 = (int)(((long)h * OH) / H) - 1, oh1 = (int)(((long)(h + 1) * OH + H - 1) / H) + 1;
    int ow0 = (int)(((long)w * OW) / W) - 1, ow1 = (int)(((long)(w + 1) * OW + W - 1) / W) + 1;
    if (oh0 < 0) oh0 = 0;
    if (ow0 < 0) ow0 = 0;
    if (oh1 > OH) oh1 = OH;
    if (ow1 > OW) ow1 = OW;
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    for (int oh = oh0; oh < oh1; ++oh) {
      const int hs = ad_start(oh, H, OH), he = ad_end(oh, H, OH);
      if (h < hs || h >= he) continue;
      for (int ow = ow0; ow < ow1; ++ow) {
        const int ws = ad_start(ow, W, OW), we = ad_end(ow, W, OW);
        if (w < ws || w >= we) continue;
        float g[VW];
        vload<T, VW>(dy + (((long)n * OH + oh) * OW + ow) * dcs + c0, g);
        const float cnt = (float)((he - hs) * (we - ws));
#pragma unroll
        for (int e = 0; e < VW; ++e) s[e] += g[e] / cnt;
      }
    }
    vstore_acc<T, VW>(dx + pix * ocs + c0, s, accumulate);
  }
}

// ---- bilinear resize, align_corners=False (PyTorch upsample_bilinear2d semantics) ----
__device__ __forceinline__ void bl_src(int o, int in, int out, int& i0, int& i1, float& l1) {
  float scale = (float)in / (float)out;
  float src = ((float)o + 0.5f) * scale - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
}

template <typename T, int VW>
__global__ void __launch_bounds__(256) bilinear_kernel(const T* x, int xcs, int N, int H, int W, int C, T* y, int ycs,
                                                       int OH, int OW) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * OH * OW;
  POOL_LOOP(L, npix, G) {
    int n, oh, ow;
    pix_nhw(pix, OH, OW, n, oh, ow);
    const int c0 = cg * VW;
    int h0, h1, w0, w1;
    float lh, lw;
    bl_src(oh, H, OH, h0, h1, lh);
    bl_src(ow, W, OW, w0, w1, lw);
    const T* b = x + (long)n * H * W * xcs + c0;
    float a00[VW], a01[VW], a10[VW], a11[VW];
    vload<T, VW>(b + ((long)h0 * W + w0) * xcs, a00);
    vload<T, VW>(b + ((long)h0 * W + w1) * xcs, a01);
    vload<T, VW>(b + ((long)h1 * W + w0) * xcs, a10);
    vload<T, VW>(b + ((long)h1 * W + w1) * xcs, a11);
#pragma unroll
    for (int e = 0; e < VW; ++e)
      a00[e] = (1.f - lh) * ((1.f - lw) * a00[e] + lw * a01[e]) + lh * ((1.f - lw) * a10[e] + lw * a11[e]);
    vstore<T, VW>(y + pix * ycs + c0, a00);
  }
}

template <typename T, int VW>
__global__ void __launch_bounds__(256) bilinear_bwd_kernel(const T* dy, int dcs, int N, int H, int W, int C, T* dx,
                                                           int ocs, int OH, int OW, int accumulate) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    // outputs whose source taps may include (h, w): oh in a window around (h + 0.5) * OH / H
    const int rh = OH / H + 2, rw = OW / W + 2;
    const int ohc = (int)(((float)h + 0.5f) * (float)OH / (float)H);
    const int owc = (int)(((float)w + 0.5f) * (float)OW / (float)W);
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    for (int oh = max(0, ohc - rh); oh < min(OH, ohc + rh + 1); ++oh) {
      int h0, h1;
      float lh;
      bl_src(oh, H, OH, h0, h1, lh);
      const float wh = (h0 == h ? 1.f - lh : 0.f) + (h1 == h ? lh : 0.f);
      if (wh == 0.f) continue;
      for (int ow = max(0, owc - rw); ow < min(OW, owc + rw + 1); ++ow) {
        int w0, w1;
        float lw;
        bl_src(ow, W, OW, w0, w1, lw);
        const float ww = (w0 == w ? 1.f - lw : 0.f) + (w1 == w ? lw : 0.f);
        if (ww == 0.f) continue;
        float g[VW];
        vload<T, VW>(dy + (((long)n * OH + oh) * OW + ow) * dcs + c0, g);
#pragma unroll
        for (int e = 0; e < VW; ++e) s[e] += wh * ww * g[e];
      }
    }
    vstore_acc<T, VW>(dx + pix * ocs + c0, s, accumulate);
  }
}

// ---- nearest upsample, integer factor s ----
template <typename T, int VW>
__global__ void __launch_bounds__(256) upsample_nearest_kernel(const T* x, int xcs, int N, int H, int W, int C, T* y,
                                                               int ycs, int s) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const int OH = H * s, OW = W * s;
  const long npix = (long)N * OH * OW;
  POOL_LOOP(L, npix, G) {
    int n, oh, ow;
    pix_nhw(pix, OH, OW, n, oh, ow);
    const int c0 = cg * VW;
    float v[VW];
    vload<T, VW>(x + (((long)n * H + oh / s) * W + ow / s) * xcs + c0, v);
    vstore<T, VW>(y + pix * ycs + c0, v);
  }
}

template <typename T, int VW>
__global__ void __launch_bounds__(256) upsample_nearest_bwd_kernel(const T* dy, int dcs, int N, int H, int W, int C,
                                                                   T* dx, int ocs, int s, int accumulate) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const int OH = H * s, OW = W * s;
  const long npix = (long)N * H * W;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    float acc[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) acc[e] = 0.f;
    for (int a = 0; a < s; ++a)
      for (int b = 0; b < s; ++b) {
        float g[VW];
        vload<T, VW>(dy + (((long)n * OH + h * s + a) * OW + w * s + b) * dcs + c0, g);
#pragma unroll
        for (int e = 0; e < VW; ++e) acc[e] += g[e];
      }
    vstore_acc<T, VW>(dx + pix * ocs + c0, acc, accumulate);
  }
}

}  // namespace adr

using namespace adr;

// Kernels run with VW = 16 / sizeof(T) channels per thread when C, every channel / image stride and every
// pointer allow 16-byte accesses, else VW = 1. Grid: one block per (256 / G) pixels, capped.
static bool vec_ok(int C, int vw, std::initializer_list<long> strides, std::initializer_list<const void*> ptrs) {
  if (C % vw) return false;
  for (long s : strides)
    if (s % vw) return false;
  for (const void* p : ptrs)
    if ((uintptr_t)p % 16) return false;
  return true;
}
static dim3 pool_grid(long npix, int G) {
  const long rpb = G <= 256 ? 256 / G : 1;
  long b = (npix + rpb - 1) / rpb;
  if (b > 65536) b = 65536;
  return dim3((unsigned)(b < 1 ? 1 : b));
}

#define P(t, x) ((t*)(x))
#define VW_OF(dtype) ((dtype) == ADR_BF16 ? 8 : 4)
#define GOF(dtype, vec, C) ((C) / ((vec) ? VW_OF(dtype) : 1))

extern "C" int adr_maxpool(int dtype, const void* x, int xcs, void* y, int ycs, uint8_t* arg, int N, int H, int W,
                           int C, int k, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  ADR_REQUIRE(k % 2 == 1 && k * k <= 255, "maxpool: k=%d", k);
  const bool v = vec_ok(C, VW_OF(dtype), {xcs, ycs}, {x, y});
  const dim3 g = pool_grid((long)N * H * W, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((maxpool_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, x), xcs, P(__bf16, y), ycs, arg, N, H, W, C, k);
    else hipLaunchKernelGGL((maxpool_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, x), xcs, P(__bf16, y), ycs, arg, N, H, W, C, k);
  } else {
    if (v) hipLaunchKernelGGL((maxpool_kernel<float, 4>), g, dim3(256), 0, st, P(const float, x), xcs, P(float, y), ycs, arg, N, H, W, C, k);
    else hipLaunchKernelGGL((maxpool_kernel<float, 1>), g, dim3(256), 0, st, P(const float, x), xcs, P(float, y), ycs, arg, N, H, W, C, k);
  }
  return check_launch("adr_maxpool");
}

extern "C" int adr_maxpool_bwd(int dtype, const void* dy, int dcs, const uint8_t* arg, void* dx, int ocs, int N, int H,
                               int W, int C, int k, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {dcs, ocs}, {dy, dx});
  const dim3 g = pool_grid((long)N * H * W, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((maxpool_bwd_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, dy), dcs, arg, P(__bf16, dx), ocs, N, H, W, C, k, accumulate);
    else hipLaunchKernelGGL((maxpool_bwd_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, dy), dcs, arg, P(__bf16, dx), ocs, N, H, W, C, k, accumulate);
  } else {
    if (v) hipLaunchKernelGGL((maxpool_bwd_kernel<float, 4>), g, dim3(256), 0, st, P(const float, dy), dcs, arg, P(float, dx), ocs, N, H, W, C, k, accumulate);
    else hipLaunchKernelGGL((maxpool_bwd_kernel<float, 1>), g, dim3(256), 0, st, P(const float, dy), dcs, arg, P(float, dx), ocs, N, H, W, C, k, accumulate);
  }
  return check_launch("adr_maxpool_bwd");
}

extern "C" int adr_axis_mean(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* oh, long ohn,
                             void* ow, long own, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {xcs, ohn, own}, {x, oh, ow});
  const dim3 g = dim3(H + W, N);
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((axis_mean_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, oh), ohn, P(__bf16, ow), own);
    else hipLaunchKernelGGL((axis_mean_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, oh), ohn, P(__bf16, ow), own);
  } else {
    if (v) hipLaunchKernelGGL((axis_mean_kernel<float, 4>), g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, oh), ohn, P(float, ow), own);
    else hipLaunchKernelGGL((axis_mean_kernel<float, 1>), g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, oh), ohn, P(float, ow), own);
  }
  return check_launch("adr_axis_mean");
}

extern "C" int adr_axis_mean_bwd(int dtype, const void* dh, long dhn, const void* dw, long dwn, void* dx, int ocs,
                                 int N, int H, int W, int C, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {dhn, dwn, ocs}, {dh, dw, dx});
  const dim3 g = pool_grid((long)N * H * W, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((axis_mean_bwd_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, dh), dhn, P(const __bf16, dw), dwn, P(__bf16, dx), ocs, N, H, W, C, accumulate);
    else hipLaunchKernelGGL((axis_mean_bwd_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, dh), dhn, P(const __bf16, dw), dwn, P(__bf16, dx), ocs, N, H, W, C, accumulate);
  } else {
    if (v) hipLaunchKernelGGL((axis_mean_bwd_kernel<float, 4>), g, dim3(256), 0, st, P(const float, dh), dhn, P(const float, dw), dwn, P(float, dx), ocs, N, H, W, C, accumulate);
    else hipLaunchKernelGGL((axis_mean_bwd_kernel<float, 1>), g, dim3(256), 0, st, P(const float, dh), dhn, P(const float, dw), dwn, P(float, dx), ocs, N, H, W, C, accumulate);
  }
  return check_launch("adr_axis_mean_bwd");
}

extern "C" int adr_gate(int dtype, const void* x, int xcs, const void* ah, long ahn, const void* aw, long awn, void* o,
                        int ocs, int N, int H, int W, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {xcs, ahn, awn, ocs}, {x, ah, aw, o});
  const dim3 g = pool_grid((long)N * H * W, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((gate_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, x), xcs, P(const __bf16, ah), ahn, P(const __bf16, aw), awn, P(__bf16, o), ocs, N, H, W, C);
    else hipLaunchKernelGGL((gate_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, x), xcs, P(const __bf16, ah), ahn, P(const __bf16, aw), awn, P(__bf16, o), ocs, N, H, W, C);
  } else {
    if (v) hipLaunchKernelGGL((gate_kernel<float, 4>), g, dim3(256), 0, st, P(const float, x), xcs, P(const float, ah), ahn, P(const float, aw), awn, P(float, o), ocs, N, H, W, C);
    else hipLaunchKernelGGL((gate_kernel<float, 1>), g, dim3(256), 0, st, P(const float, x), xcs, P(const float, ah), ahn, P(const float, aw), awn, P(float, o), ocs, N, H, W, C);
  }
  return check_launch("adr_gate");
}

extern "C" int adr_gate_bwd(int dtype, const void* x, int xcs, const void* ah, long ahn, const void* aw, long awn,
                            const void* dout, int dcs, void* dx, int ocs, void* dah, long dahn, void* daw, long dawn,
                            int N, int H, int W, int C, int accumulate, int zero_other, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {xcs, ahn, awn, dcs, ocs, dahn, dawn}, {x, ah, aw, dout, dx, dah, daw});
  const dim3 g = dim3(H + W, N);
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((gate_bwd_reduce_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, x), xcs, P(const __bf16, ah), ahn, P(const __bf16, aw), awn, P(const __bf16, dout), dcs, P(__bf16, dah), dahn, P(__bf16, daw), dawn, N, H, W, C, zero_other);
    else hipLaunchKernelGGL((gate_bwd_reduce_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, x), xcs, P(const __bf16, ah), ahn, P(const __bf16, aw), awn, P(const __bf16, dout), dcs, P(__bf16, dah), dahn, P(__bf16, daw), dawn, N, H, W, C, zero_other);
  } else {
    if (v) hipLaunchKernelGGL((gate_bwd_reduce_kernel<float, 4>), g, dim3(256), 0, st, P(const float, x), xcs, P(const float, ah), ahn, P(const float, aw), awn, P(const float, dout), dcs, P(float, dah), dahn, P(float, daw), dawn, N, H, W, C, zero_other);
    else hipLaunchKernelGGL((gate_bwd_reduce_kernel<float, 1>), g, dim3(256), 0, st, P(const float, x), xcs, P(const float, ah), ahn, P(const float, aw), awn, P(const float, dout), dcs, P(float, dah), dahn, P(float, daw), dawn, N, H, W, C, zero_other);
  }
  int rc = check_launch("adr_gate_bwd(reduce)");
  if (rc || !dx) return rc;
  {
  const dim3 g = pool_grid((long)N * H * W, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((gate_bwd_x_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, ah), ahn, P(const __bf16, aw), awn, P(const __bf16, dout), dcs, P(__bf16, dx), ocs, N, H, W, C, accumulate);
    else hipLaunchKernelGGL((gate_bwd_x_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, ah), ahn, P(const __bf16, aw), awn, P(const __bf16, dout), dcs, P(__bf16, dx), ocs, N, H, W, C, accumulate);
  } else {
    if (v) hipLaunchKernelGGL((gate_bwd_x_kernel<float, 4>), g, dim3(256), 0, st, P(const float, ah), ahn, P(const float, aw), awn, P(const float, dout), dcs, P(float, dx), ocs, N, H, W, C, accumulate);
    else hipLaunchKernelGGL((gate_bwd_x_kernel<float, 1>), g, dim3(256), 0, st, P(const float, ah), ahn, P(const float, aw), awn, P(const float, dout), dcs, P(float, dx), ocs, N, H, W, C, accumulate);
  }
  }
  return check_launch("adr_gate_bwd");
}

extern "C" int adr_adapool(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* y, int ycs, int OH,
                           int OW, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {xcs, ycs}, {x, y});
  const dim3 g = pool_grid((long)N * OH * OW, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((adapool_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, y), ycs, OH, OW);
    else hipLaunchKernelGGL((adapool_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, y), ycs, OH, OW);
  } else {
    if (v) hipLaunchKernelGGL((adapool_kernel<float, 4>), g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, y), ycs, OH, OW);
    else hipLaunchKernelGGL((adapool_kernel<float, 1>), g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, y), ycs, OH, OW);
  }
  return check_launch("adr_adapool");
}

extern "C" int adr_adapool_bwd(int dtype, const void* dy, int dcs, int N, int H, int W, int C, void* dx, int ocs,
                               int OH, int OW, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {dcs, ocs}, {dy, dx});
  const dim3 g = pool_grid((long)N * H * W, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((adapool_bwd_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, dy), dcs, N, H, W, C, P(__bf16, dx), ocs, OH, OW, accumulate);
    else hipLaunchKernelGGL((adapool_bwd_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, dy), dcs, N, H, W, C, P(__bf16, dx), ocs, OH, OW, accumulate);
  } else {
    if (v) hipLaunchKernelGGL((adapool_bwd_kernel<float, 4>), g, dim3(256), 0, st, P(const float, dy), dcs, N, H, W, C, P(float, dx), ocs, OH, OW, accumulate);
    else hipLaunchKernelGGL((adapool_bwd_kernel<float, 1>), g, dim3(256), 0, st, P(const float, dy), dcs, N, H, W, C, P(float, dx), ocs, OH, OW, accumulate);
  }
  return check_launch("adr_adapool_bwd");
}

extern "C" int adr_bilinear(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* y, int ycs, int OH,
                            int OW, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {xcs, ycs}, {x, y});
  const dim3 g = pool_grid((long)N * OH * OW, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((bilinear_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, y), ycs, OH, OW);
    else hipLaunchKernelGGL((bilinear_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, y), ycs, OH, OW);
  } else {
    if (v) hipLaunchKernelGGL((bilinear_kernel<float, 4>), g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, y), ycs, OH, OW);
    else hipLaunchKernelGGL((bilinear_kernel<float, 1>), g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, y), ycs, OH, OW);
  }
  return check_launch("adr_bilinear");
}

extern "C" int adr_bilinear_bwd(int dtype, const void* dy, int dcs, int N, int H, int W, int C, void* dx, int ocs,
                                int OH, int OW, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v = vec_ok(C, VW_OF(dtype), {dcs, ocs}, {dy, dx});
  const dim3 g = pool_grid((long)N * H * W, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((bilinear_bwd_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, dy), dcs, N, H, W, C, P(__bf16, dx), ocs, OH, OW, accumulate);
    else hipLaunchKernelGGL((bilinear_bwd_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, dy), dcs, N, H, W, C, P(__bf16, dx), ocs, OH, OW, accumulate);
  } else {
    if (v) hipLaunchKernelGGL((bilinear_bwd_kernel<float, 4>), g, dim3(256), 0, st, P(const float, dy), dcs, N, H, W, C, P(float, dx), ocs, OH, OW, accumulate);
    else hipLaunchKernelGGL((bilinear_bwd_kernel<float, 1>), g, dim3(256), 0, st, P(const float, dy), dcs, N, H, W, C, P(float, dx), ocs, OH, OW, accumulate);
  }
  return check_launch("adr_bilinear_bwd");
}

extern "C" int adr_upsample_nearest(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* y, int ycs,
                                    int s, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  ADR_REQUIRE(s >= 1 && s <= 8, "upsample_nearest: factor %d", s);
  const bool v = vec_ok(C, VW_OF(dtype), {xcs, ycs}, {x, y});
  const dim3 g = pool_grid((long)N * H * W * s * s, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((upsample_nearest_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, y), ycs, s);
    else hipLaunchKernelGGL((upsample_nearest_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, y), ycs, s);
  } else {
    if (v) hipLaunchKernelGGL((upsample_nearest_kernel<float, 4>), g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, y), ycs, s);
    else hipLaunchKernelGGL((upsample_nearest_kernel<float, 1>), g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, y), ycs, s);
  }
  return check_launch("adr_upsample_nearest");
}

extern "C" int adr_upsample_nearest_bwd(int dtype, const void* dy, int dcs, int N, int H, int W, int C, void* dx,
                                        int ocs, int s, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  ADR_REQUIRE(s >= 1 && s <= 8, "upsample_nearest_bwd: factor %d", s);
  const bool v = vec_ok(C, VW_OF(dtype), {dcs, ocs}, {dy, dx});
  const dim3 g = pool_grid((long)N * H * W, GOF(dtype, v, C));
  if (dtype == ADR_BF16) {
    if (v) hipLaunchKernelGGL((upsample_nearest_bwd_kernel<__bf16, 8>), g, dim3(256), 0, st, P(const __bf16, dy), dcs, N, H, W, C, P(__bf16, dx), ocs, s, accumulate);
    else hipLaunchKernelGGL((upsample_nearest_bwd_kernel<__bf16, 1>), g, dim3(256), 0, st, P(const __bf16, dy), dcs, N, H, W, C, P(__bf16, dx), ocs, s, accumulate);
  } else {
    if (v) hipLaunchKernelGGL((upsample_nearest_bwd_kernel<float, 4>), g, dim3(256), 0, st, P(const float, dy), dcs, N, H, W, C, P(float, dx), ocs, s, accumulate);
    else hipLaunchKernelGGL((upsample_nearest_bwd_kernel<float, 1>), g, dim3(256), 0, st, P(const float, dy), dcs, N, H, W, C, P(float, dx), ocs, s, accumulate);
  }
  return check_launch("adr_upsample_nearest_bwd");
}
