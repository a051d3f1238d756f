// Pooling / resampling kernels on NHWC views, forward and backward (gather form, deterministic).
//   * max pool k x k, stride 1, pad k/2 (SPPF, block.py:177-196): first maximum in row-major window order,
//     as PyTorch's CPU kernel picks it, so gradients route to the same element.
//   * axis means (row means over W, column means over H) and the separable gate
//     out = x * a_h[n,h,c] * a_w[n,w,c]  (ELA_HSFPN block.py:1418-1424; CoordAtt head.py:689-707).
//   * adaptive average pooling, any in/out size (MLCA block.py:1558-1581; CrossScaleAttentionTSSA :2455).
//   * bilinear resize, align_corners=False (CrossScaleAttentionTSSA block.py:2459-2462).
#include "adr_common.h"

namespace adr {

__device__ __forceinline__ int ad_start(int o, int in, int out) { return (int)(((long)o * in) / out); }
__device__ __forceinline__ int ad_end(int o, int in, int out) { return (int)(((long)(o + 1) * in + out - 1) / out); }

// ---- max pool (stride 1) ----
template <typename T>
__global__ void __launch_bounds__(256) maxpool_kernel(const T* x, int xcs, T* y, int ycs, uint8_t* arg, int N, int H,
                                                      int W, int C, int k) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  int p = k / 2;
  float best = -INFINITY;
  int bi = 0;
  for (int dy = 0; dy < k; ++dy) {
    int ih = h - p + dy;
    if (ih < 0 || ih >= H) continue;
    for (int dx = 0; dx < k; ++dx) {
      int iw = w - p + dx;
      if (iw < 0 || iw >= W) continue;
      float v = to_f(x[(((long)n * H + ih) * W + iw) * xcs + c]);
      if (v > best || isnan(v)) {
        best = v;
        bi = dy * k + dx;
      }
    }
  }
  y[pix * ycs + c] = from_f<T>(best);
  arg[i] = (uint8_t)bi;
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const T* dy, int dcs, const uint8_t* arg, T* dx, int ocs,
                                                          int N, int H, int W, int C, int k, int accumulate) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  int p = k / 2;
  float s = 0.f;
  // outputs (oh, ow) whose window contains (h, w): oh in [h-p, h+p]
  for (int oh = h - p; oh <= h + p; ++oh) {
    if (oh < 0 || oh >= H) continue;
    int dyy = h - (oh - p);
    for (int ow = w - p; ow <= w + p; ++ow) {
      if (ow < 0 || ow >= W) continue;
      int dxx = w - (ow - p);
      long o = ((long)n * H + oh) * W + ow;
      if (arg[o * C + c] == dyy * k + dxx) s += to_f(dy[o * dcs + c]);
    }
  }
  T* q = dx + pix * ocs + c;
  *q = from_f<T>(accumulate ? to_f(*q) + s : s);
}

// ---- axis means: blocks [0, H) -> row means, [H, H+W) -> column means ----
template <typename T>
__global__ void __launch_bounds__(256) axis_mean_kernel(const T* x, int xcs, int N, int H, int W, int C, T* oh,
                                                        long ohn, T* ow, long own) {
  int n = blockIdx.y, b = blockIdx.x;
  bool row = b < H;
  int idx = row ? b : b - H;
  int L = row ? W : H;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < L; ++j) {
      int hh = row ? idx : j, ww = row ? j : idx;
      s += to_f(x[(((long)n * H + hh) * W + ww) * xcs + c]);
    }
    s /= (float)L;
    if (row) oh[n * ohn + (long)idx * C + c] = from_f<T>(s);
    else ow[n * own + (long)idx * C + c] = from_f<T>(s);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) axis_mean_bwd_kernel(const T* dh, long dhn, const T* dw, long dwn, T* dx,
                                                            int ocs, int N, int H, int W, int C, int accumulate) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  float g = to_f(dh[n * dhn + (long)h * C + c]) / (float)W + to_f(dw[n * dwn + (long)w * C + c]) / (float)H;
  T* q = dx + pix * ocs + c;
  *q = from_f<T>(accumulate ? to_f(*q) + g : g);
}

// ---- separable gate: out = (x ? x : 1) * ah[n,h,c] * aw[n,w,c] ----
template <typename T>
__global__ void __launch_bounds__(256) gate_kernel(const T* x, int xcs, const T* ah, long ahn, const T* aw, long awn,
                                                   T* o, int ocs, int N, int H, int W, int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  float a = to_f(ah[n * ahn + (long)h * C + c]) * to_f(aw[n * awn + (long)w * C + c]);
  float v = x ? to_f(x[pix * xcs + c]) * a : a;
  o[pix * ocs + c] = from_f<T>(v);
}

// gate backward: blocks [0,H): dah[n,h,c] = sum_w dout*x*aw ; [H,H+W): daw[n,w,c] = sum_h dout*x*ah
template <typename T>
__global__ void __launch_bounds__(256) gate_bwd_reduce_kernel(const T* x, int xcs, const T* ah, long ahn, const T* aw,
                                                              long awn, const T* dout, int dcs, T* dah, long dahn,
                                                              T* daw, long dawn, int N, int H, int W, int C) {
  int n = blockIdx.y, b = blockIdx.x;
  bool row = b < H;
  int idx = row ? b : b - H;
  int L = row ? W : H;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < L; ++j) {
      int hh = row ? idx : j, ww = row ? j : idx;
      long pix = ((long)n * H + hh) * W + ww;
      float xv = x ? to_f(x[pix * xcs + c]) : 1.f;
      float other = row ? to_f(aw[n * awn + (long)ww * C + c]) : to_f(ah[n * ahn + (long)hh * C + c]);
      s += to_f(dout[pix * dcs + c]) * xv * other;
    }
    if (row) dah[n * dahn + (long)idx * C + c] = from_f<T>(s);
    else daw[n * dawn + (long)idx * C + c] = from_f<T>(s);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gate_bwd_x_kernel(const T* ah, long ahn, const T* aw, long awn, const T* dout,
                                                         int dcs, T* dx, int ocs, int N, int H, int W, int C,
                                                         int accumulate) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  float g = to_f(dout[pix * dcs + c]) * to_f(ah[n * ahn + (long)h * C + c]) * to_f(aw[n * awn + (long)w * C + c]);
  T* q = dx + pix * ocs + c;
  *q = from_f<T>(accumulate ? to_f(*q) + g : g);
}

// ---- adaptive average pool ----
template <typename T>
__global__ void __launch_bounds__(256) adapool_kernel(const T* x, int xcs, int N, int H, int W, int C, T* y, int ycs,
                                                      int OH, int OW) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * OH * OW * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int ow = (int)(pix % OW);
  long r = pix / OW;
  int oh = (int)(r % OH);
  int n = (int)(r / OH);
  int hs = ad_start(oh, H, OH), he = ad_end(oh, H, OH), ws = ad_start(ow, W, OW), we = ad_end(ow, W, OW);
  float s = 0.f;
  for (int h = hs; h < he; ++h)
    for (int w = ws; w < we; ++w) s += to_f(x[(((long)n * H + h) * W + w) * xcs + c]);
  y[pix * ycs + c] = from_f<T>(s / (float)((he - hs) * (we - ws)));
}

template <typename T>
__global__ void __launch_bounds__(256) adapool_bwd_kernel(const T* dy, int dcs, int N, int H, int W, int C, T* dx,
                                                          int ocs, int OH, int OW, int accumulate) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  // candidate output rows: those whose [start, end) contains h
  int oh0 = (int)(((long)h * OH) / H) - 1, oh1 = (int)(((long)(h + 1) * OH + H - 1) / H) + 1;
  int ow0 = (int)(((long)w * OW) / W) - 1, ow1 = (int)(((long)(w + 1) * OW + W - 1) / W) + 1;
  if (oh0 < 0) oh0 = 0;
  if (ow0 < 0) ow0 = 0;
  if (oh1 > OH) oh1 = OH;
  if (ow1 > OW) ow1 = OW;
  float s = 0.f;
  for (int oh = oh0; oh < oh1; ++oh) {
    int hs = ad_start(oh, H, OH), he = ad_end(oh, H, OH);
    if (h < hs || h >= he) continue;
    for (int ow = ow0; ow < ow1; ++ow) {
      int ws = ad_start(ow, W, OW), we = ad_end(ow, W, OW);
      if (w < ws || w >= we) continue;
      s += to_f(dy[(((long)n * OH + oh) * OW + ow) * dcs + c]) / (float)((he - hs) * (we - ws));
    }
  }
  T* q = dx + pix * ocs + c;
  *q = from_f<T>(accumulate ? to_f(*q) + s : s);
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

template <typename T>
__global__ void __launch_bounds__(256) bilinear_kernel(const T* x, int xcs, int N, int H, int W, int C, T* y, int ycs,
                                                       int OH, int OW) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * OH * OW * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int ow = (int)(pix % OW);
  long r = pix / OW;
  int oh = (int)(r % OH);
  int n = (int)(r / OH);
  int h0, h1, w0, w1;
  float lh, lw;
  bl_src(oh, H, OH, h0, h1, lh);
  bl_src(ow, W, OW, w0, w1, lw);
  const T* b = x + (long)n * H * W * xcs + c;
  float v = (1.f - lh) * ((1.f - lw) * to_f(b[((long)h0 * W + w0) * xcs]) + lw * to_f(b[((long)h0 * W + w1) * xcs])) +
            lh * ((1.f - lw) * to_f(b[((long)h1 * W + w0) * xcs]) + lw * to_f(b[((long)h1 * W + w1) * xcs]));
  y[pix * ycs + c] = from_f<T>(v);
}

template <typename T>
__global__ void __launch_bounds__(256) bilinear_bwd_kernel(const T* dy, int dcs, int N, int H, int W, int C, T* dx,
                                                           int ocs, int OH, int OW, int accumulate) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  // outputs whose source taps may include (h, w): oh in a window around (h + 0.5) * OH / H
  int rh = OH / H + 2, rw = OW / W + 2;
  int ohc = (int)(((float)h + 0.5f) * (float)OH / (float)H);
  int owc = (int)(((float)w + 0.5f) * (float)OW / (float)W);
  float s = 0.f;
  for (int oh = max(0, ohc - rh); oh < min(OH, ohc + rh + 1); ++oh) {
    int h0, h1;
    float lh;
    bl_src(oh, H, OH, h0, h1, lh);
    float wh = (h0 == h ? 1.f - lh : 0.f) + (h1 == h ? lh : 0.f);
    if (wh == 0.f) continue;
    for (int ow = max(0, owc - rw); ow < min(OW, owc + rw + 1); ++ow) {
      int w0, w1;
      float lw;
      bl_src(ow, W, OW, w0, w1, lw);
      float ww = (w0 == w ? 1.f - lw : 0.f) + (w1 == w ? lw : 0.f);
      if (ww == 0.f) continue;
      s += wh * ww * to_f(dy[(((long)n * OH + oh) * OW + ow) * dcs + c]);
    }
  }
  T* q = dx + pix * ocs + c;
  *q = from_f<T>(accumulate ? to_f(*q) + s : s);
}

}  // namespace adr

using namespace adr;

#define DISPATCH(dtype, KERN, grid, ...)                                                                   \
  do {                                                                                                     \
    if ((dtype) == ADR_BF16) hipLaunchKernelGGL(KERN<__bf16>, grid, dim3(256), 0, st, __VA_ARGS__);        \
    else hipLaunchKernelGGL(KERN<float>, grid, dim3(256), 0, st, __VA_ARGS__);                             \
  } while (0)

#define P(t, x) ((t*)(x))

extern "C" int adr_maxpool(int dtype, const void* x, int xcs, void* y, int ycs, uint8_t* arg, int N, int H, int W,
                           int C, int k, void* stream) {
  ADR_REQUIRE(k % 2 == 1 && k * k <= 255, "maxpool: k=%d", k);
  hipStream_t st = (hipStream_t)stream;
  long total = (long)N * H * W * C;
  dim3 g(cdiv(total, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(maxpool_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, x), xcs, P(__bf16, y), ycs, arg, N,
                       H, W, C, k);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, g, dim3(256), 0, st, P(const float, x), xcs, P(float, y), ycs, arg, N, H,
                       W, C, k);
  return check_launch("adr_maxpool");
}

extern "C" int adr_maxpool_bwd(int dtype, const void* dy, int dcs, const uint8_t* arg, void* dx, int ocs, int N, int H,
                               int W, int C, int k, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  long total = (long)N * H * W * C;
  dim3 g(cdiv(total, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, dy), dcs, arg, P(__bf16, dx),
                       ocs, N, H, W, C, k, accumulate);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, g, dim3(256), 0, st, P(const float, dy), dcs, arg, P(float, dx), ocs,
                       N, H, W, C, k, accumulate);
  return check_launch("adr_maxpool_bwd");
}

extern "C" int adr_axis_mean(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* oh, long ohn,
                             void* ow, long own, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(H + W, N);
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(axis_mean_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C,
                       P(__bf16, oh), ohn, P(__bf16, ow), own);
  else
    hipLaunchKernelGGL(axis_mean_kernel<float>, g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, oh),
                       ohn, P(float, ow), own);
  return check_launch("adr_axis_mean");
}

extern "C" int adr_axis_mean_bwd(int dtype, const void* dh, long dhn, const void* dw, long dwn, void* dx, int ocs,
                                 int N, int H, int W, int C, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(cdiv((long)N * H * W * C, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(axis_mean_bwd_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, dh), dhn,
                       P(const __bf16, dw), dwn, P(__bf16, dx), ocs, N, H, W, C, accumulate);
  else
    hipLaunchKernelGGL(axis_mean_bwd_kernel<float>, g, dim3(256), 0, st, P(const float, dh), dhn, P(const float, dw),
                       dwn, P(float, dx), ocs, N, H, W, C, accumulate);
  return check_launch("adr_axis_mean_bwd");
}

extern "C" int adr_gate(int dtype, const void* x, int xcs, const void* ah, long ahn, const void* aw, long awn, void* o,
                        int ocs, int N, int H, int W, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(cdiv((long)N * H * W * C, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(gate_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, x), xcs, P(const __bf16, ah), ahn,
                       P(const __bf16, aw), awn, P(__bf16, o), ocs, N, H, W, C);
  else
    hipLaunchKernelGGL(gate_kernel<float>, g, dim3(256), 0, st, P(const float, x), xcs, P(const float, ah), ahn,
                       P(const float, aw), awn, P(float, o), ocs, N, H, W, C);
  return check_launch("adr_gate");
}

extern "C" int adr_gate_bwd(int dtype, const void* x, int xcs, const void* ah, long ahn, const void* aw, long awn,
                            const void* dout, int dcs, void* dx, int ocs, void* dah, long dahn, void* daw, long dawn,
                            int N, int H, int W, int C, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g2(H + W, N);
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(gate_bwd_reduce_kernel<__bf16>, g2, dim3(256), 0, st, P(const __bf16, x), xcs,
                       P(const __bf16, ah), ahn, P(const __bf16, aw), awn, P(const __bf16, dout), dcs, P(__bf16, dah),
                       dahn, P(__bf16, daw), dawn, N, H, W, C);
  else
    hipLaunchKernelGGL(gate_bwd_reduce_kernel<float>, g2, dim3(256), 0, st, P(const float, x), xcs, P(const float, ah),
                       ahn, P(const float, aw), awn, P(const float, dout), dcs, P(float, dah), dahn, P(float, daw),
                       dawn, N, H, W, C);
  int rc = check_launch("adr_gate_bwd(reduce)");
  if (rc || !dx) return rc;
  dim3 g(cdiv((long)N * H * W * C, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(gate_bwd_x_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, ah), ahn, P(const __bf16, aw),
                       awn, P(const __bf16, dout), dcs, P(__bf16, dx), ocs, N, H, W, C, accumulate);
  else
    hipLaunchKernelGGL(gate_bwd_x_kernel<float>, g, dim3(256), 0, st, P(const float, ah), ahn, P(const float, aw), awn,
                       P(const float, dout), dcs, P(float, dx), ocs, N, H, W, C, accumulate);
  return check_launch("adr_gate_bwd");
}

extern "C" int adr_adapool(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* y, int ycs, int OH,
                           int OW, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(cdiv((long)N * OH * OW * C, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(adapool_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, y),
                       ycs, OH, OW);
  else
    hipLaunchKernelGGL(adapool_kernel<float>, g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, y), ycs,
                       OH, OW);
  return check_launch("adr_adapool");
}

extern "C" int adr_adapool_bwd(int dtype, const void* dy, int dcs, int N, int H, int W, int C, void* dx, int ocs,
                               int OH, int OW, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(cdiv((long)N * H * W * C, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(adapool_bwd_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, dy), dcs, N, H, W, C,
                       P(__bf16, dx), ocs, OH, OW, accumulate);
  else
    hipLaunchKernelGGL(adapool_bwd_kernel<float>, g, dim3(256), 0, st, P(const float, dy), dcs, N, H, W, C,
                       P(float, dx), ocs, OH, OW, accumulate);
  return check_launch("adr_adapool_bwd");
}

extern "C" int adr_bilinear(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* y, int ycs, int OH,
                            int OW, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(cdiv((long)N * OH * OW * C, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(bilinear_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, x), xcs, N, H, W, C, P(__bf16, y),
                       ycs, OH, OW);
  else
    hipLaunchKernelGGL(bilinear_kernel<float>, g, dim3(256), 0, st, P(const float, x), xcs, N, H, W, C, P(float, y),
                       ycs, OH, OW);
  return check_launch("adr_bilinear");
}

extern "C" int adr_bilinear_bwd(int dtype, const void* dy, int dcs, int N, int H, int W, int C, void* dx, int ocs,
                                int OH, int OW, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(cdiv((long)N * H * W * C, 256));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(bilinear_bwd_kernel<__bf16>, g, dim3(256), 0, st, P(const __bf16, dy), dcs, N, H, W, C,
                       P(__bf16, dx), ocs, OH, OW, accumulate);
  else
    hipLaunchKernelGGL(bilinear_bwd_kernel<float>, g, dim3(256), 0, st, P(const float, dy), dcs, N, H, W, C,
                       P(float, dx), ocs, OH, OW, accumulate);
  return check_launch("adr_bilinear_bwd");
}
