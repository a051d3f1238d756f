// C2PTSSA building blocks (reference nn/modules/block.py:2376-2710), forward + backward, NHWC:
//   * depthwise k x k conv + bias (ProgressiveFeatureFusion :2589-2593, EDFFN dwconv :2387, MonaOp mona.py:15-17)
//   * AdaptiveDynamicTanh apply: out = (sum_i tanh(alpha_i x) * imp[n,i]) * w[c] + b[c]  (:2547-2575)
//   * TSSA token statistics per (image, head) (CrossScaleAttentionTSSA :2465-2477):
//       qn = q / max(|q|, 1e-12); Pi = softmax_tokens(temp * sum_d qn^2); attn[d] = 1 / (1 + sum_n Pi k^2);
//       out = -v * Pi * attn
//   * mean over the stacked scales (:2484-2486)
//   * EDFFN 8x8-patch spectral filter as a per-channel 64x64 real operator (:2399-2413): reflect pad to a
//     multiple of 8, y_patch = M_c x_patch with M_c = sum_uv fft[c,u,v] B_uv (B_uv = irfft2(e_uv * rfft2(.)),
//     a constant basis built once on the host in float64), crop. Backward folds the reflected border and
//     returns dfft[c,uv] = <B_uv, sum_patches dy x^T>.
#include "adr_common.h"
#include <cstdlib>
#include <type_traits>

namespace adr {

// ---------------- depthwise conv ----------------
// depthwise k x k, stride 1, pad k/2. BWD = false: y = dwconv(x, w) + b; BWD = true: dx (+)= dwconv^T(dy, w)
// (taps mirrored). The block stages w tap-major ([t][c]) in LDS so each tap is two 16-byte LDS reads per
// 8-channel vector instead of eight strided global loads.
template <typename T, bool BWD, int KS>
__global__ void __launch_bounds__(256) dw_kernel(const T* __restrict__ x, int xcs, const float* __restrict__ w,
                                                 const float* __restrict__ b, T* __restrict__ y, int ycs, int N, int H,
                                                 int W, int C, int kr, int accumulate) {
  constexpr int V = 16 / sizeof(T);
  const int k = KS > 0 ? KS : kr;
  extern __shared__ float wl[];  // [k*k][C]
  const int kk = k * k;
  for (int i = threadIdx.x; i < kk * C; i += 256) {
    const int c = i / kk, t = i % kk;
    wl[t * C + c] = w[i];
  }
  __syncthreads();
  const unsigned G = C / V;
  const unsigned total = (unsigned)N * H * W * G;
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const unsigned pix = i / G;
  const int c0 = (int)(i - pix * G) * V;
  int n, hh, ww;
  pix_nhw(pix, H, W, n, hh, ww);
  const int p = k / 2;
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = (!BWD && b) ? b[c0 + e] : 0.f;
  const T* xb = x + (long)n * H * W * xcs + c0;
#pragma unroll
  for (int ky = 0; ky < (KS > 0 ? KS : 1); ++ky)
    for (int ky2 = 0; ky2 < (KS > 0 ? 1 : k); ++ky2) {
      const int kyy = KS > 0 ? ky : ky2;
      const int ih = BWD ? hh - kyy + p : hh + kyy - p;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int kx = 0; kx < (KS > 0 ? KS : 1); ++kx)
        for (int kx2 = 0; kx2 < (KS > 0 ? 1 : k); ++kx2) {
          const int kxx = KS > 0 ? kx : kx2;
          const int iw = BWD ? ww - kxx + p : ww + kxx - p;
          if (iw < 0 || iw >= W) continue;
          const u32x4 v = ld16(xb + ((long)ih * W + iw) * xcs);
          const T* e = reinterpret_cast<const T*>(&v);
          const float* wt = wl + (kyy * k + kxx) * C + c0;
#pragma unroll
          for (int q = 0; q < V; ++q) acc[q] += to_f(e[q]) * wt[q];
        }
    }
  T* dst = y + (long)pix * ycs + c0;
  if (BWD && accumulate) {
    const u32x4 pv = ld16(dst);
    const T* pe = reinterpret_cast<const T*>(&pv);
#pragma unroll
    for (int q = 0; q < V; ++q) acc[q] += to_f(pe[q]);
  }
  u32x4 o;
  T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
  for (int q = 0; q < V; ++q) oe[q] = from_f<T>(acc[q]);
  st16(dst, o);
}

// partial[chunk][t][c] = sum over the chunk's pixels of dy * x(shifted by tap t); grid (chunks, k*k)
template <typename T>
__global__ void __launch_bounds__(256) dw_bwd_w_kernel(const T* x, int xcs, const T* dy, int dcs, int N, int H, int W,
                                                       int C, int k, int rows_per_chunk, float* partial) {
  constexpr int V = 16 / sizeof(T);
  __shared__ float sh[256 * V];
  const int chunk = blockIdx.x, t = blockIdx.y;
  const int G = C / V, rpp = 256 / G;
  const int tid = threadIdx.x, g = tid % G, r0 = tid / G;
  const int ky = t / k, kx = t % k, p = k / 2;
  const int npix = N * H * W;
  const int beg = chunk * rows_per_chunk, end = min(npix, beg + rows_per_chunk);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  if (r0 < rpp) {
    int n, hh, ww;
    pix_nhw(beg + r0, H, W, n, hh, ww);
    const int dw_ = rpp % W, dh_ = rpp / W;  // advance (n, hh, ww) by rpp pixels without dividing
    for (int pix = beg + r0; pix < end; pix += rpp) {
      const int ih = hh + ky - p, iw = ww + kx - p;
      if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
        const u32x4 dv = ld16(dy + (long)pix * dcs + g * V);
        const u32x4 xv = ld16(x + (((long)n * H + ih) * W + iw) * xcs + g * V);
        const T* de = reinterpret_cast<const T*>(&dv);
        const T* xe = reinterpret_cast<const T*>(&xv);
#pragma unroll
        for (int q = 0; q < V; ++q) acc[q] += to_f(de[q]) * to_f(xe[q]);
      }
      ww += dw_;
      hh += dh_;
      if (ww >= W) {
        ww -= W;
        ++hh;
      }
      while (hh >= H) {
        hh -= H;
        ++n;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < V; ++q) sh[tid * V + q] = acc[q];
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    int gg = c / V, e = c % V;
    float s = 0.f;
    for (int rr = 0; rr < rpp; ++rr) s += sh[(gg + rr * G) * V + e];
    partial[((long)chunk * k * k + t) * C + c] = s;
  }
}

// Whole-image depthwise kernels for small maps (the 20x20 C2PTSSA / EDFFN / Mona path): block per (image,
// CB-channel slab); the zero-padded input image (and dy) are staged once in LDS as bf16/fp32 rows of CB
// channels, every LDS access is one 16-byte vector of VW channels.
template <typename T>
__device__ __forceinline__ void stage_img(const T* src, int cs, int H, int W, int pad, int cb0, int C, int CB, T* dst) {
  constexpr int VW = 16 / sizeof(T), U = 8;  // U loads in flight per thread (a load-store loop serialises latencies)
  const int Hp = H + 2 * pad, Wp = W + 2 * pad, nv = CB / VW, tot = Hp * Wp * nv;
  for (int i0 = threadIdx.x; i0 < tot; i0 += U * blockDim.x) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * blockDim.x;
      const int pp = i / nv, cv = i % nv;
      const int yy = pp / Wp - pad, xx = pp % Wp - pad;
      const int c = cb0 + cv * VW;
      v[u] = (u32x4){0u, 0u, 0u, 0u};
      if (i < tot && yy >= 0 && yy < H && xx >= 0 && xx < W && c < C) v[u] = ld16(src + ((long)yy * W + xx) * cs + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * blockDim.x;
      if (i < tot) *reinterpret_cast<u32x4*>(dst + (long)(i / nv) * CB + (i % nv) * VW) = v[u];
    }
  }
}

// the padded image staged as fp32 in LDS (converted once, not per tap read): CB channels per pixel row
template <typename T, int CBT>
__device__ __forceinline__ void stage_img_f32(const T* src, int cs, int H, int W, int pad, int cb0, int C, int CB,
                                              float* dst) {
  constexpr int VW = (int)(16 / sizeof(T)) < CBT ? (int)(16 / sizeof(T)) : CBT;  // a 4-channel slab: 8-byte bf16 reads
  constexpr int U = 8;  // loads in flight per thread
  const int Hp = H + 2 * pad, Wp = W + 2 * pad, nv = CB / VW, tot = Hp * Wp * nv;
  for (int i0 = threadIdx.x; i0 < tot; i0 += U * blockDim.x) {
    float f[U][VW];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * blockDim.x;
      const int pp = i / nv, cv = i % nv;
      const int yy = pp / Wp - pad, xx = pp % Wp - pad;
      const int c = cb0 + cv * VW;
#pragma unroll
      for (int e = 0; e < VW; ++e) f[u][e] = 0.f;
      if (i < tot && yy >= 0 && yy < H && xx >= 0 && xx < W && c < C) vload<T, VW>(src + ((long)yy * W + xx) * cs + c, f[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * blockDim.x;
      if (i >= tot) continue;
      float* d = dst + (long)(i / nv) * CB + (i % nv) * VW;
#pragma unroll
      for (int e = 0; e < VW; e += 4)
        *reinterpret_cast<f32x4*>(d + e) = (f32x4){f[u][e], f[u][e + 1], f[u][e + 2], f[u][e + 3]};
    }
  }
}

// y = dwconv(x, w) (+b) or dx (+)= dwconv^T(dy, w): items (pixel, VW-channel vector), taps from the LDS image
// EPI (eval DWConv-BN-act, adr_dwconv_fwd_act): the BatchNorm scale folds into the staged fp32 taps, the shift is
// the bias, and the activation is applied before the store — the reference's fuse_conv_and_bn on a depthwise conv.
// F32S (bf16 tensors whose fp32 padded slab fits the LDS plan): the image is converted to fp32 once at staging, so a
// tap is two 16-byte LDS reads + four v_pk_fma_f32 per 8 channels instead of eight conversions + eight FMAs — the
// kernel is VALU-bound (a 7x7 at 20x20: 27 us at ~12 TF/s). Per output the sum is bias + taps in (ky, kx) order,
// each an fp32 fma: bitwise the same for every variant.
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <typename T, bool BWD, int CB, bool EPI, bool F32S = false>
__device__ __forceinline__ void dw_img_body(const T* x, int xcs, const float* w, const float* b, T* y, int ycs, int H,
                                            int W, int C, int k, int accumulate, const float* escale, int eact) {
  constexpr int VW = 16 / sizeof(T), NV = CB / VW;
  typedef typename std::conditional<F32S, float, T>::type S;  // LDS image element
  extern __shared__ __attribute__((aligned(16))) unsigned char dwsm[];
  const int n = blockIdx.x, cb0 = blockIdx.y * CB, p = k / 2, kk = k * k;
  const int Wp = W + 2 * p;
  float* wl = reinterpret_cast<float*>(dwsm);                        // [kk][CB]
  S* xs = reinterpret_cast<S*>(dwsm + (size_t)kk * CB * sizeof(float));
  for (int i = threadIdx.x; i < kk * CB; i += 256) {
    const int t = i / CB, c = cb0 + i % CB;
    wl[i] = c < C ? w[(long)c * kk + t] * (EPI ? escale[c] : 1.f) : 0.f;
  }
  if constexpr (F32S) stage_img_f32<T, CB>(x + (long)n * H * W * xcs, xcs, H, W, p, cb0, C, CB, xs);
  else stage_img<T>(x + (long)n * H * W * xcs, xcs, H, W, p, cb0, C, CB, xs);
  __syncthreads();
  // items (pixel, VW-channel vector): 256 % NV == 0, so a thread's vector cv is fixed and it walks pixels
  // threadIdx / NV + j * (256 / NV), four at a time with the tap loop outside (a tap's weights read once per four)
  static_assert(256 % NV == 0, "dw_img_body: NV must divide the block");
  constexpr int PQ = 4, PSTEP = 256 / NV;
  const int cv = threadIdx.x % NV, c = cb0 + cv * VW;
  if (c < C) {
    for (int p0 = threadIdx.x / NV; p0 < H * W; p0 += PQ * PSTEP) {
      f32x2 acc[PQ][VW / 2];
      int base[PQ];
      bool ok[PQ];
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        const int pix = p0 + q * PSTEP;
        ok[q] = pix < H * W;
        const int pp = ok[q] ? pix : 0, oy = pp / W, ox = pp % W;
        // forward: x[oy + ky - p][ox + kx - p] = padded row oy + ky; data gradient: taps mirrored (from 2p)
        base[q] = BWD ? (oy + 2 * p) * Wp + ox + 2 * p : oy * Wp + ox;
#pragma unroll
        for (int e = 0; e < VW / 2; ++e)
          acc[q][e] = (!BWD && b) ? (f32x2){b[c + 2 * e], b[c + 2 * e + 1]} : (f32x2){0.f, 0.f};
      }
      for (int ky = 0; ky < k; ++ky)
        for (int kx = 0; kx < k; ++kx) {
          f32x2 wv[VW / 2];
          const float* wt = wl + (ky * k + kx) * CB + cv * VW;
#pragma unroll
          for (int e = 0; e < VW; e += 4) {
            const f32x4 w4 = *reinterpret_cast<const f32x4*>(wt + e);
            wv[e / 2] = (f32x2){w4[0], w4[1]};
            wv[e / 2 + 1] = (f32x2){w4[2], w4[3]};
          }
          const int toff = BWD ? -(ky * Wp + kx) : ky * Wp + kx;
#pragma unroll
          for (int q = 0; q < PQ; ++q) {
            if (!ok[q]) continue;
            const S* src = xs + ((long)(base[q] + toff)) * CB + cv * VW;
            f32x2 xv[VW / 2];
            if constexpr (sizeof(S) == 4) {
#pragma unroll
              for (int e = 0; e < VW; e += 4) {
                const f32x4 x4 = *reinterpret_cast<const f32x4*>(src + e);
                xv[e / 2] = (f32x2){x4[0], x4[1]};
                xv[e / 2 + 1] = (f32x2){x4[2], x4[3]};
              }
            } else {
              const u32x4 v = *reinterpret_cast<const u32x4*>(src);
              const T* e8 = reinterpret_cast<const T*>(&v);
#pragma unroll
              for (int e = 0; e < VW / 2; ++e) xv[e] = (f32x2){to_f(e8[2 * e]), to_f(e8[2 * e + 1])};
            }
#pragma unroll
            for (int e = 0; e < VW / 2; ++e) acc[q][e] = __builtin_elementwise_fma(xv[e], wv[e], acc[q][e]);
          }
        }
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        if (!ok[q]) continue;
        float a[VW];
#pragma unroll
        for (int e = 0; e < VW / 2; ++e) {
          a[2 * e] = acc[q][e][0];
          a[2 * e + 1] = acc[q][e][1];
        }
        T* dst = y + ((long)n * H * W + p0 + q * PSTEP) * ycs + c;
        if (BWD && accumulate) {
          const u32x4 pv = ld16(dst);
          const T* pe = reinterpret_cast<const T*>(&pv);
#pragma unroll
          for (int e = 0; e < VW; ++e) a[e] += to_f(pe[e]);
        }
        if constexpr (EPI) {
#pragma unroll
          for (int e = 0; e < VW; ++e) {
            const float v = a[e];
            a[e] = eact == ACT_SILU ? act_fwd_c<ACT_SILU, true>(v) : eact == ACT_SIGMOID ? act_fwd_c<ACT_SIGMOID, true>(v)
                                                                    : act_fwd(eact, v);
          }
        }
        u32x4 o;
        T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
        for (int e = 0; e < VW; ++e) oe[e] = from_f<T>(a[e]);
        st16(dst, o);
      }
    }
  }
}

template <typename T, bool BWD, int CB, bool F32S = false>
__global__ void __launch_bounds__(256) dw_img_kernel(const T* x, int xcs, const float* w, const float* b, T* y,
                                                     int ycs, int H, int W, int C, int k, int accumulate) {
  dw_img_body<T, BWD, CB, false, F32S>(x, xcs, w, b, y, ycs, H, W, C, k, accumulate, nullptr, 0);
}
template <int CB, bool F32S = false>
__global__ void __launch_bounds__(256) dw_img_act_kernel(const __bf16* x, int xcs, const float* w, const float* scale,
                                                         const float* shift, int act, __bf16* y, int ycs, int H, int W,
                                                         int C, int k) {
  dw_img_body<__bf16, false, CB, true, F32S>(x, xcs, w, shift, y, ycs, H, W, C, k, 0, scale, act);
}

// the depthwise conv's bias gradient for this (image, channel slab): column sums of the staged fp32 dy image,
// CB channels x (256 / CB) pixel splits combined in a fixed order; bias_part[n][2][C], half 0
template <int CB>
__device__ __forceinline__ void dw_bias_rows(const float* ds, int HW, int n, int cb0, int C, float* bias_part) {
  __shared__ float bred[256];
  constexpr int PSPL = 256 / CB;
  const int c = threadIdx.x % CB, ps = threadIdx.x / CB;
  float sacc = 0.f;
  for (int pix = ps; pix < HW; pix += PSPL) sacc += ds[(long)pix * CB + c];
  bred[threadIdx.x] = sacc;
  __syncthreads();
  if (threadIdx.x < CB) {
    float t = 0.f;
    for (int q = 0; q < PSPL; ++q) t += bred[q * CB + threadIdx.x];
    if (cb0 + (int)threadIdx.x < C) bias_part[(long)n * 2 * C + cb0 + threadIdx.x] = t;
  }
}

// weight gradient: items (tap, 4-channel group, pixel split PS) over fp32 copies of the padded image and of dy
// in LDS (converted once at staging), partial sums combined in LDS in fixed order; partial[n][t][c]
template <typename T, int CB>
__global__ void __launch_bounds__(256) dw_wgrad_img_kernel(const T* x, int xcs, const T* dy, int dcs, int H, int W,
                                                           int C, int k, float* partial, float* bias_part) {
  constexpr int NV = CB / 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char dwsm[];
  const int n = blockIdx.x, cb0 = blockIdx.y * CB, p = k / 2, kk = k * k;
  const int Hp = H + 2 * p, Wp = W + 2 * p;
  float* xs = reinterpret_cast<float*>(dwsm);
  float* ds = xs + (long)Hp * Wp * CB;
  float* red = ds + (long)H * W * CB;  // [256][4]
  stage_img_f32<T, CB>(x + (long)n * H * W * xcs, xcs, H, W, p, cb0, C, CB, xs);
  stage_img_f32<T, CB>(dy + (long)n * H * W * dcs, dcs, H, W, 0, cb0, C, CB, ds);
  __syncthreads();
  if (bias_part) dw_bias_rows<CB>(ds, H * W, n, cb0, C, bias_part);
  const int pairs = kk * NV;
  int PS = 1;  // pixel splits per (tap, group): a power of two, so split groups never straddle a 256 pass
  while (PS * 2 * pairs <= 256) PS *= 2;
  for (int base = 0; base < pairs * PS; base += 256) {
    const int it = base + threadIdx.x;
    const int pr = it / PS, ps = it % PS;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (pr < pairs) {
      const int t = pr / NV, cv = pr % NV, ky = t / k, kx = t % k;
      int oy = 0, ox = ps;  // (oy, ox) of pix, stepped by PS without dividing
      while (ox >= W) {
        ox -= W;
        ++oy;
      }
      for (int pix = ps; pix < H * W; pix += PS) {
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(ds + (long)pix * CB + cv * 4);
        const f32x4 x4 = *reinterpret_cast<const f32x4*>(xs + ((long)(oy + ky) * Wp + ox + kx) * CB + cv * 4);
        acc += d4 * x4;
        ox += PS;
        while (ox >= W) {
          ox -= W;
          ++oy;
        }
      }
    }
    *reinterpret_cast<f32x4*>(red + threadIdx.x * 4) = acc;
    __syncthreads();
    if (ps == 0 && pr < pairs) {
      const int t = pr / NV, cv = pr % NV, c = cb0 + cv * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float s2 = 0.f;
        for (int q = 0; q < PS; ++q) s2 += red[(threadIdx.x + q) * 4 + e];
        if (c + e < C) partial[((long)n * kk + t) * C + c + e] = s2;
      }
    }
    __syncthreads();
  }
}

// The same weight gradient for k in {3, 5, 7} with a sliding window along the rows: item (ky, 4-channel group, row
// split rs) walks whole output rows; per pixel it loads ONE dy vector and ONE new padded-x vector (the previous
// k - 1 stay in registers) for k taps, instead of two LDS loads per tap. The RS row splits of an item are adjacent
// lanes of one wave, combined by an xor butterfly (fixed order: deterministic).
template <typename T, int CB, int KS>
__global__ void __launch_bounds__(256) dw_wgrad_row_kernel(const T* x, int xcs, const T* dy, int dcs, int H, int W,
                                                           int C, float* partial, float* bias_part) {
  constexpr int NV = CB / 4, P = KS / 2, KK = KS * KS;
  extern __shared__ __attribute__((aligned(16))) unsigned char dwsm[];
  const int n = blockIdx.x, cb0 = blockIdx.y * CB;
  const int Hp = H + 2 * P, Wp = W + 2 * P;
  float* xs = reinterpret_cast<float*>(dwsm);
  float* ds = xs + (long)Hp * Wp * CB;
  stage_img_f32<T, CB>(x + (long)n * H * W * xcs, xcs, H, W, P, cb0, C, CB, xs);
  stage_img_f32<T, CB>(dy + (long)n * H * W * dcs, dcs, H, W, 0, cb0, C, CB, ds);
  __syncthreads();
  if (bias_part) dw_bias_rows<CB>(ds, H * W, n, cb0, C, bias_part);
  constexpr int pairs = KS * NV;
  int RS = 1;  // row splits per (ky, group): a power of two <= 64 dividing 256, so a group sits in one wave
  while (RS * 2 * pairs <= 256 && RS < 64 && RS < H) RS *= 2;
  for (int base = 0; base < pairs * RS; base += 256) {
    const int it = base + threadIdx.x;
    const int pr = it / RS, rs = it % RS;
    f32x4 acc[KS];
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) acc[kx] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (pr < pairs) {
      const int ky = pr / NV, cv = pr % NV;
      for (int oy = rs; oy < H; oy += RS) {
        const float* xr = xs + (long)(oy + ky) * Wp * CB + cv * 4;
        const float* dr = ds + (long)oy * W * CB + cv * 4;
        f32x4 xw[KS];
#pragma unroll
        for (int kx = 0; kx < KS - 1; ++kx) xw[kx] = *reinterpret_cast<const f32x4*>(xr + kx * CB);
        for (int ox = 0; ox < W; ++ox) {
          xw[KS - 1] = *reinterpret_cast<const f32x4*>(xr + (ox + KS - 1) * CB);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(dr + ox * CB);
#pragma unroll
          for (int kx = 0; kx < KS; ++kx) acc[kx] += d4 * xw[kx];
#pragma unroll
          for (int kx = 0; kx < KS - 1; ++kx) xw[kx] = xw[kx + 1];
        }
      }
    }
    for (int o = 1; o < RS; o <<= 1)
#pragma unroll
      for (int kx = 0; kx < KS; ++kx)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[kx][e] += __shfl_xor(acc[kx][e], o, 64);
    if (rs == 0 && pr < pairs) {
      const int ky = pr / NV, cv = pr % NV, c = cb0 + cv * 4;
#pragma unroll
      for (int kx = 0; kx < KS; ++kx)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (c + e < C) partial[((long)n * KK + ky * KS + kx) * C + c + e] = acc[kx][e];
    }
  }
}

// dw[c][t] = sum_chunks partial[chunk][t][c]; threads walk c fastest (coalesced partial rows), 8 chunks in flight
__global__ void dw_w_reduce_kernel(const float* partial, int chunks, int C, int kk, float* dw, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * kk) return;
  const int t = i / C, c = i - (i / C) * C;
  const float* p = partial + (long)t * C + c;
  const long stride = (long)kk * C;
  constexpr int U = 8;
  float s[U];
#pragma unroll
  for (int u = 0; u < U; ++u) s[u] = 0.f;
  int ch = 0;
  for (; ch + U <= chunks; ch += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] += p[(long)(ch + u) * stride];
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (ch + u < chunks) s[u] += p[(long)(ch + u) * stride];
  const float r = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  const int o = c * kk + t;
  dw[o] = accumulate ? dw[o] + r : r;
}

// ---------------- AdaptiveDynamicTanh ----------------
template <typename T>
__global__ void __launch_bounds__(256) adyt_fwd_kernel(const T* x, int xcs, const float* alphas, const float* imp,
                                                       const float* w, const float* b, T* y, int ycs, long npix, int HW,
                                                       int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * C) return;
  int c = (int)(i % C);
  long pix = i / C;
  int n = (int)(pix / HW);
  float xv = to_f(x[pix * xcs + c]);
  float s = 0.f;
  for (int j = 0; j < 3; ++j) s += tanhf(alphas[j] * xv) * imp[n * 3 + j];
  y[pix * ycs + c] = from_f<T>(s * w[c] + b[c]);
}

// dx, and partial[n][chunk][8][C]: {sum t_j w dout (j<3), sum x(1-t_j^2) w dout (j<3), sum S dout, sum dout}
template <typename T>
__global__ void __launch_bounds__(256) adyt_bwd_kernel(const T* x, int xcs, const T* dout, int dcs, const float* alphas,
                                                       const float* imp, const float* w, T* dx, int ocs, int HW, int C,
                                                       int rows_per_chunk, int chunks, float* partial) {
  __shared__ float sh[8][256];
  const int chunk = blockIdx.x, n = blockIdx.y;
  int tid = threadIdx.x;
  int cpt = C < 256 ? C : 256;  // threads over channels
  int rpp = 256 / cpt;
  int c = tid % cpt, r0 = tid / cpt;
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  float a[3] = {alphas[0], alphas[1], alphas[2]};
  float im[3] = {imp[n * 3], imp[n * 3 + 1], imp[n * 3 + 2]};
  int rbeg = chunk * rows_per_chunk, rend = min(HW, rbeg + rows_per_chunk);
  if (r0 < rpp) {
    for (int cc = c; cc < C; cc += cpt) {
      float wc = w[cc];
      for (int r = rbeg + r0; r < rend; r += rpp) {
        long pix = (long)n * HW + r;
        float xv = to_f(x[pix * xcs + cc]);
        float d = to_f(dout[pix * dcs + cc]);
        float g = 0.f, S = 0.f;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          float t = tanhf(a[j] * xv);
          float sech2 = 1.f - t * t;
          g += a[j] * sech2 * im[j];
          S += t * im[j];
          if (cc == c) {
            acc[j] += t * wc * d;
            acc[3 + j] += xv * sech2 * wc * d;
          }
        }
        if (cc == c) {
          acc[6] += S * d;
          acc[7] += d;
        }
        dx[pix * ocs + cc] = from_f<T>(g * wc * d);
      }
    }
  }
  // only channels c < cpt were accumulated; C <= 256 is required by the host wrapper
  for (int q = 0; q < 8; ++q) sh[q][tid] = acc[q];
  __syncthreads();
  if (tid < cpt) {
    float* out = partial + ((long)n * chunks + chunk) * 8 * C;
    for (int q = 0; q < 8; ++q) {
      float s = 0.f;
      for (int rr = 0; rr < rpp; ++rr) s += sh[q][tid + rr * cpt];
      out[q * C + tid] = s;
    }
  }
}

// collapse: dimp[n][j] = sum_{chunk,c} P0..2 ; dalpha[j] = sum_{n,chunk,c} P3..5 * imp[n][j] ; dw[c] = sum P6 ;
// db[c] = sum P7
// collapse of the per-(image, chunk) partials of adyt_bwd. Blocks [0, 3N): (n, j) -> dimp[n][j] and the
// per-image alpha term dan[n][j]; blocks [3N, 3N + C): channel c -> dw[c], db[c]. Fixed-order tree reductions.
__global__ void __launch_bounds__(256) adyt_collapse_kernel(const float* partial, int N, int chunks, int C,
                                                            float* dimp, float* dan, float* dw, float* db) {
  __shared__ double r1[256], r2[256];
  const int tid = threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (blockIdx.x < 3 * N) {
    const int n = blockIdx.x / 3, j = blockIdx.x % 3;
    for (int it = tid; it < chunks * C; it += 256) {
      const int ch = it / C, c = it % C;
      const float* p = partial + ((long)n * chunks + ch) * 8 * C;
      s1 += p[j * C + c];
      s2 += p[(3 + j) * C + c];
    }
  } else {
    const int c = blockIdx.x - 3 * N;
    for (int it = tid; it < N * chunks; it += 256) {
      const float* p = partial + (long)it * 8 * C;
      s1 += p[6 * C + c];
      s2 += p[7 * C + c];
    }
  }
  r1[tid] = s1;
  r2[tid] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      r1[tid] += r1[tid + o];
      r2[tid] += r2[tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    if (blockIdx.x < 3 * N) {
      dimp[blockIdx.x] = (float)r1[0];
      dan[blockIdx.x] = (float)r2[0];
    } else {
      dw[blockIdx.x - 3 * N] = (float)r1[0];
      db[blockIdx.x - 3 * N] = (float)r2[0];
    }
  }
}

// dalpha[j] = sum_n dan[n][j] * imp[n][j]
__global__ void adyt_alpha_kernel(const float* dan, const float* imp, int N, float* dalpha) {
  const int j = threadIdx.x;
  if (j >= 3) return;
  double da = 0.0;
  for (int n = 0; n < N; ++n) da += (double)dan[n * 3 + j] * imp[n * 3 + j];
  dalpha[j] = (float)da;
}

// ---------------- TSSA (one block per (image, head)) ----------------
// q/k/v: [b][tok][*] rows with channel stride cs; head h uses channels [h*D, (h+1)*D) of each
// Per-(image, head) block; threads = TPP tokens x LD lanes, a lane holding VW consecutive channels of the head
// (D = LD * VW): every q/k/v/dout access is a 16-byte vector, per-token sums over d are LD-lane xor shuffles,
// per-channel sums over tokens go through one LDS pass (chan_sum).
// NTH threads per block. 1024 (four times the loads in flight per image-head block) measured n-scale -0.13 ms,
// l-scale -1.1 ms, and each kernel's outputs agree with the 256-thread kernels to fp32 rounding
// (scripts/tssa_ab.py), but with them the fp32 gradient arena of the packed-head trainer test
// (test_gpu_packed_head.py) drifted 200x further from the per-level loop (2.4e-4 vs 1.2e-6 relative, uniformly
// over the backbone and neck, scripts/packed_arena_diff.py); at 512 it is 1.1e-6. Not explained; the launches run
// 512 threads.
#ifndef TSSA_NTH
#define TSSA_NTH 512
#endif
// Each thread also issues the 16-byte loads of TSSA_U of its tokens before using any (the same tokens, the same
// per-thread order of the sums: bitwise the one-token loop).
#ifndef TSSA_LOADS
#define TSSA_LOADS 4
#endif
constexpr int TSSA_U = TSSA_LOADS;
template <typename T, int VW>
__device__ __forceinline__ void vdecode(const u32x4& v, float* f) {
  static_assert(VW * sizeof(T) == 16, "16-byte token rows");
  const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
  for (int i = 0; i < VW; ++i) f[i] = to_f(e[i]);
}
template <typename T, int VW, int LD, int NTH = 1024>
__global__ void __launch_bounds__(NTH) tssa_fwd_kernel(const T* q, const T* k, const T* v, int cs, int Ntok,
                                                       const float* temp, T* out, int ocs, int oimg, int heads,
                                                       float* Pi_out, float* ss_out, float* attn_out) {
  constexpr int TPP = NTH / LD, D = LD * VW;
  extern __shared__ float Pi[];  // Ntok
  __shared__ float red[NTH * VW];
  __shared__ float at[D];
  __shared__ float sh[NTH];
  const int b = blockIdx.x / heads, h = blockIdx.x % heads;
  const int lane = threadIdx.x % LD, r0 = threadIdx.x / LD, c0 = h * D + lane * VW;
  const long base = (long)b * Ntok, bh = (long)b * heads + h;
  const float tp = temp[h];
  // pass 1: ss = sum_d (q / max(|q|, eps))^2 and the logits
  float mx = -INFINITY;
  for (int n0 = r0; n0 < Ntok; n0 += TSSA_U * TPP) {
  u32x4 qr[TSSA_U];
#pragma unroll
  for (int u = 0; u < TSSA_U; ++u)
    if (n0 + u * TPP < Ntok) qr[u] = ld16(q + (base + n0 + u * TPP) * cs + c0);
#pragma unroll
  for (int u = 0; u < TSSA_U; ++u) {
    const int n = n0 + u * TPP;
    if (n >= Ntok) continue;
    float qv[VW];
    vdecode<T, VW>(qr[u], qv);
    float s2 = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) s2 += qv[e] * qv[e];
    const float r = fmaxf(sqrtf(tok_sum<LD>(s2)), 1e-12f);
    float ssp = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const float t = qv[e] / r;
      ssp += t * t;
    }
    const float ss = tok_sum<LD>(ssp);
    if (lane == 0) {
      ss_out[bh * Ntok + n] = ss;
      Pi[n] = ss * tp;
    }
    mx = fmaxf(mx, ss * tp);
  }
  }
  sh[threadIdx.x] = mx;
  __syncthreads();
  for (int o = NTH / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] = fmaxf(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  mx = sh[0];
  __syncthreads();
  float z = 0.f;
  for (int n = threadIdx.x; n < Ntok; n += NTH) {
    const float e = __expf(Pi[n] - mx);
    Pi[n] = e;
    z += e;
  }
  z = block_sum<NTH>(z, sh);
  for (int n = threadIdx.x; n < Ntok; n += NTH) {
    Pi[n] /= z;
    Pi_out[bh * Ntok + n] = Pi[n];
  }
  __syncthreads();
  // pass 2: dots[d] = sum_n Pi k^2 -> attn
  float p[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) p[e] = 0.f;
  for (int n0 = r0; n0 < Ntok; n0 += TSSA_U * TPP) {
    u32x4 kr[TSSA_U];
#pragma unroll
    for (int u = 0; u < TSSA_U; ++u)
      if (n0 + u * TPP < Ntok) kr[u] = ld16(k + (base + n0 + u * TPP) * cs + c0);
#pragma unroll
    for (int u = 0; u < TSSA_U; ++u) {
      const int n = n0 + u * TPP;
      if (n >= Ntok) continue;
      float kv[VW];
      vdecode<T, VW>(kr[u], kv);
#pragma unroll
      for (int e = 0; e < VW; ++e) p[e] += Pi[n] * kv[e] * kv[e];
    }
  }
  chan_sum<VW, LD, NTH>(p, red, at);
  if (threadIdx.x < D) {
    const float a = 1.f / (1.f + at[threadIdx.x]);
    at[threadIdx.x] = a;
    attn_out[bh * D + threadIdx.x] = a;
  }
  __syncthreads();
  // pass 3: out = -v * Pi * attn
  for (int n0 = r0; n0 < Ntok; n0 += TSSA_U * TPP) {
    u32x4 vr[TSSA_U];
#pragma unroll
    for (int u = 0; u < TSSA_U; ++u)
      if (n0 + u * TPP < Ntok) vr[u] = ld16(v + (base + n0 + u * TPP) * cs + c0);
#pragma unroll
    for (int u = 0; u < TSSA_U; ++u) {
      const int n = n0 + u * TPP;
      if (n >= Ntok) continue;
      float vv[VW];
      vdecode<T, VW>(vr[u], vv);
#pragma unroll
      for (int e = 0; e < VW; ++e) vv[e] = -vv[e] * Pi[n] * at[lane * VW + e];
      vstore<T, VW>(out + ((long)b * oimg + n) * ocs + c0, vv);
    }
  }
}

template <typename T, int VW, int LD, int NTH = 1024>
__global__ void __launch_bounds__(NTH) tssa_bwd_kernel(const T* q, const T* k, const T* v, int cs, int Ntok,
                                                       const float* temp, const T* dout, int dcs, int dimg, int heads,
                                                       const float* Pi_in, const float* ss_in, const float* attn_in,
                                                       T* dq, T* dk, T* dv, int gcs, float* dtemp_part) {
  constexpr int TPP = NTH / LD, D = LD * VW;
  extern __shared__ float dPi[];  // Ntok
  __shared__ float red[NTH * VW];
  __shared__ float dd[D];
  __shared__ float sh[NTH];
  const int b = blockIdx.x / heads, h = blockIdx.x % heads;
  const int lane = threadIdx.x % LD, r0 = threadIdx.x / LD, c0 = h * D + lane * VW;
  const long base = (long)b * Ntok, bh = (long)b * heads + h;
  const float* Pi = Pi_in + bh * Ntok;
  const float* ss = ss_in + bh * Ntok;
  const float* attn = attn_in + bh * D;
  const float tp = temp[h];
  float at[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) at[e] = attn[lane * VW + e];
  // dattn[d] = sum_n -dout v Pi ; dv = -dout Pi attn
  float p[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) p[e] = 0.f;
  for (int n0 = r0; n0 < Ntok; n0 += TSSA_U * TPP) {
  u32x4 gr[TSSA_U], vr[TSSA_U];
#pragma unroll
  for (int u = 0; u < TSSA_U; ++u)
    if (n0 + u * TPP < Ntok) {
      gr[u] = ld16(dout + ((long)b * dimg + n0 + u * TPP) * dcs + c0);
      vr[u] = ld16(v + (base + n0 + u * TPP) * cs + c0);
    }
#pragma unroll
  for (int u = 0; u < TSSA_U; ++u) {
    const int n = n0 + u * TPP;
    if (n >= Ntok) continue;
    float g[VW], vv[VW], o[VW];
    vdecode<T, VW>(gr[u], g);
    vdecode<T, VW>(vr[u], vv);
    const float pn = Pi[n];
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      p[e] -= g[e] * vv[e] * pn;
      o[e] = -g[e] * pn * at[e];
    }
    vstore<T, VW>(dv + (base + n) * gcs + c0, o);
  }
  }
  chan_sum<VW, LD, NTH>(p, red, dd);
  if (threadIdx.x < D) dd[threadIdx.x] = -dd[threadIdx.x] * attn[threadIdx.x] * attn[threadIdx.x];  // ddots
  __syncthreads();
  // dPi[n] = sum_d (-dout v attn + ddots k^2) ; dk = ddots * Pi * 2k
  float part = 0.f;
  for (int n0 = r0; n0 < Ntok; n0 += TSSA_U * TPP) {
  u32x4 gr[TSSA_U], vr[TSSA_U], kr[TSSA_U];
#pragma unroll
  for (int u = 0; u < TSSA_U; ++u)
    if (n0 + u * TPP < Ntok) {
      gr[u] = ld16(dout + ((long)b * dimg + n0 + u * TPP) * dcs + c0);
      vr[u] = ld16(v + (base + n0 + u * TPP) * cs + c0);
      kr[u] = ld16(k + (base + n0 + u * TPP) * cs + c0);
    }
#pragma unroll
  for (int u = 0; u < TSSA_U; ++u) {
    const int n = n0 + u * TPP;
    if (n >= Ntok) continue;
    float g[VW], vv[VW], kv[VW], o[VW];
    vdecode<T, VW>(gr[u], g);
    vdecode<T, VW>(vr[u], vv);
    vdecode<T, VW>(kr[u], kv);
    const float pn = Pi[n];
    float sp = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const float ddv = dd[lane * VW + e];
      sp += -g[e] * vv[e] * at[e] + ddv * kv[e] * kv[e];
      o[e] = ddv * pn * 2.f * kv[e];
    }
    vstore<T, VW>(dk + (base + n) * gcs + c0, o);
    const float s = tok_sum<LD>(sp);
    if (lane == 0) {
      dPi[n] = s;
      part += pn * s;
    }
  }
  }
  const float dot = block_sum<NTH>(part, sh);
  // softmax backward -> dl ; dtemp partial ; dss -> dq
  float tpart = 0.f;
  for (int n0 = r0; n0 < Ntok; n0 += TSSA_U * TPP) {
  u32x4 qr[TSSA_U];
#pragma unroll
  for (int u = 0; u < TSSA_U; ++u)
    if (n0 + u * TPP < Ntok) qr[u] = ld16(q + (base + n0 + u * TPP) * cs + c0);
#pragma unroll
  for (int u = 0; u < TSSA_U; ++u) {
    const int n = n0 + u * TPP;
    if (n >= Ntok) continue;
    const float dl = Pi[n] * (dPi[n] - dot);
    if (lane == 0) tpart += dl * ss[n];
    const float dss = dl * tp;
    float qv[VW];
    vdecode<T, VW>(qr[u], qv);
    float s2 = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) s2 += qv[e] * qv[e];
    const float nrm = sqrtf(tok_sum<LD>(s2));
    const float r = fmaxf(nrm, 1e-12f);
    // dqn = 2 qn dss ; dq = dqn / r - (nrm > eps) * q (q . dqn) / r^3
    float qp = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) qp += qv[e] * (2.f * (qv[e] / r) * dss);
    const float qdq = tok_sum<LD>(qp);
    float o[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const float dqn = 2.f * (qv[e] / r) * dss;
      o[e] = dqn / r - (nrm > 1e-12f ? qv[e] * qdq / (r * r * r) : 0.f);
    }
    vstore<T, VW>(dq + (base + n) * gcs + c0, o);
  }
  }
  tpart = block_sum<NTH>(tpart, sh);
  if (threadIdx.x == 0) dtemp_part[bh] = tpart;
}

__global__ void tssa_temp_reduce_kernel(const float* part, int B, int heads, float* dtemp) {
  int h = threadIdx.x;
  if (h >= heads) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += part[b * heads + h];
  dtemp[h] = s;
}

// ---------------- mean over S stacked token groups ----------------
template <typename T>
__global__ void __launch_bounds__(256) group_mean_kernel(const T* x, int xcs, int S, int HW, T* y, int ycs, long B,
                                                         int C, int backward) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (!backward) {
    if (i >= B * HW * C) return;
    int c = (int)(i % C);
    long r = i / C;
    int n = (int)(r % HW);
    long b = r / HW;
    float s = 0.f;
    for (int g = 0; g < S; ++g) s += to_f(x[((b * S + g) * HW + n) * xcs + c]);
    y[(b * HW + n) * ycs + c] = from_f<T>(s / (float)S);
  } else {  // y: [B][S*HW] grad, x: [B][HW] upstream
    if (i >= B * S * HW * C) return;
    int c = (int)(i % C);
    long r = i / C;
    int n = (int)(r % HW);
    long bg = r / HW;
    long b = bg / S;
    y[(bg * HW + n) * ycs + c] = from_f<T>(to_f(x[(b * HW + n) * xcs + c]) / (float)S);
  }
}

// ---------------- EDFFN spectral patch filter ----------------
__device__ __forceinline__ int reflect_idx(int j, int n) { return j < n ? j : 2 * (n - 1) - j; }

// M[c][i][j] = sum_uv w[c][uv] * B[uv][i][j]
__global__ void edffn_build_kernel(const float* w, const float* Bm, int C, int nuv, float* M) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)C * 4096) return;
  int c = (int)(i / 4096), e = (int)(i % 4096);
  float s = 0.f;
  for (int u = 0; u < nuv; ++u) s += w[c * nuv + u] * Bm[(long)u * 4096 + e];
  M[i] = s;
}

// the same, 8 channels per thread (the basis element read once for 8 channels, loads of the u loop in flight):
// per output the same fp32 sum over u in order
__global__ void __launch_bounds__(256) edffn_build8_kernel(const float* w, const float* Bm, int C, int nuv, float* M) {
  const int e = blockIdx.x * 256 + threadIdx.x, c0 = blockIdx.y * 8;
  if (e >= 4096) return;
  float s[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[q] = 0.f;
#pragma unroll 4
  for (int u = 0; u < nuv; ++u) {
    const float b = Bm[(long)u * 4096 + e];
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] += w[(c0 + q) * nuv + u] * b;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) M[(long)(c0 + q) * 4096 + e] = s[q];
}

// y_patch = M_c x_patch for every 8x8 patch of channel c (transpose: M_c^T, the backward).
// Block = one channel x EDFFN_PPB patches; lane = patch position: the lane keeps its row (column for the
// transpose) of M_c in 64 registers, the wave stages each patch's 64 inputs in LDS and every lane reads them
// back as broadcasts, so M is read from memory once per block instead of once per output element.
// Forward: x reflect-padded, y written on the real (cropped) pixels. Transpose: dy read on the real pixels
// (zero elsewhere), written to the padded fp32 scratch [N][Hp][Wp][C] for the fold.
constexpr int EDFFN_PPB = 64;

template <typename T>
__global__ void __launch_bounds__(256) edffn_apply_kernel(const T* x, int xcs, const float* M, T* y, int ycs, int N,
                                                          int H, int W, int C, int transpose) {
  __shared__ float xs[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x % C, chunk = blockIdx.x / C;
  const int pw_n = (W + 7) / 8, ph_n = (H + 7) / 8, npatch = N * ph_n * pw_n;
  const float* Mc = M + (long)c * 4096;
  float mr[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) mr[j] = transpose ? Mc[j * 64 + lane] : Mc[lane * 64 + j];
  const int dy_ = lane / 8, dx_ = lane % 8;
  const int pend = min(npatch, (chunk + 1) * EDFFN_PPB);
  for (int pp = chunk * EDFFN_PPB + wave; pp < pend; pp += 4) {
    const int n = pp / (ph_n * pw_n), q = pp % (ph_n * pw_n);
    const int yy = (q / pw_n) * 8 + dy_, xx = (q % pw_n) * 8 + dx_;
    float v = 0.f;
    if (!transpose) {
      v = to_f(x[(((long)n * H + reflect_idx(yy, H)) * W + reflect_idx(xx, W)) * xcs + c]);
    } else if (yy < H && xx < W) {
      v = to_f(x[(((long)n * H + yy) * W + xx) * xcs + c]);
    }
    xs[wave][lane] = v;
    __builtin_amdgcn_wave_barrier();
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 64; j += 4) {
      const float4 b = *reinterpret_cast<const float4*>(&xs[wave][j]);
      s += mr[j] * b.x + mr[j + 1] * b.y + mr[j + 2] * b.z + mr[j + 3] * b.w;
    }
    __builtin_amdgcn_wave_barrier();
    if (!transpose) {
      if (yy < H && xx < W) y[(((long)n * H + yy) * W + xx) * ycs + c] = from_f<T>(s);
    } else {
      float* scratch = reinterpret_cast<float*>(y);
      scratch[(((long)n * ph_n * 8 + yy) * (pw_n * 8) + xx) * C + c] = s;
    }
  }
}

// The same apply on the fp32 matrix cores (bf16 tensors): block = 8 channels x 16 patches. The per-channel kernel above
// reads one 2-byte element of a 256-byte pixel row per lane (every channel block re-fetches every line): 63 us per
// call at bs 64, 20x20, C = 128. Here a 16-byte load brings a pixel's 8 channels into LDS as fp32 [ch][pos][patch]
// (pitch 17: the four k-slot row groups of an MFMA B read fall on disjoint banks), each wave runs two channels as
// D (64 positions x 16 patches) = M_c (64 x 64) * X_c (64 x 16) on v_mfma_f32_16x16x4_f32 — exact fp32 products,
// fp32 sums — with the reduction index of step js, slot g being j = 16g + js so a lane's A values are 16 consecutive
// floats of one M row (four 16-byte loads; the transpose reads M columns, lanes along i, coalesced), and the result
// goes through LDS [patch][pos][ch] so the stores are 16-byte (bf16) / 32-byte (fp32 scratch) pixel rows.
constexpr int EA_CG = 8, EA_PG = 16, EA_XP = EA_PG + 1, EA_YP = 64 * EA_CG + 4;
template <bool TR>
__global__ void __launch_bounds__(256) edffn_apply_mfma_kernel(const __bf16* x, int xcs, const float* M, void* yv,
                                                               int ycs, int N, int H, int W, int C) {
  __shared__ __attribute__((aligned(16))) float Xs[EA_CG * 64 * EA_XP];
  __shared__ __attribute__((aligned(16))) float Ys[EA_PG * EA_YP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int ncg = C / EA_CG, cg = blockIdx.x % ncg, pg = blockIdx.x / ncg;
  const int pw_n = (W + 7) / 8, ph_n = (H + 7) / 8, ppi = ph_n * pw_n, npatch = N * ppi;
  const int c0 = cg * EA_CG;
  // stage: item (patch p, position pos), p fastest
  {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int it = tid + 256 * u, pl = it % EA_PG, pos = it / EA_PG, pp = pg * EA_PG + pl;
      v[u] = (u32x4){0u, 0u, 0u, 0u};
      if (pp < npatch) {
        const int n = pp / ppi, q = pp % ppi;
        const int yy = (q / pw_n) * 8 + pos / 8, xx = (q % pw_n) * 8 + pos % 8;
        if (!TR) v[u] = ld16(x + (((long)n * H + reflect_idx(yy, H)) * W + reflect_idx(xx, W)) * xcs + c0);
        else if (yy < H && xx < W) v[u] = ld16(x + (((long)n * H + yy) * W + xx) * xcs + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int it = tid + 256 * u, pl = it % EA_PG, pos = it / EA_PG;
      const __bf16* e = reinterpret_cast<const __bf16*>(&v[u]);
#pragma unroll
      for (int ch = 0; ch < EA_CG; ++ch) Xs[(ch * 64 + pos) * EA_XP + pl] = to_f(e[ch]);
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int cc = 0; cc < 2; ++cc) {
    const int ch = wave * 2 + cc;
    const float* Mc = M + (long)(c0 + ch) * 4096;
    f32x4 acc[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) acc[it] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float a[4][16];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int i = it * 16 + cl;
      if (!TR) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 m4 = *reinterpret_cast<const f32x4*>(Mc + i * 64 + 16 * g + 4 * q);
          a[it][4 * q] = m4[0]; a[it][4 * q + 1] = m4[1]; a[it][4 * q + 2] = m4[2]; a[it][4 * q + 3] = m4[3];
        }
      } else {
#pragma unroll
        for (int js = 0; js < 16; ++js) a[it][js] = Mc[(16 * g + js) * 64 + i];
      }
    }
    const float* xb = Xs + (ch * 64 + 16 * g) * EA_XP + cl;
#pragma unroll
    for (int js = 0; js < 16; ++js) {
      const float bv = xb[js * EA_XP];
#pragma unroll
      for (int it = 0; it < 4; ++it) acc[it] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[it][js], bv, acc[it], 0, 0, 0);
    }
    // D[i = it*16 + 4g + r][patch cl]
#pragma unroll
    for (int it = 0; it < 4; ++it)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ys[cl * EA_YP + (it * 16 + 4 * g + r) * EA_CG + ch] = acc[it][r];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int it = tid + 256 * u, pl = it % EA_PG, pos = it / EA_PG, pp = pg * EA_PG + pl;
    if (pp >= npatch) continue;
    const int n = pp / ppi, q = pp % ppi;
    const int yy = (q / pw_n) * 8 + pos / 8, xx = (q % pw_n) * 8 + pos % 8;
    const float* ys = Ys + pl * EA_YP + pos * EA_CG;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(ys), hi = *reinterpret_cast<const f32x4*>(ys + 4);
    if (!TR) {
      if (yy < H && xx < W) {
        u32x4 o;
        __bf16* oe = reinterpret_cast<__bf16*>(&o);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          oe[e] = from_f<__bf16>(lo[e]);
          oe[4 + e] = from_f<__bf16>(hi[e]);
        }
        st16(reinterpret_cast<__bf16*>(yv) + (((long)n * H + yy) * W + xx) * ycs + c0, o);
      }
    } else {
      float* d = reinterpret_cast<float*>(yv) + (((long)n * ph_n * 8 + yy) * (pw_n * 8) + xx) * C + c0;
      *reinterpret_cast<f32x4*>(d) = lo;
      *reinterpret_cast<f32x4*>(d + 4) = hi;
    }
  }
}

// fold reflected padding: dx[n,h,w,c] = sum of padded-grid grads whose reflect source is (h, w)
template <typename T>
__global__ void __launch_bounds__(256) edffn_fold_kernel(const float* dpad, int H, int W, int C, long N, T* dx, int ocs) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * H * W * C) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  long n = r / H;
  int Hp = (H + 7) / 8 * 8, Wp = (W + 7) / 8 * 8;
  float s = 0.f;
  for (int a = 0; a < 2; ++a) {
    int yy = a == 0 ? h : 2 * (H - 1) - h;
    if (a == 1 && (yy < H || yy >= Hp)) continue;
    for (int bb = 0; bb < 2; ++bb) {
      int xx = bb == 0 ? w : 2 * (W - 1) - w;
      if (bb == 1 && (xx < W || xx >= Wp)) continue;
      s += dpad[((n * Hp + yy) * Wp + xx) * C + c];
    }
  }
  dx[pix * ocs + c] = from_f<T>(s);
}

// dw[c][uv] = sum_{i,j} B[uv][i][j] dM[c][i][j],  dM[c][i][j] = sum over (n, patch) dY_patch[i] * X_patch[j].
// Block per channel: lane j accumulates column j of dM over the wave's patches (64 registers, dY broadcast from
// LDS), the four waves' partials are summed in LDS in a fixed order, and the block contracts dM with the
// basis in place (no dM round trip through memory).
// dM partial per (channel, patch split): grid (C, EDFFN_DWS); 4 waves x patch stride, two patches' loads in
// flight per iteration; part[(split * C + c) * 4096 + e]
constexpr int EDFFN_DWS = 16;  // patch splits of the dM partials (16: 256 blocks of the MFMA kernel at C = 128)
template <typename T>
__global__ void __launch_bounds__(256) edffn_dw_kernel(const T* x, int xcs, const T* dy, int dcs, int N, int H, int W,
                                                       int C, float* part) {
  __shared__ float sdy[4][2][64];
  __shared__ float dM[4][4096];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int c = blockIdx.x, sp = blockIdx.y;
  const int pw_n = (W + 7) / 8, ph_n = (H + 7) / 8, npatch = N * ph_n * pw_n;
  const int per = (npatch + EDFFN_DWS - 1) / EDFFN_DWS, pbeg = sp * per, pend = min(npatch, pbeg + per);
  float acc[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) acc[i] = 0.f;
  const int dy_ = lane / 8, dx_ = lane % 8;
  auto fetch = [&](int pp, float& xv, float& gv) {
    xv = 0.f;
    gv = 0.f;
    if (pp >= pend) return;
    const int n = pp / (ph_n * pw_n), q = pp % (ph_n * pw_n);
    const int yy = (q / pw_n) * 8 + dy_, xx = (q % pw_n) * 8 + dx_;
    xv = to_f(x[(((long)n * H + reflect_idx(yy, H)) * W + reflect_idx(xx, W)) * xcs + c]);
    gv = (yy < H && xx < W) ? to_f(dy[(((long)n * H + yy) * W + xx) * dcs + c]) : 0.f;
  };
  for (int pp = pbeg + wave; pp < pend; pp += 8) {
    float x0, g0, x1, g1;
    fetch(pp, x0, g0);
    fetch(pp + 4, x1, g1);
    sdy[wave][0][lane] = g0;
    sdy[wave][1][lane] = g1;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 64; i += 4) {
      const float4 a = *reinterpret_cast<const float4*>(&sdy[wave][0][i]);
      const float4 b = *reinterpret_cast<const float4*>(&sdy[wave][1][i]);
      acc[i] += a.x * x0 + b.x * x1;
      acc[i + 1] += a.y * x0 + b.y * x1;
      acc[i + 2] += a.z * x0 + b.z * x1;
      acc[i + 3] += a.w * x0 + b.w * x1;
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int i = 0; i < 64; ++i) dM[wave][i * 64 + lane] = acc[i];
  __syncthreads();
  float* out = part + ((long)sp * C + c) * 4096;
  for (int e = tid; e < 4096; e += 256) out[e] = (dM[0][e] + dM[1][e]) + (dM[2][e] + dM[3][e]);
}

// The dM partials on the fp32 matrix cores (bf16 tensors): block = 8 channels x one of EDFFN_DWS patch splits;
// chunks of 16 patches of dY (real pixels, zero padding) and X (reflect-padded) are staged as fp32 [ch][pos][patch]
// (16-byte pixel loads), and each wave accumulates two channels' 64 x 64 dM = dY (64 x P) * X^T (P x 64) over its
// split on v_mfma_f32_16x16x4_f32 (16 f32x4 tiles per channel). The per-channel kernel above gathered one 2-byte
// element of a 256-byte pixel row per lane (48 us per call at bs 64, 20x20, C = 128). Same partial layout.
__global__ void __launch_bounds__(256) edffn_dw_mfma_kernel(const __bf16* x, int xcs, const __bf16* dy, int dcs,
                                                            int N, int H, int W, int C, float* part) {
  __shared__ __attribute__((aligned(16))) float Ds[EA_CG * 64 * EA_XP];
  __shared__ __attribute__((aligned(16))) float Xs[EA_CG * 64 * EA_XP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int ncg = C / EA_CG, cg = blockIdx.x % ncg, sp = blockIdx.x / ncg;
  const int pw_n = (W + 7) / 8, ph_n = (H + 7) / 8, ppi = ph_n * pw_n, npatch = N * ppi;
  const int nchunk = (npatch + EA_PG - 1) / EA_PG, per = (nchunk + EDFFN_DWS - 1) / EDFFN_DWS;
  const int k0 = sp * per, k1 = min(nchunk, k0 + per);
  const int c0 = cg * EA_CG;
  f32x4 acc[2][16];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[cc][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int kc = k0; kc < k1; ++kc) {
    u32x4 vx[4], vd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int it = tid + 256 * u, pl = it % EA_PG, pos = it / EA_PG, pp = kc * EA_PG + pl;
      vx[u] = vd[u] = (u32x4){0u, 0u, 0u, 0u};
      if (pp < npatch) {
        const int n = pp / ppi, q = pp % ppi;
        const int yy = (q / pw_n) * 8 + pos / 8, xx = (q % pw_n) * 8 + pos % 8;
        vx[u] = ld16(x + (((long)n * H + reflect_idx(yy, H)) * W + reflect_idx(xx, W)) * xcs + c0);
        if (yy < H && xx < W) vd[u] = ld16(dy + (((long)n * H + yy) * W + xx) * dcs + c0);
      }
    }
    __syncthreads();  // the previous chunk's MFMA reads are done
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int it = tid + 256 * u, pl = it % EA_PG, pos = it / EA_PG;
      const __bf16* ex = reinterpret_cast<const __bf16*>(&vx[u]);
      const __bf16* ed = reinterpret_cast<const __bf16*>(&vd[u]);
#pragma unroll
      for (int ch = 0; ch < EA_CG; ++ch) {
        Xs[(ch * 64 + pos) * EA_XP + pl] = to_f(ex[ch]);
        Ds[(ch * 64 + pos) * EA_XP + pl] = to_f(ed[ch]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int ch = wave * 2 + cc;
      const float* db = Ds + (ch * 64 + cl) * EA_XP + g;
      const float* xb = Xs + (ch * 64 + cl) * EA_XP + g;
#pragma unroll
      for (int ks = 0; ks < EA_PG / 4; ++ks) {
        float av[4], bv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          av[t] = db[t * 16 * EA_XP + 4 * ks];  // A[i = t*16 + cl][patch 4ks + g]
          bv[t] = xb[t * 16 * EA_XP + 4 * ks];  // B[patch 4ks + g][j = t*16 + cl]
        }
#pragma unroll
        for (int it = 0; it < 4; ++it)
#pragma unroll
          for (int jt = 0; jt < 4; ++jt)
            acc[cc][it * 4 + jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[it], bv[jt], acc[cc][it * 4 + jt], 0, 0, 0);
      }
    }
  }
  // D[i = it*16 + 4g + r][j = jt*16 + cl] -> part[(sp * C + c) * 4096 + i * 64 + j]
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
    float* out = part + ((long)sp * C + c0 + wave * 2 + cc) * 4096;
#pragma unroll
    for (int it = 0; it < 4; ++it)
#pragma unroll
      for (int jt = 0; jt < 4; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(it * 16 + 4 * g + r) * 64 + jt * 16 + cl] = acc[cc][it * 4 + jt][r];
  }
}

// dw[c][uv] (+)= sum_e B[uv][e] * sum_split part[split][c][e]; block = (channel, half of the uv rows): the split
// sum of dM_c goes to LDS (16-byte loads), then a wave per uv row reads B[uv] as 16 float4 per lane (all in flight)
// against it and reduces in a fixed order. The per-channel kernel below kept 8 scalar basis loads in flight per wave
// (43 us per call: latency on the 640 KB basis read by every block).
__global__ void __launch_bounds__(256) edffn_dw_fin2_kernel(const float* part, int C, const float* Bm, int nuv,
                                                            float* dw, int accumulate) {
  __shared__ __attribute__((aligned(16))) float dM[4096];
  const int c = blockIdx.x, half = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int e4 = threadIdx.x; e4 < 1024; e4 += 256) {
    f32x4 v[EDFFN_DWS];
#pragma unroll
    for (int sp = 0; sp < EDFFN_DWS; ++sp) v[sp] = *reinterpret_cast<const f32x4*>(part + ((long)sp * C + c) * 4096 + 4 * e4);
    f32x4 sacc = v[0];
#pragma unroll
    for (int sp = 1; sp < EDFFN_DWS; ++sp) sacc += v[sp];
    *reinterpret_cast<f32x4*>(dM + 4 * e4) = sacc;
  }
  __syncthreads();
  const int u0 = half * ((nuv + 1) / 2), u1 = min(nuv, u0 + (nuv + 1) / 2);
  for (int u = u0 + wave; u < u1; u += 4) {
    const f32x4* b = reinterpret_cast<const f32x4*>(Bm + (long)u * 4096);
    f32x4 bv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) bv[k] = b[lane + 64 * k];
    float sacc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const f32x4 m4 = *reinterpret_cast<const f32x4*>(dM + 4 * (lane + 64 * k));
      sacc += bv[k][0] * m4[0] + bv[k][1] * m4[1] + bv[k][2] * m4[2] + bv[k][3] * m4[3];
    }
    sacc = wave_sum(sacc);
    if (lane == 0) dw[c * nuv + u] = accumulate ? dw[c * nuv + u] + sacc : sacc;
  }
}

// dw[c][uv] (+)= sum_e B[uv][e] * sum_split part[split][c][e]: block per channel, fixed order
__global__ void __launch_bounds__(256) edffn_dw_fin_kernel(const float* part, int C, const float* Bm, int nuv,
                                                           float* dw, int accumulate) {
  __shared__ float dM[4096];
  const int c = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < 4096; e += 256) {
    float sacc = 0.f;
    for (int sp = 0; sp < EDFFN_DWS; ++sp) sacc += part[((long)sp * C + c) * 4096 + e];
    dM[e] = sacc;
  }
  __syncthreads();
  for (int u = wave; u < nuv; u += 4) {
    const float* b = Bm + (long)u * 4096;
    float sacc = 0.f;
    for (int e0 = lane; e0 < 4096; e0 += 64 * 8) {
      float bv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) bv[q] = b[e0 + 64 * q];  // eight loads in flight
#pragma unroll
      for (int q = 0; q < 8; ++q) sacc += bv[q] * dM[e0 + 64 * q];
    }
    sacc = wave_sum(sacc);
    if (lane == 0) dw[c * nuv + u] = accumulate ? dw[c * nuv + u] + sacc : sacc;
  }
}

}  // namespace adr

using namespace adr;

#define TDISPATCH(dtype, KERN, grid, block, sm, ...)                                                    \
  do {                                                                                                  \
    if ((dtype) == ADR_BF16) hipLaunchKernelGGL(KERN<__bf16>, grid, block, sm, st, __VA_ARGS__);         \
    else hipLaunchKernelGGL(KERN<float>, grid, block, sm, st, __VA_ARGS__);                             \
  } while (0)

static constexpr int DW_CB_BF16 = 16, DW_CB_F32 = 8, DW_CB_WG = 8;  // DW_CB_WG: weight-gradient channel slab
// ADR_DW_IMG=0 routes the forward / data gradient to the direct (global-load) kernel for A/B runs
static bool dw_img_ok() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ADR_DW_IMG");
    v = e ? atoi(e) != 0 : 1;
  }
  return v != 0;
}
// ADR_DW_ROW=0: the per-tap weight-gradient kernel instead of the sliding-window one (A/B)
static bool dw_row_ok() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ADR_DW_ROW");
    v = e ? atoi(e) != 0 : 1;
  }
  return v != 0;
}
constexpr size_t DW_LDS_MAX = 64 * 1024;
static size_t dw_img_smem_cb(int H, int W, int k, int cb) {  // weight-gradient kernel (fp32 copies in LDS)
  const int p = k / 2;
  return ((size_t)(H + 2 * p) * (W + 2 * p) + (size_t)H * W) * cb * 4 + 256 * 16;
}
// the weight-gradient kernels' channel slab: 8, or 4 when an 8-channel image pair does not fit (the l-scale 40x40
// maps); 0: the map is too large for the whole-image kernels
static int dw_wg_cb(int H, int W, int k) {
  return dw_img_smem_cb(H, W, k, DW_CB_WG) <= DW_LDS_MAX ? DW_CB_WG : dw_img_smem_cb(H, W, k, 4) <= DW_LDS_MAX ? 4 : 0;
}
static size_t dw_fwd_smem_cb(int dtype, int H, int W, int k, int cb) {  // forward / data-gradient kernel
  const int p = k / 2;
  const size_t es = dtype == ADR_BF16 ? 2 : 4;
  return (size_t)k * k * cb * 4 + (size_t)(H + 2 * p) * (W + 2 * p) * cb * es;
}
// the forward / data-gradient whole-image kernels' channel slab: 16 (bf16) / 8 (fp32), halved when the padded image
// slab does not fit 64 KB of LDS (one 16-byte vector per pixel is the floor); 0: use the direct kernel
static int dw_fwd_cb(int dtype, int H, int W, int k) {
  const int cb = dtype == ADR_BF16 ? DW_CB_BF16 : DW_CB_F32, half = cb / 2;
  return dw_fwd_smem_cb(dtype, H, W, k, cb) <= DW_LDS_MAX ? cb : dw_fwd_smem_cb(dtype, H, W, k, half) <= DW_LDS_MAX ? half : 0;
}
// bf16 with a 16-channel slab whose fp32 padded image fits 64 KB (the 20x20 maps): the F32S variant
static bool dw_f32s(int dtype, int H, int W, int k, int cb) {
  return dtype == ADR_BF16 && cb == DW_CB_BF16 && dw_fwd_smem_cb(ADR_F32, H, W, k, DW_CB_BF16) <= DW_LDS_MAX;
}
template <bool BWD>
static void dw_img_launch(int dtype, hipStream_t st, const void* x, int xcs, const float* w, const float* b, void* y,
                          int ycs, int N, int H, int W, int C, int k, int acc) {
  const int cb = dw_fwd_cb(dtype, H, W, k);
  const size_t sm = dw_fwd_smem_cb(dtype, H, W, k, cb);
  if (dw_f32s(dtype, H, W, k, cb))  // 8-channel slabs: twice the blocks of the 16-channel plan (latency-bound at 2 waves/SIMD)
    hipLaunchKernelGGL((dw_img_kernel<__bf16, BWD, DW_CB_BF16 / 2, true>), dim3(N, cdiv(C, DW_CB_BF16 / 2)), dim3(256),
                       dw_fwd_smem_cb(ADR_F32, H, W, k, DW_CB_BF16 / 2), st, (const __bf16*)x, xcs, w, b, (__bf16*)y, ycs,
                       H, W, C, k, acc);
  else if (dtype == ADR_BF16 && cb == DW_CB_BF16)
    hipLaunchKernelGGL((dw_img_kernel<__bf16, BWD, DW_CB_BF16>), dim3(N, cdiv(C, DW_CB_BF16)), dim3(256), sm, st,
                       (const __bf16*)x, xcs, w, b, (__bf16*)y, ycs, H, W, C, k, acc);
  else if (dtype == ADR_BF16)
    hipLaunchKernelGGL((dw_img_kernel<__bf16, BWD, DW_CB_BF16 / 2>), dim3(N, cdiv(C, DW_CB_BF16 / 2)), dim3(256), sm,
                       st, (const __bf16*)x, xcs, w, b, (__bf16*)y, ycs, H, W, C, k, acc);
  else if (cb == DW_CB_F32)
    hipLaunchKernelGGL((dw_img_kernel<float, BWD, DW_CB_F32>), dim3(N, cdiv(C, DW_CB_F32)), dim3(256), sm, st,
                       (const float*)x, xcs, w, b, (float*)y, ycs, H, W, C, k, acc);
  else
    hipLaunchKernelGGL((dw_img_kernel<float, BWD, DW_CB_F32 / 2>), dim3(N, cdiv(C, DW_CB_F32 / 2)), dim3(256), sm, st,
                       (const float*)x, xcs, w, b, (float*)y, ycs, H, W, C, k, acc);
}

template <typename T, bool BWD>
static void dw_launch(int k, dim3 grid, size_t sm, hipStream_t st, const T* x, int xcs, const float* w, const float* b,
                      T* y, int ycs, int N, int H, int W, int C, int acc) {
  if (k == 3)
    hipLaunchKernelGGL((dw_kernel<T, BWD, 3>), grid, dim3(256), sm, st, x, xcs, w, b, y, ycs, N, H, W, C, k, acc);
  else if (k == 5)
    hipLaunchKernelGGL((dw_kernel<T, BWD, 5>), grid, dim3(256), sm, st, x, xcs, w, b, y, ycs, N, H, W, C, k, acc);
  else if (k == 7)
    hipLaunchKernelGGL((dw_kernel<T, BWD, 7>), grid, dim3(256), sm, st, x, xcs, w, b, y, ycs, N, H, W, C, k, acc);
  else
    hipLaunchKernelGGL((dw_kernel<T, BWD, 0>), grid, dim3(256), sm, st, x, xcs, w, b, y, ycs, N, H, W, C, k, acc);
}

extern "C" int adr_dwconv_fwd(int dtype, const void* x, int xcs, const float* w, const float* b, void* y, int ycs,
                              int N, int H, int W, int C, int k, void* stream) {
  int v = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % v == 0 && xcs % v == 0 && ycs % v == 0 && k % 2 == 1, "dwconv: C=%d k=%d", C, k);
  hipStream_t st = (hipStream_t)stream;
  long total = (long)N * H * W * (C / v);
  size_t sm = (size_t)k * k * C * sizeof(float);
  ADR_REQUIRE(total < (1l << 32) && sm <= 64 * 1024, "dwconv: N*H*W*C=%ld / k=%d C=%d too large", total, k, C);
  if (dw_img_ok() && dw_fwd_cb(dtype, H, W, k) && xcs % v == 0 && ycs % v == 0) {
    dw_img_launch<false>(dtype, st, x, xcs, w, b, y, ycs, N, H, W, C, k, 0);
  } else if (dtype == ADR_BF16)
    dw_launch<__bf16, false>(k, dim3(cdiv(total, 256)), sm, st, (const __bf16*)x, xcs, w, b, (__bf16*)y, ycs, N, H, W,
                             C, 0);
  else
    dw_launch<float, false>(k, dim3(cdiv(total, 256)), sm, st, (const float*)x, xcs, w, b, (float*)y, ycs, N, H, W, C,
                            0);
  return check_launch("adr_dwconv_fwd");
}

extern "C" int adr_dwconv_fwd_act_supported(int H, int W, int C, int k) {
  return dw_img_ok() && k % 2 == 1 && C % 8 == 0 && dw_fwd_smem_cb(ADR_BF16, H, W, k, DW_CB_BF16) <= DW_LDS_MAX ? 1 : 0;
}

// Eval DWConv-BN-act (reference: Conv.forward_fuse after fuse_conv_and_bn on a depthwise Conv, nn/modules/conv.py:52-54
// / 101-106): y = act(dwconv(x, w * scale) + shift) in one launch, bf16, whole-image kernel only.
extern "C" int adr_dwconv_fwd_act(const void* x, int xcs, const float* w, const float* scale, const float* shift,
                                  int act, void* y, int ycs, int N, int H, int W, int C, int k, void* stream) {
  ADR_REQUIRE(scale && shift && xcs % 8 == 0 && ycs % 8 == 0 && act >= ACT_NONE && act <= ACT_HSWISH,
              "dwconv act: bad arguments");
  ADR_REQUIRE(adr_dwconv_fwd_act_supported(H, W, C, k), "dwconv act: H=%d W=%d C=%d k=%d not on the image kernel", H, W,
              C, k);
  hipStream_t st = (hipStream_t)stream;
  if (dw_f32s(ADR_BF16, H, W, k, DW_CB_BF16))
    hipLaunchKernelGGL((dw_img_act_kernel<DW_CB_BF16, true>), dim3(N, cdiv(C, DW_CB_BF16)), dim3(256),
                       dw_fwd_smem_cb(ADR_F32, H, W, k, DW_CB_BF16), st, (const __bf16*)x, xcs, w, scale, shift, act,
                       (__bf16*)y, ycs, H, W, C, k);
  else
    hipLaunchKernelGGL((dw_img_act_kernel<DW_CB_BF16>), dim3(N, cdiv(C, DW_CB_BF16)), dim3(256),
                       dw_fwd_smem_cb(ADR_BF16, H, W, k, DW_CB_BF16), st, (const __bf16*)x, xcs, w, scale, shift, act,
                       (__bf16*)y, ycs, H, W, C, k);
  return check_launch("adr_dwconv_fwd_act");
}

extern "C" size_t adr_dwconv_wgrad_workspace(int N, int H, int W, int C, int k) {
  long npix = (long)N * H * W;
  int chunks = cdiv(npix, 1024);
  if (chunks < N) chunks = N;  // the whole-image kernel writes one partial row per image
  return (size_t)chunks * k * k * C * sizeof(float);
}

// the depthwise weight gradient's partial rows [chunks][k*k][C] into ws; returns chunks (N on the whole-image path)
static int dw_wgrad_partials(int dtype, const void* x, int xcs, const void* dy, int dcs, int N, int H, int W, int C,
                             int k, float* ws, hipStream_t st, float* bias_part = nullptr) {
  const int v = dtype == ADR_BF16 ? 8 : 4;
  const long npix = (long)N * H * W;
  const int wcb = dw_wg_cb(H, W, k);
  if (!(wcb && xcs % v == 0 && dcs % v == 0)) {  // maps too large for LDS: the direct kernel, 1024-pixel chunks
    const int chunks = cdiv(npix, 1024);
    const dim3 g(chunks, k * k);
    if (dtype == ADR_BF16)
      hipLaunchKernelGGL(dw_bwd_w_kernel<__bf16>, g, dim3(256), 0, st, (const __bf16*)x, xcs, (const __bf16*)dy, dcs,
                         N, H, W, C, k, 1024, ws);
    else
      hipLaunchKernelGGL(dw_bwd_w_kernel<float>, g, dim3(256), 0, st, (const float*)x, xcs, (const float*)dy, dcs, N,
                         H, W, C, k, 1024, ws);
    return chunks;
  }
  // whole image in LDS (fp32 copies): the 20x20 / 40x40 C2PTSSA, EDFFN, Mona maps; one partial row per image
  const size_t ism = dw_img_smem_cb(H, W, k, wcb);
  const dim3 ig(N, cdiv(C, wcb));
#define ADR_DWWG(CBV)                                                                                               \
  if (dtype == ADR_BF16 && dw_row_ok() && (k == 3 || k == 5 || k == 7)) {                                         \
    if (k == 3)                                                                                                     \
      hipLaunchKernelGGL((dw_wgrad_row_kernel<__bf16, CBV, 3>), ig, dim3(256), ism, st, (const __bf16*)x, xcs,    \
                         (const __bf16*)dy, dcs, H, W, C, ws, bias_part);                                           \
    else if (k == 5)                                                                                                \
      hipLaunchKernelGGL((dw_wgrad_row_kernel<__bf16, CBV, 5>), ig, dim3(256), ism, st, (const __bf16*)x, xcs,    \
                         (const __bf16*)dy, dcs, H, W, C, ws, bias_part);                                           \
    else                                                                                                            \
      hipLaunchKernelGGL((dw_wgrad_row_kernel<__bf16, CBV, 7>), ig, dim3(256), ism, st, (const __bf16*)x, xcs,    \
                         (const __bf16*)dy, dcs, H, W, C, ws, bias_part);                                           \
  } else if (dtype == ADR_BF16)                                                                                     \
    hipLaunchKernelGGL((dw_wgrad_img_kernel<__bf16, CBV>), ig, dim3(256), ism, st, (const __bf16*)x, xcs,         \
                       (const __bf16*)dy, dcs, H, W, C, k, ws, bias_part);                                          \
  else                                                                                                              \
    hipLaunchKernelGGL((dw_wgrad_img_kernel<float, CBV>), ig, dim3(256), ism, st, (const float*)x, xcs,           \
                       (const float*)dy, dcs, H, W, C, k, ws, bias_part)
  if (wcb == DW_CB_WG) {
    ADR_DWWG(DW_CB_WG);
  } else {
    ADR_DWWG(4);
  }
#undef ADR_DWWG
  return N;
}

extern "C" int adr_dwconv_bwd(int dtype, const void* x, int xcs, const void* dy, int dcs, const float* w, void* dx,
                              int ocs, float* dw, int N, int H, int W, int C, int k, int accumulate,
                              int dw_accumulate, float* ws, size_t ws_bytes, void* stream) {
  int v = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % v == 0 && C / v <= 256, "dwconv_bwd: C=%d", C);
  hipStream_t st = (hipStream_t)stream;
  long total = (long)N * H * W * (C / v);
  if (dx) {
    size_t sm = (size_t)k * k * C * sizeof(float);
    ADR_REQUIRE(total < (1l << 32) && sm <= 64 * 1024, "dwconv_bwd: N*H*W*C=%ld / k=%d C=%d too large", total, k, C);
    if (dw_img_ok() && dw_fwd_cb(dtype, H, W, k) && dcs % v == 0 && ocs % v == 0)
      dw_img_launch<true>(dtype, st, dy, dcs, w, nullptr, dx, ocs, N, H, W, C, k, accumulate);
    else if (dtype == ADR_BF16)
      dw_launch<__bf16, true>(k, dim3(cdiv(total, 256)), sm, st, (const __bf16*)dy, dcs, w, nullptr, (__bf16*)dx, ocs, N,
                              H, W, C, accumulate);
    else
      dw_launch<float, true>(k, dim3(cdiv(total, 256)), sm, st, (const float*)dy, dcs, w, nullptr, (float*)dx, ocs, N, H,
                             W, C, accumulate);
  }
  if (dw) {
    ADR_REQUIRE(ws_bytes >= adr_dwconv_wgrad_workspace(N, H, W, C, k), "dwconv_bwd: workspace");
    const int chunks = dw_wgrad_partials(dtype, x, xcs, dy, dcs, N, H, W, C, k, ws, st);
    hipLaunchKernelGGL(dw_w_reduce_kernel, dim3(cdiv(C * k * k, 256)), dim3(256), 0, st, ws, chunks, C, k * k, dw,
                       dw_accumulate);
  }
  return check_launch("adr_dwconv_bwd");
}

// the weight-gradient partial rows only (the trainer reduces them at its deferred flush, batched with the conv
// weight gradients: adr_wgrad_reduce_batched with K = 1, RS = k*k); returns the row count via *chunks
extern "C" int adr_dwconv_wgrad_partials(int dtype, const void* x, int xcs, const void* dy, int dcs, int N, int H,
                                         int W, int C, int k, float* ws, size_t ws_bytes, int* chunks, void* stream) {
  const int v = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % v == 0 && C / v <= 256 && chunks && ws, "dwconv_wgrad_partials: C=%d", C);
  ADR_REQUIRE(ws_bytes >= adr_dwconv_wgrad_workspace(N, H, W, C, k), "dwconv_wgrad_partials: workspace");
  *chunks = dw_wgrad_partials(dtype, x, xcs, dy, dcs, N, H, W, C, k, ws, (hipStream_t)stream);
  return check_launch("adr_dwconv_wgrad_partials");
}

extern "C" int adr_dwconv_wgrad_bias_fusable(int dtype, int H, int W, int C, int k, int xcs, int dcs) {
  const int v = dtype == ADR_BF16 ? 8 : 4;
  return C % v == 0 && xcs % v == 0 && dcs % v == 0 && dw_wg_cb(H, W, k) ? 1 : 0;
}

extern "C" int adr_dwconv_wgrad_partials_bias(int dtype, const void* x, int xcs, const void* dy, int dcs, int N, int H,
                                              int W, int C, int k, float* ws, size_t ws_bytes, float* bias_part,
                                              int* chunks, void* stream) {
  ADR_REQUIRE(chunks && ws && bias_part && adr_dwconv_wgrad_bias_fusable(dtype, H, W, C, k, xcs, dcs),
              "dwconv_wgrad_partials_bias: H=%d W=%d C=%d k=%d not on the whole-image kernels", H, W, C, k);
  ADR_REQUIRE(ws_bytes >= adr_dwconv_wgrad_workspace(N, H, W, C, k), "dwconv_wgrad_partials_bias: workspace");
  *chunks = dw_wgrad_partials(dtype, x, xcs, dy, dcs, N, H, W, C, k, ws, (hipStream_t)stream, bias_part);
  return check_launch("adr_dwconv_wgrad_partials_bias");
}

extern "C" int adr_adyt_fwd(int dtype, const void* x, int xcs, const float* alphas, const float* imp, const float* w,
                            const float* b, void* y, int ycs, int N, int HW, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  long npix = (long)N * HW;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(adyt_fwd_kernel<__bf16>, dim3(cdiv(npix * C, 256)), dim3(256), 0, st, (const __bf16*)x, xcs,
                       alphas, imp, w, b, (__bf16*)y, ycs, npix, HW, C);
  else
    hipLaunchKernelGGL(adyt_fwd_kernel<float>, dim3(cdiv(npix * C, 256)), dim3(256), 0, st, (const float*)x, xcs, alphas,
                       imp, w, b, (float*)y, ycs, npix, HW, C);
  return check_launch("adr_adyt_fwd");
}

// rows per adyt_bwd workgroup: 256, halved until the grid has ~1024 workgroups (the C2PTSSA maps are 20x20: one
// 256-row chunk per image left half the chip idle, each thread walking 128 rows of three tanh each)
static int adyt_rows(int N, int HW) {
  int r = 256;
  while (r > 16 && (long)N * cdiv(HW, r) < 1024) r /= 2;
  return r;
}

extern "C" size_t adr_adyt_bwd_workspace(int N, int HW, int C) {
  return ((size_t)N * cdiv(HW, adyt_rows(N, HW)) * 8 * C + (size_t)N * 3) * sizeof(float);
}

extern "C" int adr_adyt_bwd(int dtype, const void* x, int xcs, const void* dout, int dcs, const float* alphas,
                            const float* imp, const float* w, void* dx, int ocs, float* dimp, float* dalpha, float* dw,
                            float* db, int N, int HW, int C, float* ws, size_t ws_bytes, void* stream) {
  ADR_REQUIRE(C <= 256, "adyt_bwd: C=%d > 256", C);
  ADR_REQUIRE(ws_bytes >= adr_adyt_bwd_workspace(N, HW, C), "adyt_bwd: workspace");
  hipStream_t st = (hipStream_t)stream;
  const int rows = adyt_rows(N, HW), chunks = cdiv(HW, rows);
  dim3 g(chunks, N);
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(adyt_bwd_kernel<__bf16>, g, dim3(256), 0, st, (const __bf16*)x, xcs, (const __bf16*)dout, dcs,
                       alphas, imp, w, (__bf16*)dx, ocs, HW, C, rows, chunks, ws);
  else
    hipLaunchKernelGGL(adyt_bwd_kernel<float>, g, dim3(256), 0, st, (const float*)x, xcs, (const float*)dout, dcs,
                       alphas, imp, w, (float*)dx, ocs, HW, C, rows, chunks, ws);
  float* dan = ws + (size_t)N * chunks * 8 * C;
  hipLaunchKernelGGL(adyt_collapse_kernel, dim3(3 * N + C), dim3(256), 0, st, ws, N, chunks, C, dimp, dan, dw, db);
  hipLaunchKernelGGL(adyt_alpha_kernel, dim3(1), dim3(64), 0, st, dan, imp, N, dalpha);
  return check_launch("adr_adyt_bwd");
}

extern "C" int adr_tssa_fwd(int dtype, const void* q, const void* k, const void* v, int cs, int B, int Ntok, int heads,
                            int D, const float* temp, void* out, int ocs, int oimg, float* Pi, float* ss, float* attn,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int vw = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(D == 64 && cs % vw == 0 && ocs % vw == 0, "tssa: head dim %d (64 supported) / strides", D);
  const size_t sm = Ntok * sizeof(float);
  ADR_REQUIRE(sm <= 64 * 1024, "tssa: Ntok=%d too large", Ntok);
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL((tssa_fwd_kernel<__bf16, 8, 8, TSSA_NTH>), dim3(B * heads), dim3(TSSA_NTH), sm, st, (const __bf16*)q,
                       (const __bf16*)k, (const __bf16*)v, cs, Ntok, temp, (__bf16*)out, ocs, oimg, heads, Pi, ss,
                       attn);
  else
    hipLaunchKernelGGL((tssa_fwd_kernel<float, 4, 16, TSSA_NTH>), dim3(B * heads), dim3(TSSA_NTH), sm, st, (const float*)q,
                       (const float*)k, (const float*)v, cs, Ntok, temp, (float*)out, ocs, oimg, heads, Pi, ss, attn);
  return check_launch("adr_tssa_fwd");
}

extern "C" int adr_tssa_bwd(int dtype, const void* q, const void* k, const void* v, int cs, int B, int Ntok, int heads,
                            int D, const float* temp, const void* dout, int dcs, int dimg, const float* Pi,
                            const float* ss,
                            const float* attn, void* dq, void* dk, void* dv, int gcs, float* dtemp, float* ws,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int vw = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(D == 64 && cs % vw == 0 && dcs % vw == 0 && gcs % vw == 0, "tssa_bwd: head dim %d / strides", D);
  const size_t sm = Ntok * sizeof(float);
  ADR_REQUIRE(sm <= 64 * 1024, "tssa_bwd: Ntok=%d too large", Ntok);
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL((tssa_bwd_kernel<__bf16, 8, 8, TSSA_NTH>), dim3(B * heads), dim3(TSSA_NTH), sm, st, (const __bf16*)q,
                       (const __bf16*)k, (const __bf16*)v, cs, Ntok, temp, (const __bf16*)dout, dcs, dimg, heads, Pi,
                       ss, attn, (__bf16*)dq, (__bf16*)dk, (__bf16*)dv, gcs, ws);
  else
    hipLaunchKernelGGL((tssa_bwd_kernel<float, 4, 16, TSSA_NTH>), dim3(B * heads), dim3(TSSA_NTH), sm, st, (const float*)q,
                       (const float*)k, (const float*)v, cs, Ntok, temp, (const float*)dout, dcs, dimg, heads, Pi, ss,
                       attn, (float*)dq, (float*)dk, (float*)dv, gcs, ws);
  hipLaunchKernelGGL(tssa_temp_reduce_kernel, dim3(1), dim3(64), 0, st, ws, B, heads, dtemp);
  return check_launch("adr_tssa_bwd");
}

extern "C" int adr_group_mean(int dtype, const void* x, int xcs, int S, int HW, void* y, int ycs, int B, int C,
                              int backward, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  long total = (long)B * (backward ? S : 1) * HW * C;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(group_mean_kernel<__bf16>, dim3(cdiv(total, 256)), dim3(256), 0, st, (const __bf16*)x, xcs, S,
                       HW, (__bf16*)y, ycs, (long)B, C, backward);
  else
    hipLaunchKernelGGL(group_mean_kernel<float>, dim3(cdiv(total, 256)), dim3(256), 0, st, (const float*)x, xcs, S, HW,
                       (float*)y, ycs, (long)B, C, backward);
  return check_launch("adr_group_mean");
}

extern "C" int adr_edffn_build(const float* w, const float* basis, int C, int nuv, float* M, void* stream) {
  if (C % 8 == 0)
    hipLaunchKernelGGL(edffn_build8_kernel, dim3(16, C / 8), dim3(256), 0, (hipStream_t)stream, w, basis, C, nuv, M);
  else
    hipLaunchKernelGGL(edffn_build_kernel, dim3(cdiv((long)C * 4096, 256)), dim3(256), 0, (hipStream_t)stream, w, basis,
                       C, nuv, M);
  return check_launch("adr_edffn_build");
}

// the matrix-core apply: bf16 tensors, 8-channel groups, 16-byte aligned channel rows (ADR_EDFFN_MFMA=0: the
// per-channel kernel, A/B)
static bool edffn_mfma_ok(int dtype, int C, int xcs, int ycs, const void* p0 = nullptr, const void* p1 = nullptr) {
  const char* e = getenv("ADR_EDFFN_MFMA");  // read per call: tests compare the two paths in one process
  const bool v = e ? atoi(e) != 0 : true;
  return v && dtype == ADR_BF16 && C % EA_CG == 0 && xcs % 8 == 0 && ycs % 8 == 0 &&
         ((uintptr_t)p0 & 15) == 0 && ((uintptr_t)p1 & 15) == 0;  // 16-byte pixel-row loads / stores
}

extern "C" int adr_edffn_fwd(int dtype, const void* x, int xcs, const float* M, void* y, int ycs, int N, int H, int W,
                             int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  ADR_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && H >= 4 && W >= 4, "edffn: N=%d H=%d W=%d C=%d", N, H, W, C);
  const long np = (long)N * ((H + 7) / 8) * ((W + 7) / 8);
  dim3 grid((unsigned)(cdiv(np, EDFFN_PPB) * C));
  if (edffn_mfma_ok(dtype, C, xcs, ycs, x, y))
    hipLaunchKernelGGL(edffn_apply_mfma_kernel<false>, dim3((unsigned)(C / EA_CG * cdiv(np, EA_PG))), dim3(256), 0, st,
                       (const __bf16*)x, xcs, M, y, ycs, N, H, W, C);
  else if (dtype == ADR_BF16)
    hipLaunchKernelGGL(edffn_apply_kernel<__bf16>, grid, dim3(256), 0, st, (const __bf16*)x, xcs, M, (__bf16*)y, ycs,
                       N, H, W, C, 0);
  else
    hipLaunchKernelGGL(edffn_apply_kernel<float>, grid, dim3(256), 0, st, (const float*)x, xcs, M, (float*)y, ycs, N,
                       H, W, C, 0);
  return check_launch("adr_edffn_fwd");
}

static size_t edffn_pad_floats(int N, int H, int W, int C) {
  const size_t hp = (H + 7) / 8 * 8, wp = (W + 7) / 8 * 8;
  return (size_t)N * hp * wp * C;
}

// padded dx scratch + the per-split spectral-weight partials
extern "C" size_t adr_edffn_bwd_workspace(int N, int H, int W, int C) {
  return (edffn_pad_floats(N, H, W, C) + (size_t)EDFFN_DWS * C * 4096) * sizeof(float);
}

extern "C" int adr_edffn_bwd(int dtype, const void* x, int xcs, const void* dy, int dcs, const float* M,
                             const float* basis, int nuv, void* dx, int ocs, float* dw, int N, int H, int W, int C,
                             int dw_accumulate, float* ws, size_t ws_bytes, void* stream) {
  ADR_REQUIRE(ws_bytes >= adr_edffn_bwd_workspace(N, H, W, C), "edffn_bwd: workspace");
  ADR_REQUIRE(N > 0 && H >= 4 && W >= 4 && C > 0, "edffn_bwd: N=%d H=%d W=%d C=%d", N, H, W, C);
  hipStream_t st = (hipStream_t)stream;
  const long np = (long)N * ((H + 7) / 8) * ((W + 7) / 8);
  dim3 grid((unsigned)(cdiv(np, EDFFN_PPB) * C));
  float* dpad = ws;
  if (edffn_mfma_ok(dtype, C, dcs, 8, dy))
    hipLaunchKernelGGL(edffn_apply_mfma_kernel<true>, dim3((unsigned)(C / EA_CG * cdiv(np, EA_PG))), dim3(256), 0, st,
                       (const __bf16*)dy, dcs, M, (void*)dpad, 0, N, H, W, C);
  else if (dtype == ADR_BF16)
    hipLaunchKernelGGL(edffn_apply_kernel<__bf16>, grid, dim3(256), 0, st, (const __bf16*)dy, dcs, M, (__bf16*)dpad, 0,
                       N, H, W, C, 1);
  else
    hipLaunchKernelGGL(edffn_apply_kernel<float>, grid, dim3(256), 0, st, (const float*)dy, dcs, M, (float*)dpad, 0,
                       N, H, W, C, 1);
  long total = (long)N * H * W * C;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(edffn_fold_kernel<__bf16>, dim3(cdiv(total, 256)), dim3(256), 0, st, dpad, H, W, C, (long)N,
                       (__bf16*)dx, ocs);
  else
    hipLaunchKernelGGL(edffn_fold_kernel<float>, dim3(cdiv(total, 256)), dim3(256), 0, st, dpad, H, W, C, (long)N,
                       (float*)dx, ocs);
  if (dw) {
    float* part = ws + edffn_pad_floats(N, H, W, C);
    if (edffn_mfma_ok(dtype, C, xcs, dcs, x, dy))
      hipLaunchKernelGGL(edffn_dw_mfma_kernel, dim3((unsigned)(C / EA_CG * EDFFN_DWS)), dim3(256), 0, st,
                         (const __bf16*)x, xcs, (const __bf16*)dy, dcs, N, H, W, C, part);
    else if (dtype == ADR_BF16)
      hipLaunchKernelGGL(edffn_dw_kernel<__bf16>, dim3(C, EDFFN_DWS), dim3(256), 0, st, (const __bf16*)x, xcs,
                         (const __bf16*)dy, dcs, N, H, W, C, part);
    else
      hipLaunchKernelGGL(edffn_dw_kernel<float>, dim3(C, EDFFN_DWS), dim3(256), 0, st, (const float*)x, xcs,
                         (const float*)dy, dcs, N, H, W, C, part);
    if (edffn_mfma_ok(dtype, C, xcs, dcs, x, dy))
      hipLaunchKernelGGL(edffn_dw_fin2_kernel, dim3(C, 2), dim3(256), 0, st, part, C, basis, nuv, dw, dw_accumulate);
    else
      hipLaunchKernelGGL(edffn_dw_fin_kernel, dim3(C), dim3(256), 0, st, part, C, basis, nuv, dw, dw_accumulate);
  }
  return check_launch("adr_edffn_bwd");
}
