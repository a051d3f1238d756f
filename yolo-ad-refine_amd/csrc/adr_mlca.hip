// MLCA — mixed local channel attention (reference nn/modules/block.py:1540-1584), fused:
//   fwd1  local[n][p][c]   = adaptive_avg_pool(x, 5)                    (p = i*5 + j, bins as PyTorch)
//   fwd2  per image:  seq[p*C + c] = local[p][c]   (the reference's (pos, chan)-interleaved sequence)
//                     att_l = sigmoid(conv1d_k(seq))  viewed back as [p][c]
//                     g[c] = mean_p local[p][c];   sig_g[n][c] = sigmoid(conv1d_k(g))
//        mix   att[n][p=(i,j)][c] = (1 - lw) * mean_{r in rows(i)} sig_g[r][c] + lw * att_l[n][p][c]
//              — the reference pools the (C, B, 1)-shaped global attention with adaptive_avg_pool2d(.., [5,5])
//              (block.py:1578), i.e. over the BATCH axis: rows(i) = [floor(i*B/5), ceil((i+1)*B/5)). Kept
//              bit-for-bit in semantics (it couples images of one per-GPU batch, exactly as the reference does).
//   fwd3  out = res + y * up(att)  with up = adaptive_avg_pool(att, (H, W))  (Bottleneck_MLCA :1594)
// Backward mirrors it: bwd1 reduces dout*y into the 5x5 bins (adjoint of up), bwd2 back-propagates through the
// sigmoids / both Conv1d(1,1,k) (weight grads per image, summed later), bwd3 forms
// dy = dout * up(att) + adjoint_pool(dlocal).  All deterministic (no atomics).
#include "adr_common.h"
#include <initializer_list>

namespace adr {

static constexpr int LS = 5;  // local_size
__device__ __forceinline__ int a_s(int o, int in, int out) { return (int)(((long)o * in) / out); }
__device__ __forceinline__ int a_e(int o, int in, int out) { return (int)(((long)(o + 1) * in + out - 1) / out); }

// fwd1: grid (25, N); local fp32 [N][25][C]. Threads = channel groups (VW channels) x pixel splits of the bin,
// fixed-order LDS combine.
template <typename T, int VW>
__global__ void __launch_bounds__(256) mlca_pool_kernel(const T* x, int xcs, int H, int W, int C, float* local) {
  __shared__ float red[256 * VW];
  const int p = blockIdx.x, n = blockIdx.y;
  const int i = p / LS, j = p % LS;
  const int hs = a_s(i, H, LS), he = a_e(i, H, LS), ws = a_s(j, W, LS), we = a_e(j, W, LS);
  const int bw = we - ws, cnt = (he - hs) * bw;
  const float inv = 1.f / (float)cnt;
  const int G = C / VW;
  for (int cb = 0; cb < G; cb += 256) {
    const int gn = min(256, G - cb), S = 256 / gn;
    const int cg = cb + threadIdx.x % gn, sp = threadIdx.x / gn, c0 = cg * VW;
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    if (sp < S)
      for (int q = sp; q < cnt; q += S) {
        const int h = hs + q / bw, w = ws + q % bw;
        float v[VW];
        vload<T, VW>(x + (((long)n * H + h) * W + w) * xcs + c0, v);
#pragma unroll
        for (int e = 0; e < VW; ++e) s[e] += v[e];
      }
#pragma unroll
    for (int e = 0; e < VW; ++e) red[threadIdx.x * VW + e] = s[e];
    __syncthreads();
    if (threadIdx.x < gn) {
#pragma unroll
      for (int e = 0; e < VW; ++e) {
        float t = 0.f;
        for (int r = 0; r < S; ++r) t += red[(r * gn + threadIdx.x) * VW + e];
        local[((long)n * LS * LS + p) * C + c0 + e] = t * inv;
      }
    }
    __syncthreads();
  }
}

// fwd2: one block per image. att fp32 [N][25][C]; saves sig_l [N][25*C] (sequence order) and sig_g [N][C]
__global__ void __launch_bounds__(256) mlca_att_kernel(const float* local, int C, const float* wl, const float* wg,
                                                       int k, float* sig_l, float* sig_g) {
  int n = blockIdx.x;
  const float* L = local + (long)n * LS * LS * C;
  int L_len = LS * LS * C, pad = (k - 1) / 2;
  extern __shared__ float sm[];
  float* g = sm;       // C
  float* sg = sm + C;  // C
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int p = 0; p < LS * LS; ++p) s += L[p * C + c];
    g[c] = s / (float)(LS * LS);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float y = 0.f;
    for (int t = 0; t < k; ++t) {
      int q = c + t - pad;
      if (q >= 0 && q < C) y += wg[t] * g[q];
    }
    float s = 1.f / (1.f + __expf(-y));
    sg[c] = s;
    sig_g[(long)n * C + c] = s;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < L_len; idx += 256) {
    float y = 0.f;
    for (int t = 0; t < k; ++t) {
      int q = idx + t - pad;
      if (q >= 0 && q < L_len) y += wl[t] * L[q];  // L is already in sequence order p*C + c
    }
    sig_l[(long)n * L_len + idx] = 1.f / (1.f + __expf(-y));
  }
}

// att[n][p][c] = (1-lw) * mean_{r in rows(i)} sig_g[r][c] + lw * sig_l[n][p*C+c]
__global__ void mlca_mix_kernel(const float* sig_l, const float* sig_g, int N, int C, float lw, float* att) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * LS * LS * C;
  if (idx >= total) return;
  int c = (int)(idx % C);
  long r = idx / C;
  int p = (int)(r % (LS * LS));
  int i = p / LS;
  int rs = a_s(i, N, LS), re = a_e(i, N, LS);
  float g = 0.f;
  for (int b = rs; b < re; ++b) g += sig_g[(long)b * C + c];
  g /= (float)(re - rs);
  att[idx] = (1.f - lw) * g + lw * sig_l[idx];
}

// S[i][c] = sum_n sum_j datt[n][i*5+j][c]: block i; threads = (image part, channel), parts of the image sum
// combined in order through LDS (deterministic)
__global__ void __launch_bounds__(256) mlca_gsum_kernel(const float* datt, int N, int C, float* S) {
  __shared__ float red[256];
  const int i = blockIdx.x;
  for (int c0 = 0; c0 < C; c0 += 256) {
    const int cb = min(256, C - c0), P = 256 / cb;
    const int c = c0 + threadIdx.x % cb, part = threadIdx.x / cb;
    float s = 0.f;
    if (part < P)
      for (int n = part; n < N; n += P)
#pragma unroll
        for (int j = 0; j < LS; ++j) s += datt[((long)n * LS * LS + i * LS + j) * C + c];
    red[threadIdx.x] = s;
    __syncthreads();
    if ((int)threadIdx.x < cb) {
      float t = 0.f;
      for (int q = 0; q < P; ++q) t += red[q * cb + threadIdx.x];
      S[i * C + c] = t;
    }
    __syncthreads();
  }
}

// up(att)[h][w][c0..c0+VW) = mean of att over the 5x5 bins in pixel (h, w)'s window
template <int VW>
__device__ __forceinline__ void up_att(const float* A, int C, int h, int w, int H, int W, int c0, float* out) {
  const int is = a_s(h, LS, H), ie = a_e(h, LS, H), js = a_s(w, LS, W), je = a_e(w, LS, W);
#pragma unroll
  for (int e = 0; e < VW; ++e) out[e] = 0.f;
  for (int i = is; i < ie; ++i)
    for (int j = js; j < je; ++j) {
      const float* a = A + (i * LS + j) * C + c0;
#pragma unroll
      for (int e = 0; e < VW; ++e) out[e] += a[e];
    }
  const float inv = 1.f / (float)((ie - is) * (je - js));
#pragma unroll
  for (int e = 0; e < VW; ++e) out[e] *= inv;
}

// fwd3: out = res + y * up(att)
template <typename T, int VW>
__global__ void __launch_bounds__(256) mlca_apply_kernel(const T* y, int ycs, const T* res, int rcs, const float* att,
                                                         T* out, int ocs, int N, int H, int W, int C) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    float a[VW], v[VW];
    up_att<VW>(att + (long)n * LS * LS * C, C, h, w, H, W, c0, a);
    vload<T, VW>(y + pix * ycs + c0, v);
#pragma unroll
    for (int e = 0; e < VW; ++e) v[e] *= a[e];
    if (res) {
      float r[VW];
      vload<T, VW>(res + pix * rcs + c0, r);
#pragma unroll
      for (int e = 0; e < VW; ++e) v[e] += r[e];
    }
    vstore<T, VW>(out + pix * ocs + c0, v);
  }
}

// bwd1: datt[n][p][c] = sum over pixels whose up-window includes bin p of dout*y / window_count ; grid (25, N).
// The pixels of bin (bi, bj) lie in a rectangle one row / column wider than the bin's pooling window.
template <typename T, int VW>
__global__ void __launch_bounds__(256) mlca_bwd_bins_kernel(const T* y, int ycs, const T* dout, int dcs, int H, int W,
                                                            int C, float* datt) {
  __shared__ float red[256 * VW];
  const int p = blockIdx.x, n = blockIdx.y;
  const int bi = p / LS, bj = p % LS;
  const int h0 = max(0, a_s(bi, H, LS) - 1), h1 = min(H, a_e(bi, H, LS) + 1);
  const int w0 = max(0, a_s(bj, W, LS) - 1), w1 = min(W, a_e(bj, W, LS) + 1);
  const int rw = w1 - w0, cnt = (h1 - h0) * rw;
  const int G = C / VW;
  for (int cb = 0; cb < G; cb += 256) {
    const int gn = min(256, G - cb), S = 256 / gn;
    const int cg = cb + threadIdx.x % gn, sp = threadIdx.x / gn, c0 = cg * VW;
    float s[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) s[e] = 0.f;
    if (sp < S)
      for (int q = sp; q < cnt; q += S) {
        const int h = h0 + q / rw, w = w0 + q % rw;
        const int is = a_s(h, LS, H), ie = a_e(h, LS, H);
        const int js = a_s(w, LS, W), je = a_e(w, LS, W);
        if (bi < is || bi >= ie || bj < js || bj >= je) continue;
        const float inv = 1.f / (float)((ie - is) * (je - js));
        const long pix = ((long)n * H + h) * W + w;
        float d[VW], v[VW];
        vload<T, VW>(dout + pix * dcs + c0, d);
        vload<T, VW>(y + pix * ycs + c0, v);
#pragma unroll
        for (int e = 0; e < VW; ++e) s[e] += d[e] * v[e] * inv;
      }
#pragma unroll
    for (int e = 0; e < VW; ++e) red[threadIdx.x * VW + e] = s[e];
    __syncthreads();
    if (threadIdx.x < gn) {
#pragma unroll
      for (int e = 0; e < VW; ++e) {
        float t = 0.f;
        for (int r = 0; r < S; ++r) t += red[(r * gn + threadIdx.x) * VW + e];
        datt[((long)n * LS * LS + p) * C + c0 + e] = t;
      }
    }
    __syncthreads();
  }
}

// bwd2: one block per image -> dlocal [N][25][C]; per-image weight grads dwl_part/dwg_part [N][k]
// MLCA_NT threads: one block per image walks all 25 x C bins (16 blocks at l-scale), so wider blocks put more
// loads in flight
#ifndef MLCA_NT
#define MLCA_NT 512
#endif
__global__ void __launch_bounds__(MLCA_NT) mlca_att_bwd_kernel(const float* local, const float* datt, const float* sig_l,
                                                           const float* sig_g, const float* S, int N, int C,
                                                           const float* wl, const float* wg, int k, float lw,
                                                           float* dlocal, float* dwl_part, float* dwg_part) {
  int n = blockIdx.x;
  int L_len = LS * LS * C, pad = (k - 1) / 2;
  const float* L = local + (long)n * L_len;
  const float* D = datt + (long)n * L_len;
  const float* SL = sig_l + (long)n * L_len;
  const float* SG = sig_g + (long)n * C;
  extern __shared__ float sm[];
  float* dyg = sm;                 // C   : d(pre-sigmoid global)
  float* g = sm + C;               // C   : global means
  float* dyl = sm + 2 * C;         // L_len : d(pre-sigmoid local seq)
  float* red = sm + 2 * C + L_len; // 2 * MLCA_NT scratch
  for (int c = threadIdx.x; c < C; c += MLCA_NT) {
    float m = 0.f;
    for (int p = 0; p < LS * LS; ++p) m += L[p * C + c];
    // d sig_g[n][c] = (1-lw) * sum over bins i whose batch-row window holds n of S[i][c] / |rows(i)|
    float s = 0.f;
    for (int i = 0; i < LS; ++i) {
      int rs = a_s(i, N, LS), re = a_e(i, N, LS);
      if (n >= rs && n < re) s += S[i * C + c] / (float)(re - rs);
    }
    float sgv = SG[c];
    dyg[c] = (1.f - lw) * s * sgv * (1.f - sgv);
    g[c] = m / (float)(LS * LS);
  }
  for (int idx = threadIdx.x; idx < L_len; idx += MLCA_NT) {
    float s = SL[idx];
    dyl[idx] = lw * D[idx] * s * (1.f - s);
  }
  __syncthreads();
  // weight grads: dwl[t] = sum_i dyl[i] * L[i + t - pad] ; dwg[t] = sum_c dyg[c] * g[c + t - pad]
  for (int t = 0; t < k; ++t) {
    float a = 0.f, b = 0.f;
    for (int i = threadIdx.x; i < L_len; i += MLCA_NT) {
      int q = i + t - pad;
      if (q >= 0 && q < L_len) a += dyl[i] * L[q];
    }
    for (int c = threadIdx.x; c < C; c += MLCA_NT) {
      int q = c + t - pad;
      if (q >= 0 && q < C) b += dyg[c] * g[q];
    }
    red[threadIdx.x] = a;
    red[MLCA_NT + threadIdx.x] = b;
    __syncthreads();
    for (int o = MLCA_NT / 2; o > 0; o >>= 1) {
      if (threadIdx.x < o) {
        red[threadIdx.x] += red[threadIdx.x + o];
        red[MLCA_NT + threadIdx.x] += red[MLCA_NT + threadIdx.x + o];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {  // rows [n][2][k]: the local conv's in half 0, the global conv's in half 1
      dwl_part[((long)n * 2 + 0) * k + t] = red[0];
      dwl_part[((long)n * 2 + 1) * k + t] = red[MLCA_NT];
    }
    __syncthreads();
  }
  // dlocal[q] = sum_t wl[t] * dyl[q - t + pad] + dg[c]/25 with dg[c] = sum_t wg[t] * dyg[c - t + pad]
  for (int q = threadIdx.x; q < L_len; q += MLCA_NT) {
    float s = 0.f;
    for (int t = 0; t < k; ++t) {
      int i = q - t + pad;
      if (i >= 0 && i < L_len) s += wl[t] * dyl[i];
    }
    int c = q % C;
    float dg = 0.f;
    for (int t = 0; t < k; ++t) {
      int i = c - t + pad;
      if (i >= 0 && i < C) dg += wg[t] * dyg[i];
    }
    dlocal[(long)n * L_len + q] = s + dg / (float)(LS * LS);
  }
}

// bwd3: dy = dout * up(att) + pool_adjoint(dlocal)
template <typename T, int VW>
__global__ void __launch_bounds__(256) mlca_bwd_y_kernel(const T* dout, int dcs, const float* att, const float* dlocal,
                                                         T* dy, int ocs, int N, int H, int W, int C) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const long npix = (long)N * H * W;
  POOL_LOOP(L, npix, G) {
    int n, h, w;
    pix_nhw(pix, H, W, n, h, w);
    const int c0 = cg * VW;
    float a[VW], g[VW];
    up_att<VW>(att + (long)n * LS * LS * C, C, h, w, H, W, c0, a);
    vload<T, VW>(dout + pix * dcs + c0, g);
#pragma unroll
    for (int e = 0; e < VW; ++e) g[e] *= a[e];
    // adaptive pool H -> 5 adjoint: bins (bi, bj) whose window contains (h, w); candidates around h*5/H
    const float* DL = dlocal + (long)n * LS * LS * C + c0;
    // (for H, W >= 2*LS a pixel lies in at most the bins next to floor(h*LS/H); smaller maps scan all bins)
    const int bic = h * LS / H, bjc = w * LS / W;
    const int bi0 = H < 2 * LS ? 0 : max(0, bic - 1), bi1 = H < 2 * LS ? LS - 1 : min(LS - 1, bic + 1);
    const int bj0 = W < 2 * LS ? 0 : max(0, bjc - 1), bj1 = W < 2 * LS ? LS - 1 : min(LS - 1, bjc + 1);
    for (int bi = bi0; bi <= bi1; ++bi) {
      const int hs = a_s(bi, H, LS), he = a_e(bi, H, LS);
      if (h < hs || h >= he) continue;
      for (int bj = bj0; bj <= bj1; ++bj) {
        const int ws = a_s(bj, W, LS), we = a_e(bj, W, LS);
        if (w < ws || w >= we) continue;
        const float inv = 1.f / (float)((he - hs) * (we - ws));
        const float* d = DL + (bi * LS + bj) * C;
#pragma unroll
        for (int e = 0; e < VW; ++e) g[e] += d[e] * inv;
      }
    }
    vstore<T, VW>(dy + pix * ocs + c0, g);
  }
}

// the local and global 1-D conv weight gradients from the per-image rows [rows][2][cols]: block 0 sums half 0 into
// out0, block 1 half 1 into out1 — one launch for both (cols <= blockDim)
__global__ void sum_rows_kernel(const float* part, int rows, int cols, float* out0, float* out1) {
  const int c = threadIdx.x;
  if (c >= cols) return;
  const float* p = part + (long)blockIdx.x * cols;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += p[(long)r * 2 * cols + c];
  (blockIdx.x ? out1 : out0)[c] = s;
}

}  // namespace adr

using namespace adr;

// VW = 16 / sizeof(T) channels per thread when C, the channel strides and the pointers allow 16-byte accesses
static bool mlca_vec(int dtype, int C, std::initializer_list<long> strides, std::initializer_list<const void*> ptrs) {
  const int vw = dtype == ADR_BF16 ? 8 : 4;
  if (C % vw) return false;
  for (long s : strides)
    if (s % vw) return false;
  for (const void* p : ptrs)
    if ((uintptr_t)p % 16) return false;
  return true;
}
static dim3 mlca_grid(long npix, int dtype, bool v, int C) {
  const int G = C / (v ? (dtype == ADR_BF16 ? 8 : 4) : 1);
  const long rpb = G <= 256 ? 256 / G : 1;
  long b = (npix + rpb - 1) / rpb;
  return dim3((unsigned)(b > 65536 ? 65536 : (b < 1 ? 1 : b)));
}
// launches KERN<TT, VW> with TT bound to the storage type inside the argument list
#define MLCA_DISPATCH(dtype, v, KERN, grid, ...)                                                  \
  do {                                                                                          \
    if ((dtype) == ADR_BF16) {                                                                  \
      using TT = __bf16;                                                                        \
      if (v) hipLaunchKernelGGL((KERN<TT, 8>), grid, dim3(256), 0, st, __VA_ARGS__);            \
      else hipLaunchKernelGGL((KERN<TT, 1>), grid, dim3(256), 0, st, __VA_ARGS__);              \
    } else {                                                                                    \
      using TT = float;                                                                         \
      if (v) hipLaunchKernelGGL((KERN<TT, 4>), grid, dim3(256), 0, st, __VA_ARGS__);            \
      else hipLaunchKernelGGL((KERN<TT, 1>), grid, dim3(256), 0, st, __VA_ARGS__);              \
    }                                                                                           \
  } while (0)

extern "C" int adr_mlca_fwd(int dtype, const void* y, int ycs, const void* res, int rcs, void* out, int ocs, int N,
                            int H, int W, int C, const float* wl, const float* wg, int k, float local_weight,
                            float* local, float* att, float* sig_l, float* sig_g, void* stream) {
  ADR_REQUIRE(k % 2 == 1 && k <= 15, "mlca: k=%d", k);
  hipStream_t st = (hipStream_t)stream;
  const bool v = mlca_vec(dtype, C, {ycs, rcs, ocs}, {y, res, out});
  MLCA_DISPATCH(dtype, v, mlca_pool_kernel, dim3(LS * LS, N), (const TT*)y, ycs, H, W, C, local);
  size_t sm = 2 * C * sizeof(float);
  hipLaunchKernelGGL(mlca_att_kernel, dim3(N), dim3(256), sm, st, local, C, wl, wg, k, sig_l, sig_g);
  long natt = (long)N * LS * LS * C;
  hipLaunchKernelGGL(mlca_mix_kernel, dim3(cdiv(natt, 256)), dim3(256), 0, st, sig_l, sig_g, N, C, local_weight, att);
  MLCA_DISPATCH(dtype, v, mlca_apply_kernel, mlca_grid((long)N * H * W, dtype, v, C), (const TT*)y, ycs,
                (const TT*)res, rcs, att, (TT*)out, ocs, N, H, W, C);
  return check_launch("adr_mlca_fwd");
}

// ws layout: datt [N][25][C] | dlocal [N][25][C] | weight-gradient rows [N][2][k] | S [5][C] (floats)
extern "C" size_t adr_mlca_bwd_workspace(int N, int C, int k) {
  return ((size_t)N * LS * LS * C * 2 + (size_t)N * k * 2 + (size_t)LS * C) * sizeof(float);
}

extern "C" int adr_mlca_bwd(int dtype, const void* y, int ycs, const void* dout, int dcs, void* dy, int ocs, int N,
                            int H, int W, int C, const float* wl, const float* wg, int k, float local_weight,
                            const float* local, const float* att, const float* sig_l, const float* sig_g, float* dwl,
                            float* dwg, float* ws, size_t ws_bytes, void* stream) {
  ADR_REQUIRE(ws_bytes >= adr_mlca_bwd_workspace(N, C, k), "mlca_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* datt = ws;
  float* dlocal = ws + (size_t)N * LS * LS * C;
  float* dwl_part = dlocal + (size_t)N * LS * LS * C;  // [N][2][k] per-image weight-gradient rows
  float* dwg_part = dwl_part + (size_t)N * k;           // (unused by the kernels: both halves live in dwl_part)
  float* S = dwg_part + (size_t)N * k;
  const bool v = mlca_vec(dtype, C, {ycs, dcs, ocs}, {y, dout, dy});
  MLCA_DISPATCH(dtype, v, mlca_bwd_bins_kernel, dim3(LS * LS, N), (const TT*)y, ycs, (const TT*)dout, dcs, H, W, C,
                datt);
  size_t sm = (2 * C + LS * LS * C + 2 * MLCA_NT) * sizeof(float);
  ADR_REQUIRE(sm <= 160 * 1024, "mlca_bwd: C=%d too large for the per-image LDS plan", C);
  hipLaunchKernelGGL(mlca_gsum_kernel, dim3(LS), dim3(256), 0, st, datt, N, C, S);
  hipLaunchKernelGGL(mlca_att_bwd_kernel, dim3(N), dim3(MLCA_NT), sm, st, local, datt, sig_l, sig_g, S, N, C, wl, wg, k,
                     local_weight, dlocal, dwl_part, dwg_part);
  MLCA_DISPATCH(dtype, v, mlca_bwd_y_kernel, mlca_grid((long)N * H * W, dtype, v, C), (const TT*)dout, dcs, att,
                dlocal, (TT*)dy, ocs, N, H, W, C);
  ADR_REQUIRE(k <= 64, "mlca_bwd: kernel size %d", k);
  ADR_REQUIRE((dwl == nullptr) == (dwg == nullptr), "mlca_bwd: dwl and dwg both given or both NULL");
  if (dwl) hipLaunchKernelGGL(sum_rows_kernel, dim3(2), dim3(64), 0, st, dwl_part, N, k, dwl, dwg);
  return check_launch("adr_mlca_bwd");
}
