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

namespace adr {

static constexpr int LS = 5;  // local_size
__device__ __forceinline__ int a_s(int o, int in, int out) { return (int)(((long)o * in) / out); }
__device__ __forceinline__ int a_e(int o, int in, int out) { return (int)(((long)(o + 1) * in + out - 1) / out); }

// fwd1: grid (25, N); local fp32 [N][25][C]
template <typename T>
__global__ void __launch_bounds__(256) mlca_pool_kernel(const T* x, int xcs, int H, int W, int C, float* local) {
  int p = blockIdx.x, n = blockIdx.y;
  int i = p / LS, j = p % LS;
  int hs = a_s(i, H, LS), he = a_e(i, H, LS), ws = a_s(j, W, LS), we = a_e(j, W, LS);
  float inv = 1.f / (float)((he - hs) * (we - ws));
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) s += to_f(x[(((long)n * H + h) * W + w) * xcs + c]);
    local[((long)n * LS * LS + p) * C + c] = s * inv;
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

// S[i][c] = sum_n sum_j datt[n][i*5+j][c]
__global__ void mlca_gsum_kernel(const float* datt, int N, int C, float* S) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= LS * C) return;
  int i = idx / C, c = idx % C;
  float s = 0.f;
  for (int n = 0; n < N; ++n)
    for (int j = 0; j < LS; ++j) s += datt[((long)n * LS * LS + i * LS + j) * C + c];
  S[idx] = s;
}

__device__ __forceinline__ float up_att(const float* A, int C, int h, int w, int H, int W, int c) {
  int is = a_s(h, LS, H), ie = a_e(h, LS, H), js = a_s(w, LS, W), je = a_e(w, LS, W);
  float s = 0.f;
  for (int i = is; i < ie; ++i)
    for (int j = js; j < je; ++j) s += A[(i * LS + j) * C + c];
  return s / (float)((ie - is) * (je - js));
}

// fwd3: out = res + y * up(att)
template <typename T>
__global__ void __launch_bounds__(256) mlca_apply_kernel(const T* y, int ycs, const T* res, int rcs, const float* att,
                                                         T* out, int ocs, int N, int H, int W, int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  float a = up_att(att + (long)n * LS * LS * C, C, h, w, H, W, c);
  float v = to_f(y[pix * ycs + c]) * a;
  if (res) v += to_f(res[pix * rcs + c]);
  out[pix * ocs + c] = from_f<T>(v);
}

// bwd1: datt[n][p][c] = sum over pixels whose up-window includes bin p of dout*y / window_count ; grid (25, N)
template <typename T>
__global__ void __launch_bounds__(256) mlca_bwd_bins_kernel(const T* y, int ycs, const T* dout, int dcs, int H, int W,
                                                            int C, float* datt) {
  int p = blockIdx.x, n = blockIdx.y;
  int bi = p / LS, bj = p % LS;
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.f;
    for (int h = 0; h < H; ++h) {
      int is = a_s(h, LS, H), ie = a_e(h, LS, H);
      if (bi < is || bi >= ie) continue;
      for (int w = 0; w < W; ++w) {
        int js = a_s(w, LS, W), je = a_e(w, LS, W);
        if (bj < js || bj >= je) continue;
        long pix = ((long)n * H + h) * W + w;
        s += to_f(dout[pix * dcs + c]) * to_f(y[pix * ycs + c]) / (float)((ie - is) * (je - js));
      }
    }
    datt[((long)n * LS * LS + p) * C + c] = s;
  }
}

// bwd2: one block per image -> dlocal [N][25][C]; per-image weight grads dwl_part/dwg_part [N][k]
__global__ void __launch_bounds__(256) mlca_att_bwd_kernel(const float* local, const float* datt, const float* sig_l,
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
  float* red = sm + 2 * C + L_len; // 256*2*k scratch
  for (int c = threadIdx.x; c < C; c += 256) {
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
  for (int idx = threadIdx.x; idx < L_len; idx += 256) {
    float s = SL[idx];
    dyl[idx] = lw * D[idx] * s * (1.f - s);
  }
  __syncthreads();
  // weight grads: dwl[t] = sum_i dyl[i] * L[i + t - pad] ; dwg[t] = sum_c dyg[c] * g[c + t - pad]
  for (int t = 0; t < k; ++t) {
    float a = 0.f, b = 0.f;
    for (int i = threadIdx.x; i < L_len; i += 256) {
      int q = i + t - pad;
      if (q >= 0 && q < L_len) a += dyl[i] * L[q];
    }
    for (int c = threadIdx.x; c < C; c += 256) {
      int q = c + t - pad;
      if (q >= 0 && q < C) b += dyg[c] * g[q];
    }
    red[threadIdx.x] = a;
    red[256 + threadIdx.x] = b;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (threadIdx.x < o) {
        red[threadIdx.x] += red[threadIdx.x + o];
        red[256 + threadIdx.x] += red[256 + threadIdx.x + o];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      dwl_part[(long)n * k + t] = red[0];
      dwg_part[(long)n * k + t] = red[256];
    }
    __syncthreads();
  }
  // dlocal[q] = sum_t wl[t] * dyl[q - t + pad] + dg[c]/25 with dg[c] = sum_t wg[t] * dyg[c - t + pad]
  for (int q = threadIdx.x; q < L_len; q += 256) {
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
template <typename T>
__global__ void __launch_bounds__(256) mlca_bwd_y_kernel(const T* dout, int dcs, const float* att, const float* dlocal,
                                                         T* dy, int ocs, int N, int H, int W, int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int n = (int)(r / H);
  float a = up_att(att + (long)n * LS * LS * C, C, h, w, H, W, c);
  float g = to_f(dout[pix * dcs + c]) * a;
  // adaptive pool H -> 5 adjoint: bins (bi, bj) whose window contains (h, w)
  const float* DL = dlocal + (long)n * LS * LS * C;
  for (int bi = 0; bi < LS; ++bi) {
    int hs = a_s(bi, H, LS), he = a_e(bi, H, LS);
    if (h < hs || h >= he) continue;
    for (int bj = 0; bj < LS; ++bj) {
      int ws = a_s(bj, W, LS), we = a_e(bj, W, LS);
      if (w < ws || w >= we) continue;
      g += DL[(bi * LS + bj) * C + c] / (float)((he - hs) * (we - ws));
    }
  }
  dy[pix * ocs + c] = from_f<T>(g);
}

__global__ void sum_rows_kernel(const float* part, int rows, int cols, float* out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += part[(long)r * cols + c];
  out[c] = s;
}

}  // namespace adr

using namespace adr;

extern "C" int adr_mlca_fwd(int dtype, const void* y, int ycs, const void* res, int rcs, void* out, int ocs, int N,
                            int H, int W, int C, const float* wl, const float* wg, int k, float local_weight,
                            float* local, float* att, float* sig_l, float* sig_g, void* stream) {
  ADR_REQUIRE(k % 2 == 1 && k <= 15, "mlca: k=%d", k);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(mlca_pool_kernel<__bf16>, dim3(LS * LS, N), dim3(256), 0, st, (const __bf16*)y, ycs, H, W, C,
                       local);
  else
    hipLaunchKernelGGL(mlca_pool_kernel<float>, dim3(LS * LS, N), dim3(256), 0, st, (const float*)y, ycs, H, W, C,
                       local);
  size_t sm = 2 * C * sizeof(float);
  hipLaunchKernelGGL(mlca_att_kernel, dim3(N), dim3(256), sm, st, local, C, wl, wg, k, sig_l, sig_g);
  long natt = (long)N * LS * LS * C;
  hipLaunchKernelGGL(mlca_mix_kernel, dim3(cdiv(natt, 256)), dim3(256), 0, st, sig_l, sig_g, N, C, local_weight, att);
  long total = (long)N * H * W * C;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(mlca_apply_kernel<__bf16>, dim3(cdiv(total, 256)), dim3(256), 0, st, (const __bf16*)y, ycs,
                       (const __bf16*)res, rcs, att, (__bf16*)out, ocs, N, H, W, C);
  else
    hipLaunchKernelGGL(mlca_apply_kernel<float>, dim3(cdiv(total, 256)), dim3(256), 0, st, (const float*)y, ycs,
                       (const float*)res, rcs, att, (float*)out, ocs, N, H, W, C);
  return check_launch("adr_mlca_fwd");
}

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
  float* dwl_part = dlocal + (size_t)N * LS * LS * C;
  float* dwg_part = dwl_part + (size_t)N * k;
  float* S = dwg_part + (size_t)N * k;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(mlca_bwd_bins_kernel<__bf16>, dim3(LS * LS, N), dim3(256), 0, st, (const __bf16*)y, ycs,
                       (const __bf16*)dout, dcs, H, W, C, datt);
  else
    hipLaunchKernelGGL(mlca_bwd_bins_kernel<float>, dim3(LS * LS, N), dim3(256), 0, st, (const float*)y, ycs,
                       (const float*)dout, dcs, H, W, C, datt);
  size_t sm = (2 * C + LS * LS * C + 512) * sizeof(float);
  ADR_REQUIRE(sm <= 160 * 1024, "mlca_bwd: C=%d too large for the per-image LDS plan", C);
  hipLaunchKernelGGL(mlca_gsum_kernel, dim3(cdiv(LS * C, 256)), dim3(256), 0, st, datt, N, C, S);
  hipLaunchKernelGGL(mlca_att_bwd_kernel, dim3(N), dim3(256), sm, st, local, datt, sig_l, sig_g, S, N, C, wl, wg, k,
                     local_weight, dlocal, dwl_part, dwg_part);
  long total = (long)N * H * W * C;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(mlca_bwd_y_kernel<__bf16>, dim3(cdiv(total, 256)), dim3(256), 0, st, (const __bf16*)dout, dcs,
                       att, dlocal, (__bf16*)dy, ocs, N, H, W, C);
  else
    hipLaunchKernelGGL(mlca_bwd_y_kernel<float>, dim3(cdiv(total, 256)), dim3(256), 0, st, (const float*)dout, dcs,
                       att, dlocal, (float*)dy, ocs, N, H, W, C);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(64), 0, st, dwl_part, N, k, dwl);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(64), 0, st, dwg_part, N, k, dwg);
  return check_launch("adr_mlca_bwd");
}
