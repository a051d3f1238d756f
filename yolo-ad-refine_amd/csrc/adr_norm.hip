// Normalisation (BatchNorm2d train/eval, GroupNorm) + fused activation, forward and backward, NHWC.
//
// Forward:  partial stats (from the conv epilogue or adr_nc_reduce) -> *_finalize -> scale/shift per channel
//           (BN) or per (image, channel) (GN) -> adr_affine_act:  z = act(x * scale + shift).
// Backward: adr_nc_reduce(MODE_BWD) gives per-(image, channel) partials of g = dz * act'(x*scale+shift) and of
//           g*x; *_bwd_finalize turns them into dgamma/dbeta and per-(image, channel) coefficients (A, B, C)
//           with dx = A*g + B*x + C, applied by adr_affine_act_bwd (g recomputed on the fly).
// All cross-block reductions are fixed-order (no atomics), so results are deterministic run to run.
// Reference semantics: nn.BatchNorm2d with eps 1e-3 / momentum 0.03 (utils/torch_utils.py:426-436),
// unbiased running_var update; GroupNorm(16, C) eps 1e-5 (nn/modules/head.py:613).
#include "adr_common.h"
#include <cstdio>
#include <cstdlib>

namespace adr {

enum RedMode { RED_STATS = 0, RED_BWD = 1, RED_SUM = 2 };

// partial[(n * chunks + chunk)][2][C]
template <typename T, int MODE, int ACT>
__device__ __forceinline__ void nc_reduce_body(const T* __restrict__ x, int xcs, int xco, const T* __restrict__ dz,
                                               int dcs, int dco, const float* __restrict__ scale,
                                               const float* __restrict__ shift, int per_sample, int HW, int C,
                                               int rows_per_chunk, int chunks, float* __restrict__ partial,
                                               const int chunk, const int n) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float sh[2][256 * VEC];
  const int G = C / VEC;
  const int rpp = 256 / G;  // rows per pass
  const int t = threadIdx.x;
  const int cg = t % G, r0 = t / G;
  float s1[VEC], s2[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  const int rbeg = chunk * rows_per_chunk;
  const int rend = min(HW, rbeg + rows_per_chunk);
  const int c0 = cg * VEC;
  float sc[VEC], sf[VEC];
  if (MODE == RED_BWD) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      int ci = per_sample ? n * C + c0 + e : c0 + e;
      sc[e] = scale[ci];
      sf[e] = shift[ci];
    }
  }
  if (r0 < rpp) {
    // NU rows in flight per thread: all loads of a group are issued before any is consumed
    constexpr int NU = 4;
    const T* xb = x + ((long)n * HW) * xcs + xco + c0;
    const T* db = MODE == RED_BWD ? dz + ((long)n * HW) * dcs + dco + c0 : nullptr;
    for (int r = rbeg + r0; r < rend; r += NU * rpp) {
      u32x4 xv[NU], dv[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int ru = r + u * rpp;
        if (ru < rend) {
          xv[u] = ld16(xb + (long)ru * xcs);
          if (MODE == RED_BWD) dv[u] = ld16(db + (long)ru * dcs);
        }
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (r + u * rpp >= rend) break;
        const T* xe = reinterpret_cast<const T*>(&xv[u]);
        if (MODE == RED_BWD) {
          const T* de = reinterpret_cast<const T*>(&dv[u]);
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            float xf = to_f(xe[e]);
            float g = bn_act_g<ACT, sizeof(T) == 2>(to_f(de[e]), xf, sc[e], sf[e]);
            s1[e] += g;
            s2[e] += g * xf;
          }
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            float xf = to_f(xe[e]);
            s1[e] += xf;
            s2[e] += xf * xf;
          }
        }
      }
    }
  }
  // combine rows: threads with the same cg (t = cg + G * r0)
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    sh[0][t * VEC + e] = s1[e];
    sh[1][t * VEC + e] = s2[e];
  }
  __syncthreads();
  float* out = partial + ((long)n * chunks + chunk) * 2 * C;
  for (int c = t; c < C; c += 256) {
    int g = c / VEC, e = c % VEC;
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rpp; ++r) {
      a += sh[0][(g + r * G) * VEC + e];
      b += sh[1][(g + r * G) * VEC + e];
    }
    out[c] = a;
    out[C + c] = b;
  }
}

template <typename T, int MODE, int ACT = ACT_NONE>
__global__ void __launch_bounds__(256) nc_reduce_kernel(const T* __restrict__ x, int xcs, int xco,
                                                        const T* __restrict__ dz, int dcs, int dco,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift, int per_sample, int act,
                                                        int HW, int C, int rows_per_chunk, int chunks,
                                                        float* __restrict__ partial) {
  nc_reduce_body<T, MODE, ACT>(x, xcs, xco, dz, dcs, dco, scale, shift, per_sample, HW, C, rows_per_chunk, chunks,
                               partial, blockIdx.x, blockIdx.y);
}

// Many RED_STATS reductions in one launch (the trainer defers the bias-gradient column sums of every biased conv
// to the end of backward): block b of the grid is (chunk, image) (b - start[e]) of entry e, reduced exactly as
// nc_reduce_kernel reduces it, so the partial rows — and the bias gradients — are bitwise those of one launch each.
constexpr int NCB_MAX = 48;
struct NcrBatch {
  adr_colsum_entry e[NCB_MAX];
  int start[NCB_MAX + 1];
  int count;
};
__global__ void __launch_bounds__(256) nc_reduce_batched_kernel(NcrBatch b) {
  int j = 0;
  while (j + 1 < b.count && (int)blockIdx.x >= b.start[j + 1]) ++j;
  const adr_colsum_entry& en = b.e[j];
  const int local = blockIdx.x - b.start[j];
  nc_reduce_body<__bf16, RED_STATS, ACT_NONE>((const __bf16*)en.x, en.xcs, 0, nullptr, 0, 0, nullptr, nullptr, 0,
                                              en.HW, en.C, en.rows_per_chunk, en.chunks, en.partial,
                                              local % en.chunks, local / en.chunks);
}

// block per channel: deterministic fixed-order sum over P partial rows in double. Each thread keeps four rows in
// flight (the finalize kernels are latency-bound: P is a few hundred rows on most layers), then a wave butterfly
// and one LDS exchange across the four waves.
__device__ __forceinline__ void block_sum2(double& a, double& b) {
  __shared__ double sa[4], sb[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sa[w] = a;
    sb[w] = b;
  }
  __syncthreads();
  a = (sa[0] + sa[1]) + (sa[2] + sa[3]);
  b = (sb[0] + sb[1]) + (sb[2] + sb[3]);
  __syncthreads();
}

// this thread's share of column c over P rows of [P][2][C] partials: (sum row[c], sum row[C + c])
__device__ __forceinline__ void col_sums2(const float* __restrict__ partial, int P, int C, int c, double& a, double& b) {
  double a1 = 0.0, b1 = 0.0, a2 = 0.0, b2 = 0.0, a3 = 0.0, b3 = 0.0;
  int p = threadIdx.x;
  for (; p + 768 < P; p += 1024) {
    const float* r0 = partial + (long)p * 2 * C + c;
    const long st = 256l * 2 * C;
    const float x0 = r0[0], y0 = r0[C], x1 = r0[st], y1 = r0[st + C];
    const float x2 = r0[2 * st], y2 = r0[2 * st + C], x3 = r0[3 * st], y3 = r0[3 * st + C];
    a += x0; b += y0; a1 += x1; b1 += y1; a2 += x2; b2 += y2; a3 += x3; b3 += y3;
  }
  for (; p < P; p += 256) {
    a += partial[(long)p * 2 * C + c];
    b += partial[(long)p * 2 * C + C + c];
  }
  a = (a + a1) + (a2 + a3);
  b = (b + b1) + (b2 + b3);
}

// pre-summed partial rows of a long finalize (fin_presum_kernel, below)
constexpr int FIN_PMAX = 2048, FIN_S = 256, FIN_SCRATCH = 1 << 20;  // floats
__device__ float g_fin_scratch[FIN_SCRATCH];

__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ partial, int P, int C, double count,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* running_mean,
                                                          float* running_var, float momentum, float eps,
                                                          int training, float* scale, float* shift, float* mean_out,
                                                          float* rstd_out, int presummed) {
  int c = blockIdx.x;
  if (presummed) partial = g_fin_scratch;
  double mean, var;
  if (training) {
    double a = 0.0, b = 0.0;
    col_sums2(partial, P, C, c, a, b);
    block_sum2(a, b);
    mean = a / count;
    var = b / count - mean * mean;
    if (var < 0) var = 0;
  } else {
    mean = running_mean[c];
    var = running_var[c];
  }
  if (threadIdx.x == 0) {
    double rstd = 1.0 / sqrt(var + (double)eps);
    double g = gamma ? gamma[c] : 1.0, bb = beta ? beta[c] : 0.0;
    scale[c] = (float)(g * rstd);
    shift[c] = (float)(bb - mean * g * rstd);
    if (mean_out) mean_out[c] = (float)mean;
    if (rstd_out) rstd_out[c] = (float)rstd;
    if (training && running_mean) {
      double unb = count > 1 ? var * count / (count - 1) : var;
      running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
      running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
    }
  }
}

// dgamma/dbeta and coefficients for BN backward. partial holds (sum g, sum g*x) per row.
__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(const float* __restrict__ partial, int P, int C,
                                                              double count, const float* __restrict__ mean,
                                                              const float* __restrict__ rstd,
                                                              const float* __restrict__ gamma, float* dgamma,
                                                              float* dbeta, float* A, float* B, float* Cc,
                                                              int training, int accumulate, int presummed) {
  int c = blockIdx.x;
  if (presummed) partial = g_fin_scratch;
  double a = 0.0, b = 0.0;
  col_sums2(partial, P, C, c, a, b);
  block_sum2(a, b);
  if (threadIdx.x == 0) {
    double mu = mean[c], rs = rstd[c], g = gamma ? gamma[c] : 1.0;
    double sg = a;                   // sum g
    double sgx = (b - mu * a) * rs;  // sum g * xhat
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)sgx : (float)sgx;
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)sg : (float)sg;
    double Ak = g * rs;
    if (training) {
      double Bk = -Ak * rs * sgx / count;
      double Ck = -Ak * sg / count - Bk * mu;
      A[c] = (float)Ak;
      B[c] = (float)Bk;
      Cc[c] = (float)Ck;
    } else {
      A[c] = (float)Ak;
      B[c] = 0.f;
      Cc[c] = 0.f;
    }
  }
}

// per-channel sums over an image's chunks into LDS (sa, sb): threads = (channel, chunk-part) pairs so every
// thread of the block loads, parts combined in a fixed order
__device__ __forceinline__ void gn_chan_sums(const float* partial, int n, int chunks, int C, double* sa, double* sb,
                                             double* scratch_a, double* scratch_b) {
  const int parts = C >= 256 ? 1 : 256 / C;
  for (int c0 = 0; c0 < C; c0 += 256) {
    const int c = c0 + (int)threadIdx.x % (C >= 256 ? 256 : C), part = (int)threadIdx.x / (C >= 256 ? 256 : C);
    double a = 0.0, b = 0.0;
    if (c < C && part < parts)
      for (int ch = part; ch < chunks; ch += parts) {
        const float* p = partial + ((long)n * chunks + ch) * 2 * C;
        a += p[c];
        b += p[C + c];
      }
    scratch_a[threadIdx.x] = a;
    scratch_b[threadIdx.x] = b;
    __syncthreads();
    if ((int)threadIdx.x < (C >= 256 ? 256 : C) && c < C) {
      double ta = 0.0, tb = 0.0;
      for (int q = 0; q < parts; ++q) {
        ta += scratch_a[q * (C >= 256 ? 256 : C) + threadIdx.x];
        tb += scratch_b[q * (C >= 256 ? 256 : C) + threadIdx.x];
      }
      sa[c] = ta;
      sb[c] = tb;
    }
    __syncthreads();
  }
}

// GroupNorm forward finalize: block per image; partial [n][chunks][2][C]
__global__ void __launch_bounds__(256) gn_finalize_kernel(const float* __restrict__ partial, int chunks, int C, int G,
                                                          double count, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, float* scale,
                                                          float* shift, float* mean_out, float* rstd_out) {
  const int n = blockIdx.x;
  __shared__ double gm[64], gr[64];
  __shared__ double sa[1024], sb[1024], xa[256], xb[256];
  gn_chan_sums(partial, n, chunks, C, sa, sb, xa, xb);
  const int cpg = C / G;
  for (int g = threadIdx.x; g < G; g += 256) {
    double a = 0.0, b = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      a += sa[c];
      b += sb[c];
    }
    double mu = a / count, var = b / count - mu * mu;
    if (var < 0) var = 0;
    gm[g] = mu;
    gr[g] = 1.0 / sqrt(var + (double)eps);
    mean_out[n * G + g] = (float)mu;
    rstd_out[n * G + g] = (float)gr[g];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    int g = c / cpg;
    double gg = gamma ? gamma[c] : 1.0, bb = beta ? beta[c] : 0.0;
    scale[n * C + c] = (float)(gg * gr[g]);
    shift[n * C + c] = (float)(bb - gm[g] * gg * gr[g]);
  }
}

// GroupNorm backward finalize, per image (grid N): channel sums over chunks -> group sums -> dx coefficients
// A, B, C (dx = A*g + B*x + C with per-(n,c) coefficients).
__global__ void __launch_bounds__(256) gn_bwd_coef_kernel(const float* __restrict__ partial, int chunks, int C, int G,
                                                          double count, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          const float* __restrict__ gamma, float* A, float* B,
                                                          float* Cc) {
  const int n = blockIdx.x, cpg = C / G;
  __shared__ double sa[1024], sg[1024], xa[256], xb[256];
  __shared__ double s1[64], s2[64];
  gn_chan_sums(partial, n, chunks, C, sa, sg, xa, xb);
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cpg;
    const double mu = mean[n * G + g], rs = rstd[n * G + g];
    const double a = sa[c], b = sg[c];
    const double gm = gamma ? gamma[c] : 1.0;
    sa[c] = gm * a;                  // sum dxhat
    sg[c] = gm * (b - mu * a) * rs;  // sum dxhat * xhat
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += 256) {
    double S1 = 0.0, S2 = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      S1 += sa[c];
      S2 += sg[c];
    }
    s1[g] = S1;
    s2[g] = S2;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cpg;
    const double mu = mean[n * G + g], rs = rstd[n * G + g];
    const double gm = gamma ? gamma[c] : 1.0;
    const double Bk = -rs * rs * s2[g] / count;
    A[n * C + c] = (float)(rs * gm);
    B[n * C + c] = (float)Bk;
    Cc[n * C + c] = (float)(-rs * s1[g] / count - Bk * mu);
  }
}

// GroupNorm dgamma / dbeta, per channel (grid C): fixed-order reduction over (image, chunk) of
// (sum g*x - mu_n * sum g) * rstd_n and sum g.
__device__ __forceinline__ void gn_bwd_param_body(const float* __restrict__ partial, int N, int chunks, int C, int G,
                                                  const float* __restrict__ mean, const float* __restrict__ rstd,
                                                  float* dgamma, float* dbeta, int accumulate, const int c) {
  const int g = c / (C / G);
  double sgx = 0.0, sb = 0.0;
  for (int it = threadIdx.x; it < N * chunks; it += 256) {
    const int n = it / chunks;
    const float* p = partial + (long)it * 2 * C;
    const double a = p[c], b = p[C + c];
    sgx += (b - (double)mean[n * G + g] * a) * (double)rstd[n * G + g];
    sb += a;
  }
  __shared__ double r1[256], r2[256];
  r1[threadIdx.x] = sgx;
  r2[threadIdx.x] = sb;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)r1[0] : (float)r1[0];
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)r2[0] : (float)r2[0];
  }
}

__global__ void __launch_bounds__(256) gn_bwd_param_kernel(const float* __restrict__ partial, int N, int chunks, int C,
                                                           int G, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, float* dgamma,
                                                           float* dbeta, int accumulate) {
  gn_bwd_param_body(partial, N, chunks, C, G, mean, rstd, dgamma, dbeta, accumulate, blockIdx.x);
}

// Many GroupNorm dgamma / dbeta reductions per launch (deferred to the end of backward); block b is channel
// b - start[e] of entry e, reduced exactly as gn_bwd_param_kernel does. Entries of one launch have distinct
// destinations (the host splits at a repeated one, so a shared module's contributions accumulate in order).
constexpr int GPB_MAX = 40;
struct GnParamBatch {
  adr_gnparam_entry e[GPB_MAX];
  int start[GPB_MAX + 1];
  int count;
};
__global__ void __launch_bounds__(256) gn_param_batched_kernel(GnParamBatch b) {
  int j = 0;
  while (j + 1 < b.count && (int)blockIdx.x >= b.start[j + 1]) ++j;
  const adr_gnparam_entry& en = b.e[j];
  gn_bwd_param_body(en.partial, en.N, en.chunks, en.C, en.G, en.mean, en.rstd, en.dgamma, en.dbeta, en.accumulate,
                    (int)blockIdx.x - b.start[j]);
}

// ---- Level-packed GroupNorm (AYHead's three levels in one row space). The head stores a level's (image, H, W)
//      rows back to back, P3 images first, then P4, then P5, and cuts that row space into "sub-images" of S rows,
//      S = the smallest level's H*W: level l's image is k[l] = H_l*W_l / S consecutive sub-images. The per-pixel
//      kernels (nc_reduce, affine_act, ...) then run once over all N' sub-images; only the per-image statistics
//      need the level structure: a block per (level, image) segment sums its k[l]*chunks partial rows and writes
//      the result replicated to each of its sub-images, so every later per-sub-image kernel (affine_act with
//      per_sample coefficients, gn_bwd_param over N' sub-images) reads the statistics of the whole image.
constexpr int LP_MAX = 4;
struct LevelPackArgs {
  int levels, N, chunks, C, G;
  int k[LP_MAX];
  int sub0[LP_MAX];  // first sub-image of level l
  double count[LP_MAX];
  float scale[LP_MAX];
  const float* gamma[LP_MAX];
  const float* beta[LP_MAX];
};

__device__ __forceinline__ void lp_segment(const LevelPackArgs& a, int& l, int& first, int& k) {
  l = (int)blockIdx.x / a.N;
  const int n = (int)blockIdx.x % a.N;
  k = a.k[l];
  first = a.sub0[l] + n * k;
}

__global__ void __launch_bounds__(256) gn_finalize_packed_kernel(const float* __restrict__ partial, LevelPackArgs a,
                                                                 float eps, float* scale, float* shift,
                                                                 float* mean_out, float* rstd_out) {
  int l, first, k;
  lp_segment(a, l, first, k);
  const int C = a.C, G = a.G, cpg = C / G;
  __shared__ double gm[64], gr[64];
  __shared__ double sa[1024], sb[1024], xa[256], xb[256];
  gn_chan_sums(partial + (long)first * a.chunks * 2 * C, 0, k * a.chunks, C, sa, sb, xa, xb);
  for (int g = threadIdx.x; g < G; g += 256) {
    double s = 0.0, q = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      s += sa[c];
      q += sb[c];
    }
    double mu = s / a.count[l], var = q / a.count[l] - mu * mu;
    if (var < 0) var = 0;
    gm[g] = mu;
    gr[g] = 1.0 / sqrt(var + (double)eps);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < k * G; i += 256) {
    const int j = first + i / G, g = i % G;
    mean_out[(long)j * G + g] = (float)gm[g];
    rstd_out[(long)j * G + g] = (float)gr[g];
  }
  const float* gamma = a.gamma[l];
  const float* beta = a.beta[l];
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cpg;
    const double gg = gamma ? gamma[c] : 1.0, bb = beta ? beta[c] : 0.0;
    const float sc = (float)(gg * gr[g]), sf = (float)(bb - gm[g] * gg * gr[g]);
    for (int j = first; j < first + k; ++j) {
      scale[(long)j * C + c] = sc;
      shift[(long)j * C + c] = sf;
    }
  }
}

__global__ void __launch_bounds__(256) gn_bwd_coef_packed_kernel(const float* __restrict__ partial, LevelPackArgs a,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ rstd, float* A, float* B,
                                                                 float* Cc) {
  int l, first, k;
  lp_segment(a, l, first, k);
  const int C = a.C, G = a.G, cpg = C / G;
  __shared__ double sa[1024], sg[1024], xa[256], xb[256];
  __shared__ double s1[64], s2[64];
  gn_chan_sums(partial + (long)first * a.chunks * 2 * C, 0, k * a.chunks, C, sa, sg, xa, xb);
  const float* gamma = a.gamma[l];
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cpg;
    const double mu = mean[(long)first * G + g], rs = rstd[(long)first * G + g];
    const double s = sa[c], q = sg[c];
    const double gmm = gamma ? gamma[c] : 1.0;
    sa[c] = gmm * s;
    sg[c] = gmm * (q - mu * s) * rs;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += 256) {
    double S1 = 0.0, S2 = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      S1 += sa[c];
      S2 += sg[c];
    }
    s1[g] = S1;
    s2[g] = S2;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cpg;
    const double mu = mean[(long)first * G + g], rs = rstd[(long)first * G + g];
    const double gmm = gamma ? gamma[c] : 1.0;
    const double Bk = -rs * rs * s2[g] / a.count[l];
    const float av = (float)(rs * gmm), bv = (float)Bk, cv = (float)(-rs * s1[g] / a.count[l] - Bk * mu);
    for (int j = first; j < first + k; ++j) {
      A[(long)j * C + c] = av;
      B[(long)j * C + c] = bv;
      Cc[(long)j * C + c] = cv;
    }
  }
}

// Per (level, image) segment, rows of C floats: v = (in_seg ? in[segment] : sum of in[j] over the segment's
// sub-images j) * (mean ? 1 / pixels of the image : 1), written to out[segment] (out_seg) or to every sub-image's
// row. The head's global average pool (per-sub-image sums -> per-image means), the expansion of a per-image gate
// to its sub-images, and both backwards.
__global__ void __launch_bounds__(256) seg_reduce_packed_kernel(const float* __restrict__ in, int in_seg, int out_seg,
                                                                int mean, LevelPackArgs a, float* out) {
  int l, first, k;
  lp_segment(a, l, first, k);
  const int C = a.C, seg = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += 256) {
    double s = 0.0;
    if (in_seg)
      s = in[(long)seg * C + c];
    else
      for (int j = first; j < first + k; ++j) s += in[(long)j * C + c];
    const float v = (float)(mean ? s * (double)a.scale[l] : s);
    if (out_seg)
      out[(long)seg * C + c] = v;
    else
      for (int j = first; j < first + k; ++j) out[(long)j * C + c] = v;
  }
}

// Level-packed BatchNorm (CoordAtt's pooled planes of the three head levels in one row space, each level's rows a
// segment of N * k[l] sub-images): training statistics per level, block per channel looping the levels in order,
// so the shared module's running statistics are updated level by level as the reference's per-level calls do.
// scale / shift are written per sub-image (affine_act per_sample), mean / rstd per (level, channel).
__global__ void __launch_bounds__(256) bn_finalize_packed_kernel(const float* __restrict__ partial, LevelPackArgs a,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, float* running_mean,
                                                                 float* running_var, float momentum, float eps,
                                                                 float* scale, float* shift, float* mean_out,
                                                                 float* rstd_out) {
  const int c = blockIdx.x, C = a.C;
  const double g = gamma ? gamma[c] : 1.0, bb = beta ? beta[c] : 0.0;
  for (int l = 0; l < a.levels; ++l) {
    const int subs = a.N * a.k[l];
    double s = 0.0, q = 0.0;
    col_sums2(partial + (long)a.sub0[l] * a.chunks * 2 * C, subs * a.chunks, C, c, s, q);
    block_sum2(s, q);
    const double cnt = a.count[l];
    const double mean = s / cnt;
    double var = q / cnt - mean * mean;
    if (var < 0) var = 0;
    const double rstd = 1.0 / sqrt(var + (double)eps);
    const float sc = (float)(g * rstd), sf = (float)(bb - mean * g * rstd);
    for (int j = a.sub0[l] + threadIdx.x; j < a.sub0[l] + subs; j += 256) {
      scale[(long)j * C + c] = sc;
      shift[(long)j * C + c] = sf;
    }
    if (threadIdx.x == 0) {
      mean_out[l * C + c] = (float)mean;
      rstd_out[l * C + c] = (float)rstd;
      if (running_mean) {
        const double unb = cnt > 1 ? var * cnt / (cnt - 1) : var;
        running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
        running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
      }
    }
  }
}

// its backward: per level (sum g, sum g*x) -> dx coefficients A, B, C per sub-image; dgamma / dbeta summed over the
// levels in order
__global__ void __launch_bounds__(256) bn_bwd_finalize_packed_kernel(const float* __restrict__ partial,
                                                                     LevelPackArgs a, const float* __restrict__ mean,
                                                                     const float* __restrict__ rstd,
                                                                     const float* __restrict__ gamma, float* dgamma,
                                                                     float* dbeta, float* A, float* B, float* Cc,
                                                                     int accumulate) {
  const int c = blockIdx.x, C = a.C;
  const double g = gamma ? gamma[c] : 1.0;
  double dg = 0.0, db = 0.0;
  for (int l = 0; l < a.levels; ++l) {
    const int subs = a.N * a.k[l];
    double s = 0.0, q = 0.0;
    col_sums2(partial + (long)a.sub0[l] * a.chunks * 2 * C, subs * a.chunks, C, c, s, q);
    block_sum2(s, q);
    const double cnt = a.count[l], mu = mean[l * C + c], rs = rstd[l * C + c];
    const double sgx = (q - mu * s) * rs;
    dg += sgx;
    db += s;
    const double Ak = g * rs, Bk = -Ak * rs * sgx / cnt, Ck = -Ak * s / cnt - Bk * mu;
    for (int j = a.sub0[l] + threadIdx.x; j < a.sub0[l] + subs; j += 256) {
      A[(long)j * C + c] = (float)Ak;
      B[(long)j * C + c] = (float)Bk;
      Cc[(long)j * C + c] = (float)Ck;
    }
  }
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)dg : (float)dg;
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)db : (float)db;
  }
}

// ---- GroupNorm + activation fused per image (Conv_GN / TaskDecomposition / DyDCNv2 / ELA gates: GN statistics
//      are per image, so one 1024-thread workgroup owns an image and needs no cross-workgroup reduction). Forward:
//      channel sums -> group mean / rstd -> per-channel scale/shift -> z = act(x*scale + shift), one launch
//      instead of nc_reduce + gn_finalize + affine_act. Backward: channel sums of g = dz * act'(.) and g*x ->
//      (A, B, C) -> dx = A*g + B*x + C, plus the per-image (sum g, sum g*x) rows gn_bwd_param reduces for
//      dgamma / dbeta. Fixed-order sums (per-thread fp32 over its rows, then double in LDS): deterministic. ----
constexpr int GNF_T = 1024;

// per-channel (double) sums of a per-thread accumulator over the row-threads of each channel group (one LDS image
// of GNF_T x VEC floats, reused for the second accumulator)
template <int VEC>
__device__ __forceinline__ void gnf_sum1(const float* s, int G8, int RP, int C, float* shf, double* out) {
  const int t = threadIdx.x;
  if (t / G8 < RP) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) shf[t * VEC + e] = s[e];
  }
  __syncthreads();
  for (int c = t; c < C; c += GNF_T) {
    const int g = c / VEC, e = c % VEC;
    double a = 0.0;
    for (int r = 0; r < RP; ++r) a += shf[(g + r * G8) * VEC + e];
    out[c] = a;
  }
  __syncthreads();
}

template <int VEC>
__device__ __forceinline__ void gnf_channel_sums(const float* s1, const float* s2, int G8, int RP, int C, float* shf,
                                                 double* ca, double* cb) {
  gnf_sum1<VEC>(s1, G8, RP, C, shf, ca);
  gnf_sum1<VEC>(s2, G8, RP, C, shf, cb);
}

template <typename T, int ACT>
__global__ void __launch_bounds__(GNF_T) gn_fused_fwd_kernel(const T* __restrict__ x, int xcs, int xco, T* __restrict__ z,
                                                             int zcs, int zco, const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float eps, int HW, int C,
                                                             int G, float* scale, float* shift, float* mean_out,
                                                             float* rstd_out) {
  constexpr int VEC = 16 / sizeof(T);
  extern __shared__ __attribute__((aligned(16))) unsigned char gnf_raw[];
  float* shf = reinterpret_cast<float*>(gnf_raw);                       // [GNF_T * VEC]
  double* ca = reinterpret_cast<double*>(shf + GNF_T * VEC);           // [C]
  double* cb = ca + C;                                                  // [C]
  float* sc = reinterpret_cast<float*>(cb + C);                         // [C]
  float* sf = sc + C;                                                   // [C]
  double* gstat = reinterpret_cast<double*>(sf + C);                    // [2][G]
  const int n = blockIdx.x, t = threadIdx.x;
  const int G8 = C / VEC, RP = GNF_T / G8;
  const int cg = t % G8, r0 = t / G8, c0 = cg * VEC;
  const bool act_t = r0 < RP;
  const T* xb = x + (long)n * HW * xcs + xco + c0;
  float s1[VEC], s2[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) s1[e] = s2[e] = 0.f;
  if (act_t) {
    constexpr int NU = 4;
    for (int r = r0; r < HW; r += NU * RP) {
      u32x4 v[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u)
        if (r + u * RP < HW) v[u] = ld16(xb + (long)(r + u * RP) * xcs);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (r + u * RP >= HW) break;
        const T* ve = reinterpret_cast<const T*>(&v[u]);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float f = to_f(ve[e]);
          s1[e] += f;
          s2[e] += f * f;
        }
      }
    }
  }
  gnf_channel_sums<VEC>(s1, s2, G8, RP, C, shf, ca, cb);
  const int cpg = C / G;
  const double count = (double)HW * cpg;
  for (int g = t; g < G; g += GNF_T) {
    double a = 0.0, b = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      a += ca[c];
      b += cb[c];
    }
    const double mu = a / count;
    double var = b / count - mu * mu;
    if (var < 0) var = 0;
    const double rs = 1.0 / sqrt(var + (double)eps);
    gstat[g] = mu;
    gstat[G + g] = rs;
    mean_out[n * G + g] = (float)mu;
    rstd_out[n * G + g] = (float)rs;
  }
  __syncthreads();
  for (int c = t; c < C; c += GNF_T) {
    const int g = c / cpg;
    const double gg = gamma ? gamma[c] : 1.0, bb = beta ? beta[c] : 0.0;
    const float a = (float)(gg * gstat[G + g]), b = (float)(bb - gstat[g] * gg * gstat[G + g]);
    sc[c] = a;
    sf[c] = b;
    scale[n * C + c] = a;
    shift[n * C + c] = b;
  }
  __syncthreads();
  if (!act_t) return;
  float a[VEC], b[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    a[e] = sc[c0 + e];
    b[e] = sf[c0 + e];
  }
  T* zb = z + (long)n * HW * zcs + zco + c0;
  for (int r = r0; r < HW; r += RP) {
    const u32x4 v = ld16(xb + (long)r * xcs);
    const T* ve = reinterpret_cast<const T*>(&v);
    u32x4 o;
    T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
    for (int e = 0; e < VEC; ++e) oe[e] = from_f<T>(act_fwd_c<ACT, sizeof(T) == 2>(to_f(ve[e]) * a[e] + b[e]));
    st16(zb + (long)r * zcs, o);
  }
}

template <typename T, int ACT>
__global__ void __launch_bounds__(GNF_T) gn_fused_bwd_kernel(const T* __restrict__ x, int xcs, int xco,
                                                             const T* __restrict__ dz, int dcs, int dco,
                                                             T* __restrict__ dx, int ocs, int oco,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma, int HW, int C, int G,
                                                             float* part) {
  constexpr int VEC = 16 / sizeof(T);
  extern __shared__ __attribute__((aligned(16))) unsigned char gnf_raw[];
  float* shf = reinterpret_cast<float*>(gnf_raw);
  double* ca = reinterpret_cast<double*>(shf + GNF_T * VEC);
  double* cb = ca + C;
  float* cA = reinterpret_cast<float*>(cb + C);
  float* cB = cA + C;
  float* cC = cB + C;
  double* gsum = reinterpret_cast<double*>(cC + C + (C & 1));  // [2][G] (8-byte aligned)
  const int n = blockIdx.x, t = threadIdx.x;
  const int G8 = C / VEC, RP = GNF_T / G8;
  const int cg = t % G8, r0 = t / G8, c0 = cg * VEC;
  const bool act_t = r0 < RP;
  float sc[VEC], sf[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    sc[e] = act_t ? scale[n * C + c0 + e] : 0.f;
    sf[e] = act_t ? shift[n * C + c0 + e] : 0.f;
  }
  const T* xb = x + (long)n * HW * xcs + xco + c0;
  const T* db = dz + (long)n * HW * dcs + dco + c0;
  float s1[VEC], s2[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) s1[e] = s2[e] = 0.f;
  if (act_t) {
    constexpr int NU = 4;
    for (int r = r0; r < HW; r += NU * RP) {
      u32x4 xv[NU], dv[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u)
        if (r + u * RP < HW) {
          xv[u] = ld16(xb + (long)(r + u * RP) * xcs);
          dv[u] = ld16(db + (long)(r + u * RP) * dcs);
        }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (r + u * RP >= HW) break;
        const T* xe = reinterpret_cast<const T*>(&xv[u]);
        const T* de = reinterpret_cast<const T*>(&dv[u]);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float xf = to_f(xe[e]);
          const float g = to_f(de[e]) * act_bwd_c<ACT, sizeof(T) == 2>(xf * sc[e] + sf[e]);
          s1[e] += g;
          s2[e] += g * xf;
        }
      }
    }
  }
  gnf_channel_sums<VEC>(s1, s2, G8, RP, C, shf, ca, cb);
  const int cpg = C / G;
  const double count = (double)HW * cpg;
  for (int c = t; c < C; c += GNF_T) {
    part[((long)n * 2) * C + c] = (float)ca[c];      // (sum g, sum g*x) rows for gn_bwd_param (chunks = 1)
    part[((long)n * 2 + 1) * C + c] = (float)cb[c];
  }
  for (int g = t; g < G; g += GNF_T) {
    const double mu = mean[n * G + g], rs = rstd[n * G + g];
    double S1 = 0.0, S2 = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      const double gm = gamma ? gamma[c] : 1.0;
      S1 += gm * ca[c];                   // sum dxhat
      S2 += gm * (cb[c] - mu * ca[c]) * rs;  // sum dxhat * xhat
    }
    gsum[g] = S1;
    gsum[G + g] = S2;
  }
  __syncthreads();
  for (int c = t; c < C; c += GNF_T) {
    const int g = c / cpg;
    const double mu = mean[n * G + g], rs = rstd[n * G + g];
    const double gm = gamma ? gamma[c] : 1.0;
    const double Bk = -rs * rs * gsum[G + g] / count;
    cA[c] = (float)(rs * gm);
    cB[c] = (float)Bk;
    cC[c] = (float)(-rs * gsum[g] / count - Bk * mu);
  }
  __syncthreads();
  if (!act_t) return;
  float A[VEC], B[VEC], Cc[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    A[e] = cA[c0 + e];
    B[e] = cB[c0 + e];
    Cc[e] = cC[c0 + e];
  }
  T* ob = dx + (long)n * HW * ocs + oco + c0;
  for (int r = r0; r < HW; r += RP) {
    const u32x4 xv = ld16(xb + (long)r * xcs);
    const u32x4 dv = ld16(db + (long)r * dcs);
    const T* xe = reinterpret_cast<const T*>(&xv);
    const T* de = reinterpret_cast<const T*>(&dv);
    u32x4 o;
    T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float xf = to_f(xe[e]);
      const float g = to_f(de[e]) * act_bwd_c<ACT, sizeof(T) == 2>(xf * sc[e] + sf[e]);
      oe[e] = from_f<T>(A[e] * g + B[e] * xf + Cc[e]);
    }
    st16(ob + (long)r * ocs, o);
  }
}

static size_t gnf_smem(int vec, int C, int G) {
  return (size_t)GNF_T * vec * 4 + (size_t)2 * C * 8 + (size_t)4 * C * 4 + 8 + (size_t)2 * G * 8;
}

// z = act(x * scale + shift) (+ res) ; NHWC; scale/shift per channel or per (n, channel). With res (a residual
// branch: Bottleneck's x + cv2(...)) the activation is rounded to T first and the sum rounded again — bitwise the
// affine_act + adr_ew add pair it replaces
template <typename T, int ACT>
__global__ void __launch_bounds__(256) affine_act_kernel(const T* __restrict__ x, int xcs, int xco, T* __restrict__ z,
                                                         int zcs, int zco, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, int per_sample, int act,
                                                         long npix, int HW, int C, const T* __restrict__ res,
                                                         int rcs) {
  constexpr int VEC = 16 / sizeof(T);
  const PixLanes L(C / VEC);
  if (!L.active) return;
  const int c0 = L.cg * VEC;
  float sc[VEC], sh[VEC];
  int ncur = -1;
  if (!per_sample) {
    ld_coef<VEC>(scale + c0, sc);
    ld_coef<VEC>(shift + c0, sh);
  }
  for (long pix = (long)blockIdx.x * L.rpb + L.r0; pix < npix; pix += (long)gridDim.x * L.rpb) {
    const u32x4 v = ld16(x + pix * xcs + xco + c0);
    if (per_sample) {
      const int n = (int)((unsigned long)pix / (unsigned)HW);
      if (n != ncur) {
        ncur = n;
        ld_coef<VEC>(scale + n * C + c0, sc);
        ld_coef<VEC>(shift + n * C + c0, sh);
      }
    }
    const T* e = reinterpret_cast<const T*>(&v);
    u32x4 o;
    T* oe = reinterpret_cast<T*>(&o);
    if (res) {
      const u32x4 rv = ld16(res + pix * rcs + c0);
      const T* re = reinterpret_cast<const T*>(&rv);
#pragma unroll
      for (int k = 0; k < VEC; ++k)
        oe[k] = from_f<T>(to_f(from_f<T>(bn_act_fwd_elem<ACT, sizeof(T) == 2>(to_f(e[k]), sc[k], sh[k]))) +
                          to_f(re[k]));
    } else {
#pragma unroll
      for (int k = 0; k < VEC; ++k) oe[k] = from_f<T>(bn_act_fwd_elem<ACT, sizeof(T) == 2>(to_f(e[k]), sc[k], sh[k]));
    }
    st16(z + pix * zcs + zco + c0, o);
  }
}

// dx = A*g + B*x + C with g = dz * act'(x*scale+shift) ; optional accumulate into dx
template <typename T, int ACT>
__global__ void __launch_bounds__(256) affine_act_bwd_kernel(const T* __restrict__ x, int xcs, int xco,
                                                             const T* __restrict__ dz, int dcs, int dco,
                                                             T* __restrict__ dx, int ocs, int oco,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ A,
                                                             const float* __restrict__ B,
                                                             const float* __restrict__ Cc, int per_sample,
                                                             int coef_per_sample, int act, long npix, int HW, int C,
                                                             int accumulate) {
  constexpr int VEC = 16 / sizeof(T);
  const PixLanes L(C / VEC);
  if (!L.active) return;
  const int c0 = L.cg * VEC;
  float sc[VEC], sh[VEC], ca[VEC], cbv[VEC], cc[VEC];
  int ns = -1, nc = -1;
  if (!per_sample) {
    ld_coef<VEC>(scale + c0, sc);
    ld_coef<VEC>(shift + c0, sh);
  }
  if (!coef_per_sample) {
    ld_coef<VEC>(A + c0, ca);
    ld_coef<VEC>(B + c0, cbv);
    ld_coef<VEC>(Cc + c0, cc);
  }
  for (long pix = (long)blockIdx.x * L.rpb + L.r0; pix < npix; pix += (long)gridDim.x * L.rpb) {
    const u32x4 xv = ld16(x + pix * xcs + xco + c0);
    const u32x4 dv = ld16(dz + pix * dcs + dco + c0);
    u32x4 prev = {0u, 0u, 0u, 0u};
    if (accumulate) prev = ld16(dx + pix * ocs + oco + c0);
    if (per_sample || coef_per_sample) {
      const int n = (int)((unsigned long)pix / (unsigned)HW);
      if (per_sample && n != ns) {
        ns = n;
        ld_coef<VEC>(scale + n * C + c0, sc);
        ld_coef<VEC>(shift + n * C + c0, sh);
      }
      if (coef_per_sample && n != nc) {
        nc = n;
        ld_coef<VEC>(A + n * C + c0, ca);
        ld_coef<VEC>(B + n * C + c0, cbv);
        ld_coef<VEC>(Cc + n * C + c0, cc);
      }
    }
    const T* xe = reinterpret_cast<const T*>(&xv);
    const T* de = reinterpret_cast<const T*>(&dv);
    const T* pe = reinterpret_cast<const T*>(&prev);
    u32x4 o;
    T* oe = reinterpret_cast<T*>(&o);
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const float xf = to_f(xe[k]);
      const float g = bn_act_g<ACT, sizeof(T) == 2>(to_f(de[k]), xf, sc[k], sh[k]);
      float r = bn_act_bwd_lin(g, xf, ca[k], cbv[k], cc[k]);
      if (accumulate) r += to_f(pe[k]);
      oe[k] = from_f<T>(r);
    }
    st16(dx + pix * ocs + oco + c0, o);
  }
}

// out[c] (+)= sum_p partial[p][which][c]
__global__ void __launch_bounds__(256) partial_sum_kernel(const float* __restrict__ partial, int P, int C, int which,
                                                          float* out, int accumulate) {
  int c = blockIdx.x;
  double a = 0.0, b = 0.0;
  for (int p = threadIdx.x; p < P; p += 256) a += partial[(long)p * 2 * C + which * C + c];
  block_sum2(a, b);
  if (threadIdx.x == 0) out[c] = accumulate ? out[c] + (float)a : (float)a;
}

// Many partial sums per launch (the trainer defers the bias gradients to the end of backward): block j of the
// grid reduces channel j - start[e] of entry e exactly as partial_sum_kernel does (same order).
constexpr int PSB_MAX = 80;
struct PsumBatch {
  adr_psum_entry e[PSB_MAX];
  int start[PSB_MAX + 1];
  int count;
};
__global__ void __launch_bounds__(256) partial_sum_batched_kernel(PsumBatch b) {
  int j = 0;
  while (j + 1 < b.count && (int)blockIdx.x >= b.start[j + 1]) ++j;
  const adr_psum_entry& en = b.e[j];
  const int c = blockIdx.x - b.start[j];
  double a = 0.0, z = 0.0;
  for (int p = threadIdx.x; p < en.P; p += 256) a += en.partial[(long)p * 2 * en.C + en.which * en.C + c];
  block_sum2(a, z);
  if (threadIdx.x == 0) en.out[c] = en.accumulate ? en.out[c] + (float)a : (float)a;
}

static int grid_for(long npix, int G) {
  const long rpb = 256 / G;  // pixels per block pass (PixLanes)
  long b = (npix + rpb - 1) / rpb;
  if (b > 65536) b = 65536;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace adr

using namespace adr;

extern "C" int adr_nc_reduce_chunks(int HW, int rows_per_chunk) { return cdiv(HW, rows_per_chunk); }

extern "C" int adr_nc_reduce(int dtype, int mode, const void* x, int xcs, int xco, const void* dz, int dcs, int dco,
                             const float* scale, const float* shift, int per_sample, int act, int N, int HW, int C,
                             int rows_per_chunk, float* partial, void* stream) {
  int vec = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % vec == 0 && C / vec <= 256, "nc_reduce: C=%d unsupported", C);
  ADR_REQUIRE(xcs % vec == 0 && xco % vec == 0 && dcs % vec == 0 && dco % vec == 0, "nc_reduce: misaligned view");
  ADR_REQUIRE(mode == RED_STATS || mode == RED_BWD || mode == RED_SUM, "nc_reduce: mode");
  int chunks = cdiv(HW, rows_per_chunk);
  dim3 grid(chunks, N);
  hipStream_t st = (hipStream_t)stream;
  if (mode == RED_BWD) {
#define ADR_NCR(A)                                                                                                  \
  if (dtype == ADR_BF16)                                                                                            \
    hipLaunchKernelGGL((nc_reduce_kernel<__bf16, RED_BWD, A>), grid, dim3(256), 0, st, (const __bf16*)x, xcs, xco,  \
                       (const __bf16*)dz, dcs, dco, scale, shift, per_sample, act, HW, C, rows_per_chunk, chunks,   \
                       partial);                                                                                    \
  else                                                                                                              \
    hipLaunchKernelGGL((nc_reduce_kernel<float, RED_BWD, A>), grid, dim3(256), 0, st, (const float*)x, xcs, xco,    \
                       (const float*)dz, dcs, dco, scale, shift, per_sample, act, HW, C, rows_per_chunk, chunks,    \
                       partial)
    ADR_ACT_DISPATCH(act, ADR_NCR);
#undef ADR_NCR
  } else {
    if (dtype == ADR_BF16)
      hipLaunchKernelGGL((nc_reduce_kernel<__bf16, RED_STATS>), grid, dim3(256), 0, st, (const __bf16*)x, xcs, xco,
                         (const __bf16*)nullptr, 0, 0, scale, shift, per_sample, act, HW, C, rows_per_chunk, chunks,
                         partial);
    else
      hipLaunchKernelGGL((nc_reduce_kernel<float, RED_STATS>), grid, dim3(256), 0, st, (const float*)x, xcs, xco,
                         (const float*)nullptr, 0, 0, scale, shift, per_sample, act, HW, C, rows_per_chunk, chunks,
                         partial);
  }
  return check_launch("adr_nc_reduce");
}

// ADR_FIN_PRESUM=0: the single-launch finalize at every P (A/B; read per call, so a test can switch it in-process)
static bool fin_presum_off() {
  const char* e = getenv("ADR_FIN_PRESUM");
  return e && atoi(e) == 0;
}

// Long finalizes (P > 4096 partial rows, > 2048 at C >= 256: the 160^2 / 320^2 layers, P = 6 400 - 25 600 at bs 64) are two
// launches: the per-channel kernels above read one 4-byte column per block, so a block's P row reads are P separate
// cache lines and every channel block walks the same lines (14 us at P = 12 800, C = 32; 45 us at C = 256, against
// 3 us for P = 50). fin_presum_kernel first sums blocks of `rb` consecutive rows of all 2C columns with coalesced
// reads over the whole chip (double accumulation, fixed order) into the device-global scratch, and the finalize
// reduces those <= FIN_S rows. Deterministic (the split depends on P only); the finalizes of a process are issued
// on one stream (the scratch is not per-stream).

__global__ void __launch_bounds__(256) fin_presum_kernel(const float* __restrict__ partial, int P, int C2, int rb) {
  float* out = g_fin_scratch;
  __shared__ double red[256];
  const int p0 = blockIdx.x * rb, p1 = min(P, p0 + rb);
  for (int c0 = 0; c0 < C2; c0 += 256) {
    const int cw = min(256, C2 - c0), parts = 256 / cw;  // threads = (column, row part)
    const int c = c0 + (int)threadIdx.x % cw, part = (int)threadIdx.x / cw;
    double a = 0.0;
    if (part < parts)
      for (int p = p0 + part; p < p1; p += parts) a += partial[(long)p * C2 + c];
    red[threadIdx.x] = a;
    __syncthreads();
    if ((int)threadIdx.x < cw) {
      double t = 0.0;
      for (int q = 0; q < parts; ++q) t += red[q * cw + threadIdx.x];
      out[(long)blockIdx.x * C2 + c] = (float)t;
    }
    __syncthreads();
  }
}

// long finalize: pre-sum the caller's [P][2][C] rows into the scratch (returns 1, P becomes the scratch rows)
static int fin_rows(const float* partial, int& P, int C, hipStream_t st) {
  // measured (scripts/finalize_micro.py): the extra launch pays from P = 6 400 at every C and from P = 3 200 at C >= 256
  if (!partial || P <= FIN_PMAX || (P <= 2 * FIN_PMAX && C < 256) || (long)FIN_S * 2 * C > FIN_SCRATCH ||
      fin_presum_off())
    return 0;
  const int rb = (P + FIN_S - 1) / FIN_S, S = (P + rb - 1) / rb;
  hipLaunchKernelGGL(fin_presum_kernel, dim3(S), dim3(256), 0, st, partial, P, 2 * C, rb);
  P = S;
  return 1;
}

extern "C" int adr_bn_finalize(const float* partial, int P, int C, double count, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, float momentum, float eps, int training,
                               float* scale, float* shift, float* mean, float* rstd, void* stream) {
  ADR_REQUIRE(C > 0, "bn_finalize: C");
  hipStream_t st = (hipStream_t)stream;
  const int pre = training ? fin_rows(partial, P, C, st) : 0;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, partial, P, C, count, gamma, beta,
                     running_mean, running_var, momentum, eps, training, scale, shift, mean, rstd, pre);
  return check_launch("adr_bn_finalize");
}

extern "C" int adr_bn_bwd_finalize(const float* partial, int P, int C, double count, const float* mean,
                                   const float* rstd, const float* gamma, float* dgamma, float* dbeta, float* A,
                                   float* B, float* Cc, int training, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int pre = fin_rows(partial, P, C, st);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, partial, P, C, count, mean,
                     rstd, gamma, dgamma, dbeta, A, B, Cc, training, accumulate, pre);
  return check_launch("adr_bn_bwd_finalize");
}

extern "C" int adr_gn_finalize(const float* partial, int N, int chunks, int C, int G, double count, const float* gamma,
                               const float* beta, float eps, float* scale, float* shift, float* mean, float* rstd,
                               void* stream) {
  ADR_REQUIRE(G <= 64 && C <= 1024 && C % G == 0, "gn_finalize: G=%d C=%d", G, C);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, partial, chunks, C, G, count,
                     gamma, beta, eps, scale, shift, mean, rstd);
  return check_launch("adr_gn_finalize");
}

extern "C" int adr_gn_bwd_finalize(const float* partial, int N, int chunks, int C, int G, double count,
                                   const float* mean, const float* rstd, const float* gamma, float* dgamma,
                                   float* dbeta, float* A, float* B, float* Cc, int accumulate, void* stream) {
  ADR_REQUIRE(G <= 64 && C <= 1024 && C % G == 0, "gn_bwd_finalize: G=%d C=%d", G, C);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(gn_bwd_coef_kernel, dim3(N), dim3(256), 0, st, partial, chunks, C, G, count, mean, rstd, gamma, A,
                     B, Cc);
  if (dgamma || dbeta)
    hipLaunchKernelGGL(gn_bwd_param_kernel, dim3(C), dim3(256), 0, st, partial, N, chunks, C, G, mean, rstd, dgamma,
                       dbeta, accumulate);
  return check_launch("adr_gn_bwd_finalize");
}

static int affine_act_impl(int dtype, const void* x, int xcs, int xco, const void* res, int rcs, void* z, int zcs,
                           int zco, const float* scale, const float* shift, int per_sample, int act, int N, int HW,
                           int C, void* stream) {
  int vec = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % vec == 0 && xcs % vec == 0 && xco % vec == 0 && zcs % vec == 0 && zco % vec == 0,
              "affine_act: misaligned view (C=%d)", C);
  ADR_REQUIRE(!res || rcs % vec == 0, "affine_act: misaligned residual view");
  long npix = (long)N * HW;
  ADR_REQUIRE(C / vec <= 256, "affine_act: C=%d too wide", C);
  int grid = grid_for(npix, C / vec);
  hipStream_t st = (hipStream_t)stream;
#define ADR_AA(A)                                                                                                   \
  if (dtype == ADR_BF16)                                                                                            \
    hipLaunchKernelGGL((affine_act_kernel<__bf16, A>), dim3(grid), dim3(256), 0, st, (const __bf16*)x, xcs, xco,    \
                       (__bf16*)z, zcs, zco, scale, shift, per_sample, act, npix, HW, C, (const __bf16*)res, rcs);  \
  else                                                                                                              \
    hipLaunchKernelGGL((affine_act_kernel<float, A>), dim3(grid), dim3(256), 0, st, (const float*)x, xcs, xco,      \
                       (float*)z, zcs, zco, scale, shift, per_sample, act, npix, HW, C, (const float*)res, rcs)
  ADR_ACT_DISPATCH(act, ADR_AA);
#undef ADR_AA
  return check_launch("adr_affine_act");
}

extern "C" int adr_affine_act(int dtype, const void* x, int xcs, int xco, void* z, int zcs, int zco,
                              const float* scale, const float* shift, int per_sample, int act, int N, int HW, int C,
                              void* stream) {
  return affine_act_impl(dtype, x, xcs, xco, nullptr, 0, z, zcs, zco, scale, shift, per_sample, act, N, HW, C, stream);
}

extern "C" int adr_affine_act_res(int dtype, const void* x, int xcs, int xco, const void* res, int rcs, void* z,
                                  int zcs, int zco, const float* scale, const float* shift, int per_sample, int act,
                                  int N, int HW, int C, void* stream) {
  ADR_REQUIRE(res, "affine_act_res: residual");
  return affine_act_impl(dtype, x, xcs, xco, res, rcs, z, zcs, zco, scale, shift, per_sample, act, N, HW, C, stream);
}

extern "C" int adr_affine_act_bwd(int dtype, const void* x, int xcs, int xco, const void* dz, int dcs, int dco,
                                  void* dx, int ocs, int oco, const float* scale, const float* shift, const float* A,
                                  const float* B, const float* Cc, int per_sample, int coef_per_sample, int act,
                                  int N, int HW, int C, int accumulate, void* stream) {
  int vec = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % vec == 0 && xcs % vec == 0 && xco % vec == 0 && dcs % vec == 0 && dco % vec == 0 &&
                  ocs % vec == 0 && oco % vec == 0,
              "affine_act_bwd: misaligned view");
  long npix = (long)N * HW;
  ADR_REQUIRE(C / vec <= 256, "affine_act_bwd: C=%d too wide", C);
  int grid = grid_for(npix, C / vec);
  hipStream_t st = (hipStream_t)stream;
#define ADR_AAB(AC)                                                                                                 \
  if (dtype == ADR_BF16)                                                                                            \
    hipLaunchKernelGGL((affine_act_bwd_kernel<__bf16, AC>), dim3(grid), dim3(256), 0, st, (const __bf16*)x, xcs,   \
                       xco, (const __bf16*)dz, dcs, dco, (__bf16*)dx, ocs, oco, scale, shift, A, B, Cc, per_sample, \
                       coef_per_sample, act, npix, HW, C, accumulate);                                              \
  else                                                                                                              \
    hipLaunchKernelGGL((affine_act_bwd_kernel<float, AC>), dim3(grid), dim3(256), 0, st, (const float*)x, xcs, xco, \
                       (const float*)dz, dcs, dco, (float*)dx, ocs, oco, scale, shift, A, B, Cc, per_sample,        \
                       coef_per_sample, act, npix, HW, C, accumulate)
  ADR_ACT_DISPATCH(act, ADR_AAB);
#undef ADR_AAB
  return check_launch("adr_affine_act_bwd");
}

extern "C" int adr_nc_reduce_batched(const adr_colsum_entry* entries, int count, void* stream) {
  ADR_REQUIRE(count >= 0 && (count == 0 || entries), "nc_reduce_batched: count=%d", count);
  for (int b0 = 0; b0 < count; b0 += NCB_MAX) {
    NcrBatch nb{};
    nb.count = count - b0 < NCB_MAX ? count - b0 : NCB_MAX;
    long blocks = 0;
    for (int j = 0; j < nb.count; ++j) {
      const adr_colsum_entry& en = entries[b0 + j];
      ADR_REQUIRE(en.x && en.partial && en.N > 0 && en.HW > 0 && en.C % 8 == 0 && en.C / 8 <= 256 &&
                      en.xcs % 8 == 0 && ((uintptr_t)en.x & 15) == 0 && en.rows_per_chunk > 0 &&
                      en.chunks == cdiv(en.HW, en.rows_per_chunk),
                  "nc_reduce_batched: entry %d", b0 + j);
      nb.e[j] = en;
      nb.start[j] = (int)blocks;
      blocks += (long)en.N * en.chunks;
    }
    ADR_REQUIRE(blocks < (1l << 31), "nc_reduce_batched: grid");
    nb.start[nb.count] = (int)blocks;
    if (getenv("ADR_DEBUG_NCB"))  // entry table for profiling (one line per entry)
      for (int j = 0; j < nb.count; ++j)
        fprintf(stderr, "ncb %d: N=%d HW=%d C=%d xcs=%d rows=%d chunks=%d blocks=%d\n", b0 + j, nb.e[j].N, nb.e[j].HW,
                nb.e[j].C, nb.e[j].xcs, nb.e[j].rows_per_chunk, nb.e[j].chunks, nb.e[j].N * nb.e[j].chunks);
    hipLaunchKernelGGL(nc_reduce_batched_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, nb);
  }
  return check_launch("adr_nc_reduce_batched");
}

extern "C" int adr_partial_sum_batched(const adr_psum_entry* entries, int count, void* stream) {
  ADR_REQUIRE(count >= 0 && (count == 0 || entries), "partial_sum_batched: count=%d", count);
  for (int b0 = 0; b0 < count; b0 += PSB_MAX) {
    PsumBatch pb{};
    pb.count = count - b0 < PSB_MAX ? count - b0 : PSB_MAX;
    int blocks = 0;
    for (int j = 0; j < pb.count; ++j) {
      const adr_psum_entry& en = entries[b0 + j];
      ADR_REQUIRE(en.partial && en.out && en.P > 0 && en.C > 0, "partial_sum_batched: entry %d", b0 + j);
      for (int q = 0; q < j; ++q)
        ADR_REQUIRE(pb.e[q].out != en.out, "partial_sum_batched: entries %d and %d share a destination", b0 + q, b0 + j);
      pb.e[j] = en;
      pb.start[j] = blocks;
      blocks += en.C;
    }
    pb.start[pb.count] = blocks;
    hipLaunchKernelGGL(partial_sum_batched_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, pb);
  }
  return check_launch("adr_partial_sum_batched");
}

extern "C" int adr_partial_sum(const float* partial, int P, int C, int which, float* out, int accumulate,
                               void* stream) {
  hipLaunchKernelGGL(partial_sum_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, partial, P, C, which, out,
                     accumulate);
  return check_launch("adr_partial_sum");
}

extern "C" int adr_gn_fused_supported(int dtype, int C, int G) {
  const int vec = dtype == ADR_BF16 ? 8 : 4;
  return C % vec == 0 && C / vec <= GNF_T && G > 0 && C % G == 0 && gnf_smem(vec, C, G) + (size_t)C * 4 <= 64 * 1024;
}

extern "C" int adr_gn_act_fused(int dtype, const void* x, int xcs, int xco, void* z, int zcs, int zco,
                                const float* gamma, const float* beta, float eps, int N, int HW, int C, int G, int act,
                                float* scale, float* shift, float* mean, float* rstd, void* stream) {
  const int vec = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(N > 0 && HW > 0 && C % vec == 0 && C / vec <= GNF_T && G > 0 && C % G == 0 && xcs % vec == 0 &&
                  xco % vec == 0 && zcs % vec == 0 && zco % vec == 0,
              "gn_act_fused: N=%d HW=%d C=%d G=%d (views must be 16-byte aligned)", N, HW, C, G);
  const size_t sm = gnf_smem(vec, C, G);
  ADR_REQUIRE(sm <= 64 * 1024, "gn_act_fused: C=%d needs %zu bytes of LDS", C, sm);
  hipStream_t st = (hipStream_t)stream;
#define ADR_GNF(A)                                                                                                  \
  if (dtype == ADR_BF16)                                                                                            \
    hipLaunchKernelGGL((gn_fused_fwd_kernel<__bf16, A>), dim3(N), dim3(GNF_T), sm, st, (const __bf16*)x, xcs, xco,  \
                       (__bf16*)z, zcs, zco, gamma, beta, eps, HW, C, G, scale, shift, mean, rstd);                 \
  else                                                                                                              \
    hipLaunchKernelGGL((gn_fused_fwd_kernel<float, A>), dim3(N), dim3(GNF_T), sm, st, (const float*)x, xcs, xco,    \
                       (float*)z, zcs, zco, gamma, beta, eps, HW, C, G, scale, shift, mean, rstd)
  ADR_ACT_DISPATCH(act, ADR_GNF);
#undef ADR_GNF
  return check_launch("adr_gn_act_fused");
}

extern "C" int adr_gn_act_bwd_fused(int dtype, const void* x, int xcs, int xco, const void* dz, int dcs, int dco,
                                    void* dx, int ocs, int oco, const float* scale, const float* shift,
                                    const float* mean, const float* rstd, const float* gamma, int N, int HW, int C,
                                    int G, int act, float* partial, void* stream) {
  const int vec = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(N > 0 && HW > 0 && C % vec == 0 && C / vec <= GNF_T && G > 0 && C % G == 0 && xcs % vec == 0 &&
                  xco % vec == 0 && dcs % vec == 0 && dco % vec == 0 && ocs % vec == 0 && oco % vec == 0,
              "gn_act_bwd_fused: N=%d HW=%d C=%d G=%d (views must be 16-byte aligned)", N, HW, C, G);
  const size_t sm = gnf_smem(vec, C, G) + (size_t)C * 4;
  ADR_REQUIRE(sm <= 64 * 1024, "gn_act_bwd_fused: C=%d needs %zu bytes of LDS", C, sm);
  hipStream_t st = (hipStream_t)stream;
#define ADR_GNB(A)                                                                                                  \
  if (dtype == ADR_BF16)                                                                                            \
    hipLaunchKernelGGL((gn_fused_bwd_kernel<__bf16, A>), dim3(N), dim3(GNF_T), sm, st, (const __bf16*)x, xcs, xco,  \
                       (const __bf16*)dz, dcs, dco, (__bf16*)dx, ocs, oco, scale, shift, mean, rstd, gamma, HW, C, \
                       G, partial);                                                                                 \
  else                                                                                                              \
    hipLaunchKernelGGL((gn_fused_bwd_kernel<float, A>), dim3(N), dim3(GNF_T), sm, st, (const float*)x, xcs, xco,    \
                       (const float*)dz, dcs, dco, (float*)dx, ocs, oco, scale, shift, mean, rstd, gamma, HW, C, G, \
                       partial)
  ADR_ACT_DISPATCH(act, ADR_GNB);
#undef ADR_GNB
  return check_launch("adr_gn_act_bwd_fused");
}

extern "C" int adr_gn_param_grad_batched(const adr_gnparam_entry* entries, int count, void* stream) {
  ADR_REQUIRE(count >= 0 && (count == 0 || entries), "gn_param_grad_batched: count=%d", count);
  int b0 = 0;
  while (b0 < count) {
    GnParamBatch gb{};
    int blocks = 0, j = 0;
    for (; j < GPB_MAX && b0 + j < count; ++j) {
      const adr_gnparam_entry& en = entries[b0 + j];
      ADR_REQUIRE(en.partial && en.mean && en.rstd && (en.dgamma || en.dbeta) && en.N > 0 && en.chunks > 0 &&
                      en.G > 0 && en.C % en.G == 0,
                  "gn_param_grad_batched: entry %d", b0 + j);
      bool dup = false;
      for (int q = 0; q < j; ++q)
        dup |= (en.dgamma && gb.e[q].dgamma == en.dgamma) || (en.dbeta && gb.e[q].dbeta == en.dbeta);
      if (dup) break;  // a repeated destination starts the next launch (program-order accumulation)
      gb.e[j] = en;
      gb.start[j] = blocks;
      blocks += en.C;
    }
    gb.count = j;
    gb.start[j] = blocks;
    hipLaunchKernelGGL(gn_param_batched_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, gb);
    b0 += j;
  }
  return check_launch("adr_gn_param_grad_batched");
}

// host side of the level-packed statistics: k[l] sub-images per image of level l, `sub_rows` rows per sub-image
static int level_pack_args(LevelPackArgs& a, int levels, const int* k, int N, int chunks, int sub_rows, int C, int G,
                           const void* const* gamma, const void* const* beta, const char* who) {
  ADR_REQUIRE(levels >= 1 && levels <= LP_MAX && k && N > 0 && chunks > 0 && sub_rows > 0 && C > 0,
              "%s: levels=%d N=%d chunks=%d sub_rows=%d", who, levels, N, chunks, sub_rows);
  ADR_REQUIRE(G > 0 && G <= 64 && C <= 1024 && C % G == 0, "%s: G=%d C=%d", who, G, C);
  a = LevelPackArgs{};
  a.levels = levels;
  a.N = N;
  a.chunks = chunks;
  a.C = C;
  a.G = G;
  int sub = 0;
  for (int l = 0; l < levels; ++l) {
    ADR_REQUIRE(k[l] > 0, "%s: k[%d]=%d", who, l, k[l]);
    a.k[l] = k[l];
    a.sub0[l] = sub;
    sub += N * k[l];
    a.count[l] = (double)k[l] * sub_rows * (C / G);
    a.scale[l] = 1.0f / ((float)k[l] * sub_rows);
    a.gamma[l] = gamma ? (const float*)gamma[l] : nullptr;
    a.beta[l] = beta ? (const float*)beta[l] : nullptr;
  }
  return 0;
}

extern "C" int adr_gn_finalize_packed(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows,
                                      int C, int G, const void* const* gamma, const void* const* beta, float eps,
                                      float* scale, float* shift, float* mean, float* rstd, void* stream) {
  LevelPackArgs a;
  if (int rc = level_pack_args(a, levels, k, N, chunks, sub_rows, C, G, gamma, beta, "gn_finalize_packed")) return rc;
  hipLaunchKernelGGL(gn_finalize_packed_kernel, dim3(levels * N), dim3(256), 0, (hipStream_t)stream, partial, a, eps,
                     scale, shift, mean, rstd);
  return check_launch("adr_gn_finalize_packed");
}

// Gradient of a per-image gate s feeding a GroupNorm (TaskDecomposition: GN(s_b * conv(feat)), head.py:651-667).
// GN is invariant to s up to eps, so dL/ds = sum(dZ * Z) / s is the eps-sized residue of a cancelling sum; from the
// backward's fp32 group statistics it is exact algebra: with Z = mu + Zhat/rstd and sum(Zhat) = 0,
//   sum_{i in g} dZ_i Z_i = sum_{i in g} dY'_i Zhat_i * (1 - var * rstd^2) = eps * rstd^2 * sum_{i in g} dY'_i Zhat_i,
// dY' = gamma * g, sum_{i in g} dY' Zhat = sum_{c in g} gamma_c * rstd * (sum g*x - mu * sum g)   (partial rows).
// Block per (level, image) segment; writes dL/ds / into the segment's first sub-image, 0 into the others (the
// gate's per-sub-image expansion sums them back).
__global__ void __launch_bounds__(256) gn_gate_grad_packed_kernel(const float* __restrict__ partial, LevelPackArgs a,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ rstd, float eps,
                                                                  const float* __restrict__ gate, float* dgate) {
  int l, first, k;
  lp_segment(a, l, first, k);
  const int C = a.C, G = a.G, cpg = C / G;
  __shared__ double sa[1024], sg[1024], xa[256], xb[256];
  __shared__ double red[256];
  gn_chan_sums(partial + (long)first * a.chunks * 2 * C, 0, k * a.chunks, C, sa, sg, xa, xb);
  const float* gamma = a.gamma[l];
  double t = 0.0;
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cpg;
    const double mu = mean[(long)first * G + g], rs = rstd[(long)first * G + g];
    const double gmm = gamma ? gamma[c] : 1.0;
    t += (double)eps * rs * rs * gmm * (sg[c] - mu * sa[c]) * rs;
  }
  red[threadIdx.x] = t;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  for (int j = threadIdx.x; j < k; j += 256) {
    float v = 0.0f;
    if (j == 0) {
      const double s = (double)gate[first];
      v = (float)(red[0] / (fabs(s) > 1e-30 ? s : 1e-30));
    }
    dgate[first + j] = v;
  }
}

extern "C" int adr_gn_gate_grad(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows,
                                int C, int G, const void* const* gamma, const float* mean, const float* rstd,
                                float eps, const float* gate, float* dgate, void* stream) {
  LevelPackArgs a;
  if (int rc = level_pack_args(a, levels, k, N, chunks, sub_rows, C, G, gamma, nullptr, "gn_gate_grad")) return rc;
  hipLaunchKernelGGL(gn_gate_grad_packed_kernel, dim3(levels * N), dim3(256), 0, (hipStream_t)stream, partial, a,
                     mean, rstd, eps, gate, dgate);
  return check_launch("adr_gn_gate_grad");
}

extern "C" int adr_gn_bwd_coef_packed(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows,
                                      int C, int G, const void* const* gamma, const float* mean, const float* rstd,
                                      float* A, float* B, float* Cc, void* stream) {
  LevelPackArgs a;
  if (int rc = level_pack_args(a, levels, k, N, chunks, sub_rows, C, G, gamma, nullptr, "gn_bwd_coef_packed")) return rc;
  hipLaunchKernelGGL(gn_bwd_coef_packed_kernel, dim3(levels * N), dim3(256), 0, (hipStream_t)stream, partial, a, mean,
                     rstd, A, B, Cc);
  return check_launch("adr_gn_bwd_coef_packed");
}

static int bn_pack_args(LevelPackArgs& a, int levels, const int* k, int N, int chunks, int sub_rows, int C,
                        const char* who) {
  if (int rc = level_pack_args(a, levels, k, N, chunks, sub_rows, C, 1, nullptr, nullptr, who)) return rc;
  for (int l = 0; l < levels; ++l) a.count[l] = (double)N * k[l] * sub_rows;  // a level's rows over all images
  return 0;
}

extern "C" int adr_bn_finalize_packed(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows,
                                      int C, const float* gamma, const float* beta, float* running_mean,
                                      float* running_var, float momentum, float eps, float* scale, float* shift,
                                      float* mean, float* rstd, void* stream) {
  LevelPackArgs a;
  if (int rc = bn_pack_args(a, levels, k, N, chunks, sub_rows, C, "bn_finalize_packed")) return rc;
  hipLaunchKernelGGL(bn_finalize_packed_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, partial, a, gamma, beta,
                     running_mean, running_var, momentum, eps, scale, shift, mean, rstd);
  return check_launch("adr_bn_finalize_packed");
}

extern "C" int adr_bn_bwd_finalize_packed(const float* partial, int levels, const int* k, int N, int chunks,
                                          int sub_rows, int C, const float* mean, const float* rstd,
                                          const float* gamma, float* dgamma, float* dbeta, float* A, float* B,
                                          float* Cc, int accumulate, void* stream) {
  LevelPackArgs a;
  if (int rc = bn_pack_args(a, levels, k, N, chunks, sub_rows, C, "bn_bwd_finalize_packed")) return rc;
  hipLaunchKernelGGL(bn_bwd_finalize_packed_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, partial, a, mean, rstd,
                     gamma, dgamma, dbeta, A, B, Cc, accumulate);
  return check_launch("adr_bn_bwd_finalize_packed");
}

extern "C" int adr_seg_reduce_packed(const float* in, int in_per_seg, int out_per_seg, int mean, int levels,
                                     const int* k, int N, int sub_rows, int C, float* out, void* stream) {
  LevelPackArgs a;
  if (int rc = level_pack_args(a, levels, k, N, 1, sub_rows, C, 1, nullptr, nullptr, "seg_reduce_packed")) return rc;
  ADR_REQUIRE(in && out && in != out, "seg_reduce_packed: in place / null");
  hipLaunchKernelGGL(seg_reduce_packed_kernel, dim3(levels * N), dim3(256), 0, (hipStream_t)stream, in, in_per_seg,
                     out_per_seg, mean, a, out);
  return check_launch("adr_seg_reduce_packed");
}

extern "C" int adr_gn_param_grad(const float* partial, int N, int C, int G, const float* mean, const float* rstd,
                                 float* dgamma, float* dbeta, int accumulate, void* stream) {
  ADR_REQUIRE(G > 0 && C % G == 0, "gn_param_grad: C=%d G=%d", C, G);
  hipLaunchKernelGGL(gn_bwd_param_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, partial, N, 1, C, G, mean, rstd,
                     dgamma, dbeta, accumulate);
  return check_launch("adr_gn_param_grad");
}
