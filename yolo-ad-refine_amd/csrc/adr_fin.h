// In-kernel normalisation finalize: the workgroup that writes the LAST partial-statistics row of a reduction
// turns the rows into the BatchNorm / GroupNorm coefficients itself, so no separate *_finalize launch follows the
// producer (a conv epilogue, adr_nc_reduce).
//
// Arrival protocol (measured correct and free of the L2-writeback fences: scripts/probes/lastblock_probe.hip).
// gfx950 has one L2 per XCD and they are not coherent with each other, so the rows travel through agent-scope
// coherent stores / loads (relaxed atomics: the write goes through to the coherence point, the read bypasses a
// stale L2 line) instead of plain stores plus a release/acquire fence pair (an L2 writeback + invalidate per
// workgroup). A workgroup drains its stores (s_waitcnt), then one lane increments the reduction's arrival counter;
// the workgroup that sees count == total - 1 is the last one, reads every row and resets the counter to zero
// (counters are caller-owned, zero on entry and left zero). No workgroup ever waits for another.
//
// Deterministic: rows are summed in a fixed order in double, independent of which workgroup finishes. Large
// reductions go through two levels: groups of `gs` consecutive rows (the last arrival of each group writes the
// group's double row into scratch), then the group rows.
#pragma once
#include "adr_common.h"

namespace adr {

enum FinKind { FIN_BN_FWD = 0, FIN_BN_BWD = 1, FIN_GN_FWD = 2, FIN_GN_BWD = 3 };

// adr_norm_fin plus the row geometry the producer fills in
struct FinArgs {
  adr_norm_fin f;
  int on;       // 0: plain producer (no arrival)
  int P;        // partial rows per column tile (BN) / per image (GN: chunks)
  int gs;       // rows per level-1 group
  int ngroups;  // ceil(P / gs); 1 = single level
};

__device__ __forceinline__ void st_coh(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_coh(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_coh(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every thread of the block calls this after its coherent row stores; returns (block-uniform) whether this block
// arrived last. `flag` is an LDS word.
__device__ __forceinline__ bool fin_arrive(unsigned* cnt, unsigned total, unsigned* flag) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool last = *flag == total - 1;
  __syncthreads();  // flag is reused by the next arrival
  if (last && threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return last;
}

// Fixed-order column sums of rows [r0, r1) of a row-major matrix (row stride ld elements). Column j < 2 * nc is
// element c0 + j of the row's first half (j < nc) or C + c0 + j - nc of its second half. Needs 2 * nc <= 256;
// out[j] (LDS, 256 doubles) receives the sums; tmp is LDS scratch of 256 doubles. 256 threads.
template <typename T>
__device__ __forceinline__ void fin_colsum(const T* base, long ld, int r0, int r1, int c0, int nc, int C, double* out,
                                           double* tmp) {
  const int t = threadIdx.x, ncol = 2 * nc;
  const int S = 256 / ncol;  // row subsets
  const int j = t % ncol, s = t / ncol;
  double acc = 0.0;
  if (s < S) {
    const long col = j < nc ? c0 + j : C + c0 + (j - nc);
    const T* p = base + col;
    int r = r0 + s;
    // FIN_U rows in flight (the tail is a chain of memory round trips), added in row order
    constexpr int FIN_U = 16;
    for (; r + (FIN_U - 1) * S < r1; r += FIN_U * S) {
      T v[FIN_U];
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) v[u] = ld_coh(p + (long)(r + u * S) * ld);
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) acc += (double)v[u];
    }
    for (; r < r1; r += S) acc += (double)ld_coh(p + (long)r * ld);
  }
  tmp[t] = acc;
  __syncthreads();
  if (t < ncol) {
    double a = 0.0;
    for (int q = 0; q < S; ++q) a += tmp[q * ncol + t];
    out[t] = a;
  }
  __syncthreads();
}

// BatchNorm training finalize of channel c from (sum, sum of squares) — bn_finalize_kernel's arithmetic
__device__ __forceinline__ void fin_bn_fwd_channel(const adr_norm_fin& f, int c, double a, double b) {
  const double count = f.count;
  const double mean = a / count;
  double var = b / count - mean * mean;
  if (var < 0) var = 0;
  const double rstd = 1.0 / sqrt(var + (double)f.eps);
  const double g = f.gamma ? f.gamma[c] : 1.0, bb = f.beta ? f.beta[c] : 0.0;
  f.scale[c] = (float)(g * rstd);
  f.shift[c] = (float)(bb - mean * g * rstd);
  if (f.mean) f.mean[c] = (float)mean;
  if (f.rstd) f.rstd[c] = (float)rstd;
  if (f.running_mean) {
    const double unb = count > 1 ? var * count / (count - 1) : var;
    f.running_mean[c] = (float)((1.0 - f.momentum) * f.running_mean[c] + f.momentum * mean);
    f.running_var[c] = (float)((1.0 - f.momentum) * f.running_var[c] + f.momentum * unb);
  }
}

// BatchNorm backward finalize of channel c from (sum g, sum g*x) — bn_bwd_finalize_kernel's arithmetic (training)
__device__ __forceinline__ void fin_bn_bwd_channel(const adr_norm_fin& f, int c, double a, double b) {
  const double mu = f.mean[c], rs = f.rstd[c], g = f.gamma ? f.gamma[c] : 1.0;
  const double sgx = (b - mu * a) * rs;
  if (f.dgamma) f.dgamma[c] = f.accumulate ? f.dgamma[c] + (float)sgx : (float)sgx;
  if (f.dbeta) f.dbeta[c] = f.accumulate ? f.dbeta[c] + (float)a : (float)a;
  const double Ak = g * rs;
  const double Bk = -Ak * rs * sgx / f.count;
  const double Ck = -Ak * a / f.count - Bk * mu;
  f.A[c] = (float)Ak;
  f.B[c] = (float)Bk;
  f.Cc[c] = (float)Ck;
}

// BN finalize of channels [c0, c0 + nc) of a [P][2][C] row matrix whose rows this reduction writes (the caller's
// rows are already stored with st_coh). `cnt` = this column range's counters [1 + ngroups]; `lds` >= 4 KB + 4 B.
__device__ __forceinline__ void fin_bn_tail(const FinArgs& fa, const float* rows, int row, int c0, int nc,
                                            unsigned* cnt, unsigned char* lds) {
  const adr_norm_fin& f = fa.f;
  double* out = reinterpret_cast<double*>(lds);
  double* tmp = out + 256;
  unsigned* flag = reinterpret_cast<unsigned*>(tmp + 256);
  const int C = f.C;
  const long ld = 2l * C;
  const int g = row / fa.gs;
  const int gsz = min(fa.gs, fa.P - g * fa.gs);
  if (!fin_arrive(cnt + 1 + g, (unsigned)gsz, flag)) return;
  const bool single = fa.ngroups == 1;
  for (int cc = 0; cc < nc; cc += 128) {
    const int n = min(128, nc - cc);
    fin_colsum<float>(rows, ld, g * fa.gs, g * fa.gs + gsz, c0 + cc, n, C, out, tmp);
    if (single) {
      for (int j = threadIdx.x; j < n; j += 256) {
        if (f.kind == FIN_BN_FWD) fin_bn_fwd_channel(f, c0 + cc + j, out[j], out[n + j]);
        else fin_bn_bwd_channel(f, c0 + cc + j, out[j], out[n + j]);
      }
    } else {
      double* grow = f.scratch + (long)g * ld;
      for (int j = threadIdx.x; j < 2 * n; j += 256)
        st_coh(grow + (j < n ? c0 + cc + j : C + c0 + cc + (j - n)), out[j]);
    }
    __syncthreads();
  }
  if (single || !fin_arrive(cnt, (unsigned)fa.ngroups, flag)) return;
  for (int cc = 0; cc < nc; cc += 128) {
    const int n = min(128, nc - cc);
    fin_colsum<double>(f.scratch, ld, 0, fa.ngroups, c0 + cc, n, C, out, tmp);
    for (int j = threadIdx.x; j < n; j += 256) {
      if (f.kind == FIN_BN_FWD) fin_bn_fwd_channel(f, c0 + cc + j, out[j], out[n + j]);
      else fin_bn_bwd_channel(f, c0 + cc + j, out[j], out[n + j]);
    }
    __syncthreads();
  }
}

// GroupNorm finalize of image n (rows [n * P, (n + 1) * P) of [N * P][2][C], P = chunks): statistics and
// per-(image, channel) scale / shift (FIN_GN_FWD, gn_finalize_kernel's arithmetic) or the backward coefficients
// A / B / C (FIN_GN_BWD, gn_bwd_coef_kernel's). The caller has arrived on the image's counter and is last.
// lds >= (2 * C + 2 * 256 + 2 * 64) doubles.
__device__ __forceinline__ void fin_gn_image(const FinArgs& fa, const float* rows, int n, unsigned char* lds) {
  const adr_norm_fin& f = fa.f;
  const int C = f.C, G = f.G, cpg = C / G;
  double* sa = reinterpret_cast<double*>(lds);
  double* sb = sa + C;
  double* out = sb + C;
  double* tmp = out + 256;
  double* g1 = tmp + 256;
  double* g2 = g1 + 64;
  for (int cc = 0; cc < C; cc += 128) {
    const int m = min(128, C - cc);
    fin_colsum<float>(rows, 2l * C, n * fa.P, (n + 1) * fa.P, cc, m, C, out, tmp);
    for (int j = threadIdx.x; j < m; j += 256) {
      sa[cc + j] = out[j];
      sb[cc + j] = out[m + j];
    }
    __syncthreads();
  }
  if (f.kind == FIN_GN_FWD) {
    for (int g = threadIdx.x; g < G; g += 256) {
      double a = 0.0, b = 0.0;
      for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
        a += sa[c];
        b += sb[c];
      }
      const double mu = a / f.count;
      double var = b / f.count - mu * mu;
      if (var < 0) var = 0;
      g1[g] = mu;
      g2[g] = 1.0 / sqrt(var + (double)f.eps);
      f.mean[n * G + g] = (float)mu;
      f.rstd[n * G + g] = (float)g2[g];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      const int g = c / cpg;
      const double gg = f.gamma ? f.gamma[c] : 1.0, bb = f.beta ? f.beta[c] : 0.0;
      f.scale[n * C + c] = (float)(gg * g2[g]);
      f.shift[n * C + c] = (float)(bb - g1[g] * gg * g2[g]);
    }
    return;
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cpg;
    const double mu = f.mean[n * G + g], rs = f.rstd[n * G + g];
    const double a = sa[c], b = sb[c];
    const double gm = f.gamma ? f.gamma[c] : 1.0;
    sa[c] = gm * a;                  // sum dxhat
    sb[c] = gm * (b - mu * a) * rs;  // sum dxhat * xhat
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += 256) {
    double S1 = 0.0, S2 = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      S1 += sa[c];
      S2 += sb[c];
    }
    g1[g] = S1;
    g2[g] = S2;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int g = c / cpg;
    const double mu = f.mean[n * G + g], rs = f.rstd[n * G + g];
    const double gm = f.gamma ? f.gamma[c] : 1.0;
    const double Bk = -rs * rs * g2[g] / f.count;
    f.A[n * C + c] = (float)(rs * gm);
    f.B[n * C + c] = (float)Bk;
    f.Cc[n * C + c] = (float)(-rs * g1[g] / f.count - Bk * mu);
  }
}

// host: level-1 group size for P rows (about sqrt(P), so both levels read a similar number of rows)
inline int fin_group_rows(int P) {
  if (P <= 128) return P > 0 ? P : 1;  // one level
  int gs = 16;
  while ((long)gs * gs < P && gs < 512) gs *= 2;
  return gs;
}

// host: fill the row geometry and check the caller's buffers (BN kinds: P rows per column tile, `tiles` column
// tiles; GN kinds: N images of P rows)
int fin_setup(const adr_norm_fin* f, int P, int tiles, int N, FinArgs& fa);

}  // namespace adr
