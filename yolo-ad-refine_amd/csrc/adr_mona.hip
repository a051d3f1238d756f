// The 697 L10 variant, C2TSSA_DYT_Mona_EDFFN (reference nn/modules/block.py:1624-1709, nn/modules/mona.py),
// forward + backward, NHWC:
//   * DynamicTanh (block.py:1624-1641, channels_first): y = tanh(alpha * x) * w[c] + b[c]
//   * Mona's norm-and-mix prologue (mona.py:5-10, 55-58): y = LayerNorm_C(x) * gamma[c] + x * gammax[c], the
//     LayerNorm over the channels of each pixel (LayerNorm2d, eps 1e-5) with its own weight / bias
//   * AttentionTSSA core (block.py:1646-1683) between the qkv and to_out linears, per image b and head h over the
//     token axis n (w = qkv(x) viewed (b, h, n, d)):
//        wn = w / max(||w[b,h,:,d]||_n, 1e-12)                (F.normalize dim=-2: over TOKENS)
//        Pi[b,:,n] = softmax over HEADS of temp[h] * sum_d wn^2 (nn.Softmax(dim=1) on (b, h, n))
//        dots[d] = sum_n Pi[n] / (sum_m Pi[m] + 1e-8) * w[n,d]^2 ; attn = 1 / (1 + dots)
//        out = -w * Pi[n] * attn[d]
//   * dropout with a counter-based hash mask (Mona.dropout p = 0.1 in training; mona.py:44, 63)
// Per-channel parameter gradients are fixed-order two-stage reductions (partials per row chunk, then one
// finalize block), so results are deterministic.
#include "adr_common.h"

namespace adr {

// ---------------- DynamicTanh ----------------
template <typename T, int VW>
__global__ void __launch_bounds__(256) dyt_fwd_kernel(const T* x, int xcs, const float* alpha, const float* w,
                                                      const float* b, T* y, int ycs, long npix, int C) {
  const int G = C / VW;
  const PoolLanes L(G);
  if (!L.active) return;
  const float a = alpha[0];
  POOL_LOOP(L, npix, G) {
    const int c0 = cg * VW;
    float v[VW];
    vload<T, VW>(x + pix * xcs + c0, v);
#pragma unroll
    for (int e = 0; e < VW; ++e) v[e] = tanhf(a * v[e]) * w[c0 + e] + b[c0 + e];
    vstore<T, VW>(y + pix * ycs + c0, v);
  }
}

// dx = dy * w * a * (1 - t^2); partial[chunk][3][C] = (sum dy*t, sum dy, sum dy*w*x*(1-t^2)) per channel.
// grid = row chunks; threads = (256 / G) pixel rows x G channel groups.
template <typename T, int VW>
__global__ void __launch_bounds__(256) dyt_bwd_kernel(const T* x, int xcs, const T* dy, int dcs, const float* alpha,
                                                      const float* w, T* dx, int ocs, long npix, int C, int rows,
                                                      float* partial) {
  __shared__ float red[3][256 * VW];
  const int G = C / VW, rpp = 256 / G;
  const int t = threadIdx.x, cg = t % G, r0 = t / G, c0 = cg * VW;
  const float a = alpha[0];
  float s0[VW], s1[VW], s2[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) s0[e] = s1[e] = s2[e] = 0.f;
  const long beg = (long)blockIdx.x * rows, end = min(npix, beg + rows);
  if (r0 < rpp)
    for (long pix = beg + r0; pix < end; pix += rpp) {
      float xv[VW], g[VW], o[VW];
      vload<T, VW>(x + pix * xcs + c0, xv);
      vload<T, VW>(dy + pix * dcs + c0, g);
#pragma unroll
      for (int e = 0; e < VW; ++e) {
        const float th = tanhf(a * xv[e]), d1 = 1.f - th * th;
        const float gw = g[e] * w[c0 + e];
        o[e] = gw * a * d1;
        s0[e] += g[e] * th;
        s1[e] += g[e];
        s2[e] += gw * xv[e] * d1;
      }
      vstore<T, VW>(dx + pix * ocs + c0, o);
    }
#pragma unroll
  for (int e = 0; e < VW; ++e) {
    red[0][t * VW + e] = s0[e];
    red[1][t * VW + e] = s1[e];
    red[2][t * VW + e] = s2[e];
  }
  __syncthreads();
  float* out = partial + (long)blockIdx.x * 3 * C;
  for (int i = t; i < 3 * C; i += 256) {
    const int q = i / C, c = i % C, g = c / VW, e = c % VW;
    float s = 0.f;
    for (int r = 0; r < rpp; ++r) s += red[q][(r * G + g) * VW + e];
    out[i] = s;
  }
}

// ---------------- LayerNorm-over-channels mix ----------------
// one pixel per L = C / VW lanes (L a power of two <= 64); pixel statistics by xor shuffles within the L lanes
template <int L>
__device__ __forceinline__ float lane_group_sum(float v) {
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int VW, int L>
__global__ void __launch_bounds__(256) ln_mix_fwd_kernel(const T* x, int xcs, const float* lw, const float* lb,
                                                         const float* gamma, const float* gammax, T* y, int ycs,
                                                         float* mean, float* rstd, long npix, float eps) {
  constexpr int C = L * VW, PPB = 256 / L;
  const int lane = threadIdx.x % L, c0 = lane * VW;
  for (long pix = (long)blockIdx.x * PPB + threadIdx.x / L; pix < npix; pix += (long)gridDim.x * PPB) {
    float v[VW];
    vload<T, VW>(x + pix * xcs + c0, v);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) s += v[e];
    const float mu = lane_group_sum<L>(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) q += (v[e] - mu) * (v[e] - mu);
    const float rs = rsqrtf(lane_group_sum<L>(q) / (float)C + eps);
    float o[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const int c = c0 + e;
      o[e] = ((v[e] - mu) * rs * lw[c] + lb[c]) * gamma[c] + v[e] * gammax[c];
    }
    vstore<T, VW>(y + pix * ycs + c0, o);
    if (lane == 0) {
      mean[pix] = mu;
      rstd[pix] = rs;
    }
  }
}

// dx, and partial[chunk][4][C] = (sum dz*gamma*xhat, sum dz*gamma, sum dz*(xhat*lw + lb), sum dz*x)
template <typename T, int VW, int L>
__global__ void __launch_bounds__(256) ln_mix_bwd_kernel(const T* x, int xcs, const T* dz, int dcs, const float* lw,
                                                         const float* lb, const float* gamma, const float* gammax,
                                                         const float* mean, const float* rstd, T* dx, int ocs,
                                                         long npix, int rows, float* partial) {
  constexpr int C = L * VW, PPB = 256 / L;
  __shared__ float red[4][256 * VW];
  const int lane = threadIdx.x % L, prow = threadIdx.x / L, c0 = lane * VW;
  float s[4][VW];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < VW; ++e) s[q][e] = 0.f;
  const long beg = (long)blockIdx.x * rows, end = min(npix, beg + rows);
  for (long pix = beg + prow; pix < end; pix += PPB) {
    float v[VW], g[VW], xh[VW], dxh[VW];
    vload<T, VW>(x + pix * xcs + c0, v);
    vload<T, VW>(dz + pix * dcs + c0, g);
    const float mu = mean[pix], rs = rstd[pix];
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const int c = c0 + e;
      xh[e] = (v[e] - mu) * rs;
      const float gg = g[e] * gamma[c];
      dxh[e] = gg * lw[c];
      a1 += dxh[e];
      a2 += dxh[e] * xh[e];
      s[0][e] += gg * xh[e];
      s[1][e] += gg;
      s[2][e] += g[e] * (xh[e] * lw[c] + lb[c]);
      s[3][e] += g[e] * v[e];
    }
    const float m1 = lane_group_sum<L>(a1) / (float)C, m2 = lane_group_sum<L>(a2) / (float)C;
    float o[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) o[e] = rs * (dxh[e] - m1 - xh[e] * m2) + g[e] * gammax[c0 + e];
    vstore<T, VW>(dx + pix * ocs + c0, o);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < VW; ++e) red[q][threadIdx.x * VW + e] = s[q][e];
  __syncthreads();
  float* out = partial + (long)blockIdx.x * 4 * C;
  for (int i = threadIdx.x; i < 4 * C; i += 256) {
    const int q = i / C, c = i % C, ln = c / VW, e = c % VW;
    float t = 0.f;
    for (int r = 0; r < PPB; ++r) t += red[q][(r * L + ln) * VW + e];
    out[i] = t;
  }
}

// dst_q[c] (+)= sum_chunk partial[chunk][q][c] for q < Q (null dst skipped); quantity `scal_q` is further summed
// over c into scal_dst[0]. One block, fixed order.
__global__ void __launch_bounds__(256) colsum_kernel(const float* partial, int chunks, int Q, int C, float* d0,
                                                     float* d1, float* d2, float* d3, int accumulate, int scal_q,
                                                     float* scal_dst) {
  __shared__ float sc[256];
  float* dst[4] = {d0, d1, d2, d3};
  float mine = 0.f;
  for (int i = threadIdx.x; i < Q * C; i += 256) {
    const int q = i / C, c = i % C;
    float s = 0.f;
    for (int k = 0; k < chunks; ++k) s += partial[((long)k * Q + q) * C + c];
    if (q == scal_q) mine += s;
    else if (q < 4 && dst[q]) dst[q][c] = accumulate ? dst[q][c] + s : s;
  }
  sc[threadIdx.x] = mine;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sc[threadIdx.x] += sc[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && scal_q >= 0 && scal_dst) scal_dst[0] = accumulate ? scal_dst[0] + sc[0] : sc[0];
}

// ---------------- AttentionTSSA core ----------------
// Block per (b, h): threads = TPP token rows x LD lanes; lane covers VW channels of the head's D.
struct Tssa1Args {
  const void* w;  // tokens (B, N, C) with token stride cs, C = H * D
  int cs, B, N, H, D;
  const float* temp;  // [H]
  float* nrm;         // [B][H][D]  ||w||_n per channel
  float* s;           // [B][H][N]  temp * sum_d wn^2
  float* pi;          // [B][H][N]
  float* attn;        // [B][H][D]
  float* z;           // [B][H]     sum_n Pi + 1e-8
  void* out;          // (B, N, C) tokens, stride ocs
  int ocs;
  const void* g;      // dout tokens, stride gcs
  int gcs;
  float* ddots;       // [B][H][D]
  float* dpi;         // [B][H][N]
  void* dw;           // (B, N, C) gradient tokens, stride dwcs
  int dwcs;
  float* dtemp;       // [B][H] partials
};

// stats: nrm[d], s[n]
template <typename T, int VW, int LD>
__global__ void __launch_bounds__(256) tssa1_stats_kernel(Tssa1Args a) {
  constexpr int TPP = 256 / LD, D = LD * VW;
  __shared__ float red[256 * VW];
  __shared__ float inv[D];
  const int b = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x % LD, r0 = threadIdx.x / LD, c0 = h * D + lane * VW;
  const T* w = (const T*)a.w + (long)b * a.N * a.cs;
  float p[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) p[e] = 0.f;
  for (int n = r0; n < a.N; n += TPP) {
    float v[VW];
    vload<T, VW>(w + (long)n * a.cs + c0, v);
#pragma unroll
    for (int e = 0; e < VW; ++e) p[e] += v[e] * v[e];
  }
  chan_sum<VW, LD>(p, red, inv);
  const long bh = (long)b * a.H + h;
  if (threadIdx.x < D) {
    const float nr = sqrtf(inv[threadIdx.x]);
    a.nrm[bh * D + threadIdx.x] = nr;
    inv[threadIdx.x] = 1.f / fmaxf(nr, 1e-12f);
  }
  __syncthreads();
  const float tp = a.temp[h];
  for (int n = r0; n < a.N; n += TPP) {
    float v[VW];
    vload<T, VW>(w + (long)n * a.cs + c0, v);
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const float wn = v[e] * inv[lane * VW + e];
      q += wn * wn;
    }
    q = tok_sum<LD>(q);
    if (lane == 0) a.s[bh * a.N + n] = tp * q;
  }
}

// forward: Pi (softmax over heads), Z, dots -> attn, out
template <typename T, int VW, int LD>
__global__ void __launch_bounds__(256) tssa1_fwd_kernel(Tssa1Args a) {
  constexpr int TPP = 256 / LD, D = LD * VW;
  __shared__ float red[256 * VW];
  __shared__ float at[D];
  __shared__ float sh[256];
  const int b = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x % LD, r0 = threadIdx.x / LD, c0 = h * D + lane * VW;
  const T* w = (const T*)a.w + (long)b * a.N * a.cs;
  const long bh = (long)b * a.H + h;
  // Pi[n] for this head, all tokens (thread-strided), and Z
  float zs = 0.f;
  for (int n = threadIdx.x; n < a.N; n += 256) {
    float mx = -INFINITY;
    for (int k = 0; k < a.H; ++k) mx = fmaxf(mx, a.s[((long)b * a.H + k) * a.N + n]);
    float den = 0.f;
    for (int k = 0; k < a.H; ++k) den += __expf(a.s[((long)b * a.H + k) * a.N + n] - mx);
    const float pv = __expf(a.s[bh * a.N + n] - mx) / den;
    a.pi[bh * a.N + n] = pv;
    zs += pv;
  }
  const float Z = block_sum256(zs, sh) + 1e-8f;
  if (threadIdx.x == 0) a.z[bh] = Z;
  __syncthreads();  // pi visible to the block (global, same block)
  float p[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) p[e] = 0.f;
  for (int n = r0; n < a.N; n += TPP) {
    float v[VW];
    vload<T, VW>(w + (long)n * a.cs + c0, v);
    const float ph = a.pi[bh * a.N + n] / Z;
#pragma unroll
    for (int e = 0; e < VW; ++e) p[e] += ph * v[e] * v[e];
  }
  chan_sum<VW, LD>(p, red, at);
  if (threadIdx.x < D) {
    const float v = 1.f / (1.f + at[threadIdx.x]);
    at[threadIdx.x] = v;
    a.attn[bh * D + threadIdx.x] = v;
  }
  __syncthreads();
  T* out = (T*)a.out + (long)b * a.N * a.ocs;
  for (int n = r0; n < a.N; n += TPP) {
    float v[VW];
    vload<T, VW>(w + (long)n * a.cs + c0, v);
    const float pv = a.pi[bh * a.N + n];
#pragma unroll
    for (int e = 0; e < VW; ++e) v[e] = -v[e] * pv * at[lane * VW + e];
    vstore<T, VW>(out + (long)n * a.ocs + c0, v);
  }
}

// backward 1: ddots[d], dPi[n]
template <typename T, int VW, int LD>
__global__ void __launch_bounds__(256) tssa1_bwd1_kernel(Tssa1Args a) {
  constexpr int TPP = 256 / LD, D = LD * VW;
  __shared__ float red[256 * VW];
  __shared__ float dd[D];
  __shared__ float sh[256];
  const int b = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x % LD, r0 = threadIdx.x / LD, c0 = h * D + lane * VW;
  const T* w = (const T*)a.w + (long)b * a.N * a.cs;
  const T* g = (const T*)a.g + (long)b * a.N * a.gcs;
  const long bh = (long)b * a.H + h;
  const float Z = a.z[bh];
  float p[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) p[e] = 0.f;
  for (int n = r0; n < a.N; n += TPP) {
    float v[VW], gv[VW];
    vload<T, VW>(w + (long)n * a.cs + c0, v);
    vload<T, VW>(g + (long)n * a.gcs + c0, gv);
    const float pv = a.pi[bh * a.N + n];
#pragma unroll
    for (int e = 0; e < VW; ++e) p[e] -= gv[e] * v[e] * pv;  // dattn
  }
  chan_sum<VW, LD>(p, red, dd);
  if (threadIdx.x < D) {
    const float at = a.attn[bh * D + threadIdx.x];
    const float v = -dd[threadIdx.x] * at * at;  // ddots
    dd[threadIdx.x] = v;
    a.ddots[bh * D + threadIdx.x] = v;
  }
  __syncthreads();
  // dPi_direct[n] = -sum_d g w attn ; dPhat[n] = sum_d ddots w^2 ; T = sum_n dPhat Pi
  float tsum = 0.f;
  for (int n = r0; n < a.N; n += TPP) {
    float v[VW], gv[VW];
    vload<T, VW>(w + (long)n * a.cs + c0, v);
    vload<T, VW>(g + (long)n * a.gcs + c0, gv);
    float q1 = 0.f, q2 = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const int d = lane * VW + e;
      q1 -= gv[e] * v[e] * a.attn[bh * D + d];
      q2 += dd[d] * v[e] * v[e];
    }
    q1 = tok_sum<LD>(q1);
    q2 = tok_sum<LD>(q2);
    if (lane == 0) {
      a.dpi[bh * a.N + n] = q1 + q2 / Z;  // the -T/Z^2 term is added below
      tsum += q2 * a.pi[bh * a.N + n];
    }
  }
  const float Tt = block_sum256(tsum, sh);
  __syncthreads();
  for (int n = threadIdx.x; n < a.N; n += 256) a.dpi[bh * a.N + n] -= Tt / (Z * Z);
}

// backward 2: ds (softmax over heads), dtemp partial, dw
template <typename T, int VW, int LD>
__global__ void __launch_bounds__(256) tssa1_bwd2_kernel(Tssa1Args a) {
  constexpr int TPP = 256 / LD, D = LD * VW;
  __shared__ float red[256 * VW];
  __shared__ float s2[D], inv[D], clampd[D];
  __shared__ float sh[256];
  extern __shared__ float dsl[];  // [N]
  const int b = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x % LD, r0 = threadIdx.x / LD, c0 = h * D + lane * VW;
  const T* w = (const T*)a.w + (long)b * a.N * a.cs;
  const T* g = (const T*)a.g + (long)b * a.N * a.gcs;
  const long bh = (long)b * a.H + h;
  const float Z = a.z[bh], tp = a.temp[h];
  if (threadIdx.x < D) {
    const float nr = a.nrm[bh * D + threadIdx.x];
    inv[threadIdx.x] = 1.f / fmaxf(nr, 1e-12f);
    clampd[threadIdx.x] = nr < 1e-12f ? 1.f : 0.f;
  }
  for (int n = threadIdx.x; n < a.N; n += 256) {
    float dot = 0.f;
    for (int k = 0; k < a.H; ++k) {
      const long i = ((long)b * a.H + k) * a.N + n;
      dot += a.pi[i] * a.dpi[i];
    }
    const float pv = a.pi[bh * a.N + n];
    dsl[n] = pv * (a.dpi[bh * a.N + n] - dot);
  }
  __syncthreads();
  // S2[d] = sum_n ds w^2 ; dtemp = sum_n ds * sum_d wn^2
  float p[VW], dt = 0.f;
#pragma unroll
  for (int e = 0; e < VW; ++e) p[e] = 0.f;
  for (int n = r0; n < a.N; n += TPP) {
    float v[VW];
    vload<T, VW>(w + (long)n * a.cs + c0, v);
    const float ds = dsl[n];
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      p[e] += ds * v[e] * v[e];
      const float wn = v[e] * inv[lane * VW + e];
      q += wn * wn;
    }
    dt += ds * q;  // summed over the token's lanes and tokens by the block sum
  }
  chan_sum<VW, LD>(p, red, s2);
  const float dts = block_sum256(dt, sh);
  if (threadIdx.x == 0) a.dtemp[bh] = dts;
  const float Zi = 1.f / Z;
  T* dw = (T*)a.dw + (long)b * a.N * a.dwcs;
  for (int n = r0; n < a.N; n += TPP) {
    float v[VW], gv[VW];
    vload<T, VW>(w + (long)n * a.cs + c0, v);
    vload<T, VW>(g + (long)n * a.gcs + c0, gv);
    const float pv = a.pi[bh * a.N + n], ds = dsl[n];
    float o[VW];
#pragma unroll
    for (int e = 0; e < VW; ++e) {
      const int d = lane * VW + e;
      const float iv = inv[d];
      float r = -gv[e] * pv * a.attn[bh * D + d] + 2.f * a.ddots[bh * D + d] * pv * Zi * v[e];
      const float nt = clampd[d] != 0.f ? ds : ds - iv * iv * s2[d];
      r += 2.f * tp * iv * iv * v[e] * nt;
      o[e] = r;
    }
    vstore<T, VW>(dw + (long)n * a.dwcs + c0, o);
  }
}

// ---------------- dropout (counter-based hash, keep with probability 1 - p, scale 1 / (1 - p)) ----------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool keep_elem(uint64_t seed, uint64_t idx, uint32_t thresh) {
  const uint32_t h = mix32((uint32_t)idx ^ mix32((uint32_t)seed ^ mix32((uint32_t)(idx >> 32) + (uint32_t)(seed >> 32))));
  return h >= thresh;
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_kernel(const T* x, int xcs, T* y, int ycs, long npix, int C,
                                                      const int64_t* seed, uint32_t thresh, float scale) {
  const uint64_t sd = (uint64_t)seed[0];
  const long total = npix * C;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long pix = i / C;
    const int c = (int)(i - pix * C);
    const float v = to_f(x[pix * xcs + c]);
    y[pix * ycs + c] = from_f<T>(keep_elem(sd, (uint64_t)i, thresh) ? v * scale : 0.f);
  }
}

__global__ void seed_advance_kernel(int64_t* seed) {
  if (threadIdx.x == 0 && blockIdx.x == 0) seed[0] = seed[0] * 6364136223846793005LL + 1442695040888963407LL;
}

}  // namespace adr

using namespace adr;

static int vw_of(int dtype) { return dtype == ADR_BF16 ? 8 : 4; }

#define MONA_DISPATCH(dtype, KERN, grid, smem, ...)                                                  \
  do {                                                                                               \
    if ((dtype) == ADR_BF16) {                                                                       \
      using TT = __bf16;                                                                             \
      hipLaunchKernelGGL((KERN<TT, 8>), grid, dim3(256), smem, st, __VA_ARGS__);                     \
    } else {                                                                                         \
      using TT = float;                                                                              \
      hipLaunchKernelGGL((KERN<TT, 4>), grid, dim3(256), smem, st, __VA_ARGS__);                     \
    }                                                                                                \
  } while (0)

static int rows_chunk(long npix, int* chunks) {
  int rows = 256;
  while ((npix + rows - 1) / rows > 1024) rows *= 2;  // <= 1024 partial rows for the finalize block
  *chunks = (int)((npix + rows - 1) / rows);
  return rows;
}

extern "C" int adr_dyt_fwd(int dtype, const void* x, int xcs, const float* alpha, const float* w, const float* b,
                           void* y, int ycs, long npix, int C, void* stream) {
  const int v = vw_of(dtype);
  ADR_REQUIRE(C % v == 0 && C / v <= 256 && xcs % v == 0 && ycs % v == 0, "dyt_fwd: C=%d / strides", C);
  hipStream_t st = (hipStream_t)stream;
  const long rpb = 256 / (C / v);
  long g = (npix + rpb - 1) / rpb;
  if (g > 65536) g = 65536;
  MONA_DISPATCH(dtype, dyt_fwd_kernel, dim3((unsigned)g), 0, (const TT*)x, xcs, alpha, w, b, (TT*)y, ycs, npix, C);
  return check_launch("adr_dyt_fwd");
}

extern "C" size_t adr_dyt_bwd_workspace(long npix, int C) {
  int chunks;
  rows_chunk(npix, &chunks);
  return (size_t)chunks * 3 * C * sizeof(float);
}

extern "C" int adr_dyt_bwd(int dtype, const void* x, int xcs, const void* dy, int dcs, const float* alpha,
                           const float* w, void* dx, int ocs, float* dalpha, float* dw, float* db, int accumulate,
                           long npix, int C, float* ws, size_t ws_bytes, void* stream) {
  const int v = vw_of(dtype);
  ADR_REQUIRE(C % v == 0 && C / v <= 256 && xcs % v == 0 && dcs % v == 0 && ocs % v == 0, "dyt_bwd: C=%d", C);
  ADR_REQUIRE(ws_bytes >= adr_dyt_bwd_workspace(npix, C), "dyt_bwd: workspace");
  hipStream_t st = (hipStream_t)stream;
  int chunks;
  const int rows = rows_chunk(npix, &chunks);
  MONA_DISPATCH(dtype, dyt_bwd_kernel, dim3(chunks), 0, (const TT*)x, xcs, (const TT*)dy, dcs, alpha, w, (TT*)dx, ocs,
                npix, C, rows, ws);
  hipLaunchKernelGGL(colsum_kernel, dim3(1), dim3(256), 0, st, ws, chunks, 3, C, dw, db, nullptr, nullptr, accumulate,
                     2, dalpha);
  return check_launch("adr_dyt_bwd");
}

template <int VW, int L>
static void ln_fwd_launch(int dtype, dim3 g, hipStream_t st, const void* x, int xcs, const float* lw, const float* lb,
                          const float* gm, const float* gx, void* y, int ycs, float* mean, float* rstd, long npix,
                          float eps) {
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL((ln_mix_fwd_kernel<__bf16, VW, L>), g, dim3(256), 0, st, (const __bf16*)x, xcs, lw, lb, gm, gx,
                       (__bf16*)y, ycs, mean, rstd, npix, eps);
  else
    hipLaunchKernelGGL((ln_mix_fwd_kernel<float, VW, L>), g, dim3(256), 0, st, (const float*)x, xcs, lw, lb, gm, gx,
                       (float*)y, ycs, mean, rstd, npix, eps);
}
template <int VW, int L>
static void ln_bwd_launch(int dtype, dim3 g, hipStream_t st, const void* x, int xcs, const void* dz, int dcs,
                          const float* lw, const float* lb, const float* gm, const float* gx, const float* mean,
                          const float* rstd, void* dx, int ocs, long npix, int rows, float* part) {
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL((ln_mix_bwd_kernel<__bf16, VW, L>), g, dim3(256), 0, st, (const __bf16*)x, xcs,
                       (const __bf16*)dz, dcs, lw, lb, gm, gx, mean, rstd, (__bf16*)dx, ocs, npix, rows, part);
  else
    hipLaunchKernelGGL((ln_mix_bwd_kernel<float, VW, L>), g, dim3(256), 0, st, (const float*)x, xcs, (const float*)dz,
                       dcs, lw, lb, gm, gx, mean, rstd, (float*)dx, ocs, npix, rows, part);
}

// lanes per pixel for C channels: 8 bf16 / 4 fp32 per lane; supported C: 64, 128, 256 (L = 8 / 16 / 32 bf16)
static int ln_lanes(int dtype, int C) { return C / vw_of(dtype); }

extern "C" int adr_ln_mix_fwd(int dtype, const void* x, int xcs, const float* lw, const float* lb, const float* gamma,
                              const float* gammax, void* y, int ycs, float* mean, float* rstd, long npix, int C,
                              float eps, void* stream) {
  const int v = vw_of(dtype), L = ln_lanes(dtype, C);
  ADR_REQUIRE(C % v == 0 && xcs % v == 0 && ycs % v == 0 && (L == 8 || L == 16 || L == 32 || L == 64),
              "ln_mix_fwd: C=%d unsupported", C);
  hipStream_t st = (hipStream_t)stream;
  long g = (npix + 256 / L - 1) / (256 / L);
  if (g > 65536) g = 65536;
  const dim3 grid((unsigned)g);
  if (dtype == ADR_BF16) {
    if (L == 8) ln_fwd_launch<8, 8>(dtype, grid, st, x, xcs, lw, lb, gamma, gammax, y, ycs, mean, rstd, npix, eps);
    else if (L == 16) ln_fwd_launch<8, 16>(dtype, grid, st, x, xcs, lw, lb, gamma, gammax, y, ycs, mean, rstd, npix, eps);
    else if (L == 32) ln_fwd_launch<8, 32>(dtype, grid, st, x, xcs, lw, lb, gamma, gammax, y, ycs, mean, rstd, npix, eps);
    else ln_fwd_launch<8, 64>(dtype, grid, st, x, xcs, lw, lb, gamma, gammax, y, ycs, mean, rstd, npix, eps);
  } else {
    if (L == 8) ln_fwd_launch<4, 8>(dtype, grid, st, x, xcs, lw, lb, gamma, gammax, y, ycs, mean, rstd, npix, eps);
    else if (L == 16) ln_fwd_launch<4, 16>(dtype, grid, st, x, xcs, lw, lb, gamma, gammax, y, ycs, mean, rstd, npix, eps);
    else if (L == 32) ln_fwd_launch<4, 32>(dtype, grid, st, x, xcs, lw, lb, gamma, gammax, y, ycs, mean, rstd, npix, eps);
    else ln_fwd_launch<4, 64>(dtype, grid, st, x, xcs, lw, lb, gamma, gammax, y, ycs, mean, rstd, npix, eps);
  }
  return check_launch("adr_ln_mix_fwd");
}

extern "C" size_t adr_ln_mix_bwd_workspace(long npix, int C) {
  int chunks;
  rows_chunk(npix, &chunks);
  return (size_t)chunks * 4 * C * sizeof(float);
}

extern "C" int adr_ln_mix_bwd(int dtype, const void* x, int xcs, const void* dz, int dcs, const float* lw,
                              const float* lb, const float* gamma, const float* gammax, const float* mean,
                              const float* rstd, void* dx, int ocs, float* dlw, float* dlb, float* dgamma,
                              float* dgammax, int accumulate, long npix, int C, float* ws, size_t ws_bytes,
                              void* stream) {
  const int v = vw_of(dtype), L = ln_lanes(dtype, C);
  ADR_REQUIRE(C % v == 0 && xcs % v == 0 && dcs % v == 0 && ocs % v == 0 && (L == 8 || L == 16 || L == 32 || L == 64),
              "ln_mix_bwd: C=%d unsupported", C);
  ADR_REQUIRE(ws_bytes >= adr_ln_mix_bwd_workspace(npix, C), "ln_mix_bwd: workspace");
  hipStream_t st = (hipStream_t)stream;
  int chunks;
  const int rows = rows_chunk(npix, &chunks);
  const dim3 grid(chunks);
  if (dtype == ADR_BF16) {
    if (L == 8) ln_bwd_launch<8, 8>(dtype, grid, st, x, xcs, dz, dcs, lw, lb, gamma, gammax, mean, rstd, dx, ocs, npix, rows, ws);
    else if (L == 16) ln_bwd_launch<8, 16>(dtype, grid, st, x, xcs, dz, dcs, lw, lb, gamma, gammax, mean, rstd, dx, ocs, npix, rows, ws);
    else if (L == 32) ln_bwd_launch<8, 32>(dtype, grid, st, x, xcs, dz, dcs, lw, lb, gamma, gammax, mean, rstd, dx, ocs, npix, rows, ws);
    else ln_bwd_launch<8, 64>(dtype, grid, st, x, xcs, dz, dcs, lw, lb, gamma, gammax, mean, rstd, dx, ocs, npix, rows, ws);
  } else {
    if (L == 8) ln_bwd_launch<4, 8>(dtype, grid, st, x, xcs, dz, dcs, lw, lb, gamma, gammax, mean, rstd, dx, ocs, npix, rows, ws);
    else if (L == 16) ln_bwd_launch<4, 16>(dtype, grid, st, x, xcs, dz, dcs, lw, lb, gamma, gammax, mean, rstd, dx, ocs, npix, rows, ws);
    else if (L == 32) ln_bwd_launch<4, 32>(dtype, grid, st, x, xcs, dz, dcs, lw, lb, gamma, gammax, mean, rstd, dx, ocs, npix, rows, ws);
    else ln_bwd_launch<4, 64>(dtype, grid, st, x, xcs, dz, dcs, lw, lb, gamma, gammax, mean, rstd, dx, ocs, npix, rows, ws);
  }
  hipLaunchKernelGGL(colsum_kernel, dim3(1), dim3(256), 0, st, ws, chunks, 4, C, dlw, dlb, dgamma, dgammax,
                     accumulate, -1, nullptr);
  return check_launch("adr_ln_mix_bwd");
}

// AttentionTSSA: per-(image, head) statistics workspace (floats): nrm B*H*D, s B*H*N, pi B*H*N, attn B*H*D, z B*H
extern "C" size_t adr_tssa1_state_floats(int B, int N, int H, int D) {
  return (size_t)B * H * (2 * (size_t)D + 2 * (size_t)N + 1);
}

static Tssa1Args tssa1_args(int B, int N, int H, int D, float* state) {
  Tssa1Args a{};
  a.B = B; a.N = N; a.H = H; a.D = D;
  a.nrm = state;
  a.s = a.nrm + (size_t)B * H * D;
  a.pi = a.s + (size_t)B * H * N;
  a.attn = a.pi + (size_t)B * H * N;
  a.z = a.attn + (size_t)B * H * D;
  return a;
}

#define TSSA1_LAUNCH(KERN, smem)                                                                  \
  do {                                                                                            \
    if (dtype == ADR_BF16) hipLaunchKernelGGL((KERN<__bf16, 8, 8>), grid, dim3(256), smem, st, a); \
    else hipLaunchKernelGGL((KERN<float, 4, 16>), grid, dim3(256), smem, st, a);                  \
  } while (0)

extern "C" int adr_tssa1_fwd(int dtype, const void* w, int cs, int B, int N, int H, int D, const float* temp,
                             void* out, int ocs, float* state, void* stream) {
  ADR_REQUIRE(D == 64 && cs % vw_of(dtype) == 0 && ocs % vw_of(dtype) == 0 && N > 0 && H > 0,
              "tssa1_fwd: head dim %d (64 supported) / strides", D);
  hipStream_t st = (hipStream_t)stream;
  Tssa1Args a = tssa1_args(B, N, H, D, state);
  a.w = w; a.cs = cs; a.temp = temp; a.out = out; a.ocs = ocs;
  const dim3 grid(B, H);
  TSSA1_LAUNCH(tssa1_stats_kernel, 0);
  TSSA1_LAUNCH(tssa1_fwd_kernel, 0);
  return check_launch("adr_tssa1_fwd");
}

extern "C" size_t adr_tssa1_bwd_workspace(int B, int N, int H, int D) {
  return ((size_t)B * H * ((size_t)D + N + 1)) * sizeof(float);
}

extern "C" int adr_tssa1_bwd(int dtype, const void* w, int cs, int B, int N, int H, int D, const float* temp,
                             const float* state, const void* g, int gcs, void* dw, int dwcs, float* dtemp,
                             int accumulate, float* ws, size_t ws_bytes, void* stream) {
  ADR_REQUIRE(D == 64 && cs % vw_of(dtype) == 0 && gcs % vw_of(dtype) == 0 && dwcs % vw_of(dtype) == 0,
              "tssa1_bwd: head dim %d / strides", D);
  ADR_REQUIRE(ws_bytes >= adr_tssa1_bwd_workspace(B, N, H, D), "tssa1_bwd: workspace");
  ADR_REQUIRE((size_t)N * sizeof(float) <= 64 * 1024, "tssa1_bwd: %d tokens exceed the LDS plan", N);
  hipStream_t st = (hipStream_t)stream;
  Tssa1Args a = tssa1_args(B, N, H, D, const_cast<float*>(state));
  a.w = w; a.cs = cs; a.temp = temp; a.g = g; a.gcs = gcs; a.dw = dw; a.dwcs = dwcs;
  a.ddots = ws;
  a.dpi = ws + (size_t)B * H * D;
  a.dtemp = a.dpi + (size_t)B * H * N;
  const dim3 grid(B, H);
  TSSA1_LAUNCH(tssa1_bwd1_kernel, 0);
  TSSA1_LAUNCH(tssa1_bwd2_kernel, (size_t)N * sizeof(float));
  // dtemp[h] (+)= sum_b partial[b][h]
  hipLaunchKernelGGL(colsum_kernel, dim3(1), dim3(256), 0, st, a.dtemp, B, 1, H, dtemp, nullptr, nullptr, nullptr,
                     accumulate, -1, nullptr);
  return check_launch("adr_tssa1_bwd");
}

extern "C" int adr_dropout(int dtype, const void* x, int xcs, void* y, int ycs, long npix, int C, float p,
                           const int64_t* seed, void* stream) {
  ADR_REQUIRE(p >= 0.f && p < 1.f, "dropout: p=%f", (double)p);
  hipStream_t st = (hipStream_t)stream;
  const uint32_t thresh = (uint32_t)((double)p * 4294967296.0);
  const float scale = 1.f / (1.f - p);
  long g = (npix * C + 255) / 256;
  if (g > 65536) g = 65536;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(dropout_kernel<__bf16>, dim3((unsigned)g), dim3(256), 0, st, (const __bf16*)x, xcs, (__bf16*)y,
                       ycs, npix, C, seed, thresh, scale);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3((unsigned)g), dim3(256), 0, st, (const float*)x, xcs, (float*)y, ycs,
                       npix, C, seed, thresh, scale);
  return check_launch("adr_dropout");
}

extern "C" int adr_seed_advance(int64_t* seed, void* stream) {
  hipLaunchKernelGGL(seed_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, seed);
  return check_launch("adr_seed_advance");
}
