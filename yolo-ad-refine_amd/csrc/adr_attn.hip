// Flash attention (forward + backward) for the cross-scale nn.MultiheadAttention of C2PTSSA
// (reference nn/modules/block.py:2432 and :2484: self-attention over the 3*H*W stacked scale tokens,
// head_dim 64, softmax(q k^T / sqrt(64)) v, no masking, no dropout).
//
// Layout: q, k, v, o are token rows [b*L + l] with a channel stride (cs) — e.g. the packed in_proj output
// (B*L, 3E) — and head h occupies channels [h*64, h*64+64). One workgroup = 4 waves = 64 queries (forward,
// dQ) or 64 keys (dK/dV) of one (image, head); each wave owns 16 of them.
//
// MFMA mapping (16x16 tiles, bf16 v_mfma_f32_16x16x32_bf16 or exact-fp32 v_mfma_f32_16x16x4_f32):
//   "NT" products C[i][j] = sum_d A[i][d] B[j][d] read both operands as contiguous LDS rows.
//   Products that reduce over an index that sits in the C/D layout's row position (row = 4*(lane>>4)+r)
//   consume the accumulator registers directly as the B operand with a matching permutation of the
//   reduction index on the A side (bf16: k-set {4g..4g+3, 16+4g..16+4g+3} per 32-step; f32: key 4g+s per
//   4-step) — no LDS round trip for P / dS.
// The forward stores the per-query log-sum-exp; the backward recomputes P (two kernels: dK/dV keyed by
// key block, dQ keyed by query block), so there are no atomics and results are deterministic.
#include "adr_common.h"

namespace adr {

static constexpr int HD = 64;      // head dim
static constexpr int BLK = 64;     // queries or keys per workgroup
static constexpr int LDT = HD + 8; // LDS row stride (elements)

template <typename T>
__device__ __forceinline__ void load_rows(T* dst, const T* src, long row0, int L, int cs, int coff) {
  // 64 rows x 64 elems -> LDS [64][LDT]; rows >= L zero-filled
  constexpr int V = 16 / sizeof(T);
  for (int i = threadIdx.x; i < BLK * (HD / V); i += 256) {
    int r = i / (HD / V), c = (i % (HD / V)) * V;
    long row = row0 + r;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < L) v = ld16(src + row * cs + coff + c);
    st16(dst + r * LDT + c, v);
  }
}

// C[i][j] += sum_d A[i][d] * B[j][d] for i in [ai, ai+16), j in [bj, bj+16)
template <typename T>
__device__ __forceinline__ f32x4 nt_tile(const T* As, int ai, const T* Bs, int bj, f32x4 acc) {
  const int lane = threadIdx.x & 63;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int ds = 0; ds < HD / 32; ++ds) {
      bf16x8 a = *reinterpret_cast<const bf16x8*>(As + (ai + (lane & 15)) * LDT + ds * 32 + 8 * (lane >> 4));
      bf16x8 b = *reinterpret_cast<const bf16x8*>(Bs + (bj + (lane & 15)) * LDT + ds * 32 + 8 * (lane >> 4));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < HD / 4; ++s) {
      float a = As[(ai + (lane & 15)) * LDT + 4 * s + (lane >> 4)];
      float b = Bs[(bj + (lane & 15)) * LDT + 4 * s + (lane >> 4)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
  }
  return acc;
}

// acc[dt] (C rows d = dt*16 + 4g + r, cols j) += sum_k X[k][d] * Pt[k][j], where Pt (64 x 16) lives in the
// C-layout registers p[kt][r] (row k = kt*16 + 4g + r, col j = lane&15) and X is an LDS [k][d] tile.
template <typename T>
__device__ __forceinline__ void tn_reg(const T* Xs, const float (&p)[4][4], f32x4 (&acc)[4]) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 b;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        b[j] = (__bf16)p[2 * ks][j];
        b[4 + j] = (__bf16)p[2 * ks + 1][j];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = Xs[(ks * 32 + 4 * g + j) * LDT + dt * 16 + c];
          a[4 + j] = Xs[(ks * 32 + 16 + 4 * g + j) * LDT + dt * 16 + c];
        }
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[dt], 0, 0, 0);
      }
    }
  } else {
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        float b = p[kt][s];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          float a = Xs[(kt * 16 + 4 * g + s) * LDT + dt * 16 + c];
          acc[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[dt], 0, 0, 0);
        }
      }
  }
}

// ---------------- forward ----------------
template <typename T>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const T* q, const T* k, const T* v, int cs, int qo, int ko,
                                                       int vo, T* o, int ocs, int L, int heads, float scale,
                                                       float* lse) {
  __shared__ __attribute__((aligned(16))) T Qs[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Ks[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Vs[BLK * LDT];
  const int nqb = (L + BLK - 1) / BLK;
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int b = bh / heads, h = bh % heads;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const long rowb = (long)b * L;
  const int q0 = qb * BLK;
  load_rows(Qs, q, rowb + q0, L - q0, cs, qo + h * HD);
  float m = -INFINITY, lsum = 0.f;
  f32x4 oacc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) oacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const float sl2 = scale * 1.44269504088896341f;  // exp2 domain
  for (int k0 = 0; k0 < L; k0 += BLK) {
    __syncthreads();
    load_rows(Ks, k, rowb + k0, L - k0, cs, ko + h * HD);
    load_rows(Vs, v, rowb + k0, L - k0, cs, vo + h * HD);
    __syncthreads();
    float p[4][4];
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 s = nt_tile(Ks, kt * 16, Qs, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = k0 + kt * 16 + 4 * g + r;
        float val = key < L ? s[r] * sl2 : -INFINITY;
        p[kt][r] = val;
        mx = fmaxf(mx, val);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float mnew = fmaxf(m, mx);
    float alpha = exp2f(m - mnew);
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float e = exp2f(p[kt][r] - mnew);
        p[kt][r] = e;
        rs += e;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    lsum = lsum * alpha + rs;
    m = mnew;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) oacc[dt] = oacc[dt] * alpha;
    tn_reg(Vs, p, oacc);  // O^T[d][q] += V^T P^T
  }
  const int qq = q0 + wave * 16 + c;
  if (qq < L) {
    float inv = 1.f / lsum;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + 4 * g + r;
        o[(rowb + qq) * ocs + h * HD + d] = from_f<T>(oacc[dt][r] * inv);
      }
    if (g == 0) lse[(long)bh * L + qq] = (m + log2f(lsum)) * 0.69314718055994531f;  // natural-log LSE of scaled logits
  }
}

// Dvec[bh][q] = sum_d dO * O
template <typename T>
__global__ void __launch_bounds__(256) attn_dvec_kernel(const T* o, int ocs, const T* dout, int dcs, int L, int heads,
                                                        long total, float* dvec) {
  long i = (long)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  int lane = threadIdx.x & 63;
  if (i >= total) return;
  int l = (int)(i % L);
  long bh = i / L;
  long b = bh / heads;
  int h = (int)(bh % heads);
  long row = b * L + l;
  float s = to_f(o[row * ocs + h * HD + lane]) * to_f(dout[row * dcs + h * HD + lane]);
  s = wave_sum(s);
  if (lane == 0) dvec[i] = s;
}

// ---------------- backward: dK, dV (one workgroup per 64 keys) ----------------
template <typename T>
__global__ void __launch_bounds__(256) attn_bwd_kv_kernel(const T* q, const T* k, const T* v, int cs, int qo, int ko,
                                                          int vo, const T* dout, int dcs, const float* lse,
                                                          const float* dvec, int L, int heads, float scale, T* dq_unused,
                                                          T* dk, T* dv, int gcs, int gko, int gvo) {
  __shared__ __attribute__((aligned(16))) T Ks[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Vs[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Qs[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Ds[BLK * LDT];
  __shared__ float ls[BLK], dd[BLK];
  const int nkb = (L + BLK - 1) / BLK;
  const int kb = blockIdx.x % nkb;
  const int bh = blockIdx.x / nkb;
  const int b = bh / heads, h = bh % heads;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const long rowb = (long)b * L;
  const int k0 = kb * BLK;
  load_rows(Ks, k, rowb + k0, L - k0, cs, ko + h * HD);
  load_rows(Vs, v, rowb + k0, L - k0, cs, vo + h * HD);
  f32x4 dka[4], dva[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dka[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    dva[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  for (int q0 = 0; q0 < L; q0 += BLK) {
    __syncthreads();
    load_rows(Qs, q, rowb + q0, L - q0, cs, qo + h * HD);
    load_rows(Ds, dout, rowb + q0, L - q0, dcs, h * HD);
    for (int i = threadIdx.x; i < BLK; i += 256) {
      int qq = q0 + i;
      ls[i] = qq < L ? lse[(long)bh * L + qq] : INFINITY;
      dd[i] = qq < L ? dvec[(long)bh * L + qq] : 0.f;
    }
    __syncthreads();
    float p[4][4], ds[4][4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      // S[q][key], rows q = qt*16 + 4g + r, cols key = wave*16 + c
      f32x4 s = nt_tile(Qs, qt * 16, Ks, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
      f32x4 dp = nt_tile(Ds, qt * 16, Vs, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int qi = qt * 16 + 4 * g + r;
        float pv = __expf(s[r] * scale - ls[qi]);  // 0 for padded queries (ls = +inf)
        p[qt][r] = pv;
        ds[qt][r] = pv * (dp[r] - dd[qi]);
      }
    }
    tn_reg(Ds, p, dva);   // dV^T[d][key] += dO^T P
    tn_reg(Qs, ds, dka);  // dK^T[d][key] += Q^T dS
  }
  const int kk = k0 + wave * 16 + c;
  if (kk < L) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + 4 * g + r;
        dk[(rowb + kk) * gcs + gko + h * HD + d] = from_f<T>(dka[dt][r] * scale);
        dv[(rowb + kk) * gcs + gvo + h * HD + d] = from_f<T>(dva[dt][r]);
      }
  }
}

// ---------------- backward: dQ (one workgroup per 64 queries) ----------------
template <typename T>
__global__ void __launch_bounds__(256) attn_bwd_q_kernel(const T* q, const T* k, const T* v, int cs, int qo, int ko,
                                                         int vo, const T* dout, int dcs, const float* lse,
                                                         const float* dvec, int L, int heads, float scale, T* dq,
                                                         int gcs, int gqo) {
  __shared__ __attribute__((aligned(16))) T Qs[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Ds[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Ks[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Vs[BLK * LDT];
  const int nqb = (L + BLK - 1) / BLK;
  const int qb = blockIdx.x % nqb;
  const int bh = blockIdx.x / nqb;
  const int b = bh / heads, h = bh % heads;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const long rowb = (long)b * L;
  const int q0 = qb * BLK;
  load_rows(Qs, q, rowb + q0, L - q0, cs, qo + h * HD);
  load_rows(Ds, dout, rowb + q0, L - q0, dcs, h * HD);
  const int qq = q0 + wave * 16 + c;
  const float lq = qq < L ? lse[(long)bh * L + qq] : INFINITY;
  const float dq_d = qq < L ? dvec[(long)bh * L + qq] : 0.f;
  f32x4 dqa[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dqa[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < L; k0 += BLK) {
    __syncthreads();
    load_rows(Ks, k, rowb + k0, L - k0, cs, ko + h * HD);
    load_rows(Vs, v, rowb + k0, L - k0, cs, vo + h * HD);
    __syncthreads();
    float ds[4][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      // S^T[key][q], rows key = kt*16 + 4g + r, cols q = wave*16 + c
      f32x4 s = nt_tile(Ks, kt * 16, Qs, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
      f32x4 dp = nt_tile(Vs, kt * 16, Ds, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = k0 + kt * 16 + 4 * g + r;
        float pv = key < L ? __expf(s[r] * scale - lq) : 0.f;
        ds[kt][r] = pv * (dp[r] - dq_d);
      }
    }
    tn_reg(Ks, ds, dqa);  // dQ^T[d][q] += K^T dS^T
  }
  if (qq < L) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + 4 * g + r;
        dq[(rowb + qq) * gcs + gqo + h * HD + d] = from_f<T>(dqa[dt][r] * scale);
      }
  }
}

}  // namespace adr

using namespace adr;

extern "C" int adr_attn_fwd(int dtype, const void* q, const void* k, const void* v, int cs, int qo, int ko, int vo,
                            void* o, int ocs, int B, int L, int heads, int head_dim, float scale, float* lse,
                            void* stream) {
  ADR_REQUIRE(head_dim == HD, "attn: head_dim must be 64 (got %d)", head_dim);
  int vec = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(cs % vec == 0 && ocs % vec == 0 && qo % vec == 0 && ko % vec == 0 && vo % vec == 0, "attn: views");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(B * heads * cdiv(L, BLK));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(attn_fwd_kernel<__bf16>, grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                       (const __bf16*)v, cs, qo, ko, vo, (__bf16*)o, ocs, L, heads, scale, lse);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<float>, grid, dim3(256), 0, st, (const float*)q, (const float*)k,
                       (const float*)v, cs, qo, ko, vo, (float*)o, ocs, L, heads, scale, lse);
  return check_launch("adr_attn_fwd");
}

extern "C" int adr_attn_bwd(int dtype, const void* q, const void* k, const void* v, int cs, int qo, int ko, int vo,
                            const void* o, int ocs, const void* dout, int dcs, const float* lse, void* dq, void* dk,
                            void* dv, int gcs, int gqo, int gko, int gvo, int B, int L, int heads, int head_dim,
                            float scale, float* dvec_ws, void* stream) {
  ADR_REQUIRE(head_dim == HD, "attn: head_dim must be 64");
  hipStream_t st = (hipStream_t)stream;
  long total = (long)B * heads * L;
  dim3 g1(cdiv(total, 4));
  dim3 grid(B * heads * cdiv(L, BLK));
  if (dtype == ADR_BF16) {
    hipLaunchKernelGGL(attn_dvec_kernel<__bf16>, g1, dim3(256), 0, st, (const __bf16*)o, ocs, (const __bf16*)dout, dcs,
                       L, heads, total, dvec_ws);
    hipLaunchKernelGGL(attn_bwd_kv_kernel<__bf16>, grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                       (const __bf16*)v, cs, qo, ko, vo, (const __bf16*)dout, dcs, lse, dvec_ws, L, heads, scale,
                       (__bf16*)nullptr, (__bf16*)dk, (__bf16*)dv, gcs, gko, gvo);
    hipLaunchKernelGGL(attn_bwd_q_kernel<__bf16>, grid, dim3(256), 0, st, (const __bf16*)q, (const __bf16*)k,
                       (const __bf16*)v, cs, qo, ko, vo, (const __bf16*)dout, dcs, lse, dvec_ws, L, heads, scale,
                       (__bf16*)dq, gcs, gqo);
  } else {
    hipLaunchKernelGGL(attn_dvec_kernel<float>, g1, dim3(256), 0, st, (const float*)o, ocs, (const float*)dout, dcs, L,
                       heads, total, dvec_ws);
    hipLaunchKernelGGL(attn_bwd_kv_kernel<float>, grid, dim3(256), 0, st, (const float*)q, (const float*)k,
                       (const float*)v, cs, qo, ko, vo, (const float*)dout, dcs, lse, dvec_ws, L, heads, scale,
                       (float*)nullptr, (float*)dk, (float*)dv, gcs, gko, gvo);
    hipLaunchKernelGGL(attn_bwd_q_kernel<float>, grid, dim3(256), 0, st, (const float*)q, (const float*)k,
                       (const float*)v, cs, qo, ko, vo, (const float*)dout, dcs, lse, dvec_ws, L, heads, scale,
                       (float*)dq, gcs, gqo);
  }
  return check_launch("adr_attn_bwd");
}
