// Flash attention (forward + backward), no masking, no dropout, for two reference modules:
//   * the cross-scale nn.MultiheadAttention of C2PTSSA (reference nn/modules/block.py:2432 and :2484:
//     self-attention over the 3*H*W stacked scale tokens, q/k/v head_dim 64);
//   * Attention of C2PSA / PSABlock (block.py:874-927, yolo11): per head q and k of key_dim 32, v of
//     head_dim 64, interleaved per head as [q(32) k(32) v(64)] in the qkv conv output.
//
// Layout: q, k, v, o are token rows [b*L + l] with a channel stride (cs) — e.g. the packed in_proj output
// (B*L, 3E) or the NHWC qkv activation — and head h's q / k / v start at channel qo / ko / vo + h*hs (hs =
// the head stride: 64 for MHA's planar [q|k|v], 128 for PSA's interleaved heads). o and dO hold head h at
// channels [h*64, h*64+64). DQK (32 or 64) is the q/k width. One workgroup = 4 waves = 64 queries (forward,
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
#include <initializer_list>

namespace adr {

static constexpr int HD = 64;      // head dim
static constexpr int BLK = 64;     // queries or keys per workgroup
static constexpr int LDT = HD + 16;  // LDS row stride (elements): 160 bytes, an odd multiple of 32 (conflict-free
                                     // transposing reads)

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

template <typename T, int D = HD>
__device__ __forceinline__ void load_rows(T* dst, const T* src, long row0, int L, int cs, int coff) {
  // 64 rows x D elems -> LDS [64][LDT]; rows >= L zero-filled
  constexpr int V = 16 / sizeof(T);
  for (int i = threadIdx.x; i < BLK * (D / V); i += 256) {
    int r = i / (D / V), c = (i % (D / V)) * V;
    long row = row0 + r;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < L) v = ld16(src + row * cs + coff + c);
    st16(dst + r * LDT + c, v);
  }
}

// 2^x: the bare v_exp_f32 for bf16 (the softmax exponentials were most of the kernels' VALU work: ~20 VALU
// instructions per MFMA with the range-checked exp2f); exp2f in the fp32 parity mode
template <typename T>
__device__ __forceinline__ float fexp2(float x) {
  if constexpr (sizeof(T) == 2) return __builtin_amdgcn_exp2f(x);
  else return exp2f(x);
}
constexpr float LOG2E = 1.44269504088896341f;

// Register prefetch of one 64-row x D tile: load() issues the global reads of the next tile before the current
// one is consumed; store() writes them to LDS after the consumers' barrier (rows >= nrows are zero).
template <typename T, int D>
struct TilePrefetch {
  static constexpr int V = 16 / sizeof(T), CPR = D / V, CH = BLK * CPR, PER = (CH + 255) / 256;
  u32x4 r[PER];
  __device__ __forceinline__ void load(const T* src, long row0, int nrows, int cs, int coff) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + 256 * i, rr = idx / CPR, cc = (idx % CPR) * V;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (idx < CH && rr < nrows) v = ld16(src + (row0 + rr) * cs + coff + cc);
      r[i] = v;
    }
  }
  __device__ __forceinline__ void store(T* dst) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + 256 * i, rr = idx / CPR, cc = (idx % CPR) * V;
      if (idx < CH) st16(dst + rr * LDT + cc, r[i]);
    }
  }
};

// C[i][j] += sum_{d<D} A[i][d] * B[j][d] for i in [ai, ai+16), j in [bj, bj+16)
template <typename T, int D>
__device__ __forceinline__ f32x4 nt_tile(const T* As, int ai, const T* Bs, int bj, f32x4 acc) {
  const int lane = threadIdx.x & 63;
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int ds = 0; ds < D / 32; ++ds) {
      bf16x8 a = *reinterpret_cast<const bf16x8*>(As + (ai + (lane & 15)) * LDT + ds * 32 + 8 * (lane >> 4));
      bf16x8 b = *reinterpret_cast<const bf16x8*>(Bs + (bj + (lane & 15)) * LDT + ds * 32 + 8 * (lane >> 4));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < D / 4; ++s) {
      float a = As[(ai + (lane & 15)) * LDT + 4 * s + (lane >> 4)];
      float b = Bs[(bj + (lane & 15)) * LDT + 4 * s + (lane >> 4)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
  }
  return acc;
}

// acc[dt] (C rows d = dt*16 + 4g + r, cols j) += sum_k X[k][d] * Pt[k][j], where Pt (64 x 16) lives in the
// C-layout registers p[kt][r] (row k = kt*16 + 4g + r, col j = lane&15) and X is an LDS [k][d] tile, d < 16*DT.
template <typename T, int DT>
__device__ __forceinline__ void tn_reg(const T* Xs, const float (&p)[4][4], f32x4 (&acc)[DT]) {
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  if constexpr (sizeof(T) == 2) {
    // A = X^T: the reduction index k runs over LDS rows, so each fragment is two transposing LDS reads
    // (ds_read_b64_tr_b16) whose row sets {4g..4g+3} and {16+4g..16+4g+3} are exactly the k slots that the P
    // registers hold — no scalar gathers
    const int q4 = (lane >> 2) & 3, p4 = lane & 3;
    (void)c;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 b;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        b[j] = (__bf16)p[2 * ks][j];
        b[4 + j] = (__bf16)p[2 * ks + 1][j];
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const T* base = Xs + (ks * 32 + 4 * g + q4) * LDT + dt * 16 + 4 * p4;
        v4s both[2] = {__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base)),
                       __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + 16 * LDT))};
        const bf16x8 a = *reinterpret_cast<bf16x8*>(both);
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
        for (int dt = 0; dt < DT; ++dt) {
          float a = Xs[(kt * 16 + 4 * g + s) * LDT + dt * 16 + c];
          acc[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[dt], 0, 0, 0);
        }
      }
  }
}

// ---------------- forward ----------------
template <typename T, int DQK>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const T* q, const T* k, const T* v, int cs, int qo, int ko,
                                                       int vo, int hs, T* o, int ocs, int L, int heads, float scale,
                                                       float* lse) {
  __shared__ __attribute__((aligned(16))) T Qs[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Ks[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Vs[BLK * LDT];
  const int nqb = (L + BLK - 1) / BLK;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // the blocks of one (image, head) share an XCD's L2 (K / V)
  const int qb = bid % nqb;
  const int bh = bid / nqb;
  const int b = bh / heads, h = bh % heads;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const long rowb = (long)b * L;
  const int q0 = qb * BLK;
  load_rows<T, DQK>(Qs, q, rowb + q0, L - q0, cs, qo + h * hs);
  float m = -INFINITY, lsum = 0.f;
  f32x4 oacc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) oacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const float sl2 = scale * 1.44269504088896341f;  // exp2 domain
  TilePrefetch<T, DQK> pk;
  TilePrefetch<T, HD> pv;
  pk.load(k, rowb, L, cs, ko + h * hs);
  pv.load(v, rowb, L, cs, vo + h * hs);
  for (int k0 = 0; k0 < L; k0 += BLK) {
    __syncthreads();
    pk.store(Ks);
    pv.store(Vs);
    __syncthreads();
    if (k0 + BLK < L) {  // next key block in flight while this one is consumed
      pk.load(k, rowb + k0 + BLK, L - k0 - BLK, cs, ko + h * hs);
      pv.load(v, rowb + k0 + BLK, L - k0 - BLK, cs, vo + h * hs);
    }
    float p[4][4];
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 s = nt_tile<T, DQK>(Ks, kt * 16, Qs, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
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
    float alpha = fexp2<T>(m - mnew);
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float e = fexp2<T>(p[kt][r] - mnew);
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

// Dvec[bh][q] = sum_d dO * O: 64 / VW threads per (row, head), one 16-byte load of each operand per thread and an
// xor reduction over those lanes (was a wave per row with 2-byte loads: 32 us at bs 64, L 1200, 2 heads)
template <typename T>
__global__ void __launch_bounds__(256) attn_dvec_kernel(const T* o, int ocs, const T* dout, int dcs, int L, int heads,
                                                        long total, float* dvec) {
  constexpr int VW = 16 / sizeof(T), TPR = HD / VW, RPB = 256 / TPR;
  const long i = (long)blockIdx.x * RPB + threadIdx.x / TPR;
  const int j = threadIdx.x % TPR;
  float s = 0.f;
  if (i < total) {
    const int l = (int)(i % L);
    const long bh = i / L, b = bh / heads;
    const int h = (int)(bh % heads);
    const long row = b * L + l;
    const u32x4 ov = ld16(o + row * ocs + h * HD + j * VW), dv = ld16(dout + row * dcs + h * HD + j * VW);
    const T* oe = reinterpret_cast<const T*>(&ov);
    const T* de = reinterpret_cast<const T*>(&dv);
#pragma unroll
    for (int e = 0; e < VW; ++e) s += to_f(oe[e]) * to_f(de[e]);
  }
#pragma unroll
  for (int off = TPR / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (i < total && j == 0) dvec[i] = s;
}

// ---------------- backward: dK, dV (one workgroup per 64 keys) ----------------
template <typename T, int DQK>
__global__ void __launch_bounds__(256) attn_bwd_kv_kernel(const T* q, const T* k, const T* v, int cs, int qo, int ko,
                                                          int vo, int hs, const T* dout, int dcs, const float* lse,
                                                          const float* dvec, int L, int heads, float scale, T* dq_unused,
                                                          T* dk, T* dv, int gcs, int gko, int gvo) {
  __shared__ __attribute__((aligned(16))) T Ks[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Vs[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Qs[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Ds[BLK * LDT];
  __shared__ float ls[BLK], dd[BLK];
  const int nkb = (L + BLK - 1) / BLK;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // the blocks of one (image, head) share an XCD's L2 (Q / dO)
  const int kb = bid % nkb;
  const int bh = bid / nkb;
  const int b = bh / heads, h = bh % heads;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const long rowb = (long)b * L;
  const int k0 = kb * BLK;
  constexpr int KT = DQK / 16;
  load_rows<T, DQK>(Ks, k, rowb + k0, L - k0, cs, ko + h * hs);
  load_rows(Vs, v, rowb + k0, L - k0, cs, vo + h * hs);
  f32x4 dka[KT], dva[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dva[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < KT; ++i) dka[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  TilePrefetch<T, DQK> pq;
  TilePrefetch<T, HD> pd;
  float nls = INFINITY, ndd = 0.f;  // thread i < 64: the next query block's lse / dvec entry i
  auto fetch = [&](int qn) {
    pq.load(q, rowb + qn, L - qn, cs, qo + h * hs);
    pd.load(dout, rowb + qn, L - qn, dcs, h * HD);
    if (threadIdx.x < BLK) {
      const int qq = qn + threadIdx.x;
      nls = qq < L ? lse[(long)bh * L + qq] : INFINITY;
      ndd = qq < L ? dvec[(long)bh * L + qq] : 0.f;
    }
  };
  fetch(0);
  for (int q0 = 0; q0 < L; q0 += BLK) {
    __syncthreads();
    pq.store(Qs);
    pd.store(Ds);
    if (threadIdx.x < BLK) {
      ls[threadIdx.x] = nls;
      dd[threadIdx.x] = ndd;
    }
    __syncthreads();
    if (q0 + BLK < L) fetch(q0 + BLK);
    float p[4][4], ds[4][4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      // S[q][key], rows q = qt*16 + 4g + r, cols key = wave*16 + c
      f32x4 s = nt_tile<T, DQK>(Qs, qt * 16, Ks, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
      f32x4 dp = nt_tile<T, HD>(Ds, qt * 16, Vs, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int qi = qt * 16 + 4 * g + r;
        float pv = fexp2<T>((s[r] * scale - ls[qi]) * LOG2E);  // 0 for padded queries (ls = +inf)
        p[qt][r] = pv;
        ds[qt][r] = pv * (dp[r] - dd[qi]);
      }
    }
    tn_reg<T, 4>(Ds, p, dva);    // dV^T[d][key] += dO^T P
    tn_reg<T, KT>(Qs, ds, dka);  // dK^T[d][key] += Q^T dS
  }
  const int kk = k0 + wave * 16 + c;
  if (kk < L) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + 4 * g + r;
        dv[(rowb + kk) * gcs + gvo + h * hs + d] = from_f<T>(dva[dt][r]);
      }
#pragma unroll
    for (int dt = 0; dt < KT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + 4 * g + r;
        dk[(rowb + kk) * gcs + gko + h * hs + d] = from_f<T>(dka[dt][r] * scale);
      }
  }
}

// ---------------- backward: dQ (one workgroup per 64 queries) ----------------
template <typename T, int DQK>
__global__ void __launch_bounds__(256) attn_bwd_q_kernel(const T* q, const T* k, const T* v, int cs, int qo, int ko,
                                                         int vo, int hs, const T* dout, int dcs, const float* lse,
                                                         const float* dvec, int L, int heads, float scale, T* dq,
                                                         int gcs, int gqo) {
  __shared__ __attribute__((aligned(16))) T Qs[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Ds[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Ks[BLK * LDT];
  __shared__ __attribute__((aligned(16))) T Vs[BLK * LDT];
  const int nqb = (L + BLK - 1) / BLK;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // the blocks of one (image, head) share an XCD's L2 (K / V)
  const int qb = bid % nqb;
  const int bh = bid / nqb;
  const int b = bh / heads, h = bh % heads;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const long rowb = (long)b * L;
  const int q0 = qb * BLK;
  constexpr int KT = DQK / 16;
  load_rows<T, DQK>(Qs, q, rowb + q0, L - q0, cs, qo + h * hs);
  load_rows(Ds, dout, rowb + q0, L - q0, dcs, h * HD);
  const int qq = q0 + wave * 16 + c;
  const float lq = qq < L ? lse[(long)bh * L + qq] : INFINITY;
  const float dq_d = qq < L ? dvec[(long)bh * L + qq] : 0.f;
  f32x4 dqa[KT];
#pragma unroll
  for (int i = 0; i < KT; ++i) dqa[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  TilePrefetch<T, DQK> pk;
  TilePrefetch<T, HD> pv;
  pk.load(k, rowb, L, cs, ko + h * hs);
  pv.load(v, rowb, L, cs, vo + h * hs);
  for (int k0 = 0; k0 < L; k0 += BLK) {
    __syncthreads();
    pk.store(Ks);
    pv.store(Vs);
    __syncthreads();
    if (k0 + BLK < L) {
      pk.load(k, rowb + k0 + BLK, L - k0 - BLK, cs, ko + h * hs);
      pv.load(v, rowb + k0 + BLK, L - k0 - BLK, cs, vo + h * hs);
    }
    float ds[4][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      // S^T[key][q], rows key = kt*16 + 4g + r, cols q = wave*16 + c
      f32x4 s = nt_tile<T, DQK>(Ks, kt * 16, Qs, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
      f32x4 dp = nt_tile<T, HD>(Vs, kt * 16, Ds, wave * 16, (f32x4){0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = k0 + kt * 16 + 4 * g + r;
        float pv = key < L ? fexp2<T>((s[r] * scale - lq) * LOG2E) : 0.f;
        ds[kt][r] = pv * (dp[r] - dq_d);
      }
    }
    tn_reg<T, KT>(Ks, ds, dqa);  // dQ^T[d][q] += K^T dS^T
  }
  if (qq < L) {
#pragma unroll
    for (int dt = 0; dt < KT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + 4 * g + r;
        dq[(rowb + qq) * gcs + gqo + h * hs + d] = from_f<T>(dqa[dt][r] * scale);
      }
  }
}

}  // namespace adr

using namespace adr;

template <typename T, int DQK>
static void attn_fwd_launch(const void* q, const void* k, const void* v, int cs, int qo, int ko, int vo, int hs, void* o,
                            int ocs, int B, int L, int heads, float scale, float* lse, hipStream_t st) {
  dim3 grid(B * heads * cdiv(L, BLK));
  hipLaunchKernelGGL((attn_fwd_kernel<T, DQK>), grid, dim3(256), 0, st, (const T*)q, (const T*)k, (const T*)v, cs, qo,
                     ko, vo, hs, (T*)o, ocs, L, heads, scale, lse);
}

template <typename T, int DQK>
static void attn_bwd_launch(const void* q, const void* k, const void* v, int cs, int qo, int ko, int vo, int hs,
                            const void* o, int ocs, const void* dout, int dcs, const float* lse, void* dq, void* dk,
                            void* dv, int gcs, int gqo, int gko, int gvo, int B, int L, int heads, float scale,
                            float* dvec, hipStream_t st) {
  long total = (long)B * heads * L;
  dim3 grid(B * heads * cdiv(L, BLK));
  hipLaunchKernelGGL((attn_dvec_kernel<T>), dim3(cdiv(total, 256 / (HD / (16 / (int)sizeof(T))))), dim3(256), 0, st,
                     (const T*)o, ocs, (const T*)dout, dcs, L, heads, total, dvec);
  hipLaunchKernelGGL((attn_bwd_kv_kernel<T, DQK>), grid, dim3(256), 0, st, (const T*)q, (const T*)k, (const T*)v, cs,
                     qo, ko, vo, hs, (const T*)dout, dcs, lse, dvec, L, heads, scale, (T*)nullptr, (T*)dk, (T*)dv, gcs,
                     gko, gvo);
  hipLaunchKernelGGL((attn_bwd_q_kernel<T, DQK>), grid, dim3(256), 0, st, (const T*)q, (const T*)k, (const T*)v, cs,
                     qo, ko, vo, hs, (const T*)dout, dcs, lse, dvec, L, heads, scale, (T*)dq, gcs, gqo);
}

static bool attn_views_ok(int dtype, std::initializer_list<int> offs) {
  const int vec = dtype == ADR_BF16 ? 8 : 4;
  for (int x : offs)
    if (x % vec) return false;
  return true;
}

extern "C" int adr_attn_fwd(int dtype, const void* q, const void* k, const void* v, int cs, int qo, int ko, int vo,
                            int hs, void* o, int ocs, int B, int L, int heads, int qk_dim, int v_dim, float scale,
                            float* lse, void* stream) {
  ADR_REQUIRE(v_dim == HD && (qk_dim == 32 || qk_dim == 64), "attn: v_dim must be 64 and qk_dim 32 or 64 (got %d/%d)",
              v_dim, qk_dim);
  ADR_REQUIRE(attn_views_ok(dtype, {cs, ocs, qo, ko, vo, hs}), "attn: views");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16) {
    if (qk_dim == 32) attn_fwd_launch<__bf16, 32>(q, k, v, cs, qo, ko, vo, hs, o, ocs, B, L, heads, scale, lse, st);
    else attn_fwd_launch<__bf16, 64>(q, k, v, cs, qo, ko, vo, hs, o, ocs, B, L, heads, scale, lse, st);
  } else {
    if (qk_dim == 32) attn_fwd_launch<float, 32>(q, k, v, cs, qo, ko, vo, hs, o, ocs, B, L, heads, scale, lse, st);
    else attn_fwd_launch<float, 64>(q, k, v, cs, qo, ko, vo, hs, o, ocs, B, L, heads, scale, lse, st);
  }
  return check_launch("adr_attn_fwd");
}

extern "C" int adr_attn_bwd(int dtype, const void* q, const void* k, const void* v, int cs, int qo, int ko, int vo,
                            int hs, const void* o, int ocs, const void* dout, int dcs, const float* lse, void* dq,
                            void* dk, void* dv, int gcs, int gqo, int gko, int gvo, int B, int L, int heads,
                            int qk_dim, int v_dim, float scale, float* dvec_ws, void* stream) {
  ADR_REQUIRE(v_dim == HD && (qk_dim == 32 || qk_dim == 64), "attn: v_dim must be 64 and qk_dim 32 or 64");
  ADR_REQUIRE(attn_views_ok(dtype, {cs, ocs, dcs, qo, ko, vo, hs}) && ((uintptr_t)o & 15) == 0 && ((uintptr_t)dout & 15) == 0,
              "attn bwd: views");
  hipStream_t st = (hipStream_t)stream;
#define ADR_ATTN_BWD(T, D)                                                                                              \
  attn_bwd_launch<T, D>(q, k, v, cs, qo, ko, vo, hs, o, ocs, dout, dcs, lse, dq, dk, dv, gcs, gqo, gko, gvo, B, L, heads, \
                        scale, dvec_ws, st)
  if (dtype == ADR_BF16) {
    if (qk_dim == 32) ADR_ATTN_BWD(__bf16, 32);
    else ADR_ATTN_BWD(__bf16, 64);
  } else {
    if (qk_dim == 32) ADR_ATTN_BWD(float, 32);
    else ADR_ATTN_BWD(float, 64);
  }
#undef ADR_ATTN_BWD
  return check_launch("adr_attn_bwd");
}
