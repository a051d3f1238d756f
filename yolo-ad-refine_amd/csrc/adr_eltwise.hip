// Elementwise / broadcast kernels over NHWC views (16-byte vectorised, grid-stride).
//
// Covers the reference's glue arithmetic on the hot path: channel concat (torch.cat in C2f/SPPF/C2PSA,
// block.py:244-247, 194-196), residual adds (Bottleneck block.py:353), Multiply / Add (block.py:1442-1453),
// Fusion('bifpn') weighted sums (block.py:1532-1535), gates x + a*sigmoid(b) (head.py:739-747),
// activations (SiLU/GELU/ReLU/Sigmoid/Hardswish), per-image / per-channel broadcast multiplies
// (TaskDecomposition head.py:657-664, Scale head.py:797) and their backward reductions.
#include "adr_common.h"

namespace adr {

// op codes for the n-ary kernel:
//  0 copy          : o = a
//  1 axpby         : o = ca*a + cb*b               (ca/cb device scalars, null = 1)
//  2 mul           : o = a*b
//  3 fma           : o = a + b*c
//  4 act           : o = act(a)
//  5 act_bwd       : o = d(=b) * act'(a)
//  6 add3          : o = a + b + c
//  7 act_bwd_out   : o = d(=b) * act'(x) written from the OUTPUT a = act(x): relu (a > 0), sigmoid a (1 - a), as
//                    torch's threshold_backward / sigmoid_backward
//  8 mul_add       : o = T(a * b) + c, the product rounded to T first and no contraction — bitwise the mul + add
//                    pair (the HS-FPN gate and residual, Multiply then Add: yaml layers 17-18, 24-25)
enum EwOp { EW_COPY = 0, EW_AXPBY = 1, EW_MUL = 2, EW_FMA = 3, EW_ACT = 4, EW_ACT_BWD = 5, EW_ADD3 = 6,
            EW_ACT_BWD_OUT = 7, EW_MUL_ADD = 8 };

template <typename T>
__global__ void __launch_bounds__(256) ew_kernel(int op, int act, const T* a, int acs, const T* b, int bcs, const T* c,
                                                 int ccs, T* o, int ocs, long npix, int C, const float* ca,
                                                 const float* cb, int accumulate) {
  constexpr int V = VecIO<T>::V;
  const PixLanes L(C / V);
  if (!L.active) return;
  const int c0 = L.cg * V;
  const float sa = ca ? *ca : 1.f, sb = cb ? *cb : 1.f;
  for (long pix = (long)blockIdx.x * L.rpb + L.r0; pix < npix; pix += (long)gridDim.x * L.rpb) {
    float fa[V], fb[V], fc[V], fo[V];
    VecIO<T>::load(a + pix * acs + c0, fa);
    if (op == EW_AXPBY || op == EW_MUL || op == EW_FMA || op == EW_ACT_BWD || op == EW_ADD3 || op == EW_ACT_BWD_OUT ||
        op == EW_MUL_ADD)
      VecIO<T>::load(b + pix * bcs + c0, fb);
    if (op == EW_FMA || op == EW_ADD3 || op == EW_MUL_ADD) VecIO<T>::load(c + pix * ccs + c0, fc);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float r;
      switch (op) {
        case EW_COPY: r = fa[k]; break;
        case EW_AXPBY: r = sa * fa[k] + sb * fb[k]; break;
        case EW_MUL: r = fa[k] * fb[k]; break;
        case EW_FMA: r = fa[k] + fb[k] * fc[k]; break;
        case EW_ACT: r = act_fwd(act, fa[k]); break;
        case EW_ACT_BWD: r = fb[k] * act_bwd(act, fa[k]); break;
        case EW_ACT_BWD_OUT: r = act == 3 ? (fa[k] > 0.f ? fb[k] : 0.f) : fb[k] * ((1.f - fa[k]) * fa[k]); break;
        case EW_MUL_ADD: r = __fadd_rn(to_f(from_f<T>(__fmul_rn(fa[k], fb[k]))), fc[k]); break;
        default: r = fa[k] + fb[k] + fc[k]; break;
      }
      fo[k] = r;
    }
    if (accumulate) {
      float fp[V];
      VecIO<T>::load(o + pix * ocs + c0, fp);
#pragma unroll
      for (int k = 0; k < V; ++k) fo[k] += fp[k];
    }
    VecIO<T>::store(o + pix * ocs + c0, fo);
  }
}

// o = x * g[n*gns + c*gcs] (+ res) ; g fp32
template <typename T>
__global__ void __launch_bounds__(256) bcast_mul_kernel(const T* x, int xcs, const float* g, int gns, int gcs,
                                                        const T* res, int rcs, T* o, int ocs, long npix, int HW, int C,
                                                        int accumulate) {
  constexpr int V = VecIO<T>::V;
  const PixLanes L(C / V);
  if (!L.active) return;
  const int c0 = L.cg * V;
  for (long pix = (long)blockIdx.x * L.rpb + L.r0; pix < npix; pix += (long)gridDim.x * L.rpb) {
    const int n = (int)((unsigned long)pix / (unsigned)HW);
    float fx[V], fo[V];
    VecIO<T>::load(x + pix * xcs + c0, fx);
#pragma unroll
    for (int k = 0; k < V; ++k) fo[k] = fx[k] * g[(long)n * gns + (long)(c0 + k) * gcs];
    if (res) {
      float fr[V];
      VecIO<T>::load(res + pix * rcs + c0, fr);
#pragma unroll
      for (int k = 0; k < V; ++k) fo[k] += fr[k];
    }
    if (accumulate) {
      float fp[V];
      VecIO<T>::load(o + pix * ocs + c0, fp);
#pragma unroll
      for (int k = 0; k < V; ++k) fo[k] += fp[k];
    }
    VecIO<T>::store(o + pix * ocs + c0, fo);
  }
}

// out[n][c] = sum over chunks of partial[n][chunk][which][c], then optionally summed over n and/or c.
// One workgroup per output element (NT threads: 1024 when everything collapses to a scalar), fixed-order
// per-thread strides + tree combine (deterministic); the full collapse walks rows division-free, 8 loads in flight.
template <int NT>
__device__ __forceinline__ void nc_collapse_body(const float* partial, int N, int chunks, int C, int which, float* out,
                                                 int sum_n, int sum_c, int accumulate, const int idx) {
  const int outC = sum_c ? 1 : C;
  const int on = idx / outC, oc = idx % outC;
  const int nn = sum_n ? N : 1, ncc = sum_c ? C : 1;
  const int n0 = sum_n ? 0 : on, c0 = sum_c ? 0 : oc;
  const int items = nn * chunks * ncc;
  auto at = [&](int it) {
    const int r = it / ncc;
    const int c = c0 + (it - r * ncc);
    const int n = n0 + r / chunks, ch = r % chunks;
    return partial[((long)n * chunks + ch) * 2 * C + (long)which * C + c];
  };
  double s = 0.0;
  if (sum_n && sum_c && C <= NT && NT % C == 0) {
    // full collapse: thread = (channel, row lane), rows walked without index division, 8 loads in flight
    const int c = threadIdx.x % C, rstep = NT / C, R = N * chunks;
    const float* p = partial + (long)which * C + c;
    int r = threadIdx.x / C;
    for (; r + 7 * rstep < R; r += 8 * rstep) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(long)(r + u * rstep) * 2 * C];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (double)v[u];
    }
    for (; r < R; r += rstep) s += (double)p[(long)r * 2 * C];
  } else {
    int it = threadIdx.x;
    for (; it + 3 * NT < items; it += 4 * NT) {
      const float a = at(it), b = at(it + NT), c = at(it + 2 * NT), d = at(it + 3 * NT);
      s += (double)a;
      s += (double)b;
      s += (double)c;
      s += (double)d;
    }
    for (; it < items; it += NT) s += (double)at(it);
  }
  __shared__ double sh[NT];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[idx] = accumulate ? out[idx] + (float)sh[0] : (float)sh[0];
}

// no collapse (per (n, c) outputs, e.g. the head's per-sub-image pooled sums): one thread per output, its chunks
// summed in order in double — one 256-thread workgroup per output (the kernel below) spent ~27 us on the packed
// head's 1344 x 128 outputs of one or two chunks each
__global__ void __launch_bounds__(256) nc_sum_chunks_kernel(const float* __restrict__ partial, int N, int chunks,
                                                            int C, int which, float* out, int accumulate) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)N * C) return;
  const int n = (int)(idx / C), c = (int)(idx - (long)n * C);
  const float* p = partial + ((long)n * chunks * 2 + which) * C + c;
  double s = 0.0;
  for (int ch = 0; ch < chunks; ++ch) s += (double)p[(long)ch * 2 * C];
  out[idx] = accumulate ? out[idx] + (float)s : (float)s;
}

template <int NT>
__global__ void __launch_bounds__(NT) nc_collapse_kernel(const float* partial, int N, int chunks, int C, int which,
                                                         float* out, int sum_n, int sum_c, int accumulate) {
  nc_collapse_body<NT>(partial, N, chunks, C, which, out, sum_n, sum_c, accumulate, blockIdx.x);
}

// partial[n][chunk][0][c] = sum x*dz ; [1][c] = sum dz   (per image, per channel)
template <typename T>
__device__ __forceinline__ void dot_reduce_body(const T* __restrict__ x, int xcs, const T* __restrict__ dz, int dcs,
                                                int HW, int C, int rows_per_chunk, int chunks,
                                                float* __restrict__ partial, const int chunk, const int n) {
  constexpr int V = VecIO<T>::V;
  __shared__ float sh[2][256 * V];
  const int G = C / V;
  const int rpp = 256 / G;
  const int t = threadIdx.x;
  const int cg = t % G, r0 = t / G;
  float s1[V], s2[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  const int rbeg = chunk * rows_per_chunk, rend = min(HW, rbeg + rows_per_chunk);
  if (r0 < rpp) {
    constexpr int NU = 4;  // rows in flight per thread
    for (int r = rbeg + r0; r < rend; r += NU * rpp) {
      float fx[NU][V], fd[NU][V];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const long pix = (long)n * HW + r + u * rpp;
        if (r + u * rpp < rend) {
          if (x) VecIO<T>::load(x + pix * xcs + cg * V, fx[u]);
          VecIO<T>::load(dz + pix * dcs + cg * V, fd[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (r + u * rpp >= rend) break;
#pragma unroll
        for (int e = 0; e < V; ++e) {
          s1[e] += x ? fx[u][e] * fd[u][e] : 0.f;
          s2[e] += fd[u][e];
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    sh[0][t * V + e] = s1[e];
    sh[1][t * V + e] = s2[e];
  }
  __syncthreads();
  float* out = partial + ((long)n * chunks + chunk) * 2 * C;
  for (int c = t; c < C; c += 256) {
    int g = c / V, e = c % V;
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rpp; ++r) {
      a += sh[0][(g + r * G) * V + e];
      b += sh[1][(g + r * G) * V + e];
    }
    out[c] = a;
    out[C + c] = b;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dot_reduce_kernel(const T* __restrict__ x, int xcs, const T* __restrict__ dz,
                                                         int dcs, int HW, int C, int rows_per_chunk, int chunks,
                                                         float* __restrict__ partial) {
  dot_reduce_body<T>(x, xcs, dz, dcs, HW, C, rows_per_chunk, chunks, partial, blockIdx.x, blockIdx.y);
}

// Deferred scalar parameter gradients (Scale, weighted-sum weights: sum over every pixel and channel of x * dy),
// batched at the end of backward: the dot partials of all entries in one launch (block = (chunk, image) of an
// entry), then one 1024-thread workgroup per entry collapsing its partial rows — the same bodies, so the same
// fixed summation order as adr_dot_reduce + adr_nc_collapse(sum_n = sum_c = 1).
constexpr int DTB_MAX = 32;
struct DotBatch {
  adr_dotsum_entry e[DTB_MAX];
  int start[DTB_MAX + 1];
  int count;
};
__global__ void __launch_bounds__(256) dot_reduce_batched_kernel(DotBatch b) {
  int j = 0;
  while (j + 1 < b.count && (int)blockIdx.x >= b.start[j + 1]) ++j;
  const adr_dotsum_entry& en = b.e[j];
  const int local = (int)blockIdx.x - b.start[j];
  dot_reduce_body<__bf16>((const __bf16*)en.x, en.xcs, (const __bf16*)en.dz, en.dcs, en.HW, en.C, en.rows_per_chunk,
                          en.chunks, en.partial, local % en.chunks, local / en.chunks);
}
__global__ void __launch_bounds__(1024) dot_collapse_batched_kernel(DotBatch b) {
  const adr_dotsum_entry& en = b.e[blockIdx.x];
  nc_collapse_body<1024>(en.partial, en.N, en.chunks, en.C, 0, en.out, 1, 1, 0, 0);
}

// BiFPN fusion weights: w = relu(fw) / (sum relu(fw) + eps)   (block.py:1532-1535), and its backward
__global__ void fusion_weights_kernel(const float* fw, int n, float eps, float* w) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += fmaxf(fw[i], 0.f);
  for (int i = 0; i < n; ++i) w[i] = fmaxf(fw[i], 0.f) / (s + eps);
}
__global__ void fusion_weights_bwd_kernel(const float* fw, int n, float eps, const float* dw, float* dfw) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += fmaxf(fw[i], 0.f);
  float d = s + eps;
  float dot = 0.f;
  for (int i = 0; i < n; ++i) dot += dw[i] * fmaxf(fw[i], 0.f);
  for (int i = 0; i < n; ++i) {
    float g = dw[i] / d - dot / (d * d);  // d w_i / d r_j summed: dw_i/d - sum_k dw_k r_k / d^2
    dfw[i] = fw[i] > 0.f ? g : 0.f;
  }
}

__global__ void axpy_kernel(long n, float a, const float* x, float* y) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] += a * x[i];
}

// Many y += x over distinct destinations in one launch (the trainer's deferred parameter-gradient adds): 1024
// elements per workgroup, the entry found from the per-entry block offsets.
constexpr int AXB_MAX = 96;
struct AxpyBatch {
  adr_axpy_entry e[AXB_MAX];
  int start[AXB_MAX + 1];
  int count;
};
__global__ void __launch_bounds__(256) axpy_batched_kernel(AxpyBatch b) {
  int j = 0;
  while (j + 1 < b.count && (int)blockIdx.x >= b.start[j + 1]) ++j;
  const adr_axpy_entry& en = b.e[j];
  const long base = (long)(blockIdx.x - b.start[j]) * 1024 + threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long i = base + u * 256;
    if (i < en.n) en.y[i] += en.x[i];
  }
}

static int ew_grid(long npix, int G) {
  const long rpb = 256 / G;  // pixels per block pass (PixLanes)
  long b = (npix + rpb - 1) / rpb;
  if (b > 32768) b = 32768;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace adr

using namespace adr;

extern "C" int adr_ew(int dtype, int op, int act, const void* a, int acs, const void* b, int bcs, const void* c,
                      int ccs, void* o, int ocs, long npix, int C, const float* ca, const float* cb, int accumulate,
                      void* stream) {
  int v = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % v == 0 && acs % v == 0 && ocs % v == 0 && (!b || bcs % v == 0) && (!c || ccs % v == 0),
              "adr_ew: C=%d / strides must be multiples of %d", C, v);
  ADR_REQUIRE(op >= 0 && op <= 8 && (op != 7 || act == 3 || act == 4), "adr_ew: op %d act %d", op, act);
  ADR_REQUIRE(((uintptr_t)a | (uintptr_t)o | (uintptr_t)b | (uintptr_t)c) % 16 == 0, "adr_ew: pointers not 16B aligned");
  ADR_REQUIRE(C / v <= 256, "adr_ew: C=%d too wide", C);
  int g = ew_grid(npix, C / v);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(ew_kernel<__bf16>, dim3(g), dim3(256), 0, st, op, act, (const __bf16*)a, acs,
                       (const __bf16*)b, bcs, (const __bf16*)c, ccs, (__bf16*)o, ocs, npix, C, ca, cb, accumulate);
  else
    hipLaunchKernelGGL(ew_kernel<float>, dim3(g), dim3(256), 0, st, op, act, (const float*)a, acs, (const float*)b,
                       bcs, (const float*)c, ccs, (float*)o, ocs, npix, C, ca, cb, accumulate);
  return check_launch("adr_ew");
}

extern "C" int adr_bcast_mul(int dtype, const void* x, int xcs, const float* g, int gns, int gcs, const void* res,
                             int rcs, void* o, int ocs, int N, int HW, int C, int accumulate, void* stream) {
  int v = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % v == 0 && xcs % v == 0 && ocs % v == 0 && (!res || rcs % v == 0), "adr_bcast_mul: misaligned");
  long npix = (long)N * HW;
  ADR_REQUIRE(C / v <= 256, "adr_bcast_mul: C=%d too wide", C);
  int grid = ew_grid(npix, C / v);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(bcast_mul_kernel<__bf16>, dim3(grid), dim3(256), 0, st, (const __bf16*)x, xcs, g, gns, gcs,
                       (const __bf16*)res, rcs, (__bf16*)o, ocs, npix, HW, C, accumulate);
  else
    hipLaunchKernelGGL(bcast_mul_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)x, xcs, g, gns, gcs,
                       (const float*)res, rcs, (float*)o, ocs, npix, HW, C, accumulate);
  return check_launch("adr_bcast_mul");
}

extern "C" int adr_dot_reduce(int dtype, const void* x, int xcs, const void* dz, int dcs, int N, int HW, int C,
                              int rows_per_chunk, float* partial, void* stream) {
  int v = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % v == 0 && C / v <= 256 && (!x || xcs % v == 0) && dcs % v == 0, "adr_dot_reduce: C=%d", C);
  int chunks = cdiv(HW, rows_per_chunk);
  dim3 grid(chunks, N);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(dot_reduce_kernel<__bf16>, grid, dim3(256), 0, st, (const __bf16*)x, xcs, (const __bf16*)dz,
                       dcs, HW, C, rows_per_chunk, chunks, partial);
  else
    hipLaunchKernelGGL(dot_reduce_kernel<float>, grid, dim3(256), 0, st, (const float*)x, xcs, (const float*)dz, dcs,
                       HW, C, rows_per_chunk, chunks, partial);
  return check_launch("adr_dot_reduce");
}

extern "C" int adr_dotsum_batched(const adr_dotsum_entry* entries, int count, void* stream) {
  ADR_REQUIRE(count >= 0 && (count == 0 || entries), "dotsum_batched: count=%d", count);
  hipStream_t st = (hipStream_t)stream;
  for (int b0 = 0; b0 < count; b0 += DTB_MAX) {
    DotBatch db{};
    db.count = count - b0 < DTB_MAX ? count - b0 : DTB_MAX;
    long blocks = 0;
    for (int j = 0; j < db.count; ++j) {
      const adr_dotsum_entry& en = entries[b0 + j];
      ADR_REQUIRE(en.x && en.dz && en.partial && en.out && en.N > 0 && en.HW > 0 && en.C % 8 == 0 &&
                      en.C / 8 <= 256 && en.xcs % 8 == 0 && en.dcs % 8 == 0 && en.rows_per_chunk > 0 &&
                      en.chunks == cdiv(en.HW, en.rows_per_chunk),
                  "dotsum_batched: entry %d", b0 + j);
      db.e[j] = en;
      db.start[j] = (int)blocks;
      blocks += (long)en.N * en.chunks;
    }
    ADR_REQUIRE(blocks < (1l << 31), "dotsum_batched: grid");
    db.start[db.count] = (int)blocks;
    hipLaunchKernelGGL(dot_reduce_batched_kernel, dim3((unsigned)blocks), dim3(256), 0, st, db);
    hipLaunchKernelGGL(dot_collapse_batched_kernel, dim3(db.count), dim3(1024), 0, st, db);
  }
  return check_launch("adr_dotsum_batched");
}

extern "C" int adr_nc_collapse(const float* partial, int N, int chunks, int C, int which, float* out, int sum_n,
                               int sum_c, int accumulate, void* stream) {
  int outn = (sum_n ? 1 : N) * (sum_c ? 1 : C);
  if (!sum_n && !sum_c && outn > 1)
    hipLaunchKernelGGL(nc_sum_chunks_kernel, dim3(cdiv((long)outn, 256)), dim3(256), 0, (hipStream_t)stream, partial,
                       N, chunks, C, which, out, accumulate);
  else if (outn == 1)
    hipLaunchKernelGGL(nc_collapse_kernel<1024>, dim3(1), dim3(1024), 0, (hipStream_t)stream, partial, N, chunks, C,
                       which, out, sum_n, sum_c, accumulate);
  else
    hipLaunchKernelGGL(nc_collapse_kernel<256>, dim3(outn), dim3(256), 0, (hipStream_t)stream, partial, N, chunks, C,
                       which, out, sum_n, sum_c, accumulate);
  return check_launch("adr_nc_collapse");
}

extern "C" int adr_fusion_weights(const float* fw, int n, float eps, float* w, void* stream) {
  hipLaunchKernelGGL(fusion_weights_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, fw, n, eps, w);
  return check_launch("adr_fusion_weights");
}

extern "C" int adr_fusion_weights_bwd(const float* fw, int n, float eps, const float* dw, float* dfw, void* stream) {
  hipLaunchKernelGGL(fusion_weights_bwd_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, fw, n, eps, dw, dfw);
  return check_launch("adr_fusion_weights_bwd");
}

extern "C" int adr_axpy_batched(const adr_axpy_entry* entries, int count, void* stream) {
  ADR_REQUIRE(count >= 0 && (count == 0 || entries), "axpy_batched: count=%d", count);
  for (int b0 = 0; b0 < count; b0 += AXB_MAX) {
    AxpyBatch ab{};
    ab.count = count - b0 < AXB_MAX ? count - b0 : AXB_MAX;
    long blocks = 0;
    for (int j = 0; j < ab.count; ++j) {
      const adr_axpy_entry& en = entries[b0 + j];
      ADR_REQUIRE(en.x && en.y && en.n > 0, "axpy_batched: entry %d", b0 + j);
      for (int q = 0; q < j; ++q)
        ADR_REQUIRE(ab.e[q].y != en.y, "axpy_batched: entries %d and %d share a destination", b0 + q, b0 + j);
      ab.e[j] = en;
      ab.start[j] = (int)blocks;
      blocks += cdiv(en.n, 1024);
    }
    ADR_REQUIRE(blocks < (1l << 31), "axpy_batched: too many elements");
    ab.start[ab.count] = (int)blocks;
    hipLaunchKernelGGL(axpy_batched_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, ab);
  }
  return check_launch("adr_axpy_batched");
}


constexpr int CPB_MAX = 8;
struct CopyBatch {
  adr_copy_piece e[CPB_MAX];
  int start[CPB_MAX + 1];
  int count;
  unsigned npix;
};
// block b belongs to piece j (start[j] <= b < start[j+1]); a thread moves one 16-byte chunk (8 bf16 channels)
__global__ void __launch_bounds__(256) copy_pieces_kernel(CopyBatch b) {
  int j = 0;
  while (j + 1 < b.count && (int)blockIdx.x >= b.start[j + 1]) ++j;
  const adr_copy_piece& en = b.e[j];
  const unsigned c8 = (unsigned)en.C / 8u;
  const unsigned i = (unsigned)(blockIdx.x - b.start[j]) * 256u + threadIdx.x;
  if (i >= b.npix * c8) return;
  const unsigned pix = i / c8, c = (i - pix * c8) * 8u;
  st16(reinterpret_cast<__bf16*>(en.dst) + (size_t)pix * en.dcs + c,
       ld16(reinterpret_cast<const __bf16*>(en.src) + (size_t)pix * en.scs + c));
}

extern "C" int adr_copy_pieces(const adr_copy_piece* pieces, int count, long npix, void* stream) {
  ADR_REQUIRE(count >= 0 && (count == 0 || pieces) && npix >= 0 && npix < (1l << 31), "copy_pieces: count=%d npix=%ld",
              count, npix);
  for (int b0 = 0; b0 < count; b0 += CPB_MAX) {
    CopyBatch cb{};
    cb.count = count - b0 < CPB_MAX ? count - b0 : CPB_MAX;
    cb.npix = (unsigned)npix;
    long blocks = 0;
    for (int j = 0; j < cb.count; ++j) {
      const adr_copy_piece& en = pieces[b0 + j];
      ADR_REQUIRE(en.src && en.dst && en.C > 0 && en.C % 8 == 0 && en.scs % 8 == 0 && en.dcs % 8 == 0 &&
                      ((uintptr_t)en.src & 15) == 0 && ((uintptr_t)en.dst & 15) == 0 && npix * (en.C / 8) < (1l << 31),
                  "copy_pieces: piece %d (C=%d scs=%d dcs=%d)", b0 + j, en.C, en.scs, en.dcs);
      cb.e[j] = en;
      cb.start[j] = (int)blocks;
      blocks += cdiv(npix * (en.C / 8), 256);
    }
    ADR_REQUIRE(blocks < (1l << 31), "copy_pieces: grid");
    cb.start[cb.count] = (int)blocks;
    if (blocks) hipLaunchKernelGGL(copy_pieces_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, cb);
  }
  return check_launch("adr_copy_pieces");
}

extern "C" int adr_axpy(long n, float a, const float* x, float* y, void* stream) {
  if (n <= 0) return ADR_OK;
  hipLaunchKernelGGL(axpy_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, n, a, x, y);
  return check_launch("adr_axpy");
}
