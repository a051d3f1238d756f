// Shared device/host helpers for libadr_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/adr.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

namespace adr {

// ---- error plumbing (thread-local, C-ABI visible through adr_last_error) ----
void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define ADR_REQUIRE(cond, ...)                 \
  do {                                         \
    if (!(cond)) {                             \
      ::adr::set_error(__VA_ARGS__);           \
      return ADR_ERR_BAD_ARG;                  \
    }                                          \
  } while (0)

// ---- scalar conversions ----
__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(__bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float v) { return (__bf16)v; }

// 16-byte vector of T (8 bf16 or 4 f32)
template <typename T> struct Vec16 { static constexpr int N = 16 / sizeof(T); };

// XCD-aware block order: the dispatcher deals consecutive workgroup ids round-robin over the 8 XCDs (id % 8), each
// with its own L2. Logical id = rank of the block among its XCD's blocks, offset by the blocks of the XCDs before it,
// so consecutive logical ids (blocks reading the same rows) share one L2. Bijective for every nb: the XCDs below
// r = nb % 8 get one block more (a grid that is not a multiple of 8 used to keep the identity order, which spread
// e.g. the nine tap blocks of one DCN weight-gradient split over eight L2s). The results never depend on the order.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

__device__ __forceinline__ u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ void st16(void* p, u32x4 v) { *reinterpret_cast<u32x4*>(p) = v; }
// VEC consecutive fp32 coefficients (16-byte aligned: VEC-multiple channel offsets into torch allocations)
template <int VEC>
__device__ __forceinline__ void ld_coef(const float* p, float* out) {
#pragma unroll
  for (int k = 0; k < VEC; k += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p + k);
    out[k] = v[0];
    out[k + 1] = v[1];
    out[k + 2] = v[2];
    out[k + 3] = v[3];
  }
}

// ---- activations (shared by norm epilogues and elementwise kernels) ----
enum Act { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_RELU = 3, ACT_SIGMOID = 4, ACT_HSWISH = 5 };

// logistic sigmoid; FAST (the bf16 kernels) uses the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE
// division sequence — the BN/GN activation kernels are VALU-bound on exp + divide, and bf16 storage rounds far
// coarser than 1 ulp of fp32; the fp32 parity mode keeps the exact division
template <bool FAST>
__device__ __forceinline__ float sigmoid_fast(float v) {
  // exp(-v) as a bare v_exp_f32 (2^x): no denormal-range guards; -v*log2(e) beyond the fp32 range gives 0 or inf,
  // and rcp(inf) = 0, the sigmoid's own limit
  if constexpr (FAST) return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(v * -1.44269504088896341f));
  else return 1.f / (1.f + __expf(-v));
}

template <int ACT, bool FAST = false>
__device__ __forceinline__ float act_fwd_c(float v) {
  if constexpr (ACT == ACT_SILU) return FAST ? v * sigmoid_fast<true>(v) : v / (1.f + __expf(-v));
  else if constexpr (ACT == ACT_GELU) return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  else if constexpr (ACT == ACT_RELU) return v > 0.f ? v : 0.f;
  else if constexpr (ACT == ACT_SIGMOID) return sigmoid_fast<FAST>(v);
  else if constexpr (ACT == ACT_HSWISH) return v * fminf(fmaxf(v + 3.f, 0.f), 6.f) * (1.f / 6.f);
  else return v;
}
// derivative d act(v) / dv
template <int ACT, bool FAST = false>
__device__ __forceinline__ float act_bwd_c(float v) {
  if constexpr (ACT == ACT_SILU) {
    const float s = sigmoid_fast<FAST>(v);
    return s * (1.f + v * (1.f - s));
  } else if constexpr (ACT == ACT_GELU) {
    const float cdf = 0.5f * (1.f + erff(v * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * __expf(-0.5f * v * v);
    return cdf + v * pdf;
  } else if constexpr (ACT == ACT_RELU) {
    return v > 0.f ? 1.f : 0.f;
  } else if constexpr (ACT == ACT_SIGMOID) {
    const float s = sigmoid_fast<FAST>(v);
    return s * (1.f - s);
  } else if constexpr (ACT == ACT_HSWISH) {
    return v < -3.f ? 0.f : (v > 3.f ? 1.f : (2.f * v + 3.f) * (1.f / 6.f));
  } else {
    return 1.f;
  }
}

// BatchNorm-affine + activation of one element and its backward, with the fma order written out so that every
// kernel that evaluates them (affine_act / affine_act_bwd, nc_reduce's backward statistics, the conv engine's XF
// operand staging) produces the same bits:  z = act(y * s + t);  dy = A * g + B * y + C, g = dz * act'(y * s + t)
template <int ACT, bool FAST = false>
__device__ __forceinline__ float bn_act_fwd_elem(float y, float s, float t) {
  return act_fwd_c<ACT, FAST>(__builtin_fmaf(y, s, t));
}
template <int ACT, bool FAST = false>
__device__ __forceinline__ float bn_act_g(float dz, float y, float s, float t) {
  return dz * act_bwd_c<ACT, FAST>(__builtin_fmaf(y, s, t));
}
__device__ __forceinline__ float bn_act_bwd_lin(float g, float y, float A, float B, float C) {
  return __builtin_fmaf(A, g, __builtin_fmaf(B, y, C));
}

__device__ __forceinline__ float act_fwd(int act, float v) {
  switch (act) {
    case ACT_SILU: return act_fwd_c<ACT_SILU>(v);
    case ACT_GELU: return act_fwd_c<ACT_GELU>(v);
    case ACT_RELU: return act_fwd_c<ACT_RELU>(v);
    case ACT_SIGMOID: return act_fwd_c<ACT_SIGMOID>(v);
    case ACT_HSWISH: return act_fwd_c<ACT_HSWISH>(v);
    default: return v;
  }
}
__device__ __forceinline__ float act_bwd(int act, float v) {
  switch (act) {
    case ACT_SILU: return act_bwd_c<ACT_SILU>(v);
    case ACT_GELU: return act_bwd_c<ACT_GELU>(v);
    case ACT_RELU: return act_bwd_c<ACT_RELU>(v);
    case ACT_SIGMOID: return act_bwd_c<ACT_SIGMOID>(v);
    case ACT_HSWISH: return act_bwd_c<ACT_HSWISH>(v);
    default: return 1.f;
  }
}

// host: run F(std::integral_constant<int, ACT>) for a runtime activation code (kernels templated on ACT)
#define ADR_ACT_DISPATCH(act, F)                                                         \
  do {                                                                                    \
    switch (act) {                                                                        \
      case ACT_SILU: F(ACT_SILU); break;                                                  \
      case ACT_GELU: F(ACT_GELU); break;                                                  \
      case ACT_RELU: F(ACT_RELU); break;                                                  \
      case ACT_SIGMOID: F(ACT_SIGMOID); break;                                            \
      case ACT_HSWISH: F(ACT_HSWISH); break;                                              \
      default: F(ACT_NONE); break;                                                        \
    }                                                                                     \
  } while (0)

// Thread -> (channel group, pixel row) mapping for 256-thread NHWC elementwise kernels: G = C / vector width
// lanes per pixel, 256 / G pixels per block pass; the channel group is fixed for the thread's whole loop (so
// per-channel coefficients load once) and the loop has no integer division. Host guarantees G <= 256.
// 16-byte vector load / store of one NHWC channel chunk as fp32 (elementwise kernels)
template <typename T> struct VecIO {
  static constexpr int V = 16 / sizeof(T);
  __device__ static void load(const T* p, float* f) {
    u32x4 v = ld16(p);
    const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int i = 0; i < V; ++i) f[i] = to_f(e[i]);
  }
  __device__ static void store(T* p, const float* f) {
    u32x4 v;
    T* e = reinterpret_cast<T*>(&v);
#pragma unroll
    for (int i = 0; i < V; ++i) e[i] = from_f<T>(f[i]);
    st16(p, v);
  }
};

struct PixLanes {
  int cg, r0, rpb;
  bool active;
  __device__ explicit PixLanes(int G) {
    const int t = threadIdx.x;
    rpb = 256 / G;
    cg = t % G;
    r0 = t / G;
    active = r0 < rpb;
  }
};

// (image, row, column) of a flattened NHWC pixel index (< 2^32) with 32-bit unsigned divisions
__device__ __forceinline__ void pix_nhw(long pix, int H, int W, int& n, int& h, int& w) {
  const unsigned p = (unsigned)pix;
  const unsigned r = p / (unsigned)W;
  w = (int)(p - r * (unsigned)W);
  n = (int)(r / (unsigned)H);
  h = (int)(r - (unsigned)n * (unsigned)H);
}

// VW consecutive channels per thread: one 16-byte access when VW * sizeof(T) == 16, scalar otherwise (the host
// picks VW = 1 for views whose channel strides / offsets are not vector multiples).
template <typename T, int VW>
__device__ __forceinline__ void vload(const T* p, float* f) {
  if constexpr (VW * sizeof(T) == 16) {
    const u32x4 v = ld16(p);
    const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int i = 0; i < VW; ++i) f[i] = to_f(e[i]);
  } else {
#pragma unroll
    for (int i = 0; i < VW; ++i) f[i] = to_f(p[i]);
  }
}
template <typename T, int VW>
__device__ __forceinline__ void vstore(T* p, const float* f) {
  if constexpr (VW * sizeof(T) == 16) {
    u32x4 v;
    T* e = reinterpret_cast<T*>(&v);
#pragma unroll
    for (int i = 0; i < VW; ++i) e[i] = from_f<T>(f[i]);
    st16(p, v);
  } else {
#pragma unroll
    for (int i = 0; i < VW; ++i) p[i] = from_f<T>(f[i]);
  }
}
// optional accumulate into dst, then store
template <typename T, int VW>
__device__ __forceinline__ void vstore_acc(T* p, float* f, int accumulate) {
  if (accumulate) {
    float o[VW];
    vload<T, VW>(p, o);
#pragma unroll
    for (int i = 0; i < VW; ++i) f[i] += o[i];
  }
  vstore<T, VW>(p, f);
}

// thread -> (channel group, pixel lane); loops: for (pix = first; pix < npix; pix += step) for (cg ...) — the
// channel loop runs once unless C / VW > 256
struct PoolLanes {
  int cg0, cstep, r0, rpb;
  bool active;
  __device__ explicit PoolLanes(int G) {
    const int t = threadIdx.x;
    if (G <= 256) {
      rpb = 256 / G;
      cg0 = t % G;
      r0 = t / G;
      cstep = G;
    } else {
      rpb = 1;
      cg0 = t;
      r0 = 0;
      cstep = 256;
    }
    active = r0 < rpb;
  }
};
#define POOL_LOOP(L, npix, G)                                                                        \
  for (long pix = (long)blockIdx.x * (L).rpb + (L).r0; pix < (npix); pix += (long)gridDim.x * (L).rpb) \
    for (int cg = (L).cg0; cg < (G); cg += (L).cstep)

// ---- token x channel-group lane layouts (LD lanes per token, VW channels per lane, 256 threads) ----
template <int LD>
__device__ __forceinline__ float tok_sum(float v) {
#pragma unroll
  for (int o = LD / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum of one float per thread (NTH threads, sh[NTH]), result broadcast
template <int NTH>
__device__ __forceinline__ float block_sum(float v, float* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int o = NTH / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  const float r = sh[0];
  __syncthreads();
  return r;
}
// the same for 256 threads
__device__ __forceinline__ float block_sum256(float v, float* sh) {
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  const float r = sh[0];
  __syncthreads();
  return r;
}

// per-channel (d) sum over the block's token rows: red has NTH * VW floats; result in dsum[D]
template <int VW, int LD, int NTH = 256>
__device__ __forceinline__ void chan_sum(const float* part, float* red, float* dsum) {
  constexpr int TPP = NTH / LD;
  const int lane = threadIdx.x % LD;
#pragma unroll
  for (int e = 0; e < VW; ++e) red[threadIdx.x * VW + e] = part[e];
  __syncthreads();
  for (int d = threadIdx.x; d < LD * VW; d += NTH) {
    const int ln = d / VW, e = d % VW;
    float t = 0.f;
    for (int r = 0; r < TPP; ++r) t += red[(r * LD + ln) * VW + e];
    dsum[d] = t;
  }
  (void)lane;
  __syncthreads();
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// wave-level sum (64 lanes)
__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// wave-level sum on DPP (VALU only, no LDS): quad / half-row / row butterflies, then the four row sums are read
// out with v_readlane and added in a fixed order. Wave-uniform result; deterministic.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ double wave_sum_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace adr
