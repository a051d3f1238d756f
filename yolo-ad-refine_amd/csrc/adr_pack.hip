// Parameter plumbing kernels: pack fp32 PyTorch-layout weights into the kernels' KRSC operand layout
// (with the cast to the compute dtype), and unpack KRSC fp32 weight gradients back to (K, C, R, S).
#include "adr_common.h"

namespace adr {

template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ src, T* __restrict__ dst, int K, int C, int Cp, int RS,
                                   int transpose_kc) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long n = (long)K * Cp * RS;
  if (i >= n) return;
  // destination index i = (k * RS + t) * Cp + c ; channels c >= C are zero padding
  int c = (int)(i % Cp);
  long r = i / Cp;
  int t = (int)(r % RS);
  int k = (int)(r / RS);
  // source (K, C, RS) or, for ConvTranspose2d weights viewed as the equivalent conv, (C, K, RS)
  if (c >= C) {
    dst[i] = from_f<T>(0.f);
    return;
  }
  long s = transpose_kc ? ((long)c * K + k) * RS + t : ((long)k * C + c) * RS + t;
  dst[i] = from_f<T>(src[s]);
}

__global__ void unpack_weight_grad_kernel(const float* __restrict__ src, float* __restrict__ dst, int K, int C,
                                          int Cp, int RS, int transpose_kc, int accumulate) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long n = (long)K * Cp * RS;
  if (i >= n) return;
  int c = (int)(i % Cp);
  long r = i / Cp;
  int t = (int)(r % RS);
  int k = (int)(r / RS);
  if (c >= C) return;
  long s = transpose_kc ? ((long)c * K + k) * RS + t : ((long)k * C + c) * RS + t;
  dst[s] = accumulate ? dst[s] + src[i] : src[i];
}

// both operand layouts from one read of the fp32 parameter: KRSC [Kp][RS][Cp] (FWD rows) and CRSK [Cp][RS][Kp]
// (DGRAD rows); k >= K and c >= C are zero padding
template <typename T>
__global__ void pack_weight2_kernel(const float* __restrict__ src, T* __restrict__ krsc, T* __restrict__ crsk, int K,
                                    int Kp, int C, int Cp, int RS, int transpose_kc) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long n = (long)Kp * Cp * RS;
  if (i >= n) return;
  int c = (int)(i % Cp);
  long r = i / Cp;
  int t = (int)(r % RS);
  int k = (int)(r / RS);
  float v = 0.f;
  if (c < C && k < K) v = src[transpose_kc ? ((long)c * K + k) * RS + t : ((long)k * C + c) * RS + t];
  const T tv = from_f<T>(v);
  krsc[i] = tv;
  crsk[((long)c * RS + t) * Kp + k] = tv;
}

// batched pack2: one block per chunk row of the table (a chunk = up to PACK_CHUNK elements of one weight)
struct PackChunk {
  const float* src;
  void* krsc;
  void* crsk;
  int K, Kp, C, Cp, RS, tkc;
  long start, len;
};

template <typename T>
__global__ void __launch_bounds__(256) pack_weight2_batched_kernel(const PackChunk* tab) {
  const PackChunk e = tab[blockIdx.x];
  T* krsc = (T*)e.krsc;
  T* crsk = (T*)e.crsk;
  for (long i = e.start + threadIdx.x; i < e.start + e.len; i += 256) {
    const int c = (int)(i % e.Cp);
    const long r = i / e.Cp;
    const int t = (int)(r % e.RS);
    const int k = (int)(r / e.RS);
    float v = 0.f;
    if (c < e.C && k < e.K) v = e.src[e.tkc ? ((long)c * e.K + k) * e.RS + t : ((long)k * e.C + c) * e.RS + t];
    const T tv = from_f<T>(v);
    krsc[i] = tv;
    crsk[((long)c * e.RS + t) * e.Kp + k] = tv;
  }
}

// tiled pack2: one block per (weight, tap t, 64-row k tile, 64-column c tile). The fp32 weight tile is staged in LDS
// once and written out in both layouts with consecutive lanes on the contiguous axis: KRSC rows along c, CRSK rows
// along k. (The per-chunk kernel above walks KRSC order, so its CRSK stores are 2-byte writes RS * Kp elements apart:
// at the l-scale model's 25 M weights 0.91 ms per step for ~150 MB of algorithmic traffic.)
struct PackTile {
  const float* src;
  void* krsc;
  void* crsk;
  int K, Kp, C, Cp, RS, tkc;
  int t, k0, c0, pad;
};

template <typename T>
__global__ void __launch_bounds__(256) pack_weight2_tiled_kernel(const PackTile* tab) {
  __shared__ float tile[64][65];
  const PackTile e = tab[blockIdx.x];
  T* krsc = (T*)e.krsc;
  T* crsk = (T*)e.crsk;
  const int tid = threadIdx.x;
#pragma unroll 4
  for (int i = tid; i < 64 * 64; i += 256) {  // lanes along c: KRSC stores contiguous
    const int kk = i >> 6, cc = i & 63, k = e.k0 + kk, c = e.c0 + cc;
    float v = 0.f;
    if (c < e.C && k < e.K)
      v = e.src[e.tkc ? ((long)c * e.K + k) * e.RS + e.t : ((long)k * e.C + c) * e.RS + e.t];
    tile[kk][cc] = v;
    if (k < e.Kp && c < e.Cp) krsc[((long)k * e.RS + e.t) * e.Cp + c] = from_f<T>(v);
  }
  __syncthreads();
#pragma unroll 4
  for (int i = tid; i < 64 * 64; i += 256) {  // lanes along k: CRSK stores contiguous
    const int cc = i >> 6, kk = i & 63, k = e.k0 + kk, c = e.c0 + cc;
    if (k < e.Kp && c < e.Cp) crsk[((long)c * e.RS + e.t) * e.Kp + k] = from_f<T>(tile[kk][cc]);
  }
}

template <typename A, typename B>
__global__ void cast_kernel(const A* __restrict__ src, B* __restrict__ dst, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = from_f<B>(to_f(src[i]));
}

}  // namespace adr

using namespace adr;

extern "C" int adr_pack_weight(int dtype, const float* src, void* dst, int K, int C, int Cp, int RS,
                               int transpose_kc, void* stream) {
  ADR_REQUIRE(Cp >= C, "pack_weight: Cp < C");
  long n = (long)K * Cp * RS;
  ADR_REQUIRE(n > 0, "pack_weight: empty");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<__bf16>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, (__bf16*)dst, K, C, Cp,
                       RS, transpose_kc);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, (float*)dst, K, C, Cp,
                       RS, transpose_kc);
  return check_launch("adr_pack_weight");
}

extern "C" int adr_pack_weight2(int dtype, const float* src, void* krsc, void* crsk, int K, int Kp, int C, int Cp,
                                int RS, int transpose_kc, void* stream) {
  ADR_REQUIRE(K <= Kp && C <= Cp && K > 0 && C > 0 && RS > 0, "pack_weight2: K=%d Kp=%d C=%d Cp=%d", K, Kp, C, Cp);
  long n = (long)Kp * Cp * RS;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(pack_weight2_kernel<__bf16>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, (__bf16*)krsc,
                       (__bf16*)crsk, K, Kp, C, Cp, RS, transpose_kc);
  else
    hipLaunchKernelGGL(pack_weight2_kernel<float>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, (float*)krsc,
                       (float*)crsk, K, Kp, C, Cp, RS, transpose_kc);
  return check_launch("adr_pack_weight2");
}

extern "C" int adr_pack_chunk_size(void) { return (int)sizeof(PackChunk); }

extern "C" int adr_pack_weight2_batched(int dtype, const void* table, int nchunks, void* stream) {
  ADR_REQUIRE(nchunks > 0, "pack_weight2_batched: empty table");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(pack_weight2_batched_kernel<__bf16>, dim3(nchunks), dim3(256), 0, st, (const PackChunk*)table);
  else
    hipLaunchKernelGGL(pack_weight2_batched_kernel<float>, dim3(nchunks), dim3(256), 0, st, (const PackChunk*)table);
  return check_launch("adr_pack_weight2_batched");
}

extern "C" int adr_pack_tile_size(void) { return (int)sizeof(PackTile); }

extern "C" int adr_pack_weight2_tiled(int dtype, const void* table, int ntiles, void* stream) {
  ADR_REQUIRE(ntiles > 0, "pack_weight2_tiled: empty table");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(pack_weight2_tiled_kernel<__bf16>, dim3(ntiles), dim3(256), 0, st, (const PackTile*)table);
  else
    hipLaunchKernelGGL(pack_weight2_tiled_kernel<float>, dim3(ntiles), dim3(256), 0, st, (const PackTile*)table);
  return check_launch("adr_pack_weight2_tiled");
}

extern "C" int adr_unpack_weight_grad(const float* src, float* dst, int K, int C, int Cp, int RS,
                                      int transpose_kc, int accumulate, void* stream) {
  long n = (long)K * Cp * RS;
  hipLaunchKernelGGL(unpack_weight_grad_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, src, dst, K, C,
                     Cp, RS, transpose_kc, accumulate);
  return check_launch("adr_unpack_weight_grad");
}

extern "C" int adr_cast(int src_dtype, const void* src, int dst_dtype, void* dst, long n, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 g(cdiv(n, 256));
  if (src_dtype == ADR_F32 && dst_dtype == ADR_BF16)
    hipLaunchKernelGGL((cast_kernel<float, __bf16>), g, dim3(256), 0, st, (const float*)src, (__bf16*)dst, n);
  else if (src_dtype == ADR_BF16 && dst_dtype == ADR_F32)
    hipLaunchKernelGGL((cast_kernel<__bf16, float>), g, dim3(256), 0, st, (const __bf16*)src, (float*)dst, n);
  else if (src_dtype == ADR_F32 && dst_dtype == ADR_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), g, dim3(256), 0, st, (const float*)src, (float*)dst, n);
  else
    hipLaunchKernelGGL((cast_kernel<__bf16, __bf16>), g, dim3(256), 0, st, (const __bf16*)src, (__bf16*)dst, n);
  return check_launch("adr_cast");
}

// NCHW fp32 image batch -> NHWC compute dtype with channels zero-padded to Cp (detect/train.py:57-59 hands the
// model float images in [0,1]; the first conv's C=3 is padded so every conv input is 16-byte vectorisable).
template <typename T>
__global__ void image_to_nhwc_kernel(const float* __restrict__ src, T* __restrict__ dst, int N, int C, int H, int W,
                                     int Cp) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long n = (long)N * H * W * Cp;
  if (i >= n) return;
  int c = (int)(i % Cp);
  long pix = i / Cp;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int b = (int)(r / H);
  float v = c < C ? src[(((long)b * C + c) * H + h) * W + w] : 0.f;
  dst[i] = from_f<T>(v);
}

// vector form (W % 4 == 0, Cp == 8): a thread turns 4 consecutive pixels of C planes into 4 NHWC rows of 8
// channels (float4 plane reads, 16-byte row stores)
template <typename T>
__global__ void __launch_bounds__(256) image_to_nhwc8_kernel(const float* __restrict__ src, T* __restrict__ dst, int N,
                                                             int C, int H, int W) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;  // pixel quad
  const long nq = (long)N * H * W / 4;
  if (q >= nq) return;
  const long pix = q * 4;
  const long HW = (long)H * W;
  const long b = pix / HW, hw = pix % HW;
  float v[4][8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < C) f = *reinterpret_cast<const float4*>(src + (b * C + c) * HW + hw);
    v[0][c] = f.x; v[1][c] = f.y; v[2][c] = f.z; v[3][c] = f.w;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    T* o = dst + (pix + p) * 8;
    if constexpr (sizeof(T) == 2) {
      u32x4 r;
      T* e = reinterpret_cast<T*>(&r);
#pragma unroll
      for (int c = 0; c < 8; ++c) e[c] = from_f<T>(v[p][c]);
      st16(o, r);
    } else {
      st16(o, *reinterpret_cast<const u32x4*>(&v[p][0]));
      st16(o + 4, *reinterpret_cast<const u32x4*>(&v[p][4]));
    }
  }
}

// uint8 NCHW batch -> NHWC compute-dtype activation with channels zero-padded to Cp, value / 255 (preprocess_batch)
template <typename T>
__global__ void image_u8_to_nhwc_kernel(const uint8_t* __restrict__ src, T* __restrict__ dst, int N, int C, int H,
                                        int W, int Cp) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long n = (long)N * H * W * Cp;
  if (i >= n) return;
  int c = (int)(i % Cp);
  long pix = i / Cp;
  int w = (int)(pix % W);
  long r = pix / W;
  int h = (int)(r % H);
  int b = (int)(r / H);
  // x * fp32(1/255): torch's device division by a scalar (a multiplication by the reciprocal), bitwise
  float v = c < C ? (float)src[(((long)b * C + c) * H + h) * W + w] * (1.f / 255.f) : 0.f;
  dst[i] = from_f<T>(v);
}

extern "C" int adr_image_u8_to_nhwc(int dtype, const uint8_t* src, void* dst, int N, int C, int H, int W, int Cp,
                                    void* stream) {
  ADR_REQUIRE(Cp >= C && C > 0, "image_u8_to_nhwc: C=%d Cp=%d", C, Cp);
  long n = (long)N * H * W * Cp;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(image_u8_to_nhwc_kernel<__bf16>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, (__bf16*)dst, N, C, H,
                       W, Cp);
  else
    hipLaunchKernelGGL(image_u8_to_nhwc_kernel<float>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, (float*)dst, N, C, H,
                       W, Cp);
  return check_launch("adr_image_u8_to_nhwc");
}

extern "C" int adr_image_to_nhwc(int dtype, const float* src, void* dst, int N, int C, int H, int W, int Cp,
                                 void* stream) {
  long n = (long)N * H * W * Cp;
  hipStream_t st = (hipStream_t)stream;
  if (Cp == 8 && C <= 8 && W % 4 == 0) {
    const long nq = (long)N * H * W / 4;
    if (dtype == ADR_BF16)
      hipLaunchKernelGGL(image_to_nhwc8_kernel<__bf16>, dim3(cdiv(nq, 256)), dim3(256), 0, st, src, (__bf16*)dst, N, C,
                         H, W);
    else
      hipLaunchKernelGGL(image_to_nhwc8_kernel<float>, dim3(cdiv(nq, 256)), dim3(256), 0, st, src, (float*)dst, N, C, H,
                         W);
    return check_launch("adr_image_to_nhwc");
  }
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(image_to_nhwc_kernel<__bf16>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, (__bf16*)dst, N, C, H,
                       W, Cp);
  else
    hipLaunchKernelGGL(image_to_nhwc_kernel<float>, dim3(cdiv(n, 256)), dim3(256), 0, st, src, (float*)dst, N, C, H, W,
                       Cp);
  return check_launch("adr_image_to_nhwc");
}
