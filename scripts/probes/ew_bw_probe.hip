// Streaming-kernel shape probe: the BN-act backward arithmetic (dx = A*g + B*x + C, g = dz * silu'(x*s+t)) on
// bf16 NHWC rows, 2 reads + 1 write per element, in several thread/grid shapes. Prints GB/s per variant.
// build: hipcc -O3 --offload-arch=gfx950 scripts/probes/ew_bw_probe.hip -o scripts/probes/ew_bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ float bf2f(unsigned short v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float silu_g(float dz, float x, float s, float t) {
  const float v = x * s + t;
  const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-v));
  return dz * sg * (1.f + v * (1.f - sg));
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ u32x4 compute(u32x4 xv, u32x4 dv, const float* c) {
  const unsigned short* xe = reinterpret_cast<const unsigned short*>(&xv);
  const unsigned short* de = reinterpret_cast<const unsigned short*>(&dv);
  u32x4 o;
  unsigned short* oe = reinterpret_cast<unsigned short*>(&o);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float xf = bf2f(xe[k]);
    const float g = silu_g(bf2f(de[k]), xf, c[k], c[8 + k]);
    oe[k] = f2bf(c[16 + k] * g + c[24 + k] * xf + 0.01f);
  }
  return o;
}

// chunks per thread U (loads of all U issued first), grid-stride over n16 16-byte chunks; channel-group-major: the
// chunk index's low bits are the channel group (C/8 groups), so the coefficients depend on chunk % G
template <int U, bool NT>
__global__ void __launch_bounds__(256) kern(const u32x4* __restrict__ x, const u32x4* __restrict__ dz,
                                            u32x4* __restrict__ dx, long n16, int G, const float* __restrict__ coef) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long base = (long)blockIdx.x * 256 * U + threadIdx.x; base < n16; base += stride) {
    u32x4 xv[U], dv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + 256L * u;
      if (i < n16) {
        xv[u] = __builtin_nontemporal_load(x + i);
        dv[u] = __builtin_nontemporal_load(dz + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + 256L * u;
      if (i < n16) {
        float c[32];
        const int cg = (int)(i % G);
#pragma unroll
        for (int k = 0; k < 32; ++k) c[k] = coef[(k >> 3) * 256 + cg * 8 + (k & 7)];
        st<NT>(dx + i, compute(xv[u], dv[u], c));
      }
    }
  }
}
// the library's current shape: plain loads, one chunk per thread, grid = all chunks
__global__ void __launch_bounds__(256) kern_base(const u32x4* __restrict__ x, const u32x4* __restrict__ dz,
                                                 u32x4* __restrict__ dx, long n16, int G, const float* __restrict__ coef) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n16) return;
  float c[32];
  const int cg = (int)(i % G);
#pragma unroll
  for (int k = 0; k < 32; ++k) c[k] = coef[(k >> 3) * 256 + cg * 8 + (k & 7)];
  dx[i] = compute(x[i], dz[i], c);
}

int main() {
  const int C = 32;
  const long elems = 64L * 160 * 160 * C * 2;  // 104.9 M bf16 per tensor (the step's large BN-act backward x2)
  const long n16 = elems / 8;
  const int G = C / 8;
  u32x4 *x, *dz, *dx;
  float* coef;
  hipMalloc(&x, n16 * 16);
  hipMalloc(&dz, n16 * 16);
  hipMalloc(&dx, n16 * 16);
  hipMalloc(&coef, 4 * 256 * 4);
  hipMemset(x, 0x3c, n16 * 16);
  hipMemset(dz, 0x3c, n16 * 16);
  hipMemset(coef, 0, 4 * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(e0);
    const int R = 20;
    for (int r = 0; r < R; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = 1000.0 * ms / R;
    printf("%-34s %8.1f us  %7.0f GB/s\n", name, us, 3.0 * n16 * 16 / (us * 1e-6) / 1e9);
  };
  const unsigned gfull = (unsigned)((n16 + 255) / 256);
  run("base (1 chunk/thread, full grid)", [&] { kern_base<<<gfull, 256>>>(x, dz, dx, n16, G, coef); });
  run("U1 nt-loads full grid", [&] { kern<1, false><<<gfull, 256>>>(x, dz, dx, n16, G, coef); });
  run("U1 nt-loads+nt-stores full grid", [&] { kern<1, true><<<gfull, 256>>>(x, dz, dx, n16, G, coef); });
  run("U2 full grid", [&] { kern<2, false><<<(gfull + 1) / 2, 256>>>(x, dz, dx, n16, G, coef); });
  run("U2 nt-stores full grid", [&] { kern<2, true><<<(gfull + 1) / 2, 256>>>(x, dz, dx, n16, G, coef); });
  run("U4 full grid", [&] { kern<4, false><<<(gfull + 3) / 4, 256>>>(x, dz, dx, n16, G, coef); });
  for (int per : {4, 8, 16}) {
    char nm[64];
    snprintf(nm, 64, "U2 persistent %d blk/CU", per);
    run(nm, [&] { kern<2, false><<<cus * per, 256>>>(x, dz, dx, n16, G, coef); });
    snprintf(nm, 64, "U4 persistent %d blk/CU", per);
    run(nm, [&] { kern<4, false><<<cus * per, 256>>>(x, dz, dx, n16, G, coef); });
  }
  // pure copy for the ceiling: dx = x
  run("copy (1 read + 1 write) x1.5 scale", [&] { hipMemcpyAsync(dx, x, n16 * 16, hipMemcpyDeviceToDevice); });
  return 0;
}
