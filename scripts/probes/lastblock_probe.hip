// Probe: cross-workgroup "last block finishes the reduction" on gfx950 (8 XCDs, one L2 each).
// Each block writes a 32-column partial row (and a 32 KB output tile, so the L2s hold dirty lines as in a conv
// epilogue), then arrives on a counter; the block that arrives last sums every row in a fixed order and resets
// the counter. Variants:
//   0: no arrival (the partial rows are summed by a second launch) -- today's conv -> bn_finalize pair
//   1: __threadfence() before the arrival and after it (agent-scope release/acquire: L2 writeback + invalidate)
//   2: partial rows written / read with agent-scope relaxed atomics (coherent stores and loads that bypass the
//      non-coherent L2 state), a vmcnt drain before a relaxed arrival; no L2 writeback
//   3: as 2, two levels (groups of 64 rows, then the group rows)
// Checks every result against the host's fixed-order double sum (bitwise) and reports the time per launch.
// build: hipcc --offload-arch=gfx950 -O3 scripts/probes/lastblock_probe.hip -o /tmp/lastblock_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);   \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int C = 32, GS = 64;

__device__ __host__ inline float val(unsigned b, unsigned t, unsigned c) {
  unsigned h = b * 2654435761u ^ (t * 40503u + c * 2246822519u);
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  return (float)(h & 0xFFFF) * (1.f / 65536.f) - 0.5f;
}

template <int V>
__device__ __forceinline__ void st_row(float* p, float v) {
  if (V >= 2) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <int V>
__device__ __forceinline__ float ld_row(const float* p) {
  if (V >= 2) return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

// block partial of column c (threads t < C write it)
__device__ float block_partial(float* sh) {
  const int t = threadIdx.x;
  for (int c = 0; c < C; ++c) {
    float v = val(blockIdx.x, t, c);
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((t & 63) == 0) sh[(t >> 6) * C + c] = v;
  }
  __syncthreads();
  float r = 0.f;
  if (t < C) r = (sh[t] + sh[C + t]) + (sh[2 * C + t] + sh[3 * C + t]);
  return r;
}

template <int V>
__device__ bool arrive(unsigned* cnt, unsigned total) {
  __shared__ unsigned prev;
  if (V == 1) __threadfence();
  if (V >= 2) __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool last = prev == total - 1;
  if (last) {
    if (V == 1) __threadfence();
    if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return last;
}

template <int V>
__global__ void __launch_bounds__(256) k_probe(float* part, float* part2, unsigned* cnt, double* out, __bf16* tile) {
  __shared__ float sh[4 * C];
  // 32 KB of streaming output per block (dirty L2 lines, as a conv tile store)
  for (int i = threadIdx.x; i < 16384; i += 256) tile[(long)blockIdx.x * 16384 + i] = (__bf16)(float)i;
  const float r = block_partial(sh);
  if (threadIdx.x < C) st_row<V>(&part[(long)blockIdx.x * C + threadIdx.x], r);
  if (V == 0) return;
  const unsigned G = gridDim.x;
  if (V <= 2) {
    if (!arrive<V>(cnt, G)) return;
    if (threadIdx.x < C) {
      double s = 0.0;
      for (unsigned b = 0; b < G; ++b) s += ld_row<V>(&part[(long)b * C + threadIdx.x]);
      out[threadIdx.x] = s;
    }
    return;
  }
  // two levels: group of GS rows -> one double row of part2 (as 2 floats hi/lo would be needed for exactness: keep
  // the group sum in double through a float2 pair)
  const unsigned grp = blockIdx.x / GS, ng = (G + GS - 1) / GS;
  const unsigned gsz = grp + 1 < ng ? GS : G - grp * GS;
  if (!arrive<V>(cnt + 1 + grp, gsz)) return;
  if (threadIdx.x < C) {
    double s = 0.0;
    for (unsigned b = grp * GS; b < grp * GS + gsz; ++b) s += ld_row<V>(&part[(long)b * C + threadIdx.x]);
    const float hi = (float)s, lo = (float)(s - (double)hi);
    st_row<V>(&part2[(long)grp * 2 * C + threadIdx.x], hi);
    st_row<V>(&part2[(long)grp * 2 * C + C + threadIdx.x], lo);
  }
  if (!arrive<V>(cnt, ng)) return;
  if (threadIdx.x < C) {
    double s = 0.0;
    for (unsigned g = 0; g < ng; ++g)
      s += (double)ld_row<V>(&part2[(long)g * 2 * C + threadIdx.x]) + (double)ld_row<V>(&part2[(long)g * 2 * C + C + threadIdx.x]);
    out[threadIdx.x] = s;
  }
}

__global__ void __launch_bounds__(256) k_reduce(const float* part, int G, double* out) {
  if (threadIdx.x < C) {
    double s = 0.0;
    for (int b = 0; b < G; ++b) s += part[(long)b * C + threadIdx.x];
    out[threadIdx.x] = s;
  }
}

int main() {
  const int sizes[] = {200, 800, 3200, 12800, 51200};
  float *part, *part2;
  double* out;
  unsigned* cnt;
  __bf16* tile;
  CK(hipMalloc(&part, 51200l * C * 4));
  CK(hipMalloc(&part2, 1024l * 2 * C * 4));
  CK(hipMalloc(&out, C * 8));
  CK(hipMalloc(&cnt, 4096 * 4));
  CK(hipMalloc(&tile, 51200l * 16384 * 2));
  CK(hipMemset(cnt, 0, 4096 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int bad = 0;
  for (int G : sizes) {
    // host reference: the per-block partials as the device computes them (variant 0), then the fixed-order sums
    std::vector<float> hp((size_t)G * C);
    hipLaunchKernelGGL(k_probe<0>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile);
    CK(hipMemcpy(hp.data(), part, (size_t)G * C * 4, hipMemcpyDeviceToHost));
    std::vector<double> ref(C, 0.0), ref3(C, 0.0);
    for (int c = 0; c < C; ++c)
      for (int b = 0; b < G; ++b) ref[c] += hp[(size_t)b * C + c];
    const int ng = (G + GS - 1) / GS;
    for (int c = 0; c < C; ++c)
      for (int g = 0; g < ng; ++g) {
        double s = 0.0;
        for (int b = g * GS; b < std::min(G, (g + 1) * GS); ++b) s += hp[(size_t)b * C + c];
        const float hi = (float)s, lo = (float)(s - (double)hi);
        ref3[c] += (double)hi + (double)lo;
      }
    for (int v = 0; v < 4; ++v) {
      const int reps = 20;
      float ms = 0.f;
      for (int it = 0; it < reps + 2; ++it) {
        CK(hipMemset(out, 0, C * 8));
        if (it == 2) CK(hipEventRecord(e0));
        switch (v) {
          case 0:
            hipLaunchKernelGGL(k_probe<0>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile);
            hipLaunchKernelGGL(k_reduce, dim3(1), dim3(256), 0, 0, part, G, out);
            break;
          case 1: hipLaunchKernelGGL(k_probe<1>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile); break;
          case 2: hipLaunchKernelGGL(k_probe<2>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile); break;
          case 3: hipLaunchKernelGGL(k_probe<3>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile); break;
        }
        CK(hipGetLastError());
        std::vector<double> ho(C);
        CK(hipMemcpy(ho.data(), out, C * 8, hipMemcpyDeviceToHost));
        const std::vector<double>& r = v == 3 ? ref3 : ref;
        for (int c = 0; c < C; ++c)
          if (ho[c] != r[c]) {
            if (bad < 10) printf("MISMATCH G=%d v=%d it=%d c=%d got %.17g want %.17g\n", G, v, it, c, ho[c], r[c]);
            ++bad;
          }
      }
      // timing without the per-iteration host copies
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int it = 0; it < reps; ++it) {
        switch (v) {
          case 0:
            hipLaunchKernelGGL(k_probe<0>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile);
            hipLaunchKernelGGL(k_reduce, dim3(1), dim3(256), 0, 0, part, G, out);
            break;
          case 1: hipLaunchKernelGGL(k_probe<1>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile); break;
          case 2: hipLaunchKernelGGL(k_probe<2>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile); break;
          case 3: hipLaunchKernelGGL(k_probe<3>, dim3(G), dim3(256), 0, 0, part, part2, cnt, out, tile); break;
        }
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("G=%6d variant %d: %8.2f us per launch (pair for variant 0)\n", G, v, 1000.f * ms / reps);
    }
  }
  printf(bad ? "FAILED: %d mismatches\n" : "all results exact (%d mismatches)\n", bad);
  return bad ? 1 : 0;
}
