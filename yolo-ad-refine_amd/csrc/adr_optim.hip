// Fused trainer tail (reference engine/trainer.py:580-588 optimizer_step, :753-813 build_optimizer,
// utils/torch_utils.py:521-546 ModelEMA): multi-tensor gradient-norm clip (clip_grad_norm_ max_norm 10),
// SGD with Nesterov momentum and per-group weight decay / lr (torch.optim.SGD semantics), and the EMA of every
// floating-point model state entry, in two launches over a chunk table. Deterministic: the global norm is a
// fixed-order reduction of per-chunk partials, recomputed identically by every block.
#include "adr_common.h"

namespace adr {

struct OptEntry {
  float* p;          // parameter or buffer (fp32)
  float* g;          // gradient (null: no update, e.g. buffers / frozen params); zeroed after use
  float* buf;        // momentum buffer
  float* ema;        // EMA copy (null: none)
  long n;
  int group;         // 0 decay weights, 1 norm weights, 2 biases, 3 buffer / frozen (EMA only)
  int pad;
};

struct OptChunk {
  int entry;
  int pad;
  long start, len;
};

__global__ void __launch_bounds__(256) grad_sqnorm_kernel(const OptEntry* tab, const OptChunk* chunks, float* partial) {
  const OptChunk ck = chunks[blockIdx.x];
  const OptEntry e = tab[ck.entry];
  __shared__ double sh[256];
  double s = 0.0;
  if (e.g && e.group < 3) {
    const long end = ck.start + ck.len;
    for (long i0 = ck.start + threadIdx.x; i0 < end; i0 += 1024) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i0 + 256 * u < end ? e.g[i0 + 256 * u] : 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) s += (double)v[u] * v[u];
    }
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = (float)sh[0];
}

// hyper (device): [lr0, lr1, lr2, wd0, wd1, wd2, momentum, nesterov, first, ema_d] — read from memory so a
// captured graph of the step picks up the per-step schedule; clip coefficient from the partials
__global__ void __launch_bounds__(256) sgd_ema_kernel(const OptEntry* tab, const OptChunk* chunks, int nchunks,
                                                      const float* partial, float max_norm,
                                                      const float* __restrict__ hyper, float* norm_out) {
  const float lr0 = hyper[0], lr1 = hyper[1], lr2 = hyper[2], wd0 = hyper[3], wd1 = hyper[4], wd2 = hyper[5];
  const float momentum = hyper[6], ema_d = hyper[9];
  const int nesterov = hyper[7] != 0.f, first = hyper[8] != 0.f;
  __shared__ double sh[256];
  __shared__ float coef_s;
  double s = 0.0;
  for (int k = threadIdx.x; k < nchunks; k += 256) s += partial[k];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float tn = (float)sqrt(sh[0]);
    float c = max_norm > 0.f ? max_norm / (tn + 1e-6f) : 1.f;
    coef_s = c < 1.f ? c : 1.f;
    if (blockIdx.x == 0 && norm_out) norm_out[0] = tn;
  }
  __syncthreads();
  const float coef = coef_s;
  const OptChunk ck = chunks[blockIdx.x];
  const OptEntry e = tab[ck.entry];
  const float lr = e.group == 0 ? lr0 : (e.group == 1 ? lr1 : lr2);
  const float wd = e.group == 0 ? wd0 : (e.group == 1 ? wd1 : wd2);
  // U elements per thread per round, all loads issued before any store (the four arrays are distinct
  // allocations, but the compiler cannot know that), so a round keeps 4*U loads in flight per lane
  constexpr int U = 4;
  const bool upd = e.g && e.group < 3;
  const long end = ck.start + ck.len;
  for (long i0 = ck.start + threadIdx.x; i0 < end; i0 += 256 * U) {
    float p[U], g[U], b[U], m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + 256 * u;
      const bool in = i < end;
      p[u] = in ? e.p[i] : 0.f;
      g[u] = in && upd ? e.g[i] : 0.f;
      b[u] = in && upd && !first ? e.buf[i] : 0.f;
      m[u] = in && e.ema ? e.ema[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + 256 * u;
      if (i >= end) break;
      float pv = p[u];
      if (upd) {
        float gv = g[u] * coef;
        if (wd != 0.f) gv += wd * pv;
        const float bv = first ? gv : momentum * b[u] + gv;
        e.buf[i] = bv;
        e.g[i] = 0.f;  // optimizer.zero_grad() (trainer.py:586): the arena starts the next accumulation at 0
        const float step = nesterov ? gv + momentum * bv : bv;
        pv -= lr * step;
        e.p[i] = pv;
      }
      if (e.ema) e.ema[i] = ema_d * m[u] + (1.f - ema_d) * pv;
    }
  }
}

// gather scattered tensors into a flat buffer (DDP bucket) or scatter back
__global__ void __launch_bounds__(256) flat_copy_kernel(const OptEntry* tab, const OptChunk* chunks, float* flat,
                                                        const long* offsets, int to_flat) {
  const OptChunk ck = chunks[blockIdx.x];
  const OptEntry e = tab[ck.entry];
  long off = offsets[ck.entry];
  for (long i = ck.start + threadIdx.x; i < ck.start + ck.len; i += 256) {
    if (to_flat) flat[off + i] = e.g ? e.g[i] : e.p[i];
    else e.p[i] = flat[off + i];
  }
}

}  // namespace adr

using namespace adr;

extern "C" int adr_opt_entry_size(void) { return (int)sizeof(OptEntry); }
extern "C" int adr_opt_chunk_size(void) { return (int)sizeof(OptChunk); }

extern "C" int adr_opt_step(const void* tab, const void* chunks, int nchunks, float* partial, float max_norm,
                            const float* hyper, float* norm_out, void* stream) {
  ADR_REQUIRE(nchunks > 0, "opt_step: empty chunk table");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(grad_sqnorm_kernel, dim3(nchunks), dim3(256), 0, st, (const OptEntry*)tab,
                     (const OptChunk*)chunks, partial);
  hipLaunchKernelGGL(sgd_ema_kernel, dim3(nchunks), dim3(256), 0, st, (const OptEntry*)tab, (const OptChunk*)chunks,
                     nchunks, partial, max_norm, hyper, norm_out);
  return check_launch("adr_opt_step");
}

struct F32x16 {
  float v[16];
};
__global__ void set_f32_kernel(float* dst, F32x16 vals, int n) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = vals.v[threadIdx.x];
}

extern "C" int adr_set_f32(float* dst, const float* vals, int n, void* stream) {
  ADR_REQUIRE(n >= 0 && n <= 16, "set_f32: n=%d > 16", n);
  F32x16 v{};
  for (int i = 0; i < n; ++i) v.v[i] = vals[i];
  hipLaunchKernelGGL(set_f32_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dst, v, n);
  return check_launch("adr_set_f32");
}

extern "C" int adr_flat_copy(const void* tab, const void* chunks, int nchunks, float* flat, const int64_t* offsets,
                             int to_flat, void* stream) {
  hipLaunchKernelGGL(flat_copy_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, (const OptEntry*)tab,
                     (const OptChunk*)chunks, flat, (const long*)offsets, to_flat);
  return check_launch("adr_flat_copy");
}
