// AYHead-specific kernels (reference nn/modules/head.py:1049-1252):
//   * modulated deformable im2col / col2im for DyDCNv2 (mmcv ModulatedDeformConv2d semantics, head.py:751-782):
//       offset channel 2k = dy, 2k+1 = dx, mask logit channel 2K+k (sigmoid applied here, head.py:1156);
//       sample (h - pad + i + dy, w - pad + j + dx); value 0 unless -1 < py < H and -1 < px < W; each bilinear
//       corner bounds-checked. The GEMM halves (columns x W, dy x W^T, dy^T x columns) run on the MFMA engine.
//   * tiny per-image gate MLPs on pooled vectors: TaskDecomposition la_conv1/la_conv2 (head.py:633-650) and
//     AdaptiveDynamicTanh importance_gate (block.py:2521-2531), forward + backward.
//   * broadcast fill (the adjoint of a global average pool) and per-pixel scalar multiply (cls_prob gate,
//     head.py:1172).
//   * detect decode for eval: DFL softmax-expectation + dist2bbox(xywh) * stride + sigmoid(cls)
//     (head.py:1181-1204, 1236-1252; block.py:63-81; tal.py:303-327).
#include "adr_common.h"

#include <cstdint>
#include <initializer_list>

namespace adr {

// ---------------- DCNv2 ----------------
// bilinear corner weights and validity for sample point (py, px); corners (y0,x0),(y0,x0+1),(y0+1,x0),(y0+1,x0+1)
__device__ __forceinline__ bool dcn_sample(float py, float px, int H, int W, int& y0, int& x0, float* wts, bool* v) {
  float fy = floorf(py), fx = floorf(px);
  y0 = (int)fy;
  x0 = (int)fx;
  float ly = py - fy, lx = px - fx, hy = 1.f - ly, hx = 1.f - lx;
  bool inside = (py > -1.f) && (px > -1.f) && (py < (float)H) && (px < (float)W);
  v[0] = inside && y0 >= 0 && x0 >= 0;
  v[1] = inside && y0 >= 0 && x0 + 1 <= W - 1;
  v[2] = inside && y0 + 1 <= H - 1 && x0 >= 0;
  v[3] = inside && y0 + 1 <= H - 1 && x0 + 1 <= W - 1;
  wts[0] = v[0] ? hy * hx : 0.f;
  wts[1] = v[1] ? hy * lx : 0.f;
  wts[2] = v[2] ? ly * hx : 0.f;
  wts[3] = v[3] ? ly * lx : 0.f;
  return inside;
}

// cols[pix][t][c] = mask * bilinear(x, p); thread per (pix, tap, channel-vector)
template <typename T>
__global__ void __launch_bounds__(256) dcn_im2col_kernel(const T* x, int xcs, const T* om, int omcs, T* cols, int N,
                                                         int H, int W, int C) {
  constexpr int V = 16 / sizeof(T);
  const int G = C / V;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * H * W * 9 * G;
  if (i >= total) return;
  int g = (int)(i % G);
  long r = i / G;
  int t = (int)(r % 9);
  long pix = r / 9;
  int w = (int)(pix % W);
  long r2 = pix / W;
  int h = (int)(r2 % H);
  int n = (int)(r2 / H);
  const T* o = om + pix * omcs;
  float dy = to_f(o[2 * t]), dx = to_f(o[2 * t + 1]);
  float m = 1.f / (1.f + __expf(-to_f(o[18 + t])));
  float py = (float)(h - 1 + t / 3) + dy, px = (float)(w - 1 + t % 3) + dx;
  int y0, x0;
  float wt[4];
  bool vq[4];
  dcn_sample(py, px, H, W, y0, x0, wt, vq);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  const T* xb = x + (long)n * H * W * xcs + g * V;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (!vq[q]) continue;
    int yy = y0 + (q >> 1), xx = x0 + (q & 1);
    u32x4 v = ld16(xb + ((long)yy * W + xx) * xcs);
    const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int k = 0; k < V; ++k) acc[k] += wt[q] * to_f(e[k]);
  }
  u32x4 ov;
  T* oe = reinterpret_cast<T*>(&ov);
#pragma unroll
  for (int k = 0; k < V; ++k) oe[k] = from_f<T>(acc[k] * m);
  st16(cols + (pix * 9 + t) * C + g * V, ov);
}

// col2im, one kernel, lanes over channels (64-channel contiguous loads and adds).
// A wave walks a vertical strip of sampling pixels (column w, rows h0..h0+DCN_SL-1). The bilinear-corner
// contributions of its current pixel land, for offsets within +-2 pixels, inside a 7x7 cell neighbourhood,
// which the wave keeps as a PRIVATE rolling window in LDS (7 rows x 7 columns x 64 channels fp32, ring-indexed
// by row): adds are plain ds_read/ds_write read-modify-writes in program order, no LDS atomics (which run ~30x
// slower than plain LDS traffic on this part). When the strip advances a row, the row leaving the window is
// flushed to dx32 with one global float atomic per (cell, channel). Per sampling pixel that is ~7 global
// atomics per channel instead of 36 (9 taps x 4 corners) for a per-corner global scatter. Corners beyond the
// window go straight to dx32. The same pass computes d_offset / d_mask_logit from the corner values (DPP wave
// sums). All loads of a tap group are unconditional at clamped addresses (masked afterwards), so they are in
// flight together instead of each waiting behind a branch.
__device__ __forceinline__ float ld_coh(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_coh(const __bf16* p) {
  const unsigned short b = __hip_atomic_load(reinterpret_cast<const unsigned short*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
  return __uint_as_float((unsigned)b << 16);
}
__device__ __forceinline__ void st_coh(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(__bf16* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned short*>(p), __builtin_bit_cast(unsigned short, (__bf16)v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int DCN_SL = 10;             // strip length (rows per wave; 10 beat 20 and 40 by 0.1 / 0.2 ms per step)
constexpr int DCN_WIN = 7;             // window rows / columns (pixel +-3)
constexpr int DCN_CC = 64;             // channels per pass (= lanes)
constexpr int DCN_WPB = 4;             // waves per block

template <typename T>
__global__ void __launch_bounds__(256) dcn_col2im_kernel(const T* x, int xcs, const T* om, int omcs, const T* dcols,
                                                         float* dx32, T* dom, int domcs, int N, int H, int W, int C) {
  // window cells 0..48 (ring row slot * 7 + column) plus one scratch cell (49) that absorbs the adds of corners
  // outside the window or out of the image, so every corner update is the same unconditional LDS read-add-write
  constexpr int NCELL = DCN_WIN * DCN_WIN, SCRATCH = NCELL;
  __shared__ float winbuf[DCN_WPB][(NCELL + 1) * DCN_CC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* win = winbuf[wave];
  const int nstrip = (H + DCN_SL - 1) / DCN_SL;
  const long sid = (long)blockIdx.x * DCN_WPB + wave;  // (n, strip, w) with w fastest
  if (sid >= (long)N * nstrip * W) return;
  const int w = (int)(sid % W);
  const long r = sid / W;
  const int strip = (int)(r % nstrip), n = (int)(r / nstrip);
  const int hb = strip * DCN_SL, he = min(H, hb + DCN_SL);
  const T* xb = x + (long)n * H * W * xcs;  // per-image bases; offsets inside an image are 32-bit
  float* dxb = dx32 ? dx32 + (long)n * H * W * C : nullptr;  // null: offsets / mask only (deterministic dx below)
  const int wx0 = w - DCN_WIN / 2;  // window column 0
  auto flush_row = [&](int y, int slot, int c) {  // add window row y (ring slot) to dx32 and clear it
    float* row = win + slot * DCN_WIN * DCN_CC;
    const bool yok = y >= 0 && y < H && c < C;
#pragma unroll
    for (int j = 0; j < DCN_WIN; ++j) {
      const float v = row[j * DCN_CC + lane];
      const int xx = wx0 + j;
      if (dxb && yok && xx >= 0 && xx < W && v != 0.f) unsafeAtomicAdd(dxb + (y * W + xx) * C + c, v);
      row[j * DCN_CC + lane] = 0.f;
    }
  };
  for (int c0 = 0; c0 < C; c0 += DCN_CC) {
    const int c = c0 + lane;
    const int cc = min(c, C - 1);
    for (int i = 0; i <= NCELL; ++i) win[i * DCN_CC + lane] = 0.f;
    int hs = hb % DCN_WIN;  // ring slot of row h
    for (int h = hb; h < he; ++h, hs = hs + 1 == DCN_WIN ? 0 : hs + 1) {
      if (h > hb) {  // row h-4 leaves the window (its slot becomes row h+3)
        const int fs = hs - 1 - DCN_WIN / 2;
        flush_row(h - 1 - DCN_WIN / 2, fs < 0 ? fs + DCN_WIN : fs, c);
      }
      const int pix = (n * H + h) * W + w;
      const float omv = lane < 27 ? to_f(om[(long)pix * omcs + lane]) : 0.f;
      T* d = dom + (long)pix * domcs;
      const T* gcol = dcols + (long)pix * 9 * C + cc;
#pragma unroll 1
      for (int tg = 0; tg < 3; ++tg) {
        int y0[3], x0[3];
        float wt[3][4], ly[3], lx[3], m[3], g[3], xv[3][4];
        bool ok[3][4];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int t = tg * 3 + u;
          const float oy = lane_f(omv, 2 * t), ox = lane_f(omv, 2 * t + 1);
          m[u] = 1.f / (1.f + __expf(-lane_f(omv, 18 + t)));
          const float py = (float)(h - 1 + tg) + oy, px = (float)(w - 1 + u) + ox;
          dcn_sample(py, px, H, W, y0[u], x0[u], wt[u], ok[u]);
          ly[u] = py - floorf(py);
          lx[u] = px - floorf(px);
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          g[u] = to_f(gcol[(tg * 3 + u) * C]);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int yy = min(max(y0[u] + (q >> 1), 0), H - 1), xx = min(max(x0[u] + (q & 1), 0), W - 1);
            const float v = to_f(xb[(yy * W + xx) * xcs + cc]);
            xv[u][q] = ok[u][q] ? v : 0.f;
          }
        }
        if (c >= C) g[0] = g[1] = g[2] = 0.f;
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int t = tg * 3 + u;
          // d weight / d py and d px for each corner (mmcv dmcn_get_coordinate_weight)
          const float dwy[4] = {-(1.f - lx[u]), -lx[u], (1.f - lx[u]), lx[u]};
          const float dwx[4] = {-(1.f - ly[u]), (1.f - ly[u]), -ly[u], ly[u]};
          float val = 0.f, sy = 0.f, sx = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            val += wt[u][q] * xv[u][q];
            sy += dwy[q] * xv[u][q];
            sx += dwx[q] * xv[u][q];
          }
          const float gm = g[u] * m[u];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            // wt is 0 for an invalid corner; the cell choice is wave-uniform (pixel and tap only)
            const int yy = y0[u] + (q >> 1), xx = x0[u] + (q & 1);
            const int dyw = yy - h, dxw = xx - wx0;
            const bool inwin = dyw >= -(DCN_WIN / 2) && dyw <= DCN_WIN / 2 && dxw >= 0 && dxw < DCN_WIN;
            int slot = hs + dyw;
            slot = slot < 0 ? slot + DCN_WIN : (slot >= DCN_WIN ? slot - DCN_WIN : slot);
            const int cell = (ok[u][q] && inwin) ? slot * DCN_WIN + dxw : SCRATCH;
            win[cell * DCN_CC + lane] += gm * wt[u][q];
            if (dxb && ok[u][q] && !inwin && c < C) unsafeAtomicAdd(dxb + (yy * W + xx) * C + c, gm * wt[u][q]);
          }
          const float spy = wave_sum_dpp(gm * sy), spx = wave_sum_dpp(gm * sx), smk = wave_sum_dpp(g[u] * val);
          if (lane == 0) {
            // partial sums carried across channel chunks through dom itself: device-coherent loads / stores, so
            // the read-back of the previous chunk's value cannot hit a stale vector-L1 line (C >= 256 with far
            // corners lost updates that way)
            const bool first = c0 == 0, last = c0 + DCN_CC >= C;
            const float a = first ? 0.f : ld_coh(d + 2 * t), b = first ? 0.f : ld_coh(d + 2 * t + 1);
            st_coh(d + 2 * t, a + spy);
            st_coh(d + 2 * t + 1, b + spx);
            // d mask logit: raw channel sum across chunks, times sigmoid'(logit) on the last chunk
            const float e = (first ? 0.f : ld_coh(d + 18 + t)) + smk;
            st_coh(d + 18 + t, last ? e * m[u] * (1.f - m[u]) : e);
          }
        }
      }
    }
    {  // flush the rows still in the window: he-1-3 .. he-1+3, slots relative to the last row's slot
      const int ls = (he - 1) % DCN_WIN;
      for (int dy = -(DCN_WIN / 2); dy <= DCN_WIN / 2; ++dy) {
        int sl = ls + dy;
        sl = sl < 0 ? sl + DCN_WIN : (sl >= DCN_WIN ? sl - DCN_WIN : sl);
        flush_row(he - 1 + dy, sl, c);
      }
    }
  }
}

// Deterministic input gradient (parity mode): one thread per (image, channel) walks every (pixel, tap, corner)
// of its image in a fixed order and accumulates into its own (n, :, :, c) plane — plain read-modify-writes, no
// atomics, so the fp32 result is bitwise repeatable. The summation order equals the reference
// CPU loop's for one channel (pixel-major, taps in order, corners in mmcv's order).
template <typename T>
__global__ void __launch_bounds__(64) dcn_dx_serial_kernel(const T* om, int omcs, const T* dcols, float* dx32, int N,
                                                           int H, int W, int C) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)N * C) return;
  const int n = (int)(id / C), c = (int)(id % C);
  float* d = dx32 + (long)n * H * W * C + c;
  for (int h = 0; h < H; ++h)
    for (int w = 0; w < W; ++w) {
      const long pix = ((long)n * H + h) * W + w;
      const T* o = om + pix * omcs;
      for (int t = 0; t < 9; ++t) {
        const float m = 1.f / (1.f + __expf(-to_f(o[18 + t])));
        const float py = (float)(h - 1 + t / 3) + to_f(o[2 * t]), px = (float)(w - 1 + t % 3) + to_f(o[2 * t + 1]);
        int y0, x0;
        float wt[4];
        bool ok[4];
        dcn_sample(py, px, H, W, y0, x0, wt, ok);
        const float gm = to_f(dcols[(pix * 9 + t) * C + c]) * m;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (ok[q]) d[((long)(y0 + (q >> 1)) * W + x0 + (q & 1)) * C] += gm * wt[q];
      }
    }
}

// W (Cout, C, 3, 3) fp32 -> W^T as a 1x1-conv weight [(t*C + c)][co] in dtype
template <typename T>
__global__ void dcn_wT_kernel(const float* w, T* out, int Cout, int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)Cout * C * 9;
  if (i >= total) return;
  int co = (int)(i % Cout);
  long r = i / Cout;  // r = t*C + c
  int c = (int)(r % C);
  int t = (int)(r / C);
  out[i] = from_f<T>(w[((long)co * C + c) * 9 + t]);
}

// ---------------- tiny gate MLP: out = act2(W2 act1(W1 (in*scale) + b1) + b2) per image ----------------
// act: 0 none, 3 relu, 4 sigmoid, 6 softmax (over the output vector)
__device__ __forceinline__ float gact(int a, float v) {
  if (a == 3) return v > 0.f ? v : 0.f;
  if (a == 4) return 1.f / (1.f + __expf(-v));
  return v;
}

__global__ void __launch_bounds__(256) gate_mlp_kernel(const float* in, float in_scale, int Cin, const float* W1,
                                                       const float* b1, int H1, int act1, const float* W2,
                                                       const float* b2, int H2, int act2, float* hidden, float* out) {
  int n = blockIdx.x;
  extern __shared__ float sm[];
  float* xin = sm;            // Cin
  float* hid = sm + Cin;      // H1
  float* o = sm + Cin + H1;   // H2
  for (int c = threadIdx.x; c < Cin; c += 256) xin[c] = in[(long)n * Cin + c] * in_scale;
  __syncthreads();
  for (int j = threadIdx.x; j < H1; j += 256) {
    float s = b1 ? b1[j] : 0.f;
    for (int c = 0; c < Cin; ++c) s += W1[(long)j * Cin + c] * xin[c];
    hid[j] = gact(act1, s);
    hidden[(long)n * H1 + j] = hid[j];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < H2; j += 256) {
    float s = b2 ? b2[j] : 0.f;
    for (int c = 0; c < H1; ++c) s += W2[(long)j * H1 + c] * hid[c];
    o[j] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (act2 == 6) {
      float mx = -INFINITY;
      for (int j = 0; j < H2; ++j) mx = fmaxf(mx, o[j]);
      float z = 0.f;
      for (int j = 0; j < H2; ++j) z += __expf(o[j] - mx);
      for (int j = 0; j < H2; ++j) out[(long)n * H2 + j] = __expf(o[j] - mx) / z;
    } else {
      for (int j = 0; j < H2; ++j) out[(long)n * H2 + j] = gact(act2, o[j]);
    }
  }
}

// backward: given dout (N,H2) -> din (N,Cin) (times in_scale) and dW1/db1/dW2/db2 summed over images.
// Every block recomputes the small dz2 / dh stages in LDS; the output phases (din, dW1, dW2, db1, db2) are spread
// over the grid, one thread per output, image sums in a fixed order (deterministic).
// accumulate: weight/bias gradients are added to the destination (the trainer's gradient arena).
__global__ void __launch_bounds__(256) gate_mlp_bwd_kernel(const float* in, float in_scale, int Cin, const float* W1,
                                                           int H1, int act1, const float* W2, int H2, int act2,
                                                           const float* hidden, const float* out, const float* dout,
                                                           int N, float* din, float* dW1, float* db1, float* dW2,
                                                           float* db2, int accumulate) {
  extern __shared__ float sm[];
  float* dz2 = sm;           // [N][H2]
  float* dh = sm + N * H2;   // [N][H1]
  const int tid = threadIdx.x;
  for (int n = tid; n < N; n += 256) {
    const float* o = out + (long)n * H2;
    const float* d = dout + (long)n * H2;
    float dot = 0.f;
    if (act2 == 6)
      for (int j = 0; j < H2; ++j) dot += d[j] * o[j];
    for (int j = 0; j < H2; ++j)
      dz2[n * H2 + j] = act2 == 6 ? o[j] * (d[j] - dot) : (act2 == 4 ? d[j] * o[j] * (1.f - o[j]) : d[j]);
  }
  __syncthreads();
  for (int i = tid; i < N * H1; i += 256) {
    const int n = i / H1, c = i % H1;
    float s = 0.f;
    for (int j = 0; j < H2; ++j) s += W2[(long)j * H1 + c] * dz2[n * H2 + j];
    const float hv = hidden[i];
    dh[i] = (act1 == 3) ? (hv > 0.f ? s : 0.f) : (act1 == 4 ? s * hv * (1.f - hv) : s);
  }
  __syncthreads();
  // the output phases are spread over the grid (every block recomputed dz2 / dh above, a few k MACs)
  const int gt = blockIdx.x * 256 + tid, gs = gridDim.x * 256;
  for (int i = gt; i < N * Cin; i += gs) {
    const int n = i / Cin, c = i % Cin;
    float s = 0.f;
    for (int j = 0; j < H1; ++j) s += W1[(long)j * Cin + c] * dh[n * H1 + j];
    din[i] = s * in_scale;
  }
  // dW1: each block owns a contiguous run of OB outputs, its threads split the image sum P ways (part p takes
  // images p, p + P, ...), partial sums combined in part order through LDS (deterministic)
  {
    __shared__ float red[256];
    const int O = H1 * Cin, OB = (O + gridDim.x - 1) / gridDim.x;
    for (int o0 = blockIdx.x * OB; o0 < min(O, (blockIdx.x + 1) * OB); o0 += 256) {
      const int ob = min(256, min(O, (blockIdx.x + 1) * OB) - o0), P = 256 / ob;
      const int ol = tid % ob, part = tid / ob, i = o0 + ol;
      float s = 0.f;
      if (part < P) {
        const int j = i / Cin, c = i % Cin;
        for (int n = part; n < N; n += P) s += dh[n * H1 + j] * in[(long)n * Cin + c];
      }
      red[tid] = s;
      __syncthreads();
      if (tid < ob) {
        float t = 0.f;
        for (int q = 0; q < P; ++q) t += red[q * ob + tid];
        t *= in_scale;
        dW1[i] = accumulate ? dW1[i] + t : t;
      }
      __syncthreads();
    }
  }
  for (int i = gt; i < H2 * H1; i += gs) {
    const int j = i / H1, c = i % H1;
    float s = 0.f;
    for (int n = 0; n < N; ++n) s += dz2[n * H2 + j] * hidden[(long)n * H1 + c];
    dW2[i] = accumulate ? dW2[i] + s : s;
  }
  if (db1)
    for (int j = gt; j < H1; j += gs) {
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += dh[n * H1 + j];
      db1[j] = accumulate ? db1[j] + s : s;
    }
  if (db2)
    for (int j = gt; j < H2; j += gs) {
      float s = 0.f;
      for (int n = 0; n < N; ++n) s += dz2[n * H2 + j];
      db2[j] = accumulate ? db2[j] + s : s;
    }
}

// o[n, pix, c] (+)= g[n*gns + c*gcs] * s
template <typename T>
__global__ void __launch_bounds__(256) bcast_fill_kernel(const float* g, int gns, int gcs, float s, T* o, int ocs,
                                                         long npix, int HW, int C, int accumulate) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = npix * C;
  if (i >= total) return;
  int c = (int)(i % C);
  long pix = i / C;
  int n = (int)(pix / HW);
  float v = g[(long)n * gns + (long)c * gcs] * s;
  T* q = o + pix * ocs + c;
  *q = from_f<T>(accumulate ? to_f(*q) + v : v);
}

// bf16, 8 channels per thread (one 16-byte load / store; 32-bit index math): the same per-element v = g * s and
// optional accumulate as bcast_fill_kernel (was 80 us, 0.9 TB/s, on the head's 1344 x 400 x 64 gradient fill)
__global__ void __launch_bounds__(256) bcast_fill8_kernel(const float* g, int gns, int gcs, float s, __bf16* o, int ocs,
                                                          unsigned npix, unsigned HW, unsigned C8, int accumulate) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i >= npix * C8) return;
  const unsigned pix = i / C8, c = (i - pix * C8) * 8u, n = pix / HW;
  __bf16* q = o + (size_t)pix * ocs + c;
  u32x4 prev = {0u, 0u, 0u, 0u};
  if (accumulate) prev = ld16(q);
  const __bf16* pe = reinterpret_cast<const __bf16*>(&prev);
  u32x4 out;
  __bf16* oe = reinterpret_cast<__bf16*>(&out);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float v = g[(long)n * gns + (long)(c + e) * gcs] * s;
    oe[e] = from_f<__bf16>(accumulate ? to_f(pe[e]) + v : v);
  }
  st16(q, out);
}

// o = x * p[pix] (p: channel 0 of a view) ; bwd: dx = dout*p ; dp[pix] = sum_c dout*x
template <typename T>
__global__ void __launch_bounds__(256) mul_pixel_kernel(const T* x, int xcs, const T* p, int pcs, T* o, int ocs,
                                                        long npix, int C) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * C) return;
  int c = (int)(i % C);
  long pix = i / C;
  o[pix * ocs + c] = from_f<T>(to_f(x[pix * xcs + c]) * to_f(p[pix * pcs]));
}

template <typename T>
__global__ void __launch_bounds__(256) mul_pixel_bwd_kernel(const T* x, int xcs, const T* p, int pcs, const T* dout,
                                                            int dcs, T* dx, int ocs, T* dp, int dpcs, long npix, int C) {
  long pix = (long)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  int lane = threadIdx.x & 63;
  if (pix >= npix) return;
  float pv = to_f(p[pix * pcs]);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) {
    float d = to_f(dout[pix * dcs + c]);
    s += d * to_f(x[pix * xcs + c]);
    dx[pix * ocs + c] = from_f<T>(d * pv);
  }
  s = wave_sum(s);
  if (lane < dpcs) dp[pix * dpcs + lane] = from_f<T>(lane == 0 ? s : 0.f);  // the whole dp row (zeros after channel 0)
}

// 16-byte vector versions (C / V lanes per pixel, C / V a power of two <= 64; the pixel's lanes are adjacent in a wave)
template <typename T>
__global__ void __launch_bounds__(256) mul_pixel_vec_kernel(const T* x, int xcs, const T* p, int pcs, T* o, int ocs,
                                                            long npix, int C) {
  constexpr int V = VecIO<T>::V;
  const PixLanes L(C / V);
  if (!L.active) return;
  const int c0 = L.cg * V;
  for (long pix = (long)blockIdx.x * L.rpb + L.r0; pix < npix; pix += (long)gridDim.x * L.rpb) {
    float fx[V], fo[V];
    VecIO<T>::load(x + pix * xcs + c0, fx);
    const float pv = to_f(p[pix * pcs]);
#pragma unroll
    for (int k = 0; k < V; ++k) fo[k] = fx[k] * pv;
    VecIO<T>::store(o + pix * ocs + c0, fo);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) mul_pixel_bwd_vec_kernel(const T* x, int xcs, const T* p, int pcs,
                                                                const T* dout, int dcs, T* dx, int ocs, T* dp, int dpcs,
                                                                long npix, int C) {
  constexpr int V = VecIO<T>::V;
  const int G = C / V;
  const PixLanes L(G);
  if (!L.active) return;
  const int c0 = L.cg * V;
  for (long pix = (long)blockIdx.x * L.rpb + L.r0; pix < npix; pix += (long)gridDim.x * L.rpb) {
    float fx[V], fd[V], fo[V];
    VecIO<T>::load(x + pix * xcs + c0, fx);
    VecIO<T>::load(dout + pix * dcs + c0, fd);
    const float pv = to_f(p[pix * pcs]);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      fo[k] = fd[k] * pv;
      s += fd[k] * fx[k];
    }
    VecIO<T>::store(dx + pix * ocs + c0, fo);
    for (int off = G >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (L.cg < dpcs) dp[pix * dpcs + L.cg] = from_f<T>(L.cg == 0 ? s : 0.f);
    for (int c = L.cg + G; c < dpcs; c += G) dp[pix * dpcs + c] = from_f<T>(0.f);
  }
}

static bool mul_pixel_vec_ok(int dtype, long npix, int C, std::initializer_list<long> strides,
                             std::initializer_list<const void*> ptrs) {
  const int v = dtype == ADR_BF16 ? 8 : 4;
  const int G = C / v;
  if (C % v || G > 64 || (G & (G - 1))) return false;
  for (long st : strides)
    if (st % v) return false;
  for (const void* q : ptrs)
    if ((uintptr_t)q % 16) return false;
  return npix > 0;
}

static int mul_pixel_grid(long npix, int G) {
  long b = (npix + 256 / G - 1) / (256 / G);
  return (int)(b > 32768 ? 32768 : b < 1 ? 1 : b);
}

// ---------------- eval decode ----------------
// feats: nl NHWC tensors (B, no, H_i, W_i) of dtype T; y (B, 4+nc, A) fp32
// One block per 64 (image, anchor) rows: the rows (4*reg_max + nc channels each, NHWC) are staged into LDS with
// coalesced reads (consecutive threads read consecutive channels of a row); then 4 threads per anchor (one per box
// side) take the DFL expectation, and the box / class outputs are written channel-major with 64 consecutive anchors
// per store instruction.
constexpr int DEC_ROWS = 64;
constexpr int DEC_MAXCH = 4 * 16 + 128;  // reg_max 16, up to 128 classes

template <typename T>
__global__ void __launch_bounds__(256) detect_decode_kernel(const T* f0, const T* f1, const T* f2, int cs0, int cs1,
                                                            int cs2, int H0, int W0, int H1, int W1, int H2, int W2,
                                                            float s0, float s1, float s2, int B, int nc, int reg_max,
                                                            float* y) {
  __shared__ float rows[DEC_ROWS][DEC_MAXCH + 1];
  __shared__ float dist[4][DEC_ROWS];
  const int A = H0 * W0 + H1 * W1 + H2 * W2;
  const int no = 4 * reg_max + nc;
  const long i0 = (long)blockIdx.x * DEC_ROWS;
  const long total = (long)B * A;
  auto src = [&](long i, int& loc, int& W, float& st) -> const T* {
    const int a = (int)(i % A), b = (int)(i / A);
    const T* f;
    int cs, HW;
    if (a < H0 * W0) { f = f0; cs = cs0; W = W0; HW = H0 * W0; loc = a; st = s0; }
    else if (a < H0 * W0 + H1 * W1) { f = f1; cs = cs1; W = W1; HW = H1 * W1; loc = a - H0 * W0; st = s1; }
    else { f = f2; cs = cs2; W = W2; HW = H2 * W2; loc = a - H0 * W0 - H1 * W1; st = s2; }
    return f + ((long)b * HW + loc) * cs;
  };
  for (int e = threadIdx.x; e < DEC_ROWS * no; e += 256) {
    const int r = e / no, c = e - r * no;
    const long i = i0 + r;
    if (i < total) {
      int loc, W;
      float st;
      rows[r][c] = to_f(src(i, loc, W, st)[c]);
    }
  }
  __syncthreads();
  const int r = threadIdx.x & (DEC_ROWS - 1), k = threadIdx.x >> 6;  // anchor row, box side
  const long i = i0 + r;
  const bool live = i < total;
  if (live) {
    float mx = -INFINITY;
    for (int j = 0; j < reg_max; ++j) mx = fmaxf(mx, rows[r][k * reg_max + j]);
    float z = 0.f, ev = 0.f;
    for (int j = 0; j < reg_max; ++j) {
      const float ex = __expf(rows[r][k * reg_max + j] - mx);
      z += ex;
      ev += ex * (float)j;
    }
    dist[k][r] = ev / z;
  }
  __syncthreads();
  if (!live) return;
  const int a = (int)(i % A), b = (int)(i / A);
  int loc, W;
  float st;
  src(i, loc, W, st);
  const float ax = (float)(loc % W) + 0.5f, ay = (float)(loc / W) + 0.5f;
  const float x1 = ax - dist[0][r], y1 = ay - dist[1][r], x2 = ax + dist[2][r], y2 = ay + dist[3][r];
  const long base = (long)b * (4 + nc) * A + a;
  const float box = k == 0 ? (x1 + x2) * 0.5f * st : k == 1 ? (y1 + y2) * 0.5f * st : k == 2 ? (x2 - x1) * st
                                                                                             : (y2 - y1) * st;
  y[base + (long)k * A] = box;
  for (int c = k; c < nc; c += 4) y[base + (long)(4 + c) * A] = 1.f / (1.f + __expf(-rows[r][4 * reg_max + c]));
}

}  // namespace adr

using namespace adr;

extern "C" int adr_dcn_im2col(int dtype, const void* x, int xcs, const void* om, int omcs, void* cols, int N, int H,
                              int W, int C, void* stream) {
  int v = dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(C % v == 0 && xcs % v == 0, "dcn_im2col: C=%d", C);
  ADR_REQUIRE(omcs >= 27, "dcn_im2col: offset/mask tensor needs >= 27 channels");
  long total = (long)N * H * W * 9 * (C / v);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(dcn_im2col_kernel<__bf16>, dim3(cdiv(total, 256)), dim3(256), 0, st, (const __bf16*)x, xcs,
                       (const __bf16*)om, omcs, (__bf16*)cols, N, H, W, C);
  else
    hipLaunchKernelGGL(dcn_im2col_kernel<float>, dim3(cdiv(total, 256)), dim3(256), 0, st, (const float*)x, xcs,
                       (const float*)om, omcs, (float*)cols, N, H, W, C);
  return check_launch("adr_dcn_im2col");
}

extern "C" int adr_dcn_col2im(int dtype, const void* x, int xcs, const void* om, int omcs, const void* dcols,
                              float* dx32, void* dom, int domcs, int N, int H, int W, int C, int deterministic,
                              void* stream) {
  ADR_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && omcs >= 27 && domcs >= 27, "dcn_col2im: bad geometry");
  const long waves = (long)N * cdiv(H, DCN_SL) * W;
  ADR_REQUIRE(waves / DCN_WPB < (1l << 31), "dcn_col2im: grid too large");
  hipStream_t st = (hipStream_t)stream;
  float* dxa = deterministic ? nullptr : dx32;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(dcn_col2im_kernel<__bf16>, dim3(cdiv(waves, DCN_WPB)), dim3(64 * DCN_WPB), 0, st,
                       (const __bf16*)x, xcs, (const __bf16*)om, omcs, (const __bf16*)dcols, dxa, (__bf16*)dom, domcs,
                       N, H, W, C);
  else
    hipLaunchKernelGGL(dcn_col2im_kernel<float>, dim3(cdiv(waves, DCN_WPB)), dim3(64 * DCN_WPB), 0, st,
                       (const float*)x, xcs, (const float*)om, omcs, (const float*)dcols, dxa, (float*)dom, domcs, N,
                       H, W, C);
  if (deterministic) {
    const long nc = (long)N * C;
    if (dtype == ADR_BF16)
      hipLaunchKernelGGL(dcn_dx_serial_kernel<__bf16>, dim3(cdiv(nc, 64)), dim3(64), 0, st, (const __bf16*)om, omcs,
                         (const __bf16*)dcols, dx32, N, H, W, C);
    else
      hipLaunchKernelGGL(dcn_dx_serial_kernel<float>, dim3(cdiv(nc, 64)), dim3(64), 0, st, (const float*)om, omcs,
                         (const float*)dcols, dx32, N, H, W, C);
  }
  return check_launch("adr_dcn_col2im");
}

extern "C" int adr_dcn_weight_t(int dtype, const float* w, void* out, int Cout, int C, void* stream) {
  long total = (long)Cout * C * 9;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(dcn_wT_kernel<__bf16>, dim3(cdiv(total, 256)), dim3(256), 0, st, w, (__bf16*)out, Cout, C);
  else
    hipLaunchKernelGGL(dcn_wT_kernel<float>, dim3(cdiv(total, 256)), dim3(256), 0, st, w, (float*)out, Cout, C);
  return check_launch("adr_dcn_weight_t");
}

extern "C" int adr_gate_mlp(const float* in, float in_scale, int N, int Cin, const float* W1, const float* b1, int H1,
                            int act1, const float* W2, const float* b2, int H2, int act2, float* hidden, float* out,
                            void* stream) {
  size_t sm = (Cin + H1 + H2) * sizeof(float);
  hipLaunchKernelGGL(gate_mlp_kernel, dim3(N), dim3(256), sm, (hipStream_t)stream, in, in_scale, Cin, W1, b1, H1, act1,
                     W2, b2, H2, act2, hidden, out);
  return check_launch("adr_gate_mlp");
}

extern "C" int adr_gate_mlp_bwd(const float* in, float in_scale, int N, int Cin, const float* W1, int H1, int act1,
                                const float* W2, int H2, int act2, const float* hidden, const float* out,
                                const float* dout, float* din, float* dW1, float* db1, float* dW2, float* db2,
                                int accumulate, void* stream) {
  size_t sm = (size_t)N * (H1 + H2) * sizeof(float);
  ADR_REQUIRE(sm <= 64 * 1024, "gate_mlp_bwd: N=%d H1=%d H2=%d exceed the LDS budget", N, H1, H2);
  hipLaunchKernelGGL(gate_mlp_bwd_kernel, dim3(64), dim3(256), sm, (hipStream_t)stream, in, in_scale, Cin, W1, H1, act1,
                     W2, H2, act2, hidden, out, dout, N, din, dW1, db1, dW2, db2, accumulate);
  return check_launch("adr_gate_mlp_bwd");
}

extern "C" int adr_bcast_fill(int dtype, const float* g, int gns, int gcs, float s, void* o, int ocs, int N, int HW,
                              int C, int accumulate, void* stream) {
  long npix = (long)N * HW;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16 && C % 8 == 0 && ocs % 8 == 0 && ((uintptr_t)o & 15) == 0 && npix * (C / 8) < (1l << 31)) {
    hipLaunchKernelGGL(bcast_fill8_kernel, dim3(cdiv(npix * (C / 8), 256)), dim3(256), 0, st, g, gns, gcs, s,
                       (__bf16*)o, ocs, (unsigned)npix, (unsigned)HW, (unsigned)(C / 8), accumulate);
    return check_launch("adr_bcast_fill");
  }
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(bcast_fill_kernel<__bf16>, dim3(cdiv(npix * C, 256)), dim3(256), 0, st, g, gns, gcs, s,
                       (__bf16*)o, ocs, npix, HW, C, accumulate);
  else
    hipLaunchKernelGGL(bcast_fill_kernel<float>, dim3(cdiv(npix * C, 256)), dim3(256), 0, st, g, gns, gcs, s,
                       (float*)o, ocs, npix, HW, C, accumulate);
  return check_launch("adr_bcast_fill");
}

extern "C" int adr_mul_pixel(int dtype, const void* x, int xcs, const void* p, int pcs, void* o, int ocs, long npix,
                             int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (mul_pixel_vec_ok(dtype, npix, C, {xcs, ocs}, {x, o})) {
    const int v = dtype == ADR_BF16 ? 8 : 4, g = mul_pixel_grid(npix, C / v);
    if (dtype == ADR_BF16)
      hipLaunchKernelGGL(mul_pixel_vec_kernel<__bf16>, dim3(g), dim3(256), 0, st, (const __bf16*)x, xcs,
                         (const __bf16*)p, pcs, (__bf16*)o, ocs, npix, C);
    else
      hipLaunchKernelGGL(mul_pixel_vec_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, xcs,
                         (const float*)p, pcs, (float*)o, ocs, npix, C);
    return check_launch("adr_mul_pixel");
  }
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(mul_pixel_kernel<__bf16>, dim3(cdiv(npix * C, 256)), dim3(256), 0, st, (const __bf16*)x, xcs,
                       (const __bf16*)p, pcs, (__bf16*)o, ocs, npix, C);
  else
    hipLaunchKernelGGL(mul_pixel_kernel<float>, dim3(cdiv(npix * C, 256)), dim3(256), 0, st, (const float*)x, xcs,
                       (const float*)p, pcs, (float*)o, ocs, npix, C);
  return check_launch("adr_mul_pixel");
}

extern "C" int adr_mul_pixel_bwd(int dtype, const void* x, int xcs, const void* p, int pcs, const void* dout, int dcs,
                                 void* dx, int ocs, void* dp, int dpcs, long npix, int C, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  ADR_REQUIRE(dpcs >= 1 && dpcs <= 64, "mul_pixel_bwd: dp channel stride %d (the whole row is written)", dpcs);
  if (mul_pixel_vec_ok(dtype, npix, C, {xcs, dcs, ocs}, {x, dout, dx})) {
    const int v = dtype == ADR_BF16 ? 8 : 4, gv = mul_pixel_grid(npix, C / v);
    if (dtype == ADR_BF16)
      hipLaunchKernelGGL(mul_pixel_bwd_vec_kernel<__bf16>, dim3(gv), dim3(256), 0, st, (const __bf16*)x, xcs,
                         (const __bf16*)p, pcs, (const __bf16*)dout, dcs, (__bf16*)dx, ocs, (__bf16*)dp, dpcs, npix, C);
    else
      hipLaunchKernelGGL(mul_pixel_bwd_vec_kernel<float>, dim3(gv), dim3(256), 0, st, (const float*)x, xcs,
                         (const float*)p, pcs, (const float*)dout, dcs, (float*)dx, ocs, (float*)dp, dpcs, npix, C);
    return check_launch("adr_mul_pixel_bwd");
  }
  dim3 g(cdiv(npix, 4));
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(mul_pixel_bwd_kernel<__bf16>, g, dim3(256), 0, st, (const __bf16*)x, xcs, (const __bf16*)p, pcs,
                       (const __bf16*)dout, dcs, (__bf16*)dx, ocs, (__bf16*)dp, dpcs, npix, C);
  else
    hipLaunchKernelGGL(mul_pixel_bwd_kernel<float>, g, dim3(256), 0, st, (const float*)x, xcs, (const float*)p, pcs,
                       (const float*)dout, dcs, (float*)dx, ocs, (float*)dp, dpcs, npix, C);
  return check_launch("adr_mul_pixel_bwd");
}

extern "C" int adr_detect_decode(int dtype, const void* f0, const void* f1, const void* f2, int cs0, int cs1, int cs2,
                                 int H0, int W0, int H1, int W1, int H2, int W2, float s0, float s1, float s2, int B,
                                 int nc, int reg_max, float* y, void* stream) {
  long total = (long)B * (H0 * W0 + H1 * W1 + H2 * W2);
  ADR_REQUIRE(reg_max >= 1 && 4 * reg_max + nc <= DEC_MAXCH, "detect_decode: 4*reg_max + nc = %d > %d",
              4 * reg_max + nc, DEC_MAXCH);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ADR_BF16)
    hipLaunchKernelGGL(detect_decode_kernel<__bf16>, dim3(cdiv(total, DEC_ROWS)), dim3(256), 0, st, (const __bf16*)f0,
                       (const __bf16*)f1, (const __bf16*)f2, cs0, cs1, cs2, H0, W0, H1, W1, H2, W2, s0, s1, s2, B, nc,
                       reg_max, y);
  else
    hipLaunchKernelGGL(detect_decode_kernel<float>, dim3(cdiv(total, DEC_ROWS)), dim3(256), 0, st, (const float*)f0,
                       (const float*)f1, (const float*)f2, cs0, cs1, cs2, H0, W0, H1, W1, H2, W2, s0, s1, s2, B, nc,
                       reg_max, y);
  return check_launch("adr_detect_decode");
}
