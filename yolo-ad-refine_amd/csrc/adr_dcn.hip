// Fused DCNv2 for the bf16 performance path: mmcv ModulatedDeformConv2d(C, Cout, 3, stride 1, pad 1,
// bias=False, deform_groups 1) as DyDCNv2 calls it (reference nn/modules/head.py:751-782; AYHead1 :1154-1159),
// offsets / mask logits from the 27-channel spatial_conv_offset output (offset 2t = dy, 2t+1 = dx, mask 18+t,
// sigmoid applied here). No column matrix ever reaches HBM:
//
//   dcn_fwd     y[p][co]  = sum_{t,c} W[co][t][c] * m_pt * bilinear(x, p + tap_t + off_pt)[c]
//               the A operand of a v_mfma_f32_16x16x32_bf16 GEMM is SAMPLED straight into LDS: a 128-pixel tile's
//               64-channel slab of tap t is gathered (four bilinear corners, 16-byte buffer loads; invalid corners
//               read as zero through an out-of-range offset) while the previous slab is on the MFMA units.
//   dcn_wgrad   dW[co][t][c] = sum_p dy[p][co] * cols[p][t][c]: the same sampling produces the B slab of a
//               split-K GEMM over pixels (transposing LDS reads), partials [split][Cout][9][C] reduced by
//               adr_wgrad_reduce (fixed order).
//   dcn_bwd     per 8x8 pixel tile: dcols_t^T = W_t^T dy^T on MFMA (in registers, never stored), then for every
//               (pixel, tap) the offset / mask-logit gradients (reductions over channels: DPP-free cross-lane
//               xor shuffles, fixed order) and the input-gradient scatter. The scatter lands in an LDS window
//               of the tile's input neighbourhood (corners within 3 pixels of the tile: offsets up to ~2 px)
//               with LDS float atomics; the window is flushed to the fp32 input gradient with one global atomic
//               per (cell, channel), corners outside it go to global atomics directly (unordered float atomics,
//               as mmcv's own modulated_deformable_col2im_gpu_kernel; fp32 parity mode uses the
//               deterministic path in adr_head.hip).
// Sampling follows mmcv dmcn_im2col_bilinear / dmcn_get_coordinate_weight: point (h - 1 + i + dy, w - 1 + j + dx),
// zero unless -1 < py < H and -1 < px < W, every bilinear corner bounds-checked.
// Shapes: C % 64 == 0, Cout % 64 == 0, omcs % 8 == 0 and >= 32 (the head pads the 27 channels to 32).
#include <type_traits>

#include "adr_common.h"

#include <cstdlib>

namespace adr {

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

__device__ __forceinline__ v4s tr16(const __bf16* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p)); }

__device__ __forceinline__ int xcd_order(int b, int nb) { return (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3); }

constexpr unsigned OOR = 0x7FFFFFF0u;  // out-of-range buffer offset: the load returns zeros

struct Corners {
  int y0, x0;
  float ly, lx;
  float w[4];    // bilinear weights, 0 for invalid corners / outside points
  bool ok[4];
};

__device__ __forceinline__ void sample(float py, float px, int H, int W, Corners& s) {
  const float fy = floorf(py), fx = floorf(px);
  s.y0 = (int)fy;
  s.x0 = (int)fx;
  s.ly = py - fy;
  s.lx = px - fx;
  const float hy = 1.f - s.ly, hx = 1.f - s.lx;
  const bool inside = py > -1.f && px > -1.f && py < (float)H && px < (float)W;
  s.ok[0] = inside && s.y0 >= 0 && s.x0 >= 0;
  s.ok[1] = inside && s.y0 >= 0 && s.x0 + 1 <= W - 1;
  s.ok[2] = inside && s.y0 + 1 <= H - 1 && s.x0 >= 0;
  s.ok[3] = inside && s.y0 + 1 <= H - 1 && s.x0 + 1 <= W - 1;
  s.w[0] = s.ok[0] ? hy * hx : 0.f;
  s.w[1] = s.ok[1] ? hy * s.lx : 0.f;
  s.w[2] = s.ok[2] ? s.ly * hx : 0.f;
  s.w[3] = s.ok[3] ? s.ly * s.lx : 0.f;
}

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + __expf(-v)); }

// 8 bf16 -> 8 floats
__device__ __forceinline__ void unpack8(u32x4 v, float* f) {
  const __bf16* e = reinterpret_cast<const __bf16*>(&v);
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = (float)e[k];
}

}  // namespace

struct DcnArgs {
  const __bf16* x;
  const __bf16* om;
  const __bf16* w;   // fwd: KRSC [Cout][9][C]; bwd: W^T [9][C][Cout]
  const __bf16* dy;
  __bf16* y;
  float* part;       // wgrad partials [split][Cout][9][C]
  float* dx32;       // bwd: fp32 input gradient (accumulated with atomics; caller zeroes it)
  __bf16* dom;       // bwd: offset / mask-logit gradient (caller zeroes the padding channels)
  int xcs, omcs, ycs, dycs, domcs;
  int N, H, W, C, Cout;
  int x_bytes, w_bytes, dy_bytes;
  long rows_per_split;
  int splits;
};

// ------------------------------------------------------------------------------------------------------------
// forward: 128 pixels x 64 output channels per block, K = 9 taps x C in 64-channel slabs
// ------------------------------------------------------------------------------------------------------------
constexpr int FBM = 128, FLD = 72;

__global__ void __launch_bounds__(256, 2) dcn_fwd_kernel(DcnArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 As[2][FBM * FLD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][64 * FLD];
  __shared__ __attribute__((aligned(16))) __bf16 Oms[FBM * 32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long M = (long)a.N * a.H * a.W;
  const int mtiles = (int)((M + FBM - 1) / FBM), ntiles = a.Cout / 64;
  const int bid = xcd_order(blockIdx.x, gridDim.x);
  const int mt = bid / ntiles, nt = bid % ntiles;
  const long m0 = (long)mt * FBM;
  const int co0 = nt * 64;
  (void)mtiles;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);

  // offset / mask rows of the tile (first 32 channels) into LDS
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + 256 * i, r = q >> 2, ch = (q & 3) * 8;
    const long m = m0 + r;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (m < M) v = ld16(a.om + m * a.omcs + ch);
    st16(&Oms[r * 32 + ch], v);
  }
  // this thread's sampling row and channel half
  const int r = tid >> 1, hf = tid & 1;
  const long m = m0 + r;
  const bool rok = m < M;
  int n, h, w;
  pix_nhw(rok ? m : 0, a.H, a.W, n, h, w);
  const int ibase = n * a.H * a.W;
  const int cchunks = a.C / 64, steps = 9 * cchunks;
  __syncthreads();

  u32x4 raw[4][4];  // [corner][chunk]
  float cw[4];
  u32x4 rb[2];
  auto load = [&](int s) {
    const int t = s / cchunks, cc = s - t * cchunks;
    const float oy = (float)Oms[r * 32 + 2 * t], ox = (float)Oms[r * 32 + 2 * t + 1];
    const float mk = sigm((float)Oms[r * 32 + 18 + t]);
    Corners cs;
    sample((float)(h - 1 + t / 3) + oy, (float)(w - 1 + t % 3) + ox, a.H, a.W, cs);
    const int c = cc * 64 + hf * 32;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool ok = rok && cs.ok[q];
      cw[q] = ok ? cs.w[q] * mk : 0.f;
      const int pix = ibase + (cs.y0 + (q >> 1)) * a.W + cs.x0 + (q & 1);
      const unsigned base = ok ? (unsigned)(pix * a.xcs + c) * 2u : OOR;
#pragma unroll
      for (int j = 0; j < 4; ++j) raw[q][j] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? base + 16u * j : OOR, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i;
      const int row = q >> 3, ch = (q & 7) * 8;
      rb[i] = __builtin_amdgcn_raw_buffer_load_b128(
          wr, (unsigned)(((co0 + row) * 9 * a.C) + t * a.C + cc * 64 + ch) * 2u, 0, 0);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc8[8], f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc8[e] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        unpack8(raw[q][j], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc8[e] += cw[q] * f[e];
      }
      u32x4 o;
      __bf16* oe = reinterpret_cast<__bf16*>(&o);
#pragma unroll
      for (int e = 0; e < 8; ++e) oe[e] = (__bf16)acc8[e];
      st16(&As[buf][r * FLD + hf * 32 + 8 * j], o);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i;
      st16(&Bs[buf][(q >> 3) * FLD + (q & 7) * 8], rb[i]);
    }
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int wr0 = wave * 32;
  load(0);
  store(0);
  __syncthreads();
  for (int s = 0; s < steps; ++s) {
    const int cur = s & 1;
    if (s + 1 < steps) load(s + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(&As[cur][(wr0 + 16 * i + (lane & 15)) * FLD + 32 * kk + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][(16 * j + (lane & 15)) * FLD + 32 * kk + 8 * (lane >> 4)]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < steps) store(cur ^ 1);  // the other buffer was last read in step s-1 (before the barrier)
    __syncthreads();
  }
  // epilogue: bf16 image of the tile (in A buffer 0), then 16-byte row stores
  __bf16* Os = As[0];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) Os[(wr0 + 16 * i + 4 * (lane >> 4) + e) * FLD + 16 * j + (lane & 15)] = (__bf16)acc[i][j][e];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + 256 * i, row = q >> 3, ch = (q & 7) * 8;
    const long mm = m0 + row;
    if (mm < M) st16(a.y + mm * a.ycs + co0 + ch, *reinterpret_cast<const u32x4*>(&Os[row * FLD + ch]));
  }
}

// ------------------------------------------------------------------------------------------------------------
// weight gradient: block = (co tile 64, tap, c tile 64) x split over pixels; 64 pixel rows per k-step
// ------------------------------------------------------------------------------------------------------------
constexpr int WR = 64, WP = 80;  // rows per k-step; LDS row pitch (odd multiple of 16 elements: conflict-free tr reads)

__global__ void __launch_bounds__(256, 2) dcn_wgrad_kernel(DcnArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 As[WR * WP];  // dy rows [p][co]
  __shared__ __attribute__((aligned(16))) __bf16 Bs[WR * WP];  // sampled rows [p][c]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ctiles = a.C / 64, cotiles = a.Cout / 64;
  const int nbx = gridDim.x * gridDim.y;
  int b = xcd_order(blockIdx.x + blockIdx.y * gridDim.x, nbx);
  const int split = b / gridDim.x;
  b -= split * gridDim.x;
  const int ct = b % ctiles;
  b /= ctiles;
  const int t = b % 9, cot = b / 9;
  (void)cotiles;
  const int c0 = ct * 64, co0 = cot * 64;
  const long M = (long)a.N * a.H * a.W;
  const long pbeg = (long)split * a.rows_per_split;
  const long pend = min(M, pbeg + a.rows_per_split);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);
  const int ti = t / 3, tj = t % 3;

  u32x4 ra[2], rq[2][4];
  float cw[2][4];
  auto load = [&](long p0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i, row = q >> 3, ch = (q & 7) * 8;
      const long p = p0 + row;
      const bool ok = p < pend;
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(dyr, ok ? (unsigned)((int)p * a.dycs + co0 + ch) * 2u : OOR, 0, 0);
      int n = 0, h = 0, w = 0;
      pix_nhw(ok ? p : 0, a.H, a.W, n, h, w);
      const __bf16* o = a.om + (ok ? p : 0) * a.omcs;
      const float oy = (float)o[2 * t], ox = (float)o[2 * t + 1];
      const float mk = sigm((float)o[18 + t]);
      Corners cs;
      sample((float)(h - 1 + ti) + oy, (float)(w - 1 + tj) + ox, a.H, a.W, cs);
      const int ibase = n * a.H * a.W;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const bool cok = ok && cs.ok[qq];
        cw[i][qq] = cok ? cs.w[qq] * mk : 0.f;
        const int pix = ibase + (cs.y0 + (qq >> 1)) * a.W + cs.x0 + (qq & 1);
        rq[i][qq] = __builtin_amdgcn_raw_buffer_load_b128(xr, cok ? (unsigned)(pix * a.xcs + c0 + ch) * 2u : OOR, 0, 0);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i, row = q >> 3, ch = (q & 7) * 8;
      st16(&As[row * WP + ch], ra[i]);
      float s8[8], f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) s8[e] = 0.f;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        unpack8(rq[i][qq], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) s8[e] += cw[i][qq] * f[e];
      }
      u32x4 o;
      __bf16* oe = reinterpret_cast<__bf16*>(&o);
#pragma unroll
      for (int e = 0; e < 8; ++e) oe[e] = (__bf16)s8[e];
      st16(&Bs[row * WP + ch], o);
    }
  };
  // waves 2 x 2 over (co, c): 32 x 32 each
  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int row0 = 4 * g + q4;
  const __bf16* a_base = As + row0 * WP + wm * 32 + 4 * p4;
  const __bf16* b_base = Bs + row0 * WP + wn * 32 + 4 * p4;
  const int ksteps = (int)((pend - pbeg + WR - 1) / WR);
  if (ksteps > 0) {
    load(pbeg);
    store();
    __syncthreads();
  }
  for (int s = 0; s < ksteps; ++s) {
    if (s + 1 < ksteps) load(pbeg + (long)(s + 1) * WR);
#pragma unroll
    for (int u = 0; u < WR / 32; ++u) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        v4s both[2] = {tr16(a_base + u * 32 * WP + i * 16), tr16(a_base + (u * 32 + 16) * WP + i * 16)};
        fa[i] = *reinterpret_cast<bf16x8*>(both);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        v4s both[2] = {tr16(b_base + u * 32 * WP + j * 16), tr16(b_base + (u * 32 + 16) * WP + j * 16)};
        fb[j] = *reinterpret_cast<bf16x8*>(both);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (s + 1 < ksteps) {
      store();
      __syncthreads();
    }
  }
  float* part = a.part + (long)split * a.Cout * 9 * a.C;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = c0 + wn * 32 + 16 * j + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wm * 32 + 16 * i + 4 * (lane >> 4) + e;
        part[((long)co * 9 + t) * a.C + c] = acc[i][j][e];
      }
    }
}

// ------------------------------------------------------------------------------------------------------------
// data / offset / mask gradients (C == Cout == 64): 8x8 pixel tile per block, all taps
//
// Per tap: (1) lane (pixel, channel group) computes the tap's sampling point, issues its corner loads and, on
// MFMA, its column of dcols^T = W_t^T dy^T (W_t^T fragments from L2, the tile's dy fragments held in
// registers); (2) the offset / mask-logit gradients are channel reductions in-lane plus two xor shuffles,
// written straight to dom; (3) the input-gradient scatter is a second GEMM: the tap's sampling matrix S_t
// (window cell x pixel, four bilinear weights x mask per pixel column, built in LDS) times dcols (pixel x
// channel) accumulates the tile's input-gradient window — 196 cells (corners within 3 px of the tile) x 64
// channels — in fp32 MFMA accumulators across all nine taps. No LDS read-modify-write scatter at all (LDS float
// atomics measured ~4x slower than this whole kernel). At the end the window goes to the fp32 input gradient
// with one global atomic per (cell, channel); valid corners outside it are queued per tap and added with
// global atomics.
// ------------------------------------------------------------------------------------------------------------
constexpr int BT = 8;                   // tile side (pixels)
constexpr int BHALO = 3;                // window margin: corners of samples with |offset| <~ 2 px
constexpr int BWIN = BT + 2 * BHALO;    // 14 window cells per side
constexpr int BCELL = BWIN * BWIN;      // 196 cells
constexpr int BROWS = 208;              // cells padded to 13 MFMA row blocks
constexpr int SPITCH = 72;              // S_t row pitch (bf16): 64 pixels + 8
constexpr int DPITCH = 80;              // dcols row pitch (bf16): odd multiple of 16 elements for transposing reads
constexpr int BOVF = 256;               // overflow queue (out-of-window corners) per tap

// OCC = workgroups per CU the register budget is sized for: 2 (256 VGPRs, a few spilled) or 1 (AGPRs too, no spill)
template <int OCC>
__global__ void __launch_bounds__(256, OCC) dcn_bwd_kernel(DcnArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 S[BROWS * SPITCH];   // [cell][pixel]
  __shared__ __attribute__((aligned(16))) __bf16 D[64 * DPITCH];      // dcols [pixel][channel]
  __shared__ __attribute__((aligned(16))) __bf16 oms[64 * 32];
  __shared__ __attribute__((aligned(16))) __bf16 WT[2][64 * 72];     // W_t^T [c][co], two taps
  __shared__ int ovf[BOVF];                                            // pixel * 4 + corner
  __shared__ int novf[2];                                              // per-tap queue length (alternating)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tw = (a.W + BT - 1) / BT, th = (a.H + BT - 1) / BT;
  const int bid = xcd_order(blockIdx.x, gridDim.x);
  const int n = bid / (tw * th);
  const int rem = bid - n * tw * th;
  const int h0 = (rem / tw) * BT, w0 = (rem % tw) * BT;
  const int wy0 = h0 - BHALO, wx0 = w0 - BHALO;
  const int ibase = n * a.H * a.W;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);

  {
    const int p = tid >> 2, ch = (tid & 3) * 8;
    const int hh = h0 + (p >> 3), ww = w0 + (p & 7);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (hh < a.H && ww < a.W) v = ld16(a.om + (long)(ibase + hh * a.W + ww) * a.omcs + ch);
    st16(&oms[p * 32 + ch], v);
  }
  {
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int i = tid; i < BROWS * SPITCH / 8; i += 256) st16(&S[8 * i], z);
  }
  if (tid < 2) novf[tid] = 0;

  // this lane's pixel and channel group (dcols^T layout of the MFMA result: row = channel, column = pixel)
  const int pl = 16 * wave + (lane & 15);
  const int ph = h0 + (pl >> 3), pw = w0 + (pl & 7);
  const bool pok = ph < a.H && pw < a.W;
  const int g = lane >> 4;
  const long ppix = ibase + (long)ph * a.W + pw;
  bf16x8 fb[2];  // dy fragments of this lane's pixel (B operand, k = output channel)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (pok) v = ld16(a.dy + ppix * a.dycs + 32 * k + 8 * g);
    fb[k] = *reinterpret_cast<bf16x8*>(&v);
  }
  // the tap's W^T slab (LDS, loaded cooperatively) and this lane's bilinear-corner loads, both issued one tap
  // ahead: the corners into the other of two register sets, the slab through registers into the other LDS buffer
  u32x2 xv[2][4][4];
  Corners cs[2];
  float mks[2];
  u32x4 wreg[2];
  auto issue = [&](int t, auto SB) {
    constexpr int b = decltype(SB)::value;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i;
      wreg[i] = __builtin_amdgcn_raw_buffer_load_b128(wr, (unsigned)((t * 64 + (q >> 3)) * 64 + (q & 7) * 8) * 2u, 0, 0);
    }
    const float oy = (float)oms[pl * 32 + 2 * t], ox = (float)oms[pl * 32 + 2 * t + 1];
    mks[b] = sigm((float)oms[pl * 32 + 18 + t]);
    sample((float)(ph - 1 + t / 3) + oy, (float)(pw - 1 + t % 3) + ox, a.H, a.W, cs[b]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool ok = pok && cs[b].ok[q];
      const int pix = ibase + (cs[b].y0 + (q >> 1)) * a.W + cs[b].x0 + (q & 1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        xv[b][q][i] =
            __builtin_amdgcn_raw_buffer_load_b64(xr, ok ? (unsigned)(pix * a.xcs + 16 * i + 4 * g) * 2u : OOR, 0, 0);
    }
  };
  auto wstore = [&](int b) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i;
      st16(&WT[b][(q >> 3) * 72 + (q & 7) * 8], wreg[i]);
    }
  };
  // window accumulators: wave w owns channels 16 w .. +15, all 13 cell blocks
  f32x4 win[13];
#pragma unroll
  for (int b = 0; b < 13; ++b) win[b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // transposing-read lane map for the B operand of the scatter GEMM (see adr_wgrad.hip): k-slot (g, j) is
  // pixel row 4 g + j (j < 4) / 16 + 4 g + j - 4; the A operand (S) reads the same pixels as two 8-byte pieces
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  const __bf16* dtr = D + (4 * g + q4) * DPITCH + 16 * wave + 4 * p4;
  int prev[4] = {-1, -1, -1, -1};  // S cells written in the previous tap (g == 0 lanes)
  __syncthreads();  // oms / S ready
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  issue(0, B0{});
  wstore(0);
  __syncthreads();

  auto tap = [&](int t, auto SB) {
    constexpr int cur = decltype(SB)::value;
    using NB = std::integral_constant<int, 1 - cur>;
    if (t + 1 < 9) issue(t + 1, NB{});  // WT[1 - cur] was last read before the previous tap's first barrier
    const Corners& c0 = cs[cur];
    const float mk = mks[cur];
    // the sampling-matrix column of this pixel: clear the previous tap's entries, write this tap's
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (prev[q] >= 0) S[prev[q] * SPITCH + pl] = (__bf16)0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int yy = c0.y0 + (q >> 1), xx = c0.x0 + (q & 1);
        const int cy = yy - wy0, cx = xx - wx0;
        const bool valid = pok && c0.ok[q];
        const bool inwin = cy >= 0 && cy < BWIN && cx >= 0 && cx < BWIN;
        prev[q] = -1;
        if (valid && inwin) {
          prev[q] = cy * BWIN + cx;
          S[prev[q] * SPITCH + pl] = (__bf16)(mk * c0.w[q]);
        } else if (valid) {
          const int k = atomicAdd(&novf[t & 1], 1);  // at most 64 x 4 = BOVF entries
          ovf[k] = pl * 4 + q;
        }
      }
    }
    // dcols^T (64 channels x this wave's 16 pixels) = W_t^T . dy^T
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 2; ++k)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            *reinterpret_cast<const bf16x8*>(&WT[cur][(16 * i + (lane & 15)) * 72 + 32 * k + 8 * g]), fb[k], acc[i], 0,
            0, 0);
    }
    if (t + 1 < 9) wstore(1 - cur);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __bf16 v4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v4[e] = (__bf16)acc[i][e];
      *reinterpret_cast<u32x2*>(&D[pl * DPITCH + 16 * i + 4 * g]) = *reinterpret_cast<u32x2*>(v4);
    }
    // offset / mask-logit gradients: value, d/dpy, d/dpx of the bilinear sample per channel (invalid corners
    // read as zero), dotted with dcols over this lane's 16 channels, then over the four channel groups
    float smk = 0.f, spy = 0.f, spx = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float xf[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const __bf16* e = reinterpret_cast<const __bf16*>(&xv[cur][q][i]);
#pragma unroll
        for (int k = 0; k < 4; ++k) xf[q][k] = (float)e[k];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float top = xf[0][e] + c0.lx * (xf[1][e] - xf[0][e]);
        const float bot = xf[2][e] + c0.lx * (xf[3][e] - xf[2][e]);
        const float d01 = xf[1][e] - xf[0][e], d23 = xf[3][e] - xf[2][e];
        const float val = top + c0.ly * (bot - top);
        const float sy = bot - top, sx = d01 + c0.ly * (d23 - d01);
        const float gv = acc[i][e];
        smk += gv * val;
        spy += gv * sy;
        spx += gv * sx;
      }
    }
    smk += __shfl_xor(smk, 16, 64);
    smk += __shfl_xor(smk, 32, 64);
    spy += __shfl_xor(spy, 16, 64);
    spy += __shfl_xor(spy, 32, 64);
    spx += __shfl_xor(spx, 16, 64);
    spx += __shfl_xor(spx, 32, 64);
    if (g == 0 && pok) {
      __bf16* d = a.dom + ppix * a.domcs;
      d[2 * t] = (__bf16)(mk * spy);
      d[2 * t + 1] = (__bf16)(mk * spx);
      d[18 + t] = (__bf16)(smk * mk * (1.f - mk));
    }
    __syncthreads();  // S column entries and dcols complete
    if (tid == 0) novf[(t + 1) & 1] = 0;  // last read in tap t-1
    // window[cell][c] += S_t[cell][pixel] . dcols[pixel][c]  (K = 64 pixels in two 32-steps)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v4s blo = tr16(dtr + kk * 32 * DPITCH), bhi = tr16(dtr + (kk * 32 + 16) * DPITCH);
      v4s bb[2] = {blo, bhi};
      const bf16x8 fbw = *reinterpret_cast<bf16x8*>(bb);
#pragma unroll
      for (int b = 0; b < 13; ++b) {
        const __bf16* sr = S + (16 * b + (lane & 15)) * SPITCH + 32 * kk + 4 * g;
        u32x2 alo = *reinterpret_cast<const u32x2*>(sr), ahi = *reinterpret_cast<const u32x2*>(sr + 16);
        u32x2 aa[2] = {alo, ahi};
        win[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(aa), fbw, win[b], 0, 0, 0);
      }
    }
    // out-of-window corners: global atomics, one queued (pixel, corner) per wave at a time, lanes = channels
    const int nq = novf[t & 1];
    for (int k = wave; k < nq; k += 4) {
      const int pq = ovf[k], p = pq >> 2, qq = pq & 3;
      const int ph2 = h0 + (p >> 3), pw2 = w0 + (p & 7);
      const float oy2 = (float)oms[p * 32 + 2 * t], ox2 = (float)oms[p * 32 + 2 * t + 1];
      const float mk2 = sigm((float)oms[p * 32 + 18 + t]);
      Corners c2;
      sample((float)(ph2 - 1 + t / 3) + oy2, (float)(pw2 - 1 + t % 3) + ox2, a.H, a.W, c2);
      const int yy = c2.y0 + (qq >> 1), xx = c2.x0 + (qq & 1);
      unsafeAtomicAdd(a.dx32 + (long)(ibase + yy * a.W + xx) * 64 + lane, (float)D[p * DPITCH + lane] * mk2 * c2.w[qq]);
    }
    __syncthreads();  // before the next tap rewrites S / dcols
  };
#pragma unroll 1
  for (int t = 0; t < 9; t += 2) {
    tap(t, B0{});
    if (t + 1 < 9) tap(t + 1, B1{});
  }
  // flush the window: one global atomic per (cell, channel) that received anything
#pragma unroll
  for (int b = 0; b < 13; ++b)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int cell = 16 * b + 4 * g + e;
      const int yy = wy0 + cell / BWIN, xx = wx0 + cell % BWIN;
      const float v = win[b][e];
      if (cell < BCELL && v != 0.f && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
        unsafeAtomicAdd(a.dx32 + (long)(ibase + yy * a.W + xx) * 64 + 16 * wave + (lane & 15), v);
    }
}

}  // namespace adr

using namespace adr;

static int dcn_check(int N, int H, int W, int C, int Cout, int xcs, int omcs) {
  ADR_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % 64 == 0 && Cout % 64 == 0 && Cout <= 256,
              "dcn (bf16 fused): needs C %% 64 == 0 and Cout in {64..256} step 64 (C=%d Cout=%d)", C, Cout);
  ADR_REQUIRE(omcs >= 32 && omcs % 8 == 0 && xcs % 8 == 0, "dcn (bf16 fused): omcs=%d xcs=%d", omcs, xcs);
  ADR_REQUIRE((long)N * H * W * xcs < (1l << 30), "dcn (bf16 fused): activation too large for 32-bit offsets");
  return 0;
}

extern "C" int adr_dcn_fwd_bf16(const void* x, int xcs, const void* om, int omcs, const void* w_krsc, void* y, int ycs,
                                int N, int H, int W, int C, int Cout, void* stream) {
  if (int rc = dcn_check(N, H, W, C, Cout, xcs, omcs)) return rc;
  DcnArgs a{};
  a.x = (const __bf16*)x;
  a.om = (const __bf16*)om;
  a.w = (const __bf16*)w_krsc;
  a.y = (__bf16*)y;
  a.xcs = xcs;
  a.omcs = omcs;
  a.ycs = ycs;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Cout = Cout;
  a.x_bytes = (int)((long)N * H * W * xcs * 2);
  a.w_bytes = Cout * 9 * C * 2;
  const long M = (long)N * H * W;
  const int blocks = cdiv(M, FBM) * (Cout / 64);
  hipLaunchKernelGGL(dcn_fwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("adr_dcn_fwd_bf16");
}

extern "C" int adr_dcn_wgrad_bf16_splits(int N, int H, int W, int C, int Cout) {
  const long M = (long)N * H * W;
  const long steps = (M + WR - 1) / WR;
  const int tiles = 9 * (C / 64) * (Cout / 64);
  long s = 1024 / tiles + 1;  // >= ~1k blocks
  if (s > steps) s = steps;
  if (s < 1) s = 1;
  return (int)s;
}

extern "C" int adr_dcn_wgrad_bf16(const void* x, int xcs, const void* om, int omcs, const void* dy, int dycs,
                                  float* part, int splits, int N, int H, int W, int C, int Cout, void* stream) {
  if (int rc = dcn_check(N, H, W, C, Cout, xcs, omcs)) return rc;
  ADR_REQUIRE(splits >= 1, "dcn_wgrad: splits=%d", splits);
  DcnArgs a{};
  a.x = (const __bf16*)x;
  a.om = (const __bf16*)om;
  a.dy = (const __bf16*)dy;
  a.part = part;
  a.xcs = xcs;
  a.omcs = omcs;
  a.dycs = dycs;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Cout = Cout;
  a.x_bytes = (int)((long)N * H * W * xcs * 2);
  a.dy_bytes = (int)((long)N * H * W * dycs * 2);
  const long M = (long)N * H * W;
  const long steps = (M + WR - 1) / WR;
  a.rows_per_split = ((steps + splits - 1) / splits) * WR;
  a.splits = splits;
  dim3 grid(9 * (C / 64) * (Cout / 64), splits);
  hipLaunchKernelGGL(dcn_wgrad_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("adr_dcn_wgrad_bf16");
}

extern "C" int adr_dcn_bwd_bf16(const void* x, int xcs, const void* om, int omcs, const void* dy, int dycs,
                                const void* w_t, float* dx32, void* dom, int domcs, int N, int H, int W, int C, int Cout,
                                void* stream) {
  if (int rc = dcn_check(N, H, W, C, Cout, xcs, omcs)) return rc;
  ADR_REQUIRE(C == 64 && Cout == 64, "dcn_bwd (bf16 fused): C == Cout == 64 only (C=%d Cout=%d)", C, Cout);
  ADR_REQUIRE(domcs >= 27 && dycs % 8 == 0, "dcn_bwd: domcs=%d dycs=%d", domcs, dycs);
  DcnArgs a{};
  a.x = (const __bf16*)x;
  a.om = (const __bf16*)om;
  a.dy = (const __bf16*)dy;
  a.w = (const __bf16*)w_t;
  a.dx32 = dx32;
  a.dom = (__bf16*)dom;
  a.xcs = xcs;
  a.omcs = omcs;
  a.dycs = dycs;
  a.domcs = domcs;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Cout = Cout;
  a.x_bytes = (int)((long)N * H * W * xcs * 2);
  a.w_bytes = 9 * C * Cout * 2;
  const int blocks = N * cdiv(H, BT) * cdiv(W, BT);
  static const int occ = getenv("ADR_DCN_BWD_OCC") ? atoi(getenv("ADR_DCN_BWD_OCC")) : 2;
  if (occ == 1) hipLaunchKernelGGL(dcn_bwd_kernel<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(dcn_bwd_kernel<2>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("adr_dcn_bwd_bf16");
}
