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
//   dcn_bwd     per 8x8 pixel tile: the offset / mask-logit gradients of its pixels (dcols = W^T dy on MFMA,
//               dotted with the bilinear samples), and dx of its pixels GATHERED from every source whose sample
//               has a corner there (sampling matrix x dy on MFMA, then x W): dx written once in bf16, no fp32
//               buffer, no float atomics except for corners more than ~2 px away (see below; fp32 parity mode
//               uses the deterministic path in adr_head.hip).
// Sampling follows mmcv dmcn_im2col_bilinear / dmcn_get_coordinate_weight: point (h - 1 + i + dy, w - 1 + j + dx),
// zero unless -1 < py < H and -1 < px < W, every bilinear corner bounds-checked.
// Shapes: C % 64 == 0, Cout % 64 == 0 (backward: C == Cout in {64, 128, 256}), omcs % 8 == 0 and >= 32 (the
// head pads the 27 channels to 32).
#include <type_traits>

#include "adr_common.h"

#include <cstdlib>

namespace adr {

namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4s tr16(const __bf16* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p)); }

__device__ __forceinline__ int xcd_order(int b, int nb) { return xcd_remap(b, nb); }

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

// v_rcp_f32 (1 ulp) instead of the IEEE division sequence
__device__ __forceinline__ float sigm(float v) { return __builtin_amdgcn_rcpf(1.f + __expf(-v)); }

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
  __bf16* dx;        // bwd: input gradient (written once per element, far entries added afterwards)
  __bf16* dom;       // bwd: offset / mask-logit gradient (caller zeroes the padding channels)
  int xcs, omcs, ycs, dycs, domcs, dxcs;
  int N, H, W, C, Cout;
  int x_bytes, w_bytes, dy_bytes;
  long rows_per_split;
  int splits;
};

// ------------------------------------------------------------------------------------------------------------
// forward: 128 pixels x FCO output channels per block (FCO = 64, or 128 for Cout % 128 == 0: the sampled A slab
// then feeds twice the columns — the l-scale head's 256 channels sampled every slab four times), K = 9 taps x C in
// 64-channel slabs; 4 x FCO / 64 waves: 4 along the pixels x FCO / 64 along the columns. Each output element sums the
// same K steps in the same order for either FCO (bitwise equal).
// ------------------------------------------------------------------------------------------------------------
constexpr int FBM = 128, FLD = 72;
__host__ __device__ constexpr int dcn_fwd_fco(int Cout) { return Cout % 128 == 0 ? 128 : 64; }

template <int FCO>
__device__ __forceinline__ void dcn_fwd_body(const DcnArgs& a, int bid) {
  constexpr int NT = 4 * FCO;          // threads
  constexpr int SPR = NT / FBM;        // sampling threads per pixel row (2 / 4)
  constexpr int SCH = 64 / SPR / 8;    // 16-byte chunks each of them samples per corner (4 / 2)
  constexpr int OP = FCO + 8;          // epilogue image pitch
  static_assert(FBM * OP <= 2 * FBM * FLD, "epilogue image fits the A buffers");
  __shared__ __attribute__((aligned(16))) __bf16 As[2][FBM * FLD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][FCO * FLD];
  __shared__ __attribute__((aligned(16))) __bf16 Oms[FBM * 32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long M = (long)a.N * a.H * a.W;
  const int ntiles = a.Cout / FCO;
  const int mt = bid / ntiles, nt = bid % ntiles;
  const long m0 = (long)mt * FBM;
  const int co0 = nt * FCO;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);

  // offset / mask rows of the tile (first 32 channels) into LDS
  for (int q = tid; q < FBM * 4; q += NT) {
    const int r = q >> 2, ch = (q & 3) * 8;
    const long m = m0 + r;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (m < M) v = ld16(a.om + m * a.omcs + ch);
    st16(&Oms[r * 32 + ch], v);
  }
  // this thread's sampling row and channel part
  const int r = tid / SPR, hf = tid % SPR;
  const long m = m0 + r;
  const bool rok = m < M;
  int n, h, w;
  pix_nhw(rok ? m : 0, a.H, a.W, n, h, w);
  const int ibase = n * a.H * a.W;
  const int cchunks = a.C / 64, steps = 9 * cchunks;
  __syncthreads();

  u32x4 raw[4][SCH];  // [corner][chunk]
  float cw[4];
  u32x4 rb[2];
  auto load = [&](int s) {
    const int t = s / cchunks, cc = s - t * cchunks;
    const float oy = (float)Oms[r * 32 + 2 * t], ox = (float)Oms[r * 32 + 2 * t + 1];
    const float mk = sigm((float)Oms[r * 32 + 18 + t]);
    Corners cs;
    sample((float)(h - 1 + t / 3) + oy, (float)(w - 1 + t % 3) + ox, a.H, a.W, cs);
    const int c = cc * 64 + hf * (64 / SPR);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool ok = rok && cs.ok[q];
      cw[q] = ok ? cs.w[q] * mk : 0.f;
      const int pix = ibase + (cs.y0 + (q >> 1)) * a.W + cs.x0 + (q & 1);
      const unsigned base = ok ? (unsigned)(pix * a.xcs + c) * 2u : OOR;
#pragma unroll
      for (int j = 0; j < SCH; ++j) raw[q][j] = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? base + 16u * j : OOR, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // B: FCO rows x 64 channels = 2 chunks per thread
      const int q = tid + NT * i;
      const int row = q >> 3, ch = (q & 7) * 8;
      rb[i] = __builtin_amdgcn_raw_buffer_load_b128(
          wr, (unsigned)(((co0 + row) * 9 * a.C) + t * a.C + cc * 64 + ch) * 2u, 0, 0);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < SCH; ++j) {
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
      st16(&As[buf][r * FLD + hf * (64 / SPR) + 8 * j], o);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + NT * i;
      st16(&Bs[buf][(q >> 3) * FLD + (q & 7) * 8], rb[i]);
    }
  };

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int wr0 = (wave & 3) * 32, wc0 = (wave >> 2) * 64;  // 32 pixel rows x 64 columns per wave
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
        fb[j] = *reinterpret_cast<const bf16x8*>(
            &Bs[cur][(wc0 + 16 * j + (lane & 15)) * FLD + 32 * kk + 8 * (lane >> 4)]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < steps) store(cur ^ 1);  // the other buffer was last read in step s-1 (before the barrier)
    __syncthreads();
  }
  // epilogue: bf16 image of the tile (in the A buffers), then 16-byte row stores
  __bf16* Os = As[0];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Os[(wr0 + 16 * i + 4 * (lane >> 4) + e) * OP + wc0 + 16 * j + (lane & 15)] = (__bf16)acc[i][j][e];
  __syncthreads();
  for (int q = tid; q < FBM * (FCO / 8); q += NT) {
    const int row = q / (FCO / 8), ch = (q % (FCO / 8)) * 8;
    const long mm = m0 + row;
    if (mm < M) st16(a.y + mm * a.ycs + co0 + ch, *reinterpret_cast<const u32x4*>(&Os[row * OP + ch]));
  }
}

template <int FCO>
__global__ void __launch_bounds__(4 * FCO, FCO == 64 ? 2 : 1) dcn_fwd_kernel(DcnArgs a) {
  dcn_fwd_body<FCO>(a, xcd_order(blockIdx.x, gridDim.x));
}

// The AYHead's three pyramid levels in ONE launch (LevelDCNFn): block b of the grid (XCD-ordered) belongs to level l
// with start[l] <= b < start[l + 1] and runs exactly the block b - start[l] of that level's own launch, so the
// results are bitwise the per-level launches'; the P4 / P5 levels (1 / 4 and 1 / 16 of P3's tiles, latency-bound
// on their own) fill the P3 launch's tail instead of running as launches of a few hundred workgroups.
struct DcnLevels {
  DcnArgs a[3];
  float* dxf[3];
  int* flags[3];
  int start[4];
  int tiles[3];  // wgrad: tile blocks per split
  int nl;
};
__device__ __forceinline__ int dcn_level(const DcnLevels& L, int b) {
  int l = 0;
  while (l + 1 < L.nl && b >= L.start[l + 1]) ++l;
  return l;
}
template <int FCO>
__global__ void __launch_bounds__(4 * FCO, FCO == 64 ? 2 : 1) dcn_fwd_levels_kernel(DcnLevels L) {
  const int b = xcd_order(blockIdx.x, gridDim.x), l = dcn_level(L, b);
  dcn_fwd_body<FCO>(L.a[l], b - L.start[l]);
}

// ------------------------------------------------------------------------------------------------------------
// weight gradient: block = (tap, c tile 64) x split over pixels, ALL output channels (COT = Cout for 64 / 128 / 256):
// the sampled B slab of a (tap, c tile) is built once and multiplies every co row of dy — with 64-wide co tiles the
// l-scale head (Cout 256) sampled each slab four times. 64 pixel rows per k-step; each output element accumulates the
// same k-steps in the same order whatever COT is (bitwise the 64-wide tiles).
// ------------------------------------------------------------------------------------------------------------
constexpr int WR = 64, WP = 80;  // rows per k-step; LDS row pitch (odd multiple of 16 elements: conflict-free tr reads)
__host__ __device__ constexpr int dcn_wg_cot(int Cout) { return Cout == 128 || Cout == 256 ? Cout : 64; }

// (b: XCD-ordered block of the level's launch, tiles: tile blocks per split)
template <int COT>
__device__ __forceinline__ void dcn_wgrad_body(const DcnArgs& a, int b, int tiles) {
  constexpr int AP = COT + 16;               // dy row pitch: odd multiple of 16 elements
  constexpr int ACH = WR * (COT / 8) / 256;  // 16-byte dy chunks per thread and k-step
  constexpr int WCO = COT / 2, TM = WCO / 16;
  __shared__ __attribute__((aligned(16))) __bf16 As[WR * AP];  // dy rows [p][co]
  __shared__ __attribute__((aligned(16))) __bf16 Bs[WR * WP];  // sampled rows [p][c]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ctiles = a.C / 64;
  const int split = b / tiles;
  b -= split * tiles;
  const int ct = b % ctiles;
  b /= ctiles;
  const int t = b % 9, cot = b / 9;
  const int c0 = ct * 64, co0 = cot * COT;
  const long M = (long)a.N * a.H * a.W;
  const long pbeg = (long)split * a.rows_per_split;
  const long pend = min(M, pbeg + a.rows_per_split);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);
  const int ti = t / 3, tj = t % 3;

  u32x4 ra[ACH], rq[2][4];
  float cw[2][4];
  auto load = [&](long p0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int q = tid + 256 * i, row = q / (COT / 8), ch = (q % (COT / 8)) * 8;
      const long p = p0 + row;
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(dyr, p < pend ? (unsigned)((int)p * a.dycs + co0 + ch) * 2u : OOR,
                                                    0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i, row = q >> 3, ch = (q & 7) * 8;
      const long p = p0 + row;
      const bool ok = p < pend;
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
    for (int i = 0; i < ACH; ++i) {
      const int q = tid + 256 * i, row = q / (COT / 8), ch = (q % (COT / 8)) * 8;
      st16(&As[row * AP + ch], ra[i]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i, row = q >> 3, ch = (q & 7) * 8;
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
  // waves 2 x 2 over (co, c): COT/2 x 32 each
  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int row0 = 4 * g + q4;
  const __bf16* a_base = As + row0 * AP + wm * WCO + 4 * p4;
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
      bf16x8 fa[TM], fb[2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        v4s both[2] = {tr16(a_base + u * 32 * AP + i * 16), tr16(a_base + (u * 32 + 16) * AP + i * 16)};
        fa[i] = *reinterpret_cast<bf16x8*>(both);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        v4s both[2] = {tr16(b_base + u * 32 * WP + j * 16), tr16(b_base + (u * 32 + 16) * WP + j * 16)};
        fb[j] = *reinterpret_cast<bf16x8*>(both);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
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
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = c0 + wn * 32 + 16 * j + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wm * WCO + 16 * i + 4 * (lane >> 4) + e;
        part[((long)co * 9 + t) * a.C + c] = acc[i][j][e];
      }
    }
}

template <int COT>
__global__ void __launch_bounds__(256, 2) dcn_wgrad_kernel(DcnArgs a) {
  dcn_wgrad_body<COT>(a, xcd_order(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y), gridDim.x);
}
// Levels dispatch in order (P3's long split blocks first, the short P5 blocks fill the tail) and the XCD grouping is
// applied within a level: interleaving the three levels over the whole grid started long P3 blocks last (l-scale:
// 7.6 ms for the three levels in one launch against 4.1 ms as three launches)
template <int COT>
__global__ void __launch_bounds__(256, 2) dcn_wgrad_levels_kernel(DcnLevels L) {
  const int l = dcn_level(L, blockIdx.x), s0 = L.start[l];
  const int b = xcd_order(blockIdx.x - s0, L.start[l + 1] - s0);
  dcn_wgrad_body<COT>(L.a[l], b, L.tiles[l]);
}

// ------------------------------------------------------------------------------------------------------------
// data / offset / mask gradients, gathered by destination tile (C == Cout in {64, 128, 256})
//
// A block owns an 8x8 tile of pixels: as output pixels p it produces their offset / mask-logit gradients, as
// input pixels q their dx. dx is written once, in bf16, from fp32 MFMA accumulators:
//
//   phase 1 (dom): per 64-channel chunk, the chunk of x over the tile's 14x14 neighbourhood is staged in LDS
//     once; per tap, dcols^T = W_t^T dy^T for the tile's 64 pixels on MFMA (dy fragments in registers, W_t^T
//     slabs double-buffered through LDS), dotted with the bilinear samples of x and their derivatives read from
//     the staged neighbourhood (channel reductions in-lane + two xor shuffles, fixed order) -> partial sums per
//     (pixel, tap) in LDS, finalised into one 64-byte dom row per pixel.
//   phase 2 (dx): dx_q = sum_t W_t . G_t[q], G_t[q][co] = sum_{p, corner -> q} m w dy[p][co]. The sources whose
//     tap-t sample can put a corner in the tile lie in a 12x12 sub-window of the neighbourhood (|offset| < 2
//     px); their dy rows are staged once per 64-channel chunk. The tap's sampling matrix S_t [64 dest x 144 src]
//     (bilinear weight x mask, bf16; column k written and cleared only by thread k) is built in LDS, then
//     G_t^T = dy_sub^T . S_t^T and dx^T += W_t^T . G_t^T on MFMA, G_t^T passed from accumulators to the next
//     operand in registers (k order permuted identically on both operands). 32-source K steps whose S_t columns
//     are all zero for a wave's 16 destinations are skipped (bitmask built with the matrix).
//   far corners (|offset| >= ~2 px: the source is outside its destination tile's sub-window) are added by the
//     SOURCE's block in phase 1 straight from the dcols accumulators into `dxf` (fp32 side buffer, global
//     atomics) and flag the destination tile; dcn_far_apply_kernel folds flagged tiles into dx afterwards and
//     re-zeroes them. With |offsets| < 2 px nothing is flagged and dx is bitwise repeatable.
// Near/far is decided by the same arithmetic (sample()) on both sides, so each valid corner is counted once.
// ------------------------------------------------------------------------------------------------------------
constexpr int GT = 8;                  // tile side (pixels)
constexpr int GM = 3;                  // neighbourhood margin
constexpr int GWIN = GT + 2 * GM;      // 14
constexpr int GCELL = GWIN * GWIN;     // 196 neighbourhood cells (+ one zero row)
constexpr int GSUB = 12;               // per-tap source sub-window side
constexpr int GK = GSUB * GSUB;        // 144 sources per tap
constexpr int GKS = 5;                 // K steps of 32 (160)
constexpr int GSP = 168;               // S row pitch (bf16)
constexpr int GDP = 80;                // dy-window row pitch: odd multiple of 16 elements (transposing reads)
constexpr int GXP = 72;                // x-window row pitch (bf16)

__device__ __forceinline__ int gsrc_row(int k, int sy, int sx) {  // neighbourhood row of sub-window source k
  const int ky = k / GSUB, kx = k - ky * GSUB;
  return k < GK ? (ky + 1 - sy) * GWIN + kx + 1 - sx : GCELL;
}

// SB (CO >= 2): ONE phase-1 W_t^T slab instead of two (a second barrier per tap), so the 128- and 256-channel
// kernels fit two workgroups per CU (LDS 74.8 / 81.5 KB instead of 82.6 / 115.3 KB).
// LEAN (C = Cout = 64): no om rows in LDS (each lane loads the offset pair / mask logit it needs from global, one
// tap ahead), the dy window at a 64-element pitch with its 16-byte chunks XOR-swizzled by row pair (transposing
// reads stay conflict-free), S_t at a 152-element pitch (K columns 144..159 are multiplied by the dy window's
// zero row, so they may read the next row / the K-step masks placed right after S_t) and the phase-2 W_t slab at a
// 68-element pitch: 53.6 KB, three workgroups per CU instead of two (at 53.9 KB the dispatcher placed only two).
template <int CC, int CO>
struct GLds {
  static constexpr bool SB = CO >= 2;
  static constexpr bool LEAN = CC == 1 && CO == 1;
  static constexpr int PW1 = 64 * CO + 8;                                  // phase-1 slab pitch [c][co]
  static constexpr int OMS = LEAN ? 0 : GCELL * 32 * 2;                    // om rows of the neighbourhood
  static constexpr int XP = LEAN ? 68 : GXP;  // x-window pitch: 68 (34 dwords) spreads the corner reads over 32 slots
  static constexpr int P1X = GCELL * XP * 2, P1W = (SB ? 1 : 2) * 64 * PW1 * 2, P1D = 64 * 27 * 4;
  static constexpr int P1 = P1X + P1W + P1D;                               // x window | W_t^T slabs | dom sums
  static constexpr int DP = LEAN ? 64 : GDP, SP = LEAN ? 152 : GSP;        // dy-window / S_t row pitches
  static constexpr int WP = LEAN ? 68 : 72;                                // phase-2 W_t slab pitch (8-B rows)
  static constexpr int P2Y = (GCELL + 1) * DP * 2, P2S = 64 * SP * 2, P2W = 64 * WP * 2;
  static constexpr int KM = LEAN ? P2Y + P2S : -1;                         // K-step masks inside phase 2 (LEAN)
  static constexpr int P2 = P2Y + P2S + (LEAN ? 64 : 0) + P2W;             // dy window | S_t | (masks) | W_t slab
  static constexpr int TOTAL = OMS + (P1 > P2 ? P1 : P2) + (LEAN ? 0 : 64);  // + K-step masks
};
// element offset e (multiple of 4) of dy-window row `row` (LEAN: chunk pair swizzled by (row >> 1) & 3)
template <bool LEAN>
__device__ __forceinline__ int dsw(int row, int e) { return LEAN ? e ^ (((row >> 1) & 3) << 4) : e; }

template <int CC, int CO>
__device__ __forceinline__ void dcn_bwd_body(const DcnArgs& a, float* dxf, int* flags, int mode, int bid) {
  using L = GLds<CC, CO>;
  constexpr bool LEAN = L::LEAN;
  __shared__ __attribute__((aligned(16))) char smem[L::TOTAL];
  __bf16* oms = reinterpret_cast<__bf16*>(smem);
  char* reg = smem + L::OMS;
  unsigned* kmask = reinterpret_cast<unsigned*>(L::LEAN ? smem + L::KM : smem + L::TOTAL - 64);  // [2 taps][4 waves]
  constexpr int C = 64 * CC, Cout = 64 * CO;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int tw = (a.W + GT - 1) / GT, th = (a.H + GT - 1) / GT;
  const int n = bid / (tw * th);
  const int rem = bid - n * tw * th;
  const int h0 = (rem / tw) * GT, w0 = (rem % tw) * GT;
  const int wy0 = h0 - GM, wx0 = w0 - GM;
  const int ibase = n * a.H * a.W;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  const __amdgpu_buffer_rsrc_t omr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.om, (short)0, (a.N * a.H * a.W) * a.omcs * 2, 0x00020000);
  // LEAN: offset pair (2t, 2t+1) and mask logit (18+t) of pixel `pix` for tap t, zeros when !ok
  auto omload = [&](bool ok, int pix, int t, unsigned& off2, unsigned& mlog) {
    const unsigned base = (unsigned)(pix * a.omcs) * 2u;
    off2 = __builtin_amdgcn_raw_buffer_load_b32(omr, ok ? base + 4u * t : OOR, 0, 0);
    mlog = __builtin_amdgcn_raw_buffer_load_b16(omr, ok ? base + 2u * (18 + t) : OOR, 0, 0);
  };
  auto bf_lo = [](unsigned v) { return __uint_as_float(v << 16); };
  auto bf_hi = [](unsigned v) { return __uint_as_float(v & 0xFFFF0000u); };
  auto inimg = [&](int yy, int xx) { return yy >= 0 && yy < a.H && xx >= 0 && xx < a.W; };

  // offset / mask rows of the 14x14 neighbourhood (zero outside the image)
  if constexpr (!LEAN)
  for (int q = tid; q < GCELL * 4; q += 256) {
    const int cell = q >> 2, ch = (q & 3) * 8;
    const int yy = wy0 + cell / GWIN, xx = wx0 + cell % GWIN;
    st16(&oms[cell * 32 + ch], inimg(yy, xx) ? ld16(a.om + (long)(ibase + yy * a.W + xx) * a.omcs + ch) : z4);
  }

  // ---------------- phase 1: offset / mask-logit gradients of the tile's 64 output pixels ----------------
  if (!(mode & 1)) {
    __bf16* xwin = reinterpret_cast<__bf16*>(reg);
    __bf16* slab0 = reinterpret_cast<__bf16*>(reg + L::P1X);
    __bf16* slab1 = L::SB ? slab0 : slab0 + 64 * L::PW1;
    float* dsum = reinterpret_cast<float*>(reg + L::P1X + L::P1W);  // [pixel][tap][3]: mask, dy, dx sums
    for (int i = tid; i < 64 * 27; i += 256) dsum[i] = 0.f;
    const int pl = 16 * wave + (lane & 15);
    const int ph = h0 + (pl >> 3), pw = w0 + (pl & 7);
    const bool pok = ph < a.H && pw < a.W;
    const long ppix = ibase + (long)ph * a.W + pw;
    const __bf16* om_p = oms + ((ph - wy0) * GWIN + pw - wx0) * 32;
    unsigned po2 = 0u, pml = 0u;  // LEAN: this tap's offset pair / mask logit of the lane's pixel (one tap ahead)
    if constexpr (LEAN) omload(pok, (int)ppix, 0, po2, pml);
    bf16x8 fb[2 * CO];  // dy fragments of this lane's pixel (B operand, k = output channel)
#pragma unroll
    for (int k = 0; k < 2 * CO; ++k) {
      u32x4 v = z4;
      if (pok) v = ld16(a.dy + ppix * a.dycs + 32 * k + 8 * g);
      fb[k] = *reinterpret_cast<bf16x8*>(&v);
    }
    u32x4 wreg[2 * CO];
    auto wload = [&](int t, int cc) {
#pragma unroll
      for (int i = 0; i < 2 * CO; ++i) {
        const int q = tid + 256 * i, row = q / (8 * CO), cch = q - row * 8 * CO;
        wreg[i] = __builtin_amdgcn_raw_buffer_load_b128(wr, (unsigned)(((t * C + cc * 64 + row) * Cout) + cch * 8) * 2u, 0, 0);
      }
    };
    auto wstore = [&](__bf16* sl) {
#pragma unroll
      for (int i = 0; i < 2 * CO; ++i) {
        const int q = tid + 256 * i, row = q / (8 * CO), cch = q - row * 8 * CO;
        st16(&sl[row * L::PW1 + cch * 8], wreg[i]);
      }
    };
#pragma unroll 1
    for (int cc = 0; cc < CC; ++cc) {
      wload(0, cc);
      __syncthreads();  // the previous chunk's x window and slabs no longer read
      for (int q = tid; q < GCELL * 8; q += 256) {
        const int cell = q >> 3, ch = (q & 7) * 8;
        const int yy = wy0 + cell / GWIN, xx = wx0 + cell % GWIN;
        const u32x4 v = inimg(yy, xx) ? ld16(a.x + (long)(ibase + yy * a.W + xx) * a.xcs + cc * 64 + ch) : z4;
        __bf16* d = &xwin[cell * L::XP + ch];
        if constexpr (LEAN) {  // 136-byte rows: two 8-byte stores
          *reinterpret_cast<u32x2*>(d) = (u32x2){v.x, v.y};
          *reinterpret_cast<u32x2*>(d + 4) = (u32x2){v.z, v.w};
        } else {
          st16(d, v);
        }
      }
      wstore(slab0);
      if (!L::SB) wload(1, cc);
      __syncthreads();
#pragma unroll 1
      for (int t = 0; t < 9; ++t) {
        const __bf16* sl = (t & 1) ? slab1 : slab0;
        if (L::SB) {
          if (t + 1 < 9) wload(t + 1, cc);
        } else {  // two slabs: W_{t+1} (loaded during tap t-1) into the slab tap t-1 read, then fetch W_{t+2}
          if (t + 1 < 9) wstore((t & 1) ? slab0 : slab1);
          if (t + 2 < 9) wload(t + 2, cc);
        }
        f32x4 acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < 2 * CO; ++k)
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                *reinterpret_cast<const bf16x8*>(&sl[(16 * i + (lane & 15)) * L::PW1 + 32 * k + 8 * g]), fb[k], acc[i], 0,
                0, 0);
        }
        float oy, ox, ml;
        if constexpr (LEAN) {
          oy = bf_lo(po2), ox = bf_hi(po2), ml = bf_lo(pml);
          if (t + 1 < 9) omload(pok, (int)ppix, t + 1, po2, pml);
        } else {
          oy = (float)om_p[2 * t], ox = (float)om_p[2 * t + 1], ml = (float)om_p[18 + t];
        }
        const float mk = sigm(ml);
        Corners c0;
        sample((float)(ph - 1 + t / 3) + oy, (float)(pw - 1 + t % 3) + ox, a.H, a.W, c0);
        // the four corners' channels 16 i + 4 g .. +3: from the staged neighbourhood, or (corner outside it) global.
        // The bilinear value and its two slopes are linear in the corners, so the channel sums are taken per corner
        // first (D_q = sum_c dcols_c x_qc: one FMA per channel and corner) and interpolated once per lane.
        // Corners inside the 14x14 neighbourhood (|offset| < ~3 px) read the staged window; the rest are fetched
        // from global in a separate, wave-uniform branch, so the common path never waits on the memory counter
        // (the next tap's W_t^T slab loads stay in flight under the LDS reads and the FMAs).
        u32x2 xv[4][4];
        bool farq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cy = c0.y0 + (q >> 1) - wy0, cx = c0.x0 + (q & 1) - wx0;
          const bool inwin = (unsigned)cy < (unsigned)GWIN && (unsigned)cx < (unsigned)GWIN;
          farq[q] = !inwin && pok && c0.ok[q];
          const __bf16* xr0 = &xwin[(inwin ? cy * GWIN + cx : 0) * L::XP + 4 * g];
#pragma unroll
          for (int i = 0; i < 4; ++i) xv[q][i] = *reinterpret_cast<const u32x2*>(xr0 + 16 * i);
        }
        if (__ballot(farq[0] || farq[1] || farq[2] || farq[3])) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int pix = ibase + (c0.y0 + (q >> 1)) * a.W + c0.x0 + (q & 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(
                  xr, farq[q] ? (unsigned)(pix * a.xcs + cc * 64 + 16 * i + 4 * g) * 2u : OOR, 0, 0);
              if (farq[q]) xv[q][i] = v;
            }
          }
          __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) here, so the common path below carries no wait
        }
        // D_q on the packed bf16 dot unit: dcols rounded to bf16 pairs once per tap (the products are exact in
        // fp32, the sums fp32), 8 v_dot2 per corner instead of 16 conversions + 16 FMAs
        bf16x2 dp[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dp[i][0] = (bf16x2){(__bf16)acc[i][0], (__bf16)acc[i][1]};
          dp[i][1] = (bf16x2){(__bf16)acc[i][2], (__bf16)acc[i][3]};
        }
        float D[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float d = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            // whole-vector bit cast + swizzles: hipcc (ROCm 7.2) folds bit_cast(bf16x2, v.y) to v.x
            const bf16x4 v = __builtin_bit_cast(bf16x4, xv[q][i]);
            d = __builtin_amdgcn_fdot2_f32_bf16(dp[i][0], v.xy, d, false);
            d = __builtin_amdgcn_fdot2_f32_bf16(dp[i][1], v.zw, d, false);
          }
          D[q] = pok && c0.ok[q] ? d : 0.f;
        }
        const float top = D[0] + c0.lx * (D[1] - D[0]);
        const float bot = D[2] + c0.lx * (D[3] - D[2]);
        const float d01 = D[1] - D[0], d23 = D[3] - D[2];
        float smk = top + c0.ly * (bot - top);
        float spy = bot - top, spx = d01 + c0.ly * (d23 - d01);
        smk += __shfl_xor(smk, 16, 64);
        smk += __shfl_xor(smk, 32, 64);
        spy += __shfl_xor(spy, 16, 64);
        spy += __shfl_xor(spy, 32, 64);
        spx += __shfl_xor(spx, 16, 64);
        spx += __shfl_xor(spx, 32, 64);
        if (g == 0) {
          float* d = dsum + (pl * 9 + t) * 3;
          if constexpr (LEAN) {  // one channel chunk: the finished dom values
            d[0] = smk * mk * (1.f - mk);
            d[1] = mk * spy;
            d[2] = mk * spx;
          } else {
            d[0] += smk;
            d[1] += spy;
            d[2] += spx;
          }
        }
        // corners whose destination tile cannot see this source: scatter this chunk of dcols into dxf
        if (pok) {
          const int sy = t / 3 - 1, sx = t % 3 - 1;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (!c0.ok[q]) continue;
            const int yy = c0.y0 + (q >> 1), xx = c0.x0 + (q & 1);
            const int ry = ph - (yy & ~(GT - 1)) + sy, rx = pw - (xx & ~(GT - 1)) + sx;
            if (ry < -2 || ry > GSUB - 3 || rx < -2 || rx > GSUB - 3) {
              const float wq = mk * c0.w[q];
              float* dst = dxf + (long)(ibase + yy * a.W + xx) * C + cc * 64 + 4 * g;
#pragma unroll
              for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) unsafeAtomicAdd(dst + 16 * i + e, wq * acc[i][e]);
              if (g == 0) flags[(n * th + (yy >> 3)) * tw + (xx >> 3)] = 1;
            }
          }
        }
        __syncthreads();
        if (L::SB && t + 1 < 9) {  // one slab: refill it after every wave's tap-t MFMAs (barrier above)
          wstore(slab0);
          __syncthreads();
        }
      }
    }
    // dom rows: offsets d = m * sum(g * d sample / d p), mask logit d = sum(g * sample) * m (1 - m)
    if (tid < 64) {
      const int hh = h0 + (tid >> 3), ww = w0 + (tid & 7);
      if (hh < a.H && ww < a.W) {
        const __bf16* o = oms + ((hh - wy0) * GWIN + ww - wx0) * 32;
        __bf16 row[32];
#pragma unroll
        for (int k = 27; k < 32; ++k) row[k] = (__bf16)0.f;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const float* d = dsum + (tid * 9 + t) * 3;
          if constexpr (LEAN) {
            row[2 * t] = (__bf16)d[1];
            row[2 * t + 1] = (__bf16)d[2];
            row[18 + t] = (__bf16)d[0];
          } else {
            const float mk = sigm((float)o[18 + t]);
            row[2 * t] = (__bf16)(mk * d[1]);
            row[2 * t + 1] = (__bf16)(mk * d[2]);
            row[18 + t] = (__bf16)(d[0] * mk * (1.f - mk));
          }
        }
        __bf16* dst = a.dom + (long)(ibase + hh * a.W + ww) * a.domcs;
#pragma unroll
        for (int k = 0; k < 4; ++k) st16(dst + 8 * k, *reinterpret_cast<const u32x4*>(&row[8 * k]));
      }
    }
  }

  // ---------------- phase 2: dx of the tile's 64 input pixels ----------------
  if (mode & 2) return;
  __syncthreads();  // the dom rows are read out of the phase-1 sums that S_t is about to overwrite
  __bf16* dyw = reinterpret_cast<__bf16*>(reg);
  __bf16* S = reinterpret_cast<__bf16*>(reg + L::P2Y);
  __bf16* Wsl = reinterpret_cast<__bf16*>(reg + L::P2Y + L::P2S + (LEAN ? 64 : 0));
  f32x4 dxa[CC][4];  // dx^T: [c chunk][c tile] rows c = 16 i + 4 g + e, column q = 16 wave + (lane & 15)
#pragma unroll
  for (int cc = 0; cc < CC; ++cc)
#pragma unroll
    for (int i = 0; i < 4; ++i) dxa[cc][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  // neighbourhood row of this lane's sub-window sources at tap (0, 0) shift, per K step and half (-1: k >= GK, the
  // window's zero row); a tap subtracts its uniform shift sy * GWIN + sx
  int gbase[GKS][2];
#pragma unroll
  for (int kk = 0; kk < GKS; ++kk)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 32 * kk + 16 * h + 4 * g + q4;
      gbase[kk][h] = k < GK ? gsrc_row(k, 0, 0) : -1;
    }
  const __bf16* Sq = S + (16 * wave + (lane & 15)) * L::SP;  // this lane's destination row of S_t
  u32x4 wreg[2];
  auto wissue = [&](int t, int cc, int coc) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i;
      wreg[i] = __builtin_amdgcn_raw_buffer_load_b128(
          wr, (unsigned)(((t * C + cc * 64 + (q >> 3)) * Cout) + coc * 64 + (q & 7) * 8) * 2u, 0, 0);
    }
  };
  auto wst = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = tid + 256 * i;
      __bf16* d = &Wsl[(q >> 3) * L::WP + (q & 7) * 8];
      if constexpr (LEAN) {  // 136-byte rows: two 8-byte stores
        *reinterpret_cast<u32x2*>(d) = (u32x2){wreg[i].x, wreg[i].y};
        *reinterpret_cast<u32x2*>(d + 4) = (u32x2){wreg[i].z, wreg[i].w};
      } else {
        st16(d, wreg[i]);
      }
    }
  };
  bf16x8 gb[2];  // G_t^T as the B operand of dx^T += W_t^T G_t^T (k = co, slots {16 (2kk+h) + 4 g + e})
  auto dxmma = [&](int cc) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const __bf16* wrow = Wsl + (16 * i + (lane & 15)) * L::WP + 32 * kk + 4 * g;
        u32x2 aa[2] = {*reinterpret_cast<const u32x2*>(wrow), *reinterpret_cast<const u32x2*>(wrow + 16)};
        dxa[cc][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(aa), gb[kk], dxa[cc][i], 0, 0, 0);
      }
  };
  // LEAN: source k = tid's offset pair / mask logit for the coming tap (one tap ahead)
  unsigned so2 = 0u, sml = 0u;
  auto somload = [&](int t) {
    const int ky = tid / GSUB, kx = tid - ky * GSUB;
    const int py = wy0 + ky + 2 - t / 3, px = wx0 + kx + 2 - t % 3;
    omload(tid < GK && inimg(py, px), ibase + py * a.W + px, t, so2, sml);
  };
  if constexpr (LEAN) somload(0);
  // S_t starts all-zero; thread k (< 144) writes and later clears only its own column
  for (int q = tid; q < 64 * L::SP / 8; q += 256) st16(&S[8 * q], z4);
  if (tid < 8) kmask[tid] = 0u;
  int prevq[4] = {-1, -1, -1, -1};
#pragma unroll 1
  for (int coc = 0; coc < CO; ++coc) {
    wissue(0, 0, coc);
    __syncthreads();  // phase-1 buffers / the previous chunk's dy window no longer read
    for (int q = tid; q < (GCELL + 1) * 8; q += 256) {
      const int row = q >> 3, ch = (q & 7) * 8;
      const int yy = wy0 + row / GWIN, xx = wx0 + row % GWIN;
      st16(&dyw[row * L::DP + dsw<LEAN>(row, ch)], row < GCELL && inimg(yy, xx)
                                     ? ld16(a.dy + (long)(ibase + yy * a.W + xx) * a.dycs + coc * 64 + ch)
                                     : z4);
    }
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int sy = t / 3 - 1, sx = t % 3 - 1;
      const int tt = coc * 9 + t;
      __syncthreads();  // the previous tap's S_t / W slab / masks no longer read; dy window staged
      wst();
      if (CC > 1) wissue(t, 1, coc);
      else if (t + 1 < 9) wissue(t + 1, 0, coc);
      else if (coc + 1 < CO) wissue(0, 0, coc + 1);
      if (tid < 4) kmask[4 * ((tt + 1) & 1) + tid] = 0u;  // next tap's masks (read after two more barriers)
      bool hit[4] = {false, false, false, false};  // this source has entries in each wave's destination rows
      if (tid < GK) {  // source k = tid of the tap's sub-window: its corners that land in this tile
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (prevq[q] >= 0) S[prevq[q] * L::SP + tid] = (__bf16)0.f;
        const int ky = tid / GSUB, kx = tid - ky * GSUB;
        const int cy = ky + 1 - sy, cx = kx + 1 - sx;
        const int py = wy0 + cy, px = wx0 + cx;
        const bool sok = inimg(py, px);
        float oy, ox, ml;
        if constexpr (LEAN) {
          oy = bf_lo(so2), ox = bf_hi(so2), ml = bf_lo(sml);
          if (t + 1 < 9) somload(t + 1);
        } else {
          const __bf16* o = oms + (cy * GWIN + cx) * 32;
          oy = (float)o[2 * t], ox = (float)o[2 * t + 1], ml = (float)o[18 + t];
        }
        const float mk = sigm(ml);
        Corners c0;
        sample((float)(py - 1 + t / 3) + oy, (float)(px - 1 + t % 3) + ox, a.H, a.W, c0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int qy = c0.y0 + (q >> 1) - h0, qx = c0.x0 + (q & 1) - w0;
          prevq[q] = -1;
          if (sok && c0.ok[q] && qy >= 0 && qy < GT && qx >= 0 && qx < GT) {
            prevq[q] = qy * GT + qx;
            S[prevq[q] * L::SP + tid] = (__bf16)(mk * c0.w[q]);
            hit[qy >> 1] = true;
          }
        }
      }
      // K step of source k = k >> 5: each half wave is one K step, so a ballot gives the wave's two bits; then one
      // LDS atomic per wave and destination wave (same-address LDS atomics from every lane serialise)
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        const unsigned long long m = __ballot(hit[w4]);
        const unsigned b = ((unsigned)m ? 1u << (2 * wave) : 0u) | ((unsigned)(m >> 32) ? 2u << (2 * wave) : 0u);
        if (lane == 0 && b) atomicOr(&kmask[4 * (tt & 1) + w4], b);
      }
      __syncthreads();  // S_t, masks and the W slab complete
      // G_t^T (64 co x this wave's 16 destinations) = dy_sub^T . S_t^T, skipping all-zero K steps
      const unsigned km = (mode & 4) ? 0xFFFFFFFFu : kmask[4 * (tt & 1) + wave];
      f32x4 ga[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) ga[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < GKS; ++kk) {
        if (!(km & (1u << kk))) continue;
        const __bf16* sr = Sq + 32 * kk + 4 * g;
        u32x2 bs[2] = {*reinterpret_cast<const u32x2*>(sr), *reinterpret_cast<const u32x2*>(sr + 16)};
        const bf16x8 fbs = *reinterpret_cast<bf16x8*>(bs);
        const int tsh = sy * GWIN + sx;
        const int rlo = gbase[kk][0] < 0 ? GCELL : gbase[kk][0] - tsh, rhi = gbase[kk][1] < 0 ? GCELL : gbase[kk][1] - tsh;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v4s aa[2] = {tr16(dyw + rlo * L::DP + dsw<LEAN>(rlo, 16 * j + 4 * p4)),
                       tr16(dyw + rhi * L::DP + dsw<LEAN>(rhi, 16 * j + 4 * p4))};
          ga[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(aa), fbs, ga[j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        __bf16* e = reinterpret_cast<__bf16*>(&gb[kk]);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) e[4 * h + r] = (__bf16)ga[2 * kk + h][r];
      }
      dxmma(0);
#pragma unroll
      for (int cc = 1; cc < CC; ++cc) {
        __syncthreads();
        wst();
        if (cc + 1 < CC) wissue(t, cc + 1, coc);
        else if (t + 1 < 9) wissue(t + 1, 0, coc);
        else if (coc + 1 < CO) wissue(0, 0, coc + 1);
        __syncthreads();
        dxmma(cc);
      }
    }
  }
  // dx rows: lane (g, q) holds channels 16 i + 4 g .. +3 of destination q
  const int ql = 16 * wave + (lane & 15), qy = h0 + (ql >> 3), qx = w0 + (ql & 7);
  if (qy < a.H && qx < a.W) {
    __bf16* dst = a.dx + (long)(ibase + qy * a.W + qx) * a.dxcs + 4 * g;
#pragma unroll
    for (int cc = 0; cc < CC; ++cc)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __bf16 v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (__bf16)dxa[cc][i][e];
        *reinterpret_cast<u32x2*>(dst + cc * 64 + 16 * i) = *reinterpret_cast<u32x2*>(v);
      }
  }
}

template <int CC, int CO, int OCC>
__global__ void __launch_bounds__(256, OCC) dcn_bwd_kernel(DcnArgs a, float* dxf, int* flags, int mode) {
  dcn_bwd_body<CC, CO>(a, dxf, flags, mode, xcd_order(blockIdx.x, gridDim.x));
}
template <int CC, int CO, int OCC>
__global__ void __launch_bounds__(256, OCC) dcn_bwd_levels_kernel(DcnLevels L, int mode) {
  const int b = xcd_order(blockIdx.x, gridDim.x), l = dcn_level(L, b);
  dcn_bwd_body<CC, CO>(L.a[l], L.dxf[l], L.flags[l], mode, b - L.start[l]);
}

// flagged tiles: dx += dxf (far corners), then dxf and the flag back to zero
__device__ __forceinline__ void dcn_far_apply_body(const DcnArgs& a, float* dxf, int* flags, int b) {
  const int tw = (a.W + GT - 1) / GT, th = (a.H + GT - 1) / GT;
  if (flags[b] == 0) return;
  const int n = b / (tw * th), rem = b - n * tw * th;
  const int h0 = (rem / tw) * GT, w0 = (rem % tw) * GT;
  const int cq = a.C / 4;  // float4 groups per pixel
  for (int i = threadIdx.x; i < 64 * cq; i += 256) {
    const int p = i / cq, c = (i - p * cq) * 4;
    const int hh = h0 + (p >> 3), ww = w0 + (p & 7);
    if (hh >= a.H || ww >= a.W) continue;
    const long pix = (long)n * a.H * a.W + (long)hh * a.W + ww;
    float4* f = reinterpret_cast<float4*>(dxf + pix * a.C + c);
    const float4 v = *f;
    __bf16* d = a.dx + pix * a.dxcs + c;
    d[0] = (__bf16)((float)d[0] + v.x);
    d[1] = (__bf16)((float)d[1] + v.y);
    d[2] = (__bf16)((float)d[2] + v.z);
    d[3] = (__bf16)((float)d[3] + v.w);
    *f = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  if (threadIdx.x == 0) flags[b] = 0;
}
__global__ void __launch_bounds__(256) dcn_far_apply_kernel(DcnArgs a, float* dxf, int* flags) {
  dcn_far_apply_body(a, dxf, flags, blockIdx.x);
}
__global__ void __launch_bounds__(256) dcn_far_apply_levels_kernel(DcnLevels L) {
  const int b = blockIdx.x, l = dcn_level(L, b);
  dcn_far_apply_body(L.a[l], L.dxf[l], L.flags[l], b - L.start[l]);
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
  const int fco = dcn_fwd_fco(Cout);
  const int blocks = cdiv(M, FBM) * (Cout / fco);
  if (fco == 128) hipLaunchKernelGGL(dcn_fwd_kernel<128>, dim3(blocks), dim3(512), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(dcn_fwd_kernel<64>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("adr_dcn_fwd_bf16");
}

extern "C" int adr_dcn_wgrad_bf16_splits(int N, int H, int W, int C, int Cout) {
  const long M = (long)N * H * W;
  const long steps = (M + WR - 1) / WR;
  const int tiles = 9 * (C / 64) * (Cout / dcn_wg_cot(Cout));
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
  dim3 grid(9 * (C / 64) * (Cout / dcn_wg_cot(Cout)), splits);
  switch (dcn_wg_cot(Cout)) {
    case 256: hipLaunchKernelGGL(dcn_wgrad_kernel<256>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
    case 128: hipLaunchKernelGGL(dcn_wgrad_kernel<128>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
    default: hipLaunchKernelGGL(dcn_wgrad_kernel<64>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
  }
  return check_launch("adr_dcn_wgrad_bf16");
}

extern "C" int adr_dcn_bwd_bf16(const void* x, int xcs, const void* om, int omcs, const void* dy, int dycs,
                                const void* w_t, void* dx, int dxcs, void* dom, int domcs, float* dxf, int* tile_flags,
                                int N, int H, int W, int C, int Cout, void* stream) {
  if (int rc = dcn_check(N, H, W, C, Cout, xcs, omcs)) return rc;
  ADR_REQUIRE(C == Cout && (C == 64 || C == 128 || C == 256),
              "dcn_bwd (bf16 fused): C == Cout in {64, 128, 256} (C=%d Cout=%d)", C, Cout);
  ADR_REQUIRE(domcs >= 32 && domcs % 8 == 0 && dycs % 8 == 0 && dxcs % 8 == 0 && dxcs >= C,
              "dcn_bwd: domcs=%d dycs=%d dxcs=%d", domcs, dycs, dxcs);
  DcnArgs a{};
  a.x = (const __bf16*)x;
  a.om = (const __bf16*)om;
  a.dy = (const __bf16*)dy;
  a.w = (const __bf16*)w_t;
  a.dx = (__bf16*)dx;
  a.dom = (__bf16*)dom;
  a.xcs = xcs;
  a.omcs = omcs;
  a.dycs = dycs;
  a.dxcs = dxcs;
  a.domcs = domcs;
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Cout = Cout;
  a.x_bytes = (int)((long)N * H * W * xcs * 2);
  a.w_bytes = 9 * C * Cout * 2;
  hipStream_t s = (hipStream_t)stream;
  const int blocks = N * cdiv(H, GT) * cdiv(W, GT);
  static const int mode = getenv("ADR_DCN_BWD_MODE") ? atoi(getenv("ADR_DCN_BWD_MODE")) : 0;  // A/B: 1/2 skip a phase
  if (C == 64) hipLaunchKernelGGL((dcn_bwd_kernel<1, 1, 3>), dim3(blocks), dim3(256), 0, s, a, dxf, tile_flags, mode);
  else if (C == 128) hipLaunchKernelGGL((dcn_bwd_kernel<2, 2, 2>), dim3(blocks), dim3(256), 0, s, a, dxf, tile_flags, mode);
  else hipLaunchKernelGGL((dcn_bwd_kernel<4, 4, 2>), dim3(blocks), dim3(256), 0, s, a, dxf, tile_flags, mode);
  if (int rc = check_launch("adr_dcn_bwd_bf16")) return rc;
  hipLaunchKernelGGL(dcn_far_apply_kernel, dim3(blocks), dim3(256), 0, s, a, dxf, tile_flags);
  return check_launch("adr_dcn_bwd_bf16 (far corners)");
}

/* Number of 8x8 tiles (the tile_flags length adr_dcn_bwd_bf16 needs). */
extern "C" int adr_dcn_bwd_tiles(int N, int H, int W) { return N * cdiv(H, GT) * cdiv(W, GT); }

// ---- the three AYHead pyramid levels per launch (LevelDCNFn): each entry point writes exactly what its per-level
// counterpart above writes for every level (same blocks, same arithmetic), in one launch (bwd: + one far-corner
// launch) instead of one per level ----
static int dcn_levels_fill(const adr_dcn_level* lv, int levels, int xcs, int omcs, int N, int C, int Cout,
                           DcnLevels& L) {
  ADR_REQUIRE(lv && levels >= 1 && levels <= 3, "dcn levels: %d levels (1..3)", levels);
  L = DcnLevels{};
  L.nl = levels;
  for (int l = 0; l < levels; ++l) {
    if (int rc = dcn_check(N, lv[l].H, lv[l].W, C, Cout, xcs, omcs)) return rc;
    DcnArgs& a = L.a[l];
    a.x = (const __bf16*)lv[l].x;
    a.om = (const __bf16*)lv[l].om;
    a.xcs = xcs;
    a.omcs = omcs;
    a.N = N;
    a.H = lv[l].H;
    a.W = lv[l].W;
    a.C = C;
    a.Cout = Cout;
    a.x_bytes = (int)((long)N * a.H * a.W * xcs * 2);
  }
  return 0;
}

extern "C" int adr_dcn_fwd_bf16_levels(const adr_dcn_level* lv, int levels, int xcs, int omcs, const void* w_krsc,
                                       int ycs, int N, int C, int Cout, void* stream) {
  DcnLevels L;
  if (int rc = dcn_levels_fill(lv, levels, xcs, omcs, N, C, Cout, L)) return rc;
  int total = 0;
  for (int l = 0; l < levels; ++l) {
    DcnArgs& a = L.a[l];
    a.w = (const __bf16*)w_krsc;
    a.y = (__bf16*)lv[l].y;
    a.ycs = ycs;
    a.w_bytes = Cout * 9 * C * 2;
    L.start[l] = total;
    total += cdiv((long)N * a.H * a.W, FBM) * (Cout / dcn_fwd_fco(Cout));
  }
  L.start[levels] = total;
  if (dcn_fwd_fco(Cout) == 128)
    hipLaunchKernelGGL(dcn_fwd_levels_kernel<128>, dim3(total), dim3(512), 0, (hipStream_t)stream, L);
  else
    hipLaunchKernelGGL(dcn_fwd_levels_kernel<64>, dim3(total), dim3(256), 0, (hipStream_t)stream, L);
  return check_launch("adr_dcn_fwd_bf16_levels");
}

extern "C" int adr_dcn_wgrad_bf16_levels(const adr_dcn_level* lv, int levels, int xcs, int omcs, int dycs, int N,
                                         int C, int Cout, void* stream) {
  DcnLevels L;
  if (int rc = dcn_levels_fill(lv, levels, xcs, omcs, N, C, Cout, L)) return rc;
  int total = 0;
  const int tiles = 9 * (C / 64) * (Cout / dcn_wg_cot(Cout));
  for (int l = 0; l < levels; ++l) {
    DcnArgs& a = L.a[l];
    ADR_REQUIRE(lv[l].part && lv[l].splits >= 1, "dcn_wgrad levels: partials / splits of level %d", l);
    a.dy = (const __bf16*)lv[l].dy;
    a.dycs = dycs;
    a.part = lv[l].part;
    a.dy_bytes = (int)((long)N * a.H * a.W * dycs * 2);
    const long M = (long)N * a.H * a.W;
    const long steps = (M + WR - 1) / WR;
    a.rows_per_split = ((steps + lv[l].splits - 1) / lv[l].splits) * WR;
    a.splits = lv[l].splits;
    L.tiles[l] = tiles;
    L.start[l] = total;
    total += tiles * lv[l].splits;
  }
  L.start[levels] = total;
  switch (dcn_wg_cot(Cout)) {
    case 256: hipLaunchKernelGGL(dcn_wgrad_levels_kernel<256>, dim3(total), dim3(256), 0, (hipStream_t)stream, L); break;
    case 128: hipLaunchKernelGGL(dcn_wgrad_levels_kernel<128>, dim3(total), dim3(256), 0, (hipStream_t)stream, L); break;
    default: hipLaunchKernelGGL(dcn_wgrad_levels_kernel<64>, dim3(total), dim3(256), 0, (hipStream_t)stream, L); break;
  }
  return check_launch("adr_dcn_wgrad_bf16_levels");
}

extern "C" int adr_dcn_bwd_bf16_levels(const adr_dcn_level* lv, int levels, int xcs, int omcs, int dycs,
                                       const void* w_t, int dxcs, int domcs, int N, int C, int Cout, void* stream) {
  DcnLevels L;
  if (int rc = dcn_levels_fill(lv, levels, xcs, omcs, N, C, Cout, L)) return rc;
  ADR_REQUIRE(C == Cout && (C == 64 || C == 128 || C == 256),
              "dcn_bwd levels (bf16 fused): C == Cout in {64, 128, 256} (C=%d Cout=%d)", C, Cout);
  ADR_REQUIRE(domcs >= 32 && domcs % 8 == 0 && dycs % 8 == 0 && dxcs % 8 == 0 && dxcs >= C,
              "dcn_bwd levels: domcs=%d dycs=%d dxcs=%d", domcs, dycs, dxcs);
  int total = 0;
  for (int l = 0; l < levels; ++l) {
    DcnArgs& a = L.a[l];
    ADR_REQUIRE(lv[l].dxf && lv[l].flags && lv[l].dx && lv[l].dom, "dcn_bwd levels: buffers of level %d", l);
    a.dy = (const __bf16*)lv[l].dy;
    a.w = (const __bf16*)w_t;
    a.dx = (__bf16*)lv[l].dx;
    a.dom = (__bf16*)lv[l].dom;
    a.dycs = dycs;
    a.dxcs = dxcs;
    a.domcs = domcs;
    a.w_bytes = 9 * C * Cout * 2;
    L.dxf[l] = lv[l].dxf;
    L.flags[l] = lv[l].flags;
    L.start[l] = total;
    total += N * cdiv(a.H, GT) * cdiv(a.W, GT);
  }
  L.start[levels] = total;
  hipStream_t s = (hipStream_t)stream;
  static const int mode = getenv("ADR_DCN_BWD_MODE") ? atoi(getenv("ADR_DCN_BWD_MODE")) : 0;
  if (C == 64) hipLaunchKernelGGL((dcn_bwd_levels_kernel<1, 1, 3>), dim3(total), dim3(256), 0, s, L, mode);
  else if (C == 128) hipLaunchKernelGGL((dcn_bwd_levels_kernel<2, 2, 2>), dim3(total), dim3(256), 0, s, L, mode);
  else hipLaunchKernelGGL((dcn_bwd_levels_kernel<4, 4, 2>), dim3(total), dim3(256), 0, s, L, mode);
  if (int rc = check_launch("adr_dcn_bwd_bf16_levels")) return rc;
  hipLaunchKernelGGL(dcn_far_apply_levels_kernel, dim3(total), dim3(256), 0, s, L);
  return check_launch("adr_dcn_bwd_bf16_levels (far corners)");
}
