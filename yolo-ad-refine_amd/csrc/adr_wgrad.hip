// bf16 weight-gradient GEMM for NHWC convolutions (the WGRAD third of adr_gemm.hip's engine, re-tiled):
//   dw[co][tap][ci] = sum_p dy[p][co] * x[n, oy*s-p+kh, ox*s-p+kw, ci]        (p = (n, oy, ox), split over p)
// Both operands arrive as [p][channel] rows (channels contiguous in HBM). They are staged into LDS as
// plain row images — 16-byte global loads stored as 16-byte LDS writes, no scalar transposition — and the
// MFMA fragments, which need 8 consecutive reduction rows per lane, are read with gfx950's transposing
// ds_read_b64_tr_b16 (two 4-row reads per fragment).
//
// MFMA v_mfma_f32_16x16x32_bf16: lane l supplies A[l&15][k(8(l>>4)+j)] and B[k(8(l>>4)+j)][l&15], j < 8.
// The k-slot -> LDS-row map is a free permutation shared by A and B: slot (g = l>>4, j) reads row
// 4g + j (j < 4) and 16 + 4g + (j-4) (j >= 4), so the two 16-lane groups of each 32-lane half read 8
// consecutive rows; with the row pitch an odd multiple of 32 bytes those 8 rows hit 8 disjoint bank windows
// (conflict-free, MI355X bank = (addr/4) % 64 for tr reads).
//
// Tile: BM output channels x BN input channels of one tap. 4 waves as WM x WN spatial x WK reduction
// slices (WK > 1 for thin tiles, combined through LDS at the end). Split over p for parallelism; split
// partials are reduced in fixed order by adr_gemm.hip's wgrad_reduce (deterministic).
#include "adr_common.h"
#include "adr_wgrad.h"
#include <cstdlib>

namespace adr {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

struct WgArgs {
  const __bf16* x;
  const __bf16* dy;
  float* out;  // [split][K][RS][C] partials (or dw itself when splits == 1 and not accumulating)
  int n, h, w, c, xcs, xco;
  int k, r, s, sh, sw, ph, pw, ho, wo, ycs, yco;
  long red_total;
  long red_per_split;
  int ksteps;
  int ctiles;  // input-channel tiles per tap
  int x_bytes, dy_bytes;  // buffer-descriptor extents (< 2^31): out-of-range offsets read as zero
  int accumulate;
  float* bias;  // optional: [split][2][K] rows, row half 0 = sum_p dy[p][k] over the split (the conv's bias gradient)
};

__device__ __forceinline__ v4s tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}

// XCD-aware (tile, split) order: workgroups of one split read the same pixel rows of dy / x, so consecutive
// logical ids — which walk the tiles of one split — are kept on one XCD (one L2). Returns (bx, by).
__device__ __forceinline__ void wg_xcd_block(int& bx, int& by) {
  const int gx = gridDim.x, nb = gx * gridDim.y;
  int b = blockIdx.x + blockIdx.y * gx;
  b = xcd_remap(b, nb);
  by = b / gx;
  bx = b - by * gx;
}

// KU: 32*WK-row sub-steps per k-step; (bid, split): tile and split of the block. DB: two LDS stages and two register
// sets — the loads of step t+2 are issued while step t computes (two steps of MFMA work to land behind instead of one)
// and one barrier per step; the k-steps, their order and every sum are those of the single-stage loop (bitwise equal)
template <int BM, int BN, int KU, bool DB = false>
__device__ __forceinline__ void wgrad_bf16_body(const WgArgs& a, int bid, int split) {
  constexpr int WM = BM / 16 < 2 ? BM / 16 : 2;
  constexpr int WN = BN / 16 < 2 ? BN / 16 : 2;
  constexpr int WK = 4 / (WM * WN);
  constexpr int R = 32 * WK * KU;    // reduction rows per k-step
  constexpr int WROWS = BM / WM, WCOLS = BN / WN;
  constexpr int TM = WROWS / 16, TN = WCOLS / 16;
  // row pitch (elements): odd multiple of 16 elements (32 bytes)
  constexpr int PA = ((BM / 16) % 2 == 1) ? BM : BM + 16;
  constexpr int PB = ((BN / 16) % 2 == 1) ? BN : BN + 16;
  constexpr int A_CHT = R * BM / 8, B_CHT = R * BN / 8;  // 16-byte chunks per k-step
  constexpr int A_CH = (A_CHT + 255) / 256, B_CH = (B_CHT + 255) / 256;

  constexpr int NS = DB ? 2 : 1;  // LDS stages = register sets
  __shared__ __attribute__((aligned(16))) __bf16 As[NS * R * PA];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NS * R * PB];
  __shared__ float red[WK > 1 ? (WK - 1) * BM * BN : 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave / (WM * WN), wmn = wave % (WM * WN), wm = wmn / WN, wn = wmn % WN;
  const int RS = a.r * a.s;
  // bid -> (co tile, tap, ci tile)
  const int ct = bid % a.ctiles;
  bid /= a.ctiles;
  const int tap = bid % RS;
  const int mt = bid / RS;
  const int m0 = mt * BM, c0 = ct * BN;
  const int kh = tap / a.s, kw = tap % a.s;
  const long pbeg = (long)split * a.red_per_split;
  const long pend = min(a.red_total, pbeg + a.red_per_split);
  const int hw = a.ho * a.wo;

  u32x4 ra_s[NS][A_CH], rb_s[NS][B_CH];
  constexpr unsigned OOR = 0x7FFFFFF0u;
  const __amdgpu_buffer_rsrc_t x_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dy_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);
  // per B chunk: the output pixel (img, oy, ox) of its reduction row, advanced by R rows per k-step without
  // integer division (the row of a chunk is fixed across steps: pl = q / (BN / 8))
  int b_img[B_CH], b_oy[B_CH], b_ox[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int q = tid + 256 * i;
    const long p = pbeg + q / (BN / 8);
    const int pi = (int)(p < a.red_total ? p : 0);
    b_img[i] = pi / hw;
    const int rem = pi - b_img[i] * hw;
    b_oy[i] = rem / a.wo;
    b_ox[i] = rem - b_oy[i] * a.wo;
  }

  auto load = [&](int t, auto S) {
    u32x4(&ra)[A_CH] = ra_s[decltype(S)::value];
    u32x4(&rb)[B_CH] = rb_s[decltype(S)::value];
    const long p0 = pbeg + (long)t * R;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int q = tid + 256 * i;
      const int pl = q / (BM / 8), cc = q % (BM / 8);
      const long p = p0 + pl;
      const int co = m0 + cc * 8;
      const bool ok = q < A_CHT && p < pend && co < a.k;
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(dy_rs, ok ? (unsigned)((int)p * a.ycs + a.yco + co) * 2u : OOR, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int q = tid + 256 * i;
      const int pl = q / (BN / 8), cc = q % (BN / 8);
      const long p = p0 + pl;
      const int ci = c0 + cc * 8;
      bool ok = q < B_CHT && p < pend && ci < a.c;
      const int iy = b_oy[i] * a.sh - a.ph + kh, ix = b_ox[i] * a.sw - a.pw + kw;
      ok = ok && iy >= 0 && iy < a.h && ix >= 0 && ix < a.w;
      rb[i] = __builtin_amdgcn_raw_buffer_load_b128(
          x_rs, ok ? (unsigned)(((b_img[i] * a.h + iy) * a.w + ix) * a.xcs + a.xco + ci) * 2u : OOR, 0, 0);
      b_ox[i] += R;  // next k-step's row
      while (b_ox[i] >= a.wo) {
        b_ox[i] -= a.wo;
        if (++b_oy[i] >= a.ho) {
          b_oy[i] = 0;
          ++b_img[i];
        }
      }
    }
  };
  auto store = [&](auto S, int stage) {
    const u32x4(&ra)[A_CH] = ra_s[decltype(S)::value];
    const u32x4(&rb)[B_CH] = rb_s[decltype(S)::value];
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int q = tid + 256 * i;
      if (A_CHT % 256 == 0 || q < A_CHT) st16(&As[stage * R * PA + (q / (BM / 8)) * PA + (q % (BM / 8)) * 8], ra[i]);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int q = tid + 256 * i;
      if (B_CHT % 256 == 0 || q < B_CHT) st16(&Bs[stage * R * PB + (q / (BN / 8)) * PB + (q % (BN / 8)) * 8], rb[i]);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // bias column sums ride on the dy fragments already in registers (lane: output channel i*16 + (lane & 15), 8 of
  // the k-step's pixels): four v_dot2 against ones per fragment into one fp32 per row tile, in the blocks of the
  // first (tap, input-channel) tile column, by the waves of column 0 (wave-uniform); the four lane groups' sums are
  // combined at the end. (A ones-MFMA variant cost 16 accumulator registers: 3 -> 2 waves per SIMD.)
  const bool do_bias = WK == 1 && a.bias != nullptr && tap == 0 && ct == 0 && wn == 0;
  float bsum[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) bsum[i] = 0.f;
  const bf16x2 ones2 = (bf16x2){(__bf16)1.f, (__bf16)1.f};

  // transposed-read addressing: lane (g, q4, p4) -> row rb + 4g + q4 (+16), column base + 4*p4
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int row0 = 32 * wk + 4 * g + q4;
  const __bf16* a_base = As + row0 * PA + wm * WROWS + 4 * p4;
  const __bf16* b_base = Bs + row0 * PB + wn * WCOLS + 4 * p4;

  const int ksteps = a.ksteps;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, NS - 1>;
  auto compute = [&](int stage) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const __bf16* ab = a_base + stage * R * PA + u * 32 * WK * PA;
      const __bf16* bb = b_base + stage * R * PB + u * 32 * WK * PB;
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        v4s lo = tr_read(ab + i * 16);
        v4s hi = tr_read(ab + 16 * PA + i * 16);
        v4s both[2] = {lo, hi};
        fa[i] = *reinterpret_cast<bf16x8*>(both);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        v4s lo = tr_read(bb + j * 16);
        v4s hi = tr_read(bb + 16 * PB + j * 16);
        v4s both[2] = {lo, hi};
        fb[j] = *reinterpret_cast<bf16x8*>(both);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8 f = fa[i];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            bsum[i] = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){f[2 * q], f[2 * q + 1]}, ones2, bsum[i], false);
        }
      }
    }
  };
  if constexpr (DB) {
    // step t computes stage t&1 while register set t&1 receives step t+2; step t+1 (set 1-(t&1), loaded one step
    // ago) goes into the other stage, last read in step t-1 (before the previous barrier)
    load(0, S0{});
    store(S0{}, 0);
    load(1, S1{});
    __syncthreads();
    // the loads and stores are unconditional: past the last step every chunk is out of range (p >= pend: the
    // descriptor returns zeros, no memory access), and straight-line VMEM lets the compiler count the older set's
    // loads with vmcnt(4) instead of draining the just-issued prefetch with vmcnt(0) at the store
    auto step = [&](int t, auto S) {
      constexpr int cur = decltype(S)::value;
      using SO = std::integral_constant<int, 1 - cur>;
      load(t + 2, S);
      compute(cur);
      store(SO{}, 1 - cur);
      __syncthreads();
    };
    for (int t = 0; t < ksteps; t += 2) {
      step(t, S0{});
      if (t + 1 < ksteps) step(t + 1, S1{});
    }
  } else {
    if (ksteps > 0) {
      load(0, S0{});
      store(S0{}, 0);
      __syncthreads();
    }
    for (int t = 0; t < ksteps; ++t) {
      if (t + 1 < ksteps) load(t + 1, S0{});
      compute(0);
      __syncthreads();
      if (t + 1 < ksteps) {
        store(S0{}, 0);
        __syncthreads();
      }
    }
  }

  // combine the WK reduction slices (waves wk > 0 publish, wave-slice 0 sums)
  if constexpr (WK > 1) {
    if (wk > 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int rr = wm * WROWS + i * 16 + 4 * (lane >> 4) + e, cc = wn * WCOLS + j * 16 + (lane & 15);
            red[(wk - 1) * BM * BN + rr * BN + cc] = acc[i][j][e];
          }
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rr = wm * WROWS + i * 16 + 4 * (lane >> 4) + e, cc = wn * WCOLS + j * 16 + (lane & 15);
#pragma unroll
          for (int s2 = 0; s2 < WK - 1; ++s2) acc[i][j][e] += red[s2 * BM * BN + rr * BN + cc];
        }
  }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float t = bsum[i] + __shfl_xor(bsum[i], 16, 64);
      t += __shfl_xor(t, 32, 64);
      const int co = m0 + wm * WROWS + i * 16 + (lane & 15);
      if (lane < 16 && co < a.k) a.bias[(long)split * 2 * a.k + co] = t;
    }
  }
  float* part = a.out + (long)split * a.k * ((long)RS * a.c);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int ci = c0 + wn * WCOLS + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = m0 + wm * WROWS + i * 16 + 4 * (lane >> 4) + e;
        if (co < a.k && ci < a.c) {
          float* o = part + ((long)co * RS + tap) * a.c + ci;
          *o = a.accumulate ? *o + acc[i][j][e] : acc[i][j][e];
        }
      }
    }
}

template <int BM, int BN, bool DB = false>
__global__ void __launch_bounds__(256, DB ? 3 : 1) wgrad_bf16_kernel(WgArgs a) {
  int bid, split;  // block x -> tile, block y = split (XCD-aware order)
  wg_xcd_block(bid, split);
  wgrad_bf16_body<BM, BN, wg_ku(BM, BN), DB>(a, bid, split);
}

// Grouped WGRAD: the weight gradients of many convs (the deferred ones of a backward stage, one BM x BN tile shape)
// in ONE launch. Block b belongs to entry j (start[j] <= b < start[j+1]); inside it, consecutive blocks walk the
// tiles of one split (as the single launch's XCD order groups them), so each block computes exactly what the
// entry's own launch would — same tiles, splits and fixed-order partial sums: the grouped result is bitwise the
// per-conv one. Small weight gradients (a 1x1 128 -> 128 at 20 x 20 is 100 workgroups for the whole chip) stop
// costing a launch and a half-empty machine each.
constexpr int WGB_MAX = 24;
struct WgBatch {
  WgArgs e[WGB_MAX];
  int start[WGB_MAX + 1];
  int tiles[WGB_MAX];
  int count;
};
template <int BM, int BN, bool DB = false>
__global__ void __launch_bounds__(256, DB ? 3 : 1) wgrad_bf16_batched_kernel(WgBatch b) {
  int j = 0;
  while (j + 1 < b.count && (int)blockIdx.x >= b.start[j + 1]) ++j;
  // XCD-aware order within the entry (every XCD gets an eighth of each entry, so the mix of long and short entries
  // stays balanced; the blocks of one entry with the same id % 8 share an XCD whatever start[j] is)
  const int local = xcd_remap((int)blockIdx.x - b.start[j], b.start[j + 1] - b.start[j]);
  const int split = local / b.tiles[j];
  wgrad_bf16_body<BM, BN, wg_ku(BM, BN), DB>(b.e[j], local - split * b.tiles[j], split);
}


// ------------------------------------------------------------------------------------------------------------
// 3x3 / stride-1 / pad-1 weight gradient on 2-D output tiles (the WGRAD counterpart of adr_conv.hip's
// conv3_kernel): per 128-pixel TH x TW tile, the dy tile (64 output channels) and the (TH+2) x (TW+2) input
// halo (32 input channels) are staged in LDS ONCE and all nine taps accumulate from them — the per-tap kernel
// above re-gathers x and re-reads dy for every tap. Wave w owns output channels k0 + 16w .. +15 for all nine
// taps and both 16-channel input halves (18 accumulators); the MFMA reduction runs over pixels, 32 per step,
// fragments read with the transposing ds_read_b64_tr_b16 (a B row is the lane's pixel shifted by the tap in the
// halo image). Split over tiles; partials [split][K][9][C] as the general kernel writes them.
template <int TW, int KF>
__global__ void __launch_bounds__(256, 2) wgrad3_kernel(WgArgs a) {
  constexpr int TH = 128 / TW, HWW = TW + 2, NPIX = (TH + 2) * HWW;
  constexpr int KB = 16 * KF, CK = 32;       // KF = 4: wave w = k fragment w, both c halves; KF = 2: wave w =
  constexpr int NCF = KF == 4 ? 2 : 1;       // (k fragment w % 2, c half w / 2)
  constexpr int PD = KB + 16, PX = CK + 16;  // LDS pitches (elements): odd multiples of 32 bytes
  constexpr int D_CH = 128 * KB / 8 / 256;   // dy chunks per thread
  constexpr int KQ = KB / 8;                 // 16-byte chunks per dy pixel row
  constexpr int X_TOT = NPIX * CK / 8, X_CH = (X_TOT + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 Ds[128 * PD];
  __shared__ __attribute__((aligned(16))) __bf16 Xs[NPIX * PX];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ctiles = a.c / CK;
  const int wkf = wave % KF, wcf = KF == 4 ? 0 : wave / KF;
  int bx, split;
  wg_xcd_block(bx, split);
  const int kt = bx / ctiles, ct = bx - (bx / ctiles) * ctiles;
  const int k0 = kt * KB, c0 = ct * CK;
  const int H = a.ho, W = a.wo;
  const int tx = W / TW, ty = (H + TH - 1) / TH, ntile = a.n * tx * ty;
  const int t_beg = split * (int)a.red_per_split;
  const int t_end = min(ntile, t_beg + (int)a.red_per_split);

  constexpr unsigned OOR = 0x7FFFFFF0u;
  const __amdgpu_buffer_rsrc_t x_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dy_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);
  u32x4 rd[D_CH], rx[X_CH];
  auto load = [&](int tile) {
    const int img = tile / (tx * ty), trem = tile - img * (tx * ty);
    const int y0 = (trem / tx) * TH, x0 = (trem - (trem / tx) * tx) * TW;
#pragma unroll
    for (int i = 0; i < D_CH; ++i) {
      const int e = tid + 256 * i, p = e / KQ, kq = e % KQ;
      const int y = y0 + p / TW, xx = x0 + p % TW;
      const bool ok = y < H;
      rd[i] = __builtin_amdgcn_raw_buffer_load_b128(
          dy_rs, ok ? (unsigned)(((img * H + y) * W + xx) * a.ycs + a.yco + k0 + kq * 8) * 2u : OOR, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      const int e = tid + 256 * i, q = e >> 2, cq = e & 3;
      const int hy = q / HWW, hx = q - (q / HWW) * HWW;
      const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
      const bool ok = e < X_TOT && gy >= 0 && gy < a.h && gx >= 0 && gx < a.w;
      rx[i] = __builtin_amdgcn_raw_buffer_load_b128(
          x_rs, ok ? (unsigned)(((img * a.h + gy) * a.w + gx) * a.xcs + a.xco + c0 + cq * 8) * 2u : OOR, 0, 0);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < D_CH; ++i) {
      const int e = tid + 256 * i;
      st16(&Ds[(e / KQ) * PD + (e % KQ) * 8], rd[i]);
    }
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      const int e = tid + 256 * i;
      if (e < X_TOT) st16(&Xs[(e >> 2) * PX + (e & 3) * 8], rx[i]);
    }
  };

  // transposed-read lane roles (see the header comment of this file): row 4g + q4 (+16), column 4 p4
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  // fused bias column sums (see wgrad_bf16_body): the dy fragment of each 32-pixel step, in the blocks of the first
  // input-channel tile, by the waves of input-channel half 0
  const bool do_bias = a.bias != nullptr && ct == 0 && wcf == 0;
  const bf16x2 ones2 = (bf16x2){(__bf16)1.f, (__bf16)1.f};
  float bsum = 0.f;
  f32x4 acc[9][NCF];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf) acc[t][cf] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (t_beg < t_end) load(t_beg);
  for (int tile = t_beg; tile < t_end; ++tile) {
    store();
    __syncthreads();
    if (tile + 1 < t_end) load(tile + 1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int plo = ks * 32 + 4 * g + q4, phi = plo + 16;
      const __bf16* da = Ds + wkf * 16 + 4 * p4;
      v4s lo = tr_read(da + plo * PD), hi = tr_read(da + phi * PD);
      v4s both[2] = {lo, hi};
      const bf16x8 fa = *reinterpret_cast<bf16x8*>(both);
      if (do_bias) {
#pragma unroll
        for (int q = 0; q < 4; ++q) bsum = __builtin_amdgcn_fdot2_f32_bf16((bf16x2){fa[2 * q], fa[2 * q + 1]}, ones2, bsum, false);
      }
      const int qlo = (plo / TW) * HWW + plo % TW, qhi = (phi / TW) * HWW + phi % TW;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int dq = (t / 3) * HWW + (t % 3);
#pragma unroll
        for (int cf = 0; cf < NCF; ++cf) {
          const __bf16* xb = Xs + (wcf + cf) * 16 + 4 * p4;
          v4s blo = tr_read(xb + (qlo + dq) * PX), bhi = tr_read(xb + (qhi + dq) * PX);
          v4s bb[2] = {blo, bhi};
          acc[t][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, *reinterpret_cast<bf16x8*>(bb), acc[t][cf], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  if (do_bias) {  // lane (lane & 15) holds channel k0 + wkf*16 + (lane & 15) over its 8-pixel slots: combine the groups
    float t = bsum + __shfl_xor(bsum, 16, 64);
    t += __shfl_xor(t, 32, 64);
    if (lane < 16) a.bias[(long)split * 2 * a.k + k0 + wkf * 16 + lane] = t;
  }
  float* part = a.out + (long)split * a.k * (9L * a.c);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = k0 + wkf * 16 + 4 * (lane >> 4) + e, ci = c0 + (wcf + cf) * 16 + (lane & 15);
        float* o = part + ((long)co * 9 + t) * a.c + ci;
        *o = a.accumulate ? *o + acc[t][cf][e] : acc[t][cf][e];
      }
}

// ------------------------------------------------------------------------------------------------------------
// Thin-channel 3x3 weight gradient (stride 1 or 2, pad 1, C <= 16, K <= 32: the 8/16-channel convs of the first
// C3k2 bottleneck at 160x160 and the 16 -> 32 stride-2 model.1 conv), on 128-pixel TH x 16 output tiles. The
// general kernel above gathers x per tap with 8-32-channel rows (a few bytes per pixel and tap) and re-reads dy
// for all nine taps; here each tile's dy rows (KB = 16 or 32 channels, zero-padded) and its input halo
// ((TH-1)*S+3 rows x 15*S+3 columns x 16 channels, zero-padded) are staged in LDS once, and wave w accumulates
// output pixels [32w, 32w+32) of every tile for all nine taps; the four waves' sums are combined at the end.
// Partials [split][K][9][C] as the other kernels write them.
template <int S, int KB>
__global__ void __launch_bounds__(256) wgrad3t_kernel(WgArgs a) {
  constexpr int TW = 16, TH = 8, KT = KB / 16;
  constexpr int HWW = (TW - 1) * S + 3, HH = (TH - 1) * S + 3, NPIX = HH * HWW;
  constexpr int PD = KB == 16 ? 16 : 48, PX = 16;  // LDS pitches (elements): odd multiples of 32 bytes
  constexpr int KQ = KB / 8, D_TOT = 128 * KQ, D_CH = (D_TOT + 255) / 256;
  constexpr int X_TOT = NPIX * 2, X_CH = (X_TOT + 255) / 256;
  constexpr int SM_TILES = (128 * PD + NPIX * PX) * 2, SM_RED = KB * 9 * 16 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM_TILES > SM_RED ? SM_TILES : SM_RED];
  __bf16* Ds = reinterpret_cast<__bf16*>(smem);
  __bf16* Xs = Ds + 128 * PD;
  float* red = reinterpret_cast<float*>(smem);  // the wave combine reuses the tile buffers after the last tile

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bx, split;
  wg_xcd_block(bx, split);
  (void)bx;
  const int H = a.ho, W = a.wo;
  const int tx = W / TW, ty = (H + TH - 1) / TH, ntile = a.n * tx * ty;
  const int t_beg = split * (int)a.red_per_split;
  const int t_end = min(ntile, t_beg + (int)a.red_per_split);

  constexpr unsigned OOR = 0x7FFFFFF0u;
  const __amdgpu_buffer_rsrc_t x_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dy_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_bytes, 0x00020000);
  u32x4 rd[D_CH], rx[X_CH];
  auto load = [&](int tile) {
    const int img = tile / (tx * ty), trem = tile - img * (tx * ty);
    const int y0 = (trem / tx) * TH, x0 = (trem - (trem / tx) * tx) * TW;
#pragma unroll
    for (int i = 0; i < D_CH; ++i) {
      const int e = tid + 256 * i, p = e / KQ, kq = e % KQ;
      const int y = y0 + p / TW, xx = x0 + p % TW;
      const bool ok = e < D_TOT && y < H && kq * 8 < a.k;
      rd[i] = __builtin_amdgcn_raw_buffer_load_b128(
          dy_rs, ok ? (unsigned)(((img * H + y) * W + xx) * a.ycs + a.yco + kq * 8) * 2u : OOR, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      const int e = tid + 256 * i, q = e >> 1, cq = e & 1;
      const int hy = q / HWW, hx = q - (q / HWW) * HWW;
      const int gy = y0 * S - 1 + hy, gx = x0 * S - 1 + hx;
      const bool ok = e < X_TOT && cq * 8 < a.c && gy >= 0 && gy < a.h && gx >= 0 && gx < a.w;
      rx[i] = __builtin_amdgcn_raw_buffer_load_b128(
          x_rs, ok ? (unsigned)(((img * a.h + gy) * a.w + gx) * a.xcs + a.xco + cq * 8) * 2u : OOR, 0, 0);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < D_CH; ++i) {
      const int e = tid + 256 * i;
      if (e < D_TOT) st16(&Ds[(e / KQ) * PD + (e % KQ) * 8], rd[i]);
    }
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      const int e = tid + 256 * i;
      if (e < X_TOT) st16(&Xs[(e >> 1) * PX + (e & 1) * 8], rx[i]);
    }
  };

  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  f32x4 acc[9][KT];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) acc[t][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // wave w: tile pixels [32w, 32w + 32); the transposed-read rows 4g + q4 and +16
  const int plo = wave * 32 + 4 * g + q4, phi = plo + 16;
  const int qlo = (plo / TW) * S * HWW + (plo % TW) * S, qhi = (phi / TW) * S * HWW + (phi % TW) * S;

  if (t_beg < t_end) load(t_beg);
  for (int tile = t_beg; tile < t_end; ++tile) {
    store();
    __syncthreads();
    if (tile + 1 < t_end) load(tile + 1);
    bf16x8 fa[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const __bf16* da = Ds + kt * 16 + 4 * p4;
      v4s lo = tr_read(da + plo * PD), hi = tr_read(da + phi * PD);
      v4s both[2] = {lo, hi};
      fa[kt] = *reinterpret_cast<bf16x8*>(both);
    }
    const __bf16* xb = Xs + 4 * p4;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dq = (t / 3) * HWW + (t % 3);
      v4s blo = tr_read(xb + (qlo + dq) * PX), bhi = tr_read(xb + (qhi + dq) * PX);
      v4s bb[2] = {blo, bhi};
      const bf16x8 fb = *reinterpret_cast<bf16x8*>(bb);
#pragma unroll
      for (int kt = 0; kt < KT; ++kt)
        acc[t][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kt], fb, acc[t][kt], 0, 0, 0);
    }
    __syncthreads();
  }

  // combine the four waves in a fixed order (((w0 + w1) + w2) + w3), one wave's slab at a time through LDS
  __syncthreads();
  for (int w = 1; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
          for (int e = 0; e < 4; ++e) red[((kt * 16 + 4 * g + e) * 9 + t) * 16 + (lane & 15)] = acc[t][kt][e];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[t][kt][e] += red[((kt * 16 + 4 * g + e) * 9 + t) * 16 + (lane & 15)];
    }
    __syncthreads();
  }
  if (wave > 0) return;
  float* part = a.out + (long)split * a.k * (9L * a.c);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = kt * 16 + 4 * g + e, ci = lane & 15;
        const float v = acc[t][kt][e];
        if (co < a.k && ci < a.c) {
          float* o = part + ((long)co * 9 + t) * a.c + ci;
          *o = a.accumulate ? *o + v : v;
        }
      }
}

static int wg3_thin(const adr_conv_desc* d) {
  if (d->r != 3 || d->s != 3 || d->pad_h != 1 || d->pad_w != 1 || d->stride_h != d->stride_w) return 0;
  if (d->stride_h != 1 && d->stride_h != 2) return 0;
  if (d->c > 16 || d->c % 8 || d->k > 32 || d->k % 8 || d->wo % 16) return 0;
  if (d->x_cstride % 8 || d->x_coff % 8 || d->y_cstride % 8 || d->y_coff % 8) return 0;
  if (d->stride_h == 2 && (d->h != 2 * d->ho || d->w != 2 * d->wo)) return 0;
  return d->stride_h;
}

static int wg3_tw(const adr_conv_desc* d) {
  if (d->r != 3 || d->s != 3 || d->stride_h != 1 || d->stride_w != 1 || d->pad_h != 1 || d->pad_w != 1) return 0;
  if (d->c % 32 || d->k % 32) return 0;
  if (d->wo % 16 == 0 && d->ho >= 8) return 16;
  if (d->wo % 8 == 0) return 8;
  return 0;
}

// ADR_WGRAD_THIN=0 routes the thin-channel shapes back to the general kernel (A/B runs)
static bool thin_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ADR_WGRAD_THIN");
    v = e ? atoi(e) != 0 : 1;
  }
  return v != 0;
}

// the 128 x 128 tile runs double-buffered (wgrad_bf16_body<.., DB = true>, bitwise the single-stage loop);
// ADR_WG_DB=0 selects the single-stage kernel (A/B; read per launch, so a test can switch it in-process)
static bool wg_db() {
  const char* e = getenv("ADR_WG_DB");
  return e ? atoi(e) != 0 : true;
}

static int wg_pick16(int n) { return n <= 16 ? 16 : n <= 32 ? 32 : n <= 64 ? 64 : 128; }

template <int BM>
static void launch_bm(int bn, dim3 grid, const WgArgs& g, hipStream_t st) {
  switch (bn) {
    case 16: hipLaunchKernelGGL((wgrad_bf16_kernel<BM, 16>), grid, dim3(256), 0, st, g); break;
    case 32: hipLaunchKernelGGL((wgrad_bf16_kernel<BM, 32>), grid, dim3(256), 0, st, g); break;
    case 64: hipLaunchKernelGGL((wgrad_bf16_kernel<BM, 64>), grid, dim3(256), 0, st, g); break;
    default:
      if (BM == 128 && wg_db())
        hipLaunchKernelGGL((wgrad_bf16_kernel<BM, 128, true>), grid, dim3(256), 0, st, g);
      else
        hipLaunchKernelGGL((wgrad_bf16_kernel<BM, 128>), grid, dim3(256), 0, st, g);
      break;
  }
}

// tiles, k-step rows and split count for a bf16 WGRAD; splits bounded so the fp32 partials stay small
// (ADR_WG_PART_MB / ADR_WG3_PART_MB override the per-conv partial budgets of the generic / 3x3-halo plans, A/B only)
static long part_budget(const char* var, long def_mb) {
  const char* e = getenv(var);
  const long v = e ? atol(e) : def_mb;
  return (v > 0 ? v : def_mb) << 20;
}

WgPlan wgrad_bf16_plan(const adr_conv_desc* d) {
  WgPlan p;
  p.tw3 = 0;
  p.thin = thin_enabled() ? wg3_thin(d) : 0;
  if (p.thin) {
    const long ntile = (long)d->n * ((d->ho + 7) / 8) * (d->wo / 16);
    p.bm = d->k <= 16 ? 16 : 32;
    p.bn = 16;
    p.R = 128;
    p.tiles = 1;
    long s = 768;                                                // ~3 workgroups per CU
    const long by_work = ntile / 4;                              // >= 4 tiles per split
    if (s > by_work) s = by_work;
    if (s < 1) s = 1;
    const long per = (ntile + s - 1) / s;
    p.splits = (int)((ntile + per - 1) / per);
    p.per = per;
    return p;
  }
  p.tw3 = wg3_tw(d);
  if (p.tw3) {
    const int th = 128 / p.tw3;
    const long ntile = (long)d->n * ((d->ho + th - 1) / th) * (d->wo / p.tw3);
    p.bm = d->k % 64 == 0 ? 64 : 32;  // k rows per block (KF = bm / 16)
    p.bn = 32;
    p.R = 128;
    p.tiles = (d->k / p.bm) * (d->c / 32);
    long s = (768 + p.tiles - 1) / p.tiles;                      // ~3 workgroups per CU
    const long by_work = ntile / 4;                              // >= 4 tiles per split
    static const long b3 = part_budget("ADR_WG3_PART_MB", 64);
    const long by_bytes = b3 / ((long)d->k * 9 * d->c * 4);
    if (s > by_work) s = by_work;
    if (s > by_bytes) s = by_bytes;
    if (s < 1) s = 1;
    const long per = (ntile + s - 1) / s;
    p.splits = (int)((ntile + per - 1) / per);
    p.per = per;
    return p;
  }
  p.bm = wg_pick16(d->k);
  p.bn = wg_pick16(d->c);
  const int wm = p.bm / 16 < 2 ? p.bm / 16 : 2, wn = p.bn / 16 < 2 ? p.bn / 16 : 2;
  p.R = 32 * (4 / (wm * wn)) * wg_ku(p.bm, p.bn);
  const long red = (long)d->n * d->ho * d->wo;
  const long outsz = (long)d->k * d->r * d->s * d->c;
  p.tiles = cdiv(d->k, p.bm) * d->r * d->s * cdiv(d->c, p.bn);
  long s = (1024 + p.tiles - 1) / p.tiles;                  // ~4 workgroups per CU
  static const long min_ks = getenv("ADR_WG_MIN_KSTEPS") ? atol(getenv("ADR_WG_MIN_KSTEPS")) : 16;  // A/B (8 before grouping)
  const long by_work = red / ((long)p.R * min_ks);          // >= 16 k-steps per split (grouped launches fill the chip)
  // <= 24 MB of partials (stays in L2/MALL); weights above 1 MB (l-scale: 3x3 256->256, 1x1 512->512) get 96 MB so
  // their splits still fill the chip (configs[4]: 145.2 -> 142.2 ms/step; the n-scale step is unchanged)
  static const long bg = part_budget("ADR_WG_PART_MB", 24);
  static const bool bg_env = getenv("ADR_WG_PART_MB") != nullptr;
  const long by_bytes = (!bg_env && outsz * 4 > (1l << 20) ? (96l << 20) : bg) / (outsz * 4);
  if (s > by_work) s = by_work;
  if (s > by_bytes) s = by_bytes;
  if (s < 1) s = 1;
  if (s > 65535) s = 65535;
  long per = (red + s - 1) / s;
  per = (per + p.R - 1) / p.R * p.R;
  p.splits = (int)((red + per - 1) / per);
  p.per = per;
  return p;
}

// the fused bias column sums need the generic tile kernel with one reduction slice per wave (WK == 1: bm, bn >= 32)
static bool wgrad_bias_ok(const WgPlan& p) { return !p.thin && (p.tw3 || (p.bm >= 32 && p.bn >= 32)); }

static void wgrad_args(const adr_conv_desc* d, const void* x, const void* dy, float* out, int accumulate,
                       const WgPlan& p, WgArgs& g) {
  g.x = (const __bf16*)x;
  g.dy = (const __bf16*)dy;
  g.out = out;
  g.n = d->n; g.h = d->h; g.w = d->w; g.c = d->c; g.xcs = d->x_cstride; g.xco = d->x_coff;
  g.k = d->k; g.r = d->r; g.s = d->s; g.sh = d->stride_h; g.sw = d->stride_w; g.ph = d->pad_h; g.pw = d->pad_w;
  g.ho = d->ho; g.wo = d->wo; g.ycs = d->y_cstride; g.yco = d->y_coff;
  g.red_total = (long)d->n * d->ho * d->wo;
  g.red_per_split = p.per;
  g.ksteps = (int)(p.per / p.R);
  g.ctiles = cdiv(d->c, p.bn);
  g.accumulate = accumulate;
  g.x_bytes = (int)(2l * d->n * d->h * d->w * d->x_cstride);
  g.dy_bytes = (int)(2l * d->n * d->ho * d->wo * d->y_cstride);
  g.bias = nullptr;
}

int wgrad_bf16_launch(const adr_conv_desc* d, const void* x, const void* dy, float* out, int accumulate,
                      const WgPlan& p, hipStream_t st, float* bias) {
  ADR_REQUIRE(2l * d->n * d->h * d->w * d->x_cstride < (1l << 31) && 2l * d->n * d->ho * d->wo * d->y_cstride < (1l << 31),
              "conv wgrad (bf16): operand exceeds 2 GB (32-bit buffer offsets)");
  ADR_REQUIRE(!bias || wgrad_bias_ok(p), "conv wgrad (bf16): fused bias sums need the generic tile with bm, bn >= 32");
  WgArgs g;
  wgrad_args(d, x, dy, out, accumulate, p, g);
  g.bias = bias;
  dim3 grid(p.tiles, p.splits);
  if (p.thin) {
    if (p.thin == 1) {
      if (p.bm == 16) hipLaunchKernelGGL((wgrad3t_kernel<1, 16>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((wgrad3t_kernel<1, 32>), grid, dim3(256), 0, st, g);
    } else {
      if (p.bm == 16) hipLaunchKernelGGL((wgrad3t_kernel<2, 16>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((wgrad3t_kernel<2, 32>), grid, dim3(256), 0, st, g);
    }
    return check_launch("adr_conv2d_wgrad(bf16, thin 3x3 halo)");
  }
  if (p.tw3) {
    g.bias = bias;  // the 3x3 halo kernel takes the fused bias sums too
    if (p.bm == 64) {
      if (p.tw3 == 16) hipLaunchKernelGGL((wgrad3_kernel<16, 4>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((wgrad3_kernel<8, 4>), grid, dim3(256), 0, st, g);
    } else {
      if (p.tw3 == 16) hipLaunchKernelGGL((wgrad3_kernel<16, 2>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((wgrad3_kernel<8, 2>), grid, dim3(256), 0, st, g);
    }
    return check_launch("adr_conv2d_wgrad(bf16, 3x3 halo)");
  }
  switch (p.bm) {
    case 16: launch_bm<16>(p.bn, grid, g, st); break;
    case 32: launch_bm<32>(p.bn, grid, g, st); break;
    case 64: launch_bm<64>(p.bn, grid, g, st); break;
    default: launch_bm<128>(p.bn, grid, g, st); break;
  }
  return check_launch("adr_conv2d_wgrad(bf16)");
}

template <int BM>
static void launch_batch_bm(int bn, int blocks, const WgBatch& b, hipStream_t st) {
  switch (bn) {
    case 16: hipLaunchKernelGGL((wgrad_bf16_batched_kernel<BM, 16>), dim3(blocks), dim3(256), 0, st, b); break;
    case 32: hipLaunchKernelGGL((wgrad_bf16_batched_kernel<BM, 32>), dim3(blocks), dim3(256), 0, st, b); break;
    case 64: hipLaunchKernelGGL((wgrad_bf16_batched_kernel<BM, 64>), dim3(blocks), dim3(256), 0, st, b); break;
    default:
      if (BM == 128 && wg_db())
        hipLaunchKernelGGL((wgrad_bf16_batched_kernel<BM, 128, true>), dim3(blocks), dim3(256), 0, st, b);
      else
        hipLaunchKernelGGL((wgrad_bf16_batched_kernel<BM, 128>), dim3(blocks), dim3(256), 0, st, b);
      break;
  }
}

}  // namespace adr

using namespace adr;

// The WGRAD partials of `count` convs (bf16 engine), each exactly as adr_conv2d_wgrad_partials(job) would write them:
// the jobs on the generic tile kernel are grouped by tile shape into launches of up to WGB_MAX (one launch per shape
// instead of one per conv); the 3x3 halo-tile / thin-channel ones run their own launches.
extern "C" int adr_conv2d_wgrad_batched_tile(const adr_conv_desc* d) {
  if (!d || d->dtype != ADR_BF16) return 0;
  const WgPlan p = wgrad_bf16_plan(d);
  return (p.thin || p.tw3) ? 0 : p.bm * 256 + p.bn;
}

extern "C" int adr_conv2d_wgrad_bias_fusable(const adr_conv_desc* d) {
  return d && d->dtype == ADR_BF16 && wgrad_bias_ok(wgrad_bf16_plan(d)) ? 1 : 0;
}

extern "C" int adr_conv2d_wgrad_partials_bias(const adr_conv_desc* d, const void* x, const void* dy, float* out,
                                              float* bias_part, void* stream) {
  ADR_REQUIRE(d && d->dtype == ADR_BF16 && bias_part, "conv wgrad partials + bias: bf16 descriptor and bias rows");
  const WgPlan p = wgrad_bf16_plan(d);
  return wgrad_bf16_launch(d, x, dy, out, 0, p, (hipStream_t)stream, bias_part);
}

extern "C" int adr_conv2d_wgrad_partials_batched(const adr_wgrad_job* jobs, int count, void* stream) {
  ADR_REQUIRE(count >= 0 && (count == 0 || jobs), "wgrad partials batched: count=%d", count);
  hipStream_t st = (hipStream_t)stream;
  struct Pending {
    WgBatch b;
    int blocks;
  };
  // one open batch per (bm, bn) in {16, 32, 64, 128}^2
  static thread_local Pending open[4][4];
  int used[4][4] = {};
  auto idx = [](int v) { return v <= 16 ? 0 : v <= 32 ? 1 : v <= 64 ? 2 : 3; };
  auto fire = [&](int i, int j) {
    Pending& pd = open[i][j];
    const int bm = 16 << i, bn = 16 << j;
    pd.b.start[pd.b.count] = pd.blocks;
    switch (bm) {
      case 16: launch_batch_bm<16>(bn, pd.blocks, pd.b, st); break;
      case 32: launch_batch_bm<32>(bn, pd.blocks, pd.b, st); break;
      case 64: launch_batch_bm<64>(bn, pd.blocks, pd.b, st); break;
      default: launch_batch_bm<128>(bn, pd.blocks, pd.b, st); break;
    }
    used[i][j] = 0;
  };
  for (int q = 0; q < count; ++q) {
    const adr_wgrad_job& jb = jobs[q];
    const adr_conv_desc* d = &jb.d;
    ADR_REQUIRE(d->dtype == ADR_BF16, "wgrad partials batched: bf16 jobs only (job %d)", q);
    ADR_REQUIRE(2l * d->n * d->h * d->w * d->x_cstride < (1l << 31) && 2l * d->n * d->ho * d->wo * d->y_cstride < (1l << 31),
                "wgrad partials batched: operand exceeds 2 GB (job %d)", q);
    const WgPlan p = wgrad_bf16_plan(d);
    ADR_REQUIRE(!jb.accumulate || p.splits == 1, "wgrad partials batched: accumulate needs a single split (job %d)", q);
    ADR_REQUIRE(!jb.bias || wgrad_bias_ok(p), "wgrad partials batched: job %d has fused bias sums on a tile without them", q);
    if (p.thin || p.tw3) {
      if (int rc = wgrad_bf16_launch(d, jb.x, jb.dy, jb.out, jb.accumulate, p, st, jb.bias)) return rc;
      continue;
    }
    const int i = idx(p.bm), j = idx(p.bn);
    Pending& pd = open[i][j];
    if (!used[i][j]) {
      pd.b.count = 0;
      pd.blocks = 0;
      used[i][j] = 1;
    }
    const int k = pd.b.count;
    wgrad_args(d, jb.x, jb.dy, jb.out, jb.accumulate, p, pd.b.e[k]);
    pd.b.e[k].bias = jb.bias;
    pd.b.start[k] = pd.blocks;
    pd.b.tiles[k] = p.tiles;
    pd.blocks += p.tiles * p.splits;
    pd.b.count = k + 1;
    if (pd.b.count == WGB_MAX) fire(i, j);
  }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      if (used[i][j]) fire(i, j);
  return check_launch("adr_conv2d_wgrad_partials_batched");
}
