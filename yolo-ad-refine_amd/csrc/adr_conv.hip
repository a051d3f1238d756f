// bf16 implicit-GEMM convolution, forward and data-gradient, for NHWC activations on CDNA4 MFMA.
//
// One GEMM formulation for both directions (the reduction index is the flattened (tap, channel) of the
// operand the rows gather from, channels fastest, so it walks the packed weight rows contiguously):
//   FWD   y [m=(n,oy,ox)][k]  = sum_{t=(tap,c)}  x [n, oy*s-p+kh, ox*s-p+kw, c]     * Wkrsc[k][t]
//   DGRAD dx[m=(n,iy,ix)][c]  = sum_{t=(tap,k)}  dy[n, (iy+p-kh)/s, (ix+p-kw)/s, k] * Wcrsk[c][t]
// DGRAD of a stride-2 conv runs per output parity class (blockIdx.z): rows are the dx pixels (2i+py, 2j+px) and
// the reduction covers only the taps with (pixel + pad - tap) even — a quarter of them on average.
//
// Tile: 256 threads (4 waves), BM = 128 rows x BN (16..128) columns, BK = 64 reduction elements per step.
// Each 16-byte chunk of the A tile is one (row, 8 consecutive reduction elements) gather; reductions whose
// channel count is a multiple of 8 but not of 64 (the 8-channel stem, 16/32/48-channel convs) pack several
// taps into one K-step instead of zero-padding each tap to the step. Operands go global -> registers (issued
// one step ahead) -> LDS rows of 64 + 8 elements (144-byte pitch: the 16 rows a ds_read_b128 lane group reads
// fall on 16 disjoint bank quads) -> v_mfma_f32_16x16x32_bf16 fragments.
// Epilogue: accumulators (+bias) are rounded to bf16 into an LDS image of the output tile, then written with
// 16-byte row-contiguous stores; the optional train-mode BatchNorm partial sums (sum, sum of squares of the
// stored values per column) are reduced from that image in a fixed order.
#include <cstdio>
#include <type_traits>

#include "adr_common.h"

namespace adr {

enum ConvMode { CV_FWD = 0, CV_DGRAD = 1, CV_DGRAD2 = 2 };

struct ConvArgs {
  const __bf16* src;   // A gather source: x (FWD) or dy (DGRAD)
  const __bf16* wt;    // B rows: KRSC (FWD) or CRSK (DGRAD), reduction-contiguous
  __bf16* out;
  const float* bias;
  float* stats;        // [mtiles][2][N] or null
  int n;
  int sh_, sw_, scs, sco, sc;  // source image: height, width, channel stride/offset, channel count
  int rh, rw, ocs, oco;        // row image (output pixels): height, width; output channel stride/offset
  int r, s, str, ph, pw;       // kernel, stride, padding
  int N;                       // GEMM columns (output channels)
  int ktot;                    // reduction length = taps * sc
  int ntiles;
  int accumulate;
  int src_bytes, wt_bytes;     // extents of src / wt (buffer-load range checks; < 2^31)
  // eval Conv-BN-act epilogue (adr_conv2d_fwd_bf16_act): out = act(acc * escale[col] + eshift[col]), the
  // BatchNorm with running statistics and the activation applied to the fp32 accumulator (null: acc + bias)
  const float* escale;
  const float* eshift;
  int eact;
  // DGRAD: a second gradient added in the epilogue (a fan-out's pass-through gradient, adr_conv2d_dgrad_bf16_add):
  // out = conv (+ out) + addend, NHWC with channel stride adcs (null: none)
  const __bf16* addend;
  int adcs;
  // A-operand BatchNorm-activation transform (XF kernels, adr_conv2d_{fwd,dgrad}_bf16_bnact): the A source is a
  // training BatchNorm's input y (FWD: the operand is z = act(y * s + t), 0 in the padding) or the gradient dz of
  // its output (DGRAD: the operand is dy = A * g + B * y + C with g = dz * act'(y * s + t), 0 outside the image,
  // y read alongside dz); coefficients per reduction channel, the operand side-written once (unique writer) to xo.
  const __bf16* xy;
  int xycs, xy_bytes;
  const float* xs;
  const float* xt;
  const float* xA;
  const float* xB;
  const float* xC;
  int xact;
  __bf16* xo;
  int xocs;
  // BSTAT (DGRAD only, adr_conv2d_dgrad_bf16_bstat): the stored dx is the final gradient dz of a training BatchNorm-act
  // whose input y (same pixel grid, column c = BN channel c) is read alongside in the epilogue; `stats` then receives
  // per-tile (sum g, sum g * y), g = dz * act'(y * bs + bt) — the per-element terms of nc_reduce's backward mode —
  // instead of (sum, sum of squares), so the BN backward needs no statistics pass over dz and y of its own
  const __bf16* by;
  int bycs, bact;
  const float* bs;
  const float* bt;
};

constexpr int CBM = 128, CBK = 64, CLD = CBK + 8;
enum XfMode { XF_NONE = 0, XF_FWD = 1, XF_BWD = 2 };
constexpr int XMAXC = 512;  // reduction channels of the XF coefficient table (LDS)

// XF coefficients of this thread's 8 channels (loaded from the LDS table once per staged K-step: all of a thread's
// A chunks in a step share their channels)
template <int XF>
struct XfCoef {
  float s[8], t[8], A[XF == XF_BWD ? 8 : 1], B[XF == XF_BWD ? 8 : 1], C[XF == XF_BWD ? 8 : 1];
  __device__ __forceinline__ void load(const float* tab, int c) {
    ld_coef<8>(tab + c, s);
    ld_coef<8>(tab + XMAXC + c, t);
    if constexpr (XF == XF_BWD) {
      ld_coef<8>(tab + 2 * XMAXC + c, A);
      ld_coef<8>(tab + 3 * XMAXC + c, B);
      ld_coef<8>(tab + 4 * XMAXC + c, C);
    }
  }
};

// the XF transform of one 16-byte chunk (8 channels of the reduction): the element functions affine_act_kernel
// (FWD) / affine_act_bwd_kernel (BWD) use on the bf16 path, so the operand equals what those kernels store
template <int XF>
__device__ __forceinline__ u32x4 xf_chunk(u32x4 v, u32x4 yv, const XfCoef<XF>& k, int act) {
  const __bf16* e = reinterpret_cast<const __bf16*>(&v);
  const __bf16* ye = reinterpret_cast<const __bf16*>(&yv);
  u32x4 o;
  __bf16* oe = reinterpret_cast<__bf16*>(&o);
  if constexpr (XF == XF_FWD) {
    if (act == ACT_SILU) {
#pragma unroll
      for (int q = 0; q < 8; ++q) oe[q] = (__bf16)bn_act_fwd_elem<ACT_SILU, true>((float)e[q], k.s[q], k.t[q]);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) oe[q] = (__bf16)bn_act_fwd_elem<ACT_NONE, true>((float)e[q], k.s[q], k.t[q]);
    }
  } else {
    if (act == ACT_SILU) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float xf = (float)ye[q];
        oe[q] = (__bf16)bn_act_bwd_lin(bn_act_g<ACT_SILU, true>((float)e[q], xf, k.s[q], k.t[q]), xf, k.A[q], k.B[q],
                                        k.C[q]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float xf = (float)ye[q];
        oe[q] = (__bf16)bn_act_bwd_lin(bn_act_g<ACT_NONE, true>((float)e[q], xf, k.s[q], k.t[q]), xf, k.A[q],
                                        k.B[q], k.C[q]);
      }
    }
  }
  return o;
}

// stage the XF coefficient table (per reduction channel) into LDS
template <int XF>
__device__ __forceinline__ void xf_table(const ConvArgs& a, float* tab) {
  for (int c = threadIdx.x; c < a.sc; c += 256) {
    tab[c] = a.xs[c];
    tab[XMAXC + c] = a.xt[c];
    if constexpr (XF == XF_BWD) {
      tab[2 * XMAXC + c] = a.xA[c];
      tab[3 * XMAXC + c] = a.xB[c];
      tab[4 * XMAXC + c] = a.xC[c];
    }
  }
  __syncthreads();
}

// the eval epilogue's activation (block-uniform code; 0 = none keeps the plain acc + bias path: fma by 1 is exact).
// bf16 output: the hardware exp/rcp sigmoid, as the bf16 affine_act kernels use
__device__ __forceinline__ float epi_act(int act, float v) {
  switch (act) {
    case ACT_SILU: return act_fwd_c<ACT_SILU, true>(v);
    case ACT_SIGMOID: return act_fwd_c<ACT_SIGMOID, true>(v);
    case ACT_RELU: return act_fwd_c<ACT_RELU>(v);
    case ACT_GELU: return act_fwd_c<ACT_GELU>(v);
    case ACT_HSWISH: return act_fwd_c<ACT_HSWISH>(v);
    default: return v;
  }
}

// XCD-aware block order: the dispatcher deals consecutive workgroup ids round-robin over the 8 XCDs (each with
// its own L2), so the column tiles of one row tile — which read the same A rows — would land on different XCDs
// and each fetch those rows from HBM. Renumbering so that consecutive logical ids share an XCD keeps them in one
// L2 (xcd_remap, adr_common.h: bijective for every grid size).
__device__ __forceinline__ int xcd_block(int b, int nb) { return xcd_remap(b, nb); }

// Epilogue statistics of one stored 16-byte chunk (8 columns starting at col): (sum, sum of squares) of the stored
// values, or with BSTAT the BatchNorm-backward terms (g, g * y) of the stored dz against the BN input y at the same
// pixel — bn_act_g with the bf16 path's arithmetic, as nc_reduce_kernel<bf16, RED_BWD> evaluates them.
__device__ __forceinline__ void bstat_chunk(const ConvArgs& a, u32x4 v, u32x4 yv, const float* cs, const float* ct,
                                            float* s1, float* s2) {
  const __bf16* sv = reinterpret_cast<const __bf16*>(&v);
  const __bf16* ye = reinterpret_cast<const __bf16*>(&yv);
  if (a.bact == ACT_SILU) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float yf = (float)ye[e];
      const float g = bn_act_g<ACT_SILU, true>((float)sv[e], yf, cs[e], ct[e]);
      s1[e] += g;
      s2[e] += g * yf;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float yf = (float)ye[e];
      const float g = bn_act_g<ACT_NONE, true>((float)sv[e], yf, cs[e], ct[e]);
      s1[e] += g;
      s2[e] += g * yf;
    }
  }
}

template <bool BST>
struct EpiStats {
  float s1[8], s2[8], cs[BST ? 8 : 1], ct[BST ? 8 : 1];
  __device__ __forceinline__ void init(const ConvArgs& a, bool cok, int col) {
#pragma unroll
    for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
    if constexpr (BST) {
      if (cok) {
        ld_coef<8>(a.bs + col, cs);
        ld_coef<8>(a.bt + col, ct);
      }
    }
  }
  // yv: the BN input's chunk at the same pixel / columns (BSTAT; prefetched by the caller before the row loop)
  __device__ __forceinline__ void add(const ConvArgs& a, u32x4 v, u32x4 yv) {
    const __bf16* sv = reinterpret_cast<const __bf16*>(&v);
    if constexpr (BST) {
      bstat_chunk(a, v, yv, cs, ct, s1, s2);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = (float)sv[e];
        s1[e] += f;
        s2[e] += f * f;
      }
    }
  }
};

template <int BN, int MODE, bool EPI, int XF = XF_NONE, bool BST = false>
__device__ __forceinline__ void conv_bf16_body(const ConvArgs& a) {
  static_assert(!BST || MODE != CV_FWD, "BSTAT: data gradients only");
  constexpr int WAVES_N = BN >= 128 ? 2 : 1, WAVES_M = 4 / WAVES_N;
  constexpr int WROWS = CBM / WAVES_M, WCOLS = BN / WAVES_N;
  constexpr int TM = WROWS / 16, TN = WCOLS / 16;
  constexpr int A_CH = CBM * (CBK / 8) / 256;                  // 4 chunks per thread
  constexpr int B_TOT = BN * (CBK / 8), B_CH = (B_TOT + 255) / 256;
  constexpr int OPITCH = BN + 8;                               // output image pitch (elements)
  // BN = 128 double-buffers the A/B tiles (one barrier per K-step): its VGPR budget already limits it to 2
  // waves/SIMD, which the doubled LDS (73.7 KB, 2 blocks/CU) matches; narrower tiles keep one buffer and their
  // higher occupancy
  constexpr bool DB = BN == 128;
  constexpr int STAGE = (CBM + BN) * CLD;
  constexpr int SMEM_AB = (DB ? 2 : 1) * STAGE;
  constexpr int SMEM_O = CBM * OPITCH;
  constexpr int SMEM = SMEM_AB > SMEM_O ? SMEM_AB : SMEM_O;
  constexpr int RG = 256 / (BN / 8);                           // row groups of the stats epilogue
  constexpr int SMEM_BYTES = SMEM * 2 > 2 * RG * BN * 4 ? SMEM * 2 : 2 * RG * BN * 4;
  // one LDS arena: A/B tiles in the main loop, the bf16 output image in the epilogue, then (aliased, after a
  // barrier) the stats row-group sums — keeps LDS at the tile size so more blocks fit per CU
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[SMEM_BYTES];
  __bf16* smem = reinterpret_cast<__bf16*>(lds_raw);
  float (*red)[RG][BN] = reinterpret_cast<float (*)[RG][BN]>(lds_raw);
  __bf16* As = smem;
  __bf16* Bs = smem + CBM * CLD;
  auto set_stage = [&](int b) {
    As = smem + b * STAGE;
    Bs = As + CBM * CLD;
  };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int mt = bid / a.ntiles, nt = bid % a.ntiles;
  const int m0 = mt * CBM, n0 = nt * BN;

  // ---- row space (and the parity class for stride-2 DGRAD) ----
  int rows_h = a.rh, rows_w = a.rw, cy = 0, cx = 0;
  int kh0 = 0, kw0 = 0, tstep = 1, nkw = a.s, ktot = a.ktot;
  if constexpr (MODE == CV_DGRAD2) {
    // z = 0 is dispatched first: give it the class with the most taps (odd, odd: 4 of a 3x3 at pad 1), so the
    // one-tap class's short blocks fill the tail instead of trailing behind it
    cy = (3 - (int)blockIdx.z) >> 1;
    cx = (3 - (int)blockIdx.z) & 1;
    rows_h = (a.rh - cy + 1) >> 1;
    rows_w = (a.rw - cx + 1) >> 1;
    kh0 = (cy + a.ph) & 1;
    kw0 = (cx + a.pw) & 1;
    tstep = 2;
    const int nkh = (a.r - kh0 + 1) >> 1;
    nkw = (a.s - kw0 + 1) >> 1;
    ktot = nkh * nkw * a.sc;
  }
  constexpr int ystep = MODE == CV_DGRAD2 ? 2 : 1;
  const long Mrows = (long)a.n * rows_h * rows_w;
  // statistics row of this tile: the row tile, and for stride-2 DGRAD the parity class's block of rows
  const long srow = MODE == CV_DGRAD2 ? (long)blockIdx.z * (gridDim.x / a.ntiles) + mt : mt;
  if ((long)m0 >= Mrows) {  // block-uniform (a parity class smaller than the grid): its statistics row is zero
    if (a.stats && tid < BN && n0 + tid < a.N) {
      float* s = a.stats + srow * 2 * a.N + n0 + tid;
      s[0] = 0.f;
      s[a.N] = 0.f;
    }
    return;
  }
  const int hw = rows_h * rows_w;
  auto pixel_of = [&](long m) -> long {
    const long img = m / hw;
    const int rem = (int)(m - img * hw);
    return (img * a.rh + (rem / rows_w) * ystep + cy) * a.rw + (rem % rows_w) * ystep + cx;
  };

  // per-thread A rows: chunk q = tid + 256 i -> row q / 8, reduction chunk q % 8
  const int kc = tid & 7;
  // FWD and stride-1 DGRAD gather linearly: source pixel = row base + SG * (kh * sw + kw) with SG = +1 (FWD) or
  // -1 (DGRAD), so a row keeps only its base element offset and its (y, x) origin for the padding test, and a
  // chunk's address is one 32-bit add per step (the host guarantees < 2^31 elements). Stride-2 DGRAD parity
  // classes keep the general (image, y, x) form.
  constexpr bool LIN = MODE != CV_DGRAD2;
  constexpr int SG = MODE == CV_FWD ? 1 : -1;
  int r_img[A_CH], r_y[A_CH], r_x[A_CH], r_off[A_CH], r_pix[A_CH];
  bool r_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const long m = (long)m0 + (tid >> 3) + 32 * i;
    r_ok[i] = m < Mrows;
    const long mm = r_ok[i] ? m : 0;
    r_img[i] = (int)(mm / hw);
    const int rem = (int)(mm - (long)r_img[i] * hw);
    r_y[i] = (rem / rows_w) * ystep + cy;
    r_x[i] = (rem % rows_w) * ystep + cx;
    if constexpr (LIN) {
      // origin of the gather window: FWD y*str - pad (+kh) ; DGRAD y + pad (-kh)
      r_y[i] = MODE == CV_FWD ? r_y[i] * a.str - a.ph : r_y[i] + a.ph;
      r_x[i] = MODE == CV_FWD ? r_x[i] * a.str - a.pw : r_x[i] + a.pw;
      r_pix[i] = (r_img[i] * a.sh_ + r_y[i]) * a.sw_ + r_x[i];
      r_off[i] = r_pix[i] * a.scs + a.sco;
    }
  }
  // XF: coefficient table, and per register stage the chunk validity / unique-writer bits, the chunk's channel and
  // its source pixels (the second operand y and the side output use the source grid with their own strides)
  constexpr int XTAB = XF == XF_BWD ? 5 * XMAXC : XF == XF_FWD ? 2 * XMAXC : 4;
  __shared__ __attribute__((aligned(16))) float xtab[XTAB];
  if constexpr (XF != XF_NONE) xf_table<XF>(a, xtab);
  const int RS = a.r * a.s;
  const int ksteps = (ktot + CBK - 1) / CBK;

  // DB tiles keep two register stages: the global loads of step t+2 are issued while step t computes, so each
  // load has two K-steps of MFMA work to land behind (one step for the single-buffered narrow tiles)
  constexpr int NR = DB ? 2 : 1;
  static_assert(XF == XF_NONE || !DB, "XF kernels are single-buffered (BN <= 64)");
  u32x4 ra_s[NR][A_CH], rb_s[NR][B_CH];
  const u32x4 zero = {0u, 0u, 0u, 0u};
  constexpr int XA = XF == XF_BWD ? A_CH : 1;
  u32x4 xy_s[XA];          // BWD: y chunks
  int xp_s[A_CH];          // source pixel of each chunk
  unsigned xok = 0, xw = 0;
  int xc = 0;
  // Reduction-position decoder, advanced by CBK per k-step without integer division: this thread's chunk sits
  // at k = t*CBK + kc*8 = (tap ta, channel ca); (kh, kw) are the tap's kernel coordinates. The B rows use the
  // same chunk position (q & 7 == kc for every B chunk of the thread), so one decoder serves both operands.
  const int ntaps = ktot / a.sc;
  int ta = (kc * 8) / a.sc, ca = kc * 8 - ta * a.sc;
  int kh, kw;
  if constexpr (MODE == CV_DGRAD2) {
    kh = kh0 + tstep * (ta / nkw);
    kw = kw0 + tstep * (ta % nkw);
  } else {
    kh = ta / a.s;
    kw = ta - kh * a.s;
  }
  int kpos = kc * 8;  // LIN: reduction position = element offset within a B row
  auto advance = [&]() {
    kpos += CBK;
    ca += CBK;
    while (ca >= a.sc) {
      ca -= a.sc;
      ++ta;
      kw += tstep;
      if (kw >= a.s) {
        kw = kw0;
        kh += tstep;
      }
    }
  };
  // B rows n0 + q/8 (reduction-contiguous rows of RS * sc elements)
  // chunk i of this thread: row n0 + tid/8 + 32 i
  const int b_row = LIN ? ktot : RS * a.sc;
  const int b_n = n0 + (tid >> 3);
  const int b_off0 = b_n * b_row;
  auto b_ok = [&](int i) { return tid + 256 * i < B_TOT && b_n + 32 * i < a.N; };
  // LIN gathers go through buffer descriptors: a padding / out-of-range chunk gets an offset past the
  // descriptor's range and the hardware returns zeros — no branch and no zero moves per chunk
  constexpr unsigned OOR = 0x7FFFFFF0u;
  const __amdgpu_buffer_rsrc_t src_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, a.src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wt_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, a.wt_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xy_rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xy, (short)0, XF == XF_BWD ? a.xy_bytes : 0, 0x00020000);
  // XF unique writer: of the (row, tap) pairs that gather one source pixel, the one with the largest tap. FWD
  // (stride s): the next larger tap kh + s pairs with output row oy - 1; DGRAD (any stride): tap kh + 1 pairs with
  // dx row iy + 1. Only column tile 0 writes.
  auto xf_writer = [&](int i, int kh_, int kw_) -> bool {
    if (nt != 0) return false;
    if constexpr (MODE == CV_FWD)
      return (kh_ + a.str >= a.r || r_y[i] == -a.ph) && (kw_ + a.str >= a.s || r_x[i] == -a.pw);
    else if constexpr (MODE == CV_DGRAD)
      return (kh_ + 1 >= a.r || r_y[i] - a.ph + 1 >= a.rh) && (kw_ + 1 >= a.s || r_x[i] - a.pw + 1 >= a.rw);
    else
      return (kh_ + 1 >= a.r || r_y[i] + 1 >= a.rh) && (kw_ + 1 >= a.s || r_x[i] + 1 >= a.rw);
  };
  auto load = [&](auto S) {
    u32x4(&ra)[A_CH] = ra_s[decltype(S)::value];
    u32x4(&rb)[B_CH] = rb_s[decltype(S)::value];
    const bool kok = ta < ntaps;
    const int c = ca;
    if constexpr (XF != XF_NONE) {
      xok = xw = 0;
      xc = c;
    }
    if constexpr (LIN) {
      const int dy = SG * kh, dx = SG * kw;
      const int toff = (dy * a.sw_ + dx) * a.scs + c;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        const bool ok = kok && r_ok[i] && (unsigned)(r_y[i] + dy) < (unsigned)a.sh_ &&
                        (unsigned)(r_x[i] + dx) < (unsigned)a.sw_;
        ra[i] = __builtin_amdgcn_raw_buffer_load_b128(src_rs, ok ? (unsigned)(r_off[i] + toff) * 2u : OOR, 0, 0);
        if constexpr (XF != XF_NONE) {
          const int pix = r_pix[i] + dy * a.sw_ + dx;
          xp_s[i] = pix;
          xok |= (unsigned)ok << i;
          xw |= (unsigned)(ok && xf_writer(i, kh, kw)) << i;
          if constexpr (XF == XF_BWD)
            xy_s[i] = __builtin_amdgcn_raw_buffer_load_b128(xy_rs, ok ? (unsigned)(pix * a.xycs + c) * 2u : OOR, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i)
        rb[i] = __builtin_amdgcn_raw_buffer_load_b128(
            wt_rs, (b_ok(i) && kok) ? (unsigned)(b_off0 + 32 * i * b_row + kpos) * 2u : OOR, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        // parity class: ny, nx are even by construction
        const int ny = r_y[i] + a.ph - kh, nx = r_x[i] + a.pw - kw;
        const int sy = ny >> 1, sx = nx >> 1;
        const bool ok = kok && r_ok[i] && ny >= 0 && nx >= 0 && sy < a.sh_ && sx < a.sw_;
        const int pix = (r_img[i] * a.sh_ + sy) * a.sw_ + sx;
        ra[i] = ok ? ld16(a.src + (long)pix * a.scs + a.sco + c) : zero;
        if constexpr (XF != XF_NONE) {
          xp_s[i] = pix;
          xok |= (unsigned)ok << i;
          xw |= (unsigned)(ok && xf_writer(i, kh, kw)) << i;
          if constexpr (XF == XF_BWD) xy_s[i] = ok ? ld16(a.xy + (long)pix * a.xycs + c) : zero;
        }
      }
      const int tf = kh * a.s + kw;
#pragma unroll
      for (int i = 0; i < B_CH; ++i)
        rb[i] = (b_ok(i) && kok) ? ld16(a.wt + (long)(b_off0 + 32 * i * b_row) + tf * a.sc + c) : zero;
    }
    advance();
  };
  auto store = [&](auto S) {
    const u32x4(&ra)[A_CH] = ra_s[decltype(S)::value];
    const u32x4(&rb)[B_CH] = rb_s[decltype(S)::value];
    XfCoef<XF == XF_NONE ? XF_FWD : XF> xk;
    if constexpr (XF != XF_NONE) xk.load(xtab, xc);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      if constexpr (XF == XF_NONE) {
        st16(&As[((tid >> 3) + 32 * i) * CLD + kc * 8], ra[i]);
      } else {
        u32x4 v = zero;
        if ((xok >> i) & 1) v = xf_chunk<XF>(ra[i], xy_s[XF == XF_BWD ? i : 0], xk, a.xact);
        if ((xw >> i) & 1) st16(a.xo + (long)xp_s[i] * a.xocs + xc, v);
        st16(&As[((tid >> 3) + 32 * i) * CLD + kc * 8], v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int q = tid + 256 * i;
      if (B_TOT % 256 == 0 || q < B_TOT) st16(&Bs[(q >> 3) * CLD + (q & 7) * 8], rb[i]);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int wr0 = wm * WROWS, wc0 = wn * WCOLS;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, NR - 1>;
  auto compute = [&]() {
#pragma unroll
    for (int kk = 0; kk < CBK / 32; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(&As[(wr0 + i * 16 + (lane & 15)) * CLD + kk * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wc0 + j * 16 + (lane & 15)) * CLD + kk * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (DB) {
    // stage s (LDS) and register set s alternate; step t computes stage t&1 while set t&1 receives step t+2.
    // Loads and stores are unconditional: past the last step the decoder's tap is >= ntaps, every chunk reads
    // out of range (zeros, no memory access) and the stores land in a stage nobody reads again — straight-line
    // VMEM lets the compiler count the older set's loads (vmcnt(N) > 0) instead of draining the just-issued
    // prefetch with vmcnt(0) at the store
    load(S0{});
    store(S0{});
    load(S1{});
    __syncthreads();
    auto step = [&](int t, auto S) {
      constexpr int cur = decltype(S)::value;
      using SO = std::integral_constant<int, 1 - cur>;
      set_stage(cur);
      load(S);  // set cur was stored into its stage one step ago
      compute();
      set_stage(1 - cur);
      store(SO{});  // step t+1 (loaded two steps ago) into the other stage, last read in step t-1
      __syncthreads();
    };
    for (int t = 0; t < ksteps; t += 2) {
      step(t, S0{});
      if (t + 1 < ksteps) step(t + 1, S1{});
    }
  } else {
    if (ksteps > 0) {
      load(S0{});
      store(S0{});
      __syncthreads();
    }
    for (int t = 0; t < ksteps; ++t) {
      if (t + 1 < ksteps) load(S0{});
      compute();
      __syncthreads();
      if (t + 1 < ksteps) {
        store(S0{});
        __syncthreads();
      }
    }
  }

  // ---- epilogue: bf16 image of the tile in LDS, then 16-byte row stores ----
  __bf16* Os = smem;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wc0 + j * 16 + (lane & 15);
    const bool cok = n0 + col < a.N;
    const float b = (a.bias && cok) ? a.bias[n0 + col] : 0.f;
    const float es = EPI && cok ? a.escale[n0 + col] : 1.f;
    const float eb = EPI && cok ? a.eshift[n0 + col] + b : b;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Os[(wr0 + i * 16 + 4 * (lane >> 4) + e) * OPITCH + col] = 
            (__bf16)(EPI ? epi_act(a.eact, fmaf(acc[i][j][e], es, eb)) : acc[i][j][e] + b);
  }
  constexpr int CPR = BN / 8;          // 16-byte chunks per row
  constexpr int RPP = 256 / CPR;       // rows per pass
  constexpr int RPT = CBM / RPP;       // rows per thread
  const int oc = tid % CPR, orow = tid / CPR;
  const bool col_ok = n0 + oc * 8 < a.N;
  // BSTAT: the BN input rows of this thread's output chunks, in flight across the barrier and the LDS read-back
  u32x4 ypre[BST ? RPT : 1];
  if constexpr (BST) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const long m = (long)m0 + orow + k * RPP;
      ypre[k] = (m < Mrows && col_ok) ? ld16(a.by + pixel_of(m) * a.bycs + n0 + oc * 8) : u32x4{0u, 0u, 0u, 0u};
    }
  }
  __syncthreads();
  EpiStats<BST> es;
  es.init(a, col_ok, n0 + oc * 8);
  auto out_row = [&](int r, const u32x4& yv) {
    const long m = (long)m0 + r;
    if (m >= Mrows || !col_ok) return;
    u32x4 v = *reinterpret_cast<const u32x4*>(&Os[r * OPITCH + oc * 8]);
    const long pix = pixel_of(m);
    __bf16* dst = a.out + pix * a.ocs + a.oco + n0 + oc * 8;
    if (MODE != CV_FWD && a.addend) {  // one rounding for conv + previous + addend
      const u32x4 q = ld16(a.addend + pix * a.adcs + n0 + oc * 8);
      const u32x4 o = a.accumulate ? ld16(dst) : u32x4{0u, 0u, 0u, 0u};
      const __bf16 *qv = reinterpret_cast<const __bf16*>(&q), *ov = reinterpret_cast<const __bf16*>(&o);
      __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e] + (float)qv[e]);
    } else if (a.accumulate) {
      const u32x4 o = ld16(dst);
      const __bf16* ov = reinterpret_cast<const __bf16*>(&o);
      __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e]);
    }
    st16(dst, v);
    if (a.stats) es.add(a, v, yv);
  };
  if constexpr (BST) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) out_row(orow + k * RPP, ypre[k]);
  } else {
    for (int r = orow; r < CBM; r += RPP) out_row(r, ypre[0]);
  }
  if (a.stats) {  // fixed-order reduction over the row groups of each column
    __syncthreads();  // every thread is done reading the output image that `red` aliases
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[0][orow][oc * 8 + e] = es.s1[e];
      red[1][orow][oc * 8 + e] = es.s2[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      float x1 = 0.f, x2 = 0.f;
      for (int g = 0; g < RPP; ++g) {
        x1 += red[0][g][tid];
        x2 += red[1][g][tid];
      }
      float* s = a.stats + srow * 2 * a.N + n0 + tid;
      s[0] = x1;
      s[a.N] = x2;
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// 1x1 / stride-1 / unpadded contractions with a short reduction (C <= 256), FWD and stride-1 DGRAD: streaming
// GEMM. These convs move ~256 bytes per output row and do almost no math, so the per-tile kernel above is bound by
// load latency: one short K-step per tile leaves nothing to hide its gather behind (~0.3 of HBM peak). Here a block
// keeps its column tile's weights in LDS and walks a strided sequence of 128-row tiles: the next tile's rows are
// in flight (registers) while the current tile's MFMAs, epilogue and stores run. The MFMA produces C^T (weights as
// the A operand), so a lane holds four consecutive columns of one row and the output image is written to LDS with
// 8-byte stores. BatchNorm partial sums accumulate across the block's tiles: the stats rows are per block group
// (adr_conv2d_fwd_bf16_stat_tiles), still reduced in a fixed order.
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2c;

// XF_FWD (adr_conv2d_fwd_bf16_bnact): the A rows are the producer BatchNorm's input y; each staged chunk becomes
// z = act(y * s + t) (the thread's 8 reduction channels are fixed, so their coefficients live in registers) and
// column tile 0 side-writes it once (every z element exactly once: rows are pixels).
template <int BN, int MODE, int KT, bool EPI = false, int XF = XF_NONE, bool BST = false>
__device__ __forceinline__ void conv1_body(const ConvArgs& a, int groups) {
  static_assert(!BST || MODE == CV_DGRAD, "BSTAT: data gradients only");
  static_assert(MODE == CV_FWD || MODE == CV_DGRAD, "conv1: FWD or stride-1 DGRAD");
  static_assert(XF == XF_NONE || (XF == XF_FWD && MODE == CV_FWD && !EPI), "conv1: forward XF only");
  constexpr int WAVES_N = BN >= 128 ? 2 : 1, WAVES_M = 4 / WAVES_N;
  constexpr int WROWS = CBM / WAVES_M, WCOLS = BN / WAVES_N;
  constexpr int TM = WROWS / 16, TN = WCOLS / 16;
  constexpr int KP = KT + 8;                       // A / B row pitch (elements)
  constexpr int CPR_A = KT / 8;                    // 16-byte chunks per A row
  constexpr int A_CH = CBM * CPR_A / 256;          // A chunks per thread
  constexpr int B_TOT = BN * CPR_A, B_CH = (B_TOT + 255) / 256;
  constexpr int OPITCH = BN + 8;
  constexpr int CPR = BN / 8, RPP = 256 / CPR;     // output: 16-byte chunks per row, rows per pass
  constexpr int SMEM_A = CBM * KP, SMEM_B = BN * KP, SMEM_O = CBM * OPITCH;
  constexpr int SMEM_BYTES = 2 * (SMEM_A + SMEM_B + SMEM_O) > 2 * RPP * BN * 4 ? 2 * (SMEM_A + SMEM_B + SMEM_O)
                                                                                : 2 * RPP * BN * 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[SMEM_BYTES];
  __bf16* As = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* Bs = As + SMEM_A;
  __bf16* Os = Bs + SMEM_B;
  float (*red)[RPP][BN] = reinterpret_cast<float (*)[RPP][BN]>(lds_raw);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int grp = bid / a.ntiles, nt = bid % a.ntiles;
  const int n0 = nt * BN;
  const long Mrows = (long)a.n * a.rh * a.rw;
  const int mtiles = (int)((Mrows + CBM - 1) / CBM);
  constexpr unsigned OOR = 0x7FFFFFF0u;
  const __amdgpu_buffer_rsrc_t src_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, a.src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wt_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, a.wt_bytes, 0x00020000);
  const int kc = tid % CPR_A;                      // this thread's reduction chunk (same for all its A / B chunks)
  const bool kok = kc * 8 < a.ktot;
  XfCoef<XF_FWD> xk;
  if constexpr (XF == XF_FWD) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      xk.s[q] = kok ? a.xs[kc * 8 + q] : 0.f;
      xk.t[q] = kok ? a.xt[kc * 8 + q] : 0.f;
    }
  }

  // weights of the column tile, once
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int q = tid + 256 * i, row = q / CPR_A;
    if (q < B_TOT) {
      const bool ok = kok && n0 + row < a.N;
      st16(&Bs[row * KP + kc * 8], __builtin_amdgcn_raw_buffer_load_b128(
                                      wt_rs, ok ? (unsigned)((n0 + row) * a.ktot + kc * 8) * 2u : OOR, 0, 0));
    }
  }
  u32x4 ra[A_CH];
  auto load = [&](int mt) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const long m = (long)mt * CBM + (tid / CPR_A) + (256 / CPR_A) * i;
      const bool ok = kok && m < Mrows;
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(src_rs, ok ? (unsigned)(m * a.scs + a.sco + kc * 8) * 2u : OOR, 0, 0);
    }
  };
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  const int oc = tid % CPR, orow = tid / CPR;
  const bool col_ok = n0 + oc * 8 < a.N;
  float bcs[BST ? 8 : 1], bct[BST ? 8 : 1];
  if constexpr (BST) {
    if (col_ok) {
      ld_coef<8>(a.bs + n0 + oc * 8, bcs);
      ld_coef<8>(a.bt + n0 + oc * 8, bct);
    }
  }
  const int wr0 = wm * WROWS, wc0 = wn * WCOLS;
  float bias4[TN][4], es4[EPI ? TN : 1][4];  // bias, or (EPI: eval Conv-BN-act) the affine shift + bias and scale
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = n0 + wc0 + 16 * j + 4 * (lane >> 4) + e;
      const bool cok = col < a.N;
      bias4[j][e] = (a.bias && cok) ? a.bias[col] : 0.f;
      if constexpr (EPI) {
        es4[j][e] = cok ? a.escale[col] : 1.f;
        bias4[j][e] += cok ? a.eshift[col] : 0.f;
      }
    }

  int mt = grp;
  if (mt < mtiles) load(mt);
  for (; mt < mtiles; mt += groups) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      if constexpr (XF == XF_FWD) {
        const long m = (long)mt * CBM + (tid / CPR_A) + (256 / CPR_A) * i;
        const bool ok = kok && m < Mrows;
        const u32x4 v = ok ? xf_chunk<XF_FWD>(ra[i], ra[i], xk, a.xact) : u32x4{0u, 0u, 0u, 0u};
        if (ok && nt == 0) st16(a.xo + m * a.xocs + kc * 8, v);
        st16(&As[((tid / CPR_A) + (256 / CPR_A) * i) * KP + kc * 8], v);
      } else {
        st16(&As[((tid / CPR_A) + (256 / CPR_A) * i) * KP + kc * 8], ra[i]);
      }
    }
    __syncthreads();  // A tile (and, first time, the weights) in LDS; the previous tile's output image read out
    if (mt + groups < mtiles) load(mt + groups);
    f32x4 acc[TN][TM];  // C^T: rows = columns n, columns = rows m
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KT / 32; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(&As[(wr0 + i * 16 + (lane & 15)) * KP + kk * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wc0 + j * 16 + (lane & 15)) * KP + kk * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[j][i], 0, 0, 0);
    }
    // lane: row wr0 + 16 i + (lane & 15), columns wc0 + 16 j + 4 (lane >> 4) .. +3
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        __bf16 v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (EPI) v[e] = (__bf16)epi_act(a.eact, fmaf(acc[j][i][e], es4[j][e], bias4[j][e]));
          else v[e] = (__bf16)(acc[j][i][e] + bias4[j][e]);
        }
        *reinterpret_cast<u32x2c*>(&Os[(wr0 + 16 * i + (lane & 15)) * OPITCH + wc0 + 16 * j + 4 * (lane >> 4)]) =
            *reinterpret_cast<u32x2c*>(v);
      }
    constexpr int RPT = CBM / RPP;
    u32x4 ypre[BST ? RPT : 1];  // BSTAT: this thread's BN input rows, in flight across the barrier
    if constexpr (BST) {
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        const long m = (long)mt * CBM + orow + k * RPP;
        ypre[k] = (m < Mrows && col_ok) ? ld16(a.by + m * a.bycs + n0 + oc * 8) : u32x4{0u, 0u, 0u, 0u};
      }
    }
    __syncthreads();  // output image complete; every wave is done with the A tile
    if constexpr (!BST) {
      for (int r = orow; r < CBM; r += RPP) {
        const long m = (long)mt * CBM + r;
        if (m >= Mrows || !col_ok) continue;
        u32x4 v = *reinterpret_cast<const u32x4*>(&Os[r * OPITCH + oc * 8]);
        __bf16* dst = a.out + m * a.ocs + a.oco + n0 + oc * 8;
        if (MODE == CV_DGRAD && a.addend) {
          const u32x4 q = ld16(a.addend + m * a.adcs + n0 + oc * 8);
          const u32x4 o = a.accumulate ? ld16(dst) : u32x4{0u, 0u, 0u, 0u};
          const __bf16 *qv = reinterpret_cast<const __bf16*>(&q), *ov = reinterpret_cast<const __bf16*>(&o);
          __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
          for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e] + (float)qv[e]);
        } else if (a.accumulate) {
          const u32x4 o = ld16(dst);
          const __bf16* ov = reinterpret_cast<const __bf16*>(&o);
          __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
          for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e]);
        }
        st16(dst, v);
        if (a.stats) {
          const __bf16* sv = reinterpret_cast<const __bf16*>(&v);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = (float)sv[e];
            s1[e] += f;
            s2[e] += f * f;
          }
        }
      }
    } else {
    auto out_row = [&](int r, const u32x4& yv) {
      const long m = (long)mt * CBM + r;
      if (m >= Mrows || !col_ok) return;
      u32x4 v = *reinterpret_cast<const u32x4*>(&Os[r * OPITCH + oc * 8]);
      __bf16* dst = a.out + m * a.ocs + a.oco + n0 + oc * 8;
      if (MODE == CV_DGRAD && a.addend) {
        const u32x4 q = ld16(a.addend + m * a.adcs + n0 + oc * 8);
        const u32x4 o = a.accumulate ? ld16(dst) : u32x4{0u, 0u, 0u, 0u};
        const __bf16 *qv = reinterpret_cast<const __bf16*>(&q), *ov = reinterpret_cast<const __bf16*>(&o);
        __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
        for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e] + (float)qv[e]);
      } else if (a.accumulate) {
        const u32x4 o = ld16(dst);
        const __bf16* ov = reinterpret_cast<const __bf16*>(&o);
        __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
        for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e]);
      }
      st16(dst, v);
      if (a.stats) {
        if constexpr (BST) {
          bstat_chunk(a, v, yv, bcs, bct, s1, s2);
        } else {
          const __bf16* sv = reinterpret_cast<const __bf16*>(&v);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = (float)sv[e];
            s1[e] += f;
            s2[e] += f * f;
          }
        }
      }
    };
      if constexpr (BST) {
#pragma unroll
        for (int k = 0; k < RPT; ++k) out_row(orow + k * RPP, ypre[k]);
      }
    }
  }
  if (a.stats) {  // fixed-order reduction over the row groups of each column, one stats row per block group
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[0][orow][oc * 8 + e] = s1[e];
      red[1][orow][oc * 8 + e] = s2[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      float x1 = 0.f, x2 = 0.f;
      for (int g = 0; g < RPP; ++g) {
        x1 += red[0][g][tid];
        x2 += red[1][g][tid];
      }
      float* s = a.stats + (long)grp * 2 * a.N + n0 + tid;
      s[0] = x1;
      s[a.N] = x2;
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 convolutions (FWD, and DGRAD which is the same contraction with the taps mirrored):
// the implicit GEMM above gathers every input pixel once per tap, i.e. nine times through L2, and its K-steps
// are too short to hide those loads. Here a block owns a TH x TW output tile (TH*TW = 128 rows) and 64 output
// channels; per 32-channel chunk it stages the (TH+2) x (TW+2) input halo tile and the 9-tap weight slab in LDS
// ONCE and runs all nine taps out of LDS (72 MFMAs per wave per chunk), while the next chunk's loads are in
// flight in registers. A fragment row for tap (kh, kw) is the halo pixel (py + kh, px + kw) (mirrored for
// DGRAD), so the gather costs one LDS address add per tap.
constexpr int C3_CK = 32, C3_LD = C3_CK;  // chunk channels; unpadded 64-byte LDS rows, XOR-swizzled:
// the 16-byte chunk kq of row r sits in slot kq ^ ((r >> 2) & 3), so any 16 consecutive rows a ds_read_b128 lane
// group reads cover 16 disjoint bank quads (48 KB per block: 3 blocks per CU)
__device__ __forceinline__ int c3_swz(int row, int kq) { return row * C3_LD + ((kq ^ ((row >> 2) & 3)) << 3); }

// WN = 2 (the wide tile, `conv3w_kernel`): 512 threads own a 256-pixel x 128-channel tile — waves 4 along M (64 rows
// each) x 2 along N — so each staged byte of the halo and of the weight slab feeds twice the MFMA work of the
// 128 x 64 tile: the big-channel 3x3 convs (l-scale C, K >= 128) were L2-bound at ~0.37 of the bf16 MFMA peak.
template <int TW, bool DG, int BN, bool EPI, int XF = XF_NONE, int WN = 1, bool BST = false>
__device__ __forceinline__ void conv3_body(const ConvArgs& a) {
  static_assert(!BST || DG, "BSTAT: data gradients only");
  constexpr int NT = 256 * WN, PIX = 128 * WN;         // threads, tile pixels
  constexpr int TH = PIX / TW, HWW = TW + 2, NPIX = (TH + 2) * HWW;
  constexpr int A_TOT = NPIX * (C3_CK / 8), A_CH = (A_TOT + NT - 1) / NT;
  constexpr int TPP = NT / (BN * (C3_CK / 8));       // taps per pass of the threads over the weight slab
  static_assert(TPP >= 1, "conv3: BN too wide for the thread count");
  constexpr int B_CH = (9 + TPP - 1) / TPP;          // chunk i of a thread is tap i * TPP + tid / (4 BN)
  constexpr int WROWS = PIX / 4, WCOLS = BN / WN;    // 4 waves along M x WN along N
  constexpr int TM = WROWS / 16, TN = WCOLS / 16;
  constexpr int OPITCH = BN + 8, CPR = BN / 8, RPP = NT / CPR;
  constexpr int SMEM_A = NPIX * C3_LD, SMEM_B = 9 * BN * C3_LD;
  constexpr int SMEM_AB = 2 * (SMEM_A + SMEM_B), SMEM_O = 2 * PIX * OPITCH, SMEM_R = 2 * RPP * BN * 4;
  constexpr int SMEM_BYTES = SMEM_AB > SMEM_O ? (SMEM_AB > SMEM_R ? SMEM_AB : SMEM_R) : (SMEM_O > SMEM_R ? SMEM_O : SMEM_R);
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[SMEM_BYTES];
  __bf16* As = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* Bs = As + SMEM_A;
  float (*red)[RPP][BN] = reinterpret_cast<float (*)[RPP][BN]>(lds_raw);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % 4, wn = wave / 4;
  const int H = a.rh, W = a.rw;
  const int tx = W / TW, ty = (H + TH - 1) / TH;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int mt = bid / a.ntiles, nt = bid - (bid / a.ntiles) * a.ntiles;
  const int n0 = nt * BN;
  const int img = mt / (tx * ty), trem = mt - img * (tx * ty);
  const int y0 = (trem / tx) * TH, x0 = (trem - (trem / tx) * tx) * TW;

  // halo chunks of this thread: e = tid + 256 i -> halo pixel e / 4, channel quad e % 4
  constexpr unsigned OOR = 0x7FFFFFF0u;
  const __amdgpu_buffer_rsrc_t src_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, a.src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wt_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, a.wt_bytes, 0x00020000);
  int a_off[A_CH], a_pix[A_CH];
  unsigned a_in = 0;  // XF: halo chunks in the tile interior (their source pixel belongs to this tile)
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int e = tid + NT * i, q = e >> 2, hy = q / HWW, hx = q - (q / HWW) * HWW;
    const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
    const bool ok = e < A_TOT && gy >= 0 && gy < a.sh_ && gx >= 0 && gx < a.sw_;
    a_pix[i] = ok ? (img * a.sh_ + gy) * a.sw_ + gx : -1;
    a_off[i] = ok ? a_pix[i] * a.scs + a.sco + (e & 3) * 8 : -1;
    a_in |= (unsigned)(ok && hy >= 1 && hy <= TH && hx >= 1 && hx <= TW) << i;
  }
  constexpr int XTAB = XF == XF_BWD ? 5 * XMAXC : XF == XF_FWD ? 2 * XMAXC : 4;
  __shared__ __attribute__((aligned(16))) float xtab[XTAB];
  if constexpr (XF != XF_NONE) xf_table<XF>(a, xtab);
  const __amdgpu_buffer_rsrc_t xy_rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xy, (short)0, XF == XF_BWD ? a.xy_bytes : 0, 0x00020000);
  constexpr int XA = XF == XF_BWD ? A_CH : 1;
  u32x4 ry[XA];
  const int xq = (tid & 3) * 8;  // this thread's channels within a chunk step
  const int b_row = (tid >> 2) % BN, b_tap0 = tid / (4 * BN);
  const bool b_ok = n0 + b_row < a.N;
  const int b_off = (n0 + b_row) * 9 * a.sc + (tid & 3) * 8;  // + tap * sc + c0

  u32x4 ra[A_CH], rb[B_CH];
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(src_rs, a_off[i] >= 0 ? (unsigned)(a_off[i] + c0) * 2u : OOR, 0, 0);
      if constexpr (XF == XF_BWD)
        ry[i] = __builtin_amdgcn_raw_buffer_load_b128(
            xy_rs, a_pix[i] >= 0 ? (unsigned)(a_pix[i] * a.xycs + c0 + xq) * 2u : OOR, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int tap = i * TPP + b_tap0;
      rb[i] = __builtin_amdgcn_raw_buffer_load_b128(
          wt_rs, (b_ok && tap < 9) ? (unsigned)(b_off + tap * a.sc + c0) * 2u : OOR, 0, 0);
    }
  };
  auto store = [&](int c0) {
    XfCoef<XF == XF_NONE ? XF_FWD : XF> xk;
    if constexpr (XF != XF_NONE) xk.load(xtab, c0 + xq);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int e = tid + NT * i;
      if constexpr (XF == XF_NONE) {
        if (e < A_TOT) st16(&As[c3_swz(e >> 2, e & 3)], ra[i]);
      } else {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (a_pix[i] >= 0) v = xf_chunk<XF>(ra[i], ry[XF == XF_BWD ? i : 0], xk, a.xact);
        if (nt == 0 && ((a_in >> i) & 1)) st16(a.xo + (long)a_pix[i] * a.xocs + c0 + xq, v);
        if (e < A_TOT) st16(&As[c3_swz(e >> 2, e & 3)], v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int tap = i * TPP + b_tap0;
      if (tap < 9) st16(&Bs[c3_swz(tap * BN + b_row, tid & 3)], rb[i]);
    }
  };

  const int wr0 = wm * WROWS, wc0 = wn * WCOLS;
  int fq[TM];  // halo pixel of this lane's fragment row, tap (0, 0)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = wr0 + i * 16 + (lane & 15);
    fq[i] = (p / TW) * HWW + (p % TW);
  }
  const int kq = lane >> 4;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nch = a.sc / C3_CK;
  load(0);
  for (int ch = 0; ch < nch; ++ch) {
    store(ch * C3_CK);
    __syncthreads();
    if (ch + 1 < nch) load((ch + 1) * C3_CK);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int kh = t / 3, kw = t % 3;
      const int dq = DG ? (2 - kh) * HWW + (2 - kw) : kh * HWW + kw;
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(&As[c3_swz(fq[i] + dq, kq)]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(&Bs[c3_swz(t * BN + wc0 + j * 16 + (lane & 15), kq)]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // ---- epilogue (as conv_bf16_kernel): bf16 tile image in LDS, 16-byte row stores, optional BN partials ----
  __bf16* Os = reinterpret_cast<__bf16*>(lds_raw);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wc0 + j * 16 + (lane & 15);
    const bool cok = n0 + col < a.N;
    const float b = (a.bias && cok) ? a.bias[n0 + col] : 0.f;
    const float es = EPI && cok ? a.escale[n0 + col] : 1.f;
    const float eb = EPI && cok ? a.eshift[n0 + col] + b : b;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Os[(wr0 + i * 16 + 4 * (lane >> 4) + e) * OPITCH + col] = 
            (__bf16)(EPI ? epi_act(a.eact, fmaf(acc[i][j][e], es, eb)) : acc[i][j][e] + b);
  }
  const int oc = tid % CPR, orow = tid / CPR;
  const bool col_ok = n0 + oc * 8 < a.N;
  constexpr int RPT = PIX / RPP;
  u32x4 ypre[BST ? RPT : 1];  // BSTAT: this thread's BN input rows, in flight across the barrier
  if constexpr (BST) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = orow + k * RPP, y = y0 + r / TW;
      ypre[k] = (y < H && col_ok) ? ld16(a.by + ((long)(img * H + y) * W + x0 + r % TW) * a.bycs + n0 + oc * 8)
                                  : u32x4{0u, 0u, 0u, 0u};
    }
  }
  __syncthreads();
  EpiStats<BST> es;
  es.init(a, col_ok, n0 + oc * 8);
  auto out_row = [&](int r, const u32x4& yv) {
    const int y = y0 + r / TW;
    if (y >= H || !col_ok) return;
    u32x4 v = *reinterpret_cast<const u32x4*>(&Os[r * OPITCH + oc * 8]);
    const long pix = (long)(img * H + y) * W + x0 + r % TW;
    __bf16* dst = a.out + pix * a.ocs + a.oco + n0 + oc * 8;
    if (DG && a.addend) {
      const u32x4 q = ld16(a.addend + pix * a.adcs + n0 + oc * 8);
      const u32x4 o = a.accumulate ? ld16(dst) : u32x4{0u, 0u, 0u, 0u};
      const __bf16 *qv = reinterpret_cast<const __bf16*>(&q), *ov = reinterpret_cast<const __bf16*>(&o);
      __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e] + (float)qv[e]);
    } else if (a.accumulate) {
      const u32x4 o = ld16(dst);
      const __bf16* ov = reinterpret_cast<const __bf16*>(&o);
      __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e]);
    }
    st16(dst, v);
    if (a.stats) es.add(a, v, yv);
  };
  if constexpr (BST) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) out_row(orow + k * RPP, ypre[k]);
  } else {
    for (int r = orow; r < PIX; r += RPP) out_row(r, ypre[0]);
  }
  if (a.stats) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[0][orow][oc * 8 + e] = es.s1[e];
      red[1][orow][oc * 8 + e] = es.s2[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      float x1 = 0.f, x2 = 0.f;
      for (int g = 0; g < RPP; ++g) {
        x1 += red[0][g][tid];
        x2 += red[1][g][tid];
      }
      float* s = a.stats + (long)mt * 2 * a.N + n0 + tid;
      s[0] = x1;
      s[a.N] = x2;
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// 3x3 / stride-2 / pad-1 DATA GRADIENT on super-pixel halo tiles (DG2H; also nn.ConvTranspose2d(k3, s2, p1) forward).
// dx pixel (2i + py, 2j + px) of output class (py, px) reads dy only at (i + di, j + dj), di, dj in {0, 1}: class
// (0,0) one tap (kh, kw) = (1,1); (0,1) taps (1,0) / (1,2) at dj = 1 / 0; (1,0) taps (0,1) / (2,1) at di = 1 / 0;
// (1,1) the four corners. A block owns an 8 x TJ tile of super-pixels (i, j) — the 16 x 2TJ dx pixels of all four
// classes — and BN output channels. Per 32-channel chunk of dy it stages the 9 x (TJ+1) dy halo and the 9-tap weight
// slab in LDS ONCE and runs every (class, tap) out of LDS: each dy element is staged ~(9 (TJ+1)) / (8 TJ) times per
// column tile, against once per (class, tap) gather in the per-class implicit GEMM (conv_bf16_kernel<BN,
// CV_DGRAD2>), and the four classes share one launch and one weight slab. Wave w owns super-pixels 16 w .. 16 w + 15
// in all four classes: 4 + 2 + 2 + 1 = 9 (fragment, tap) MFMA units per 32-channel chunk for every wave, four
// accumulator sets, no cross-wave sums.
constexpr int G2_TI = 8, G2_TJ = 8;  // super-pixel tile rows; columns of the launched tile
template <int TJ>
struct G2Geo {
  static constexpr int NT = 32 * TJ, W = NT / 64;             // threads, waves (= fragments per class)
  static constexpr int HW = TJ + 1, NPIX = (G2_TI + 1) * HW;  // halo
  static constexpr int PIX = 4 * G2_TI * TJ;                  // dx pixels per tile (16 x 2TJ)
};
// tap q of class c: weight tap index kh * 3 + kw and the dy offsets (di, dj)
__device__ __forceinline__ void g2_tap(int c, int q, int& t, int& di, int& dj) {
  const int py = c >> 1, px = c & 1;
  const int kh = py ? ((c == 3 ? (q >> 1) : q) ? 2 : 0) : 1;
  const int kw = px ? ((c == 3 ? (q & 1) : q) ? 2 : 0) : 1;
  t = kh * 3 + kw;
  di = py && kh == 0;
  dj = px && kw == 0;
}

template <int TJ, int BN, int XF, bool BST>
__device__ __forceinline__ void dg2_body(const ConvArgs& a) {
  using G = G2Geo<TJ>;
  constexpr int NT = G::NT, W = G::W, HW = G::HW, NPIX = G::NPIX, PIX = G::PIX, DXW = 2 * TJ;
  constexpr int A_TOT = NPIX * (C3_CK / 8), A_CH = (A_TOT + NT - 1) / NT;
  constexpr int B_TOT = 9 * BN * (C3_CK / 8), B_CH = (B_TOT + NT - 1) / NT;
  constexpr int TN = BN / 16, NS = 4;  // column fragments; accumulator sets (one per output class)
  constexpr int OPITCH = BN + 8, CPR = BN / 8, RPP = NT / CPR, RPT = PIX / RPP;
  constexpr int SMEM_A = NPIX * C3_LD, SMEM_B = 9 * BN * C3_LD;
  constexpr int SMEM_AB = 2 * (SMEM_A + SMEM_B), SMEM_O = 2 * PIX * OPITCH, SMEM_R = 2 * RPP * BN * 4;
  constexpr int SMEM_BYTES = SMEM_AB > SMEM_O ? (SMEM_AB > SMEM_R ? SMEM_AB : SMEM_R) : (SMEM_O > SMEM_R ? SMEM_O : SMEM_R);
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[SMEM_BYTES];
  __bf16* As = reinterpret_cast<__bf16*>(lds_raw);
  __bf16* Bs = As + SMEM_A;
  float (*red)[RPP][BN] = reinterpret_cast<float (*)[RPP][BN]>(lds_raw);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ho = a.sh_, Wo = a.sw_, H = a.rh, Wd = a.rw;  // dy grid, dx image
  const int tx = (Wo + TJ - 1) / TJ, ty = (Ho + G2_TI - 1) / G2_TI;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int mt = bid / a.ntiles, nt = bid - mt * a.ntiles;
  const int n0 = nt * BN;
  const int img = mt / (tx * ty), trem = mt - img * (tx * ty);
  const int i0 = (trem / tx) * G2_TI, j0 = (trem - (trem / tx) * tx) * TJ;

  // halo chunks of this thread: e = tid + NT i -> halo cell e / 4 (dy pixel (i0 + cell / HW, j0 + cell % HW)),
  // channel quad e % 4
  constexpr unsigned OOR = 0x7FFFFFF0u;
  const __amdgpu_buffer_rsrc_t src_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, a.src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wt_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, a.wt_bytes, 0x00020000);
  int a_off[A_CH], a_pix[A_CH];
  unsigned a_in = 0;  // XF: halo cells inside the tile (their dy pixel's unique writer)
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int e = tid + NT * i, q = e >> 2, hy = q / HW, hx = q - (q / HW) * HW;
    const int gy = i0 + hy, gx = j0 + hx;
    const bool ok = e < A_TOT && gy < Ho && gx < Wo;
    a_pix[i] = ok ? (img * Ho + gy) * Wo + gx : -1;
    a_off[i] = ok ? a_pix[i] * a.scs + a.sco + (e & 3) * 8 : -1;
    a_in |= (unsigned)(ok && hy < G2_TI && hx < TJ) << i;
  }
  constexpr int XTAB = XF == XF_BWD ? 5 * XMAXC : 4;
  __shared__ __attribute__((aligned(16))) float xtab[XTAB];
  if constexpr (XF != XF_NONE) xf_table<XF>(a, xtab);
  const __amdgpu_buffer_rsrc_t xy_rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.xy, (short)0, XF == XF_BWD ? a.xy_bytes : 0, 0x00020000);
  constexpr int XA = XF == XF_BWD ? A_CH : 1;
  u32x4 ry[XA];
  const int xq = (tid & 3) * 8;  // this thread's channels within a chunk step
  // weight slab rows: q = tid + NT i -> row q / 4 = tap * BN + col, channel quad q % 4 (CRSK: [c][tap][k])
  int b_off[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    const int q = tid + NT * i, row = q >> 2, tap = row / BN, col = row - tap * BN;
    b_off[i] = (q < B_TOT && n0 + col < a.N) ? (n0 + col) * 9 * a.sc + tap * a.sc + (q & 3) * 8 : -1;
  }

  u32x4 ra[A_CH], rb[B_CH];
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(src_rs, a_off[i] >= 0 ? (unsigned)(a_off[i] + c0) * 2u : OOR, 0, 0);
      if constexpr (XF == XF_BWD)
        ry[i] = __builtin_amdgcn_raw_buffer_load_b128(
            xy_rs, a_pix[i] >= 0 ? (unsigned)(a_pix[i] * a.xycs + c0 + xq) * 2u : OOR, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      rb[i] = __builtin_amdgcn_raw_buffer_load_b128(wt_rs, b_off[i] >= 0 ? (unsigned)(b_off[i] + c0) * 2u : OOR, 0, 0);
  };
  auto store = [&](int c0) {
    XfCoef<XF == XF_NONE ? XF_FWD : XF> xk;
    if constexpr (XF != XF_NONE) xk.load(xtab, c0 + xq);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int e = tid + NT * i;
      if constexpr (XF == XF_NONE) {
        if (e < A_TOT) st16(&As[c3_swz(e >> 2, e & 3)], ra[i]);
      } else {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (a_pix[i] >= 0) v = xf_chunk<XF>(ra[i], ry[XF == XF_BWD ? i : 0], xk, a.xact);
        if (nt == 0 && ((a_in >> i) & 1)) st16(a.xo + (long)a_pix[i] * a.xocs + c0 + xq, v);
        if (e < A_TOT) st16(&As[c3_swz(e >> 2, e & 3)], v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int q = tid + NT * i;
      if (q < B_TOT) st16(&Bs[c3_swz(q >> 2, q & 3)], rb[i]);
    }
  };

  // accumulator set c = output class (2 py + px) of this wave's 16 super-pixels; the lane's fragment row's halo cell
  const int sp_row = 16 * wave + (lane & 15);  // super-pixel index in the tile (row-major, TJ per row)
  const int cell0 = (sp_row / TJ) * HW + (sp_row % TJ);
  const int kq = lane >> 4;
  f32x4 acc[NS][TN];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[s][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nch = a.sc / C3_CK;
  load(0);
  for (int ch = 0; ch < nch; ++ch) {
    store(ch * C3_CK);
    __syncthreads();
    if (ch + 1 < nch) load((ch + 1) * C3_CK);
#pragma unroll
    for (int c = 0; c < NS; ++c) {
#pragma unroll
      for (int q = 0; q < (c == 3 ? 4 : c == 0 ? 1 : 2); ++q) {
        int t, di, dj;
        g2_tap(c, q, t, di, dj);
        const int s = c;
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(&As[c3_swz(cell0 + di * HW + dj, kq)]);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const bf16x8 fb = *reinterpret_cast<const bf16x8*>(&Bs[c3_swz(t * BN + 16 * j + (lane & 15), kq)]);
          acc[s][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[s][j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  // ---- epilogue: bf16 image of the 16 x 2TJ dx tile in LDS, 16-byte row stores, optional statistics ----
  __bf16* Os = reinterpret_cast<__bf16*>(lds_raw);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int c = s, py = c >> 1, px = c & 1, f = wave;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = 16 * j + (lane & 15);
      const float b = (a.bias && n0 + col < a.N) ? a.bias[n0 + col] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int sp = 16 * f + 4 * (lane >> 4) + e;
        const int ly = 2 * (sp / TJ) + py, lx = 2 * (sp % TJ) + px;
        Os[(ly * DXW + lx) * OPITCH + col] = (__bf16)(acc[s][j][e] + b);
      }
    }
  }
  const int oc = tid % CPR, orow = tid / CPR;
  const bool col_ok = n0 + oc * 8 < a.N;
  const int y0 = 2 * i0, x0 = 2 * j0;
  u32x4 ypre[BST ? RPT : 1];  // BSTAT: this thread's BN input rows, in flight across the barrier
  if constexpr (BST) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const int r = orow + k * RPP, y = y0 + r / DXW, x = x0 + r % DXW;
      ypre[k] = (y < H && x < Wd && col_ok) ? ld16(a.by + ((long)(img * H + y) * Wd + x) * a.bycs + n0 + oc * 8)
                                           : u32x4{0u, 0u, 0u, 0u};
    }
  }
  __syncthreads();
  EpiStats<BST> es;
  es.init(a, col_ok, n0 + oc * 8);
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int r = orow + k * RPP, y = y0 + r / DXW, x = x0 + r % DXW;
    if (y >= H || x >= Wd || !col_ok) continue;
    u32x4 v = *reinterpret_cast<const u32x4*>(&Os[r * OPITCH + oc * 8]);
    const long pix = (long)(img * H + y) * Wd + x;
    __bf16* dst = a.out + pix * a.ocs + a.oco + n0 + oc * 8;
    if (a.addend) {
      const u32x4 qv4 = ld16(a.addend + pix * a.adcs + n0 + oc * 8);
      const u32x4 o = a.accumulate ? ld16(dst) : u32x4{0u, 0u, 0u, 0u};
      const __bf16 *qv = reinterpret_cast<const __bf16*>(&qv4), *ov = reinterpret_cast<const __bf16*>(&o);
      __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e] + (float)qv[e]);
    } else if (a.accumulate) {
      const u32x4 o = ld16(dst);
      const __bf16* ov = reinterpret_cast<const __bf16*>(&o);
      __bf16* nv = reinterpret_cast<__bf16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) nv[e] = (__bf16)((float)nv[e] + (float)ov[e]);
    }
    st16(dst, v);
    if (a.stats) es.add(a, v, ypre[BST ? k : 0]);
  }
  if (a.stats) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[0][orow][oc * 8 + e] = es.s1[e];
      red[1][orow][oc * 8 + e] = es.s2[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      float x1 = 0.f, x2 = 0.f;
      for (int g = 0; g < RPP; ++g) {
        x1 += red[0][g][tid];
        x2 += red[1][g][tid];
      }
      float* sp = a.stats + (long)mt * 2 * a.N + n0 + tid;
      sp[0] = x1;
      sp[a.N] = x2;
    }
  }
}

// entry points (the bodies are shared; the eval Conv-BN-act variants are separate symbols so the training
// kernels keep their code and register allocation)
template <int BN, int MODE>
__global__ void __launch_bounds__(256, BN <= 64 ? 4 : 2) conv_bf16_kernel(ConvArgs a) { conv_bf16_body<BN, MODE, false>(a); }
template <int BN, int MODE, int KT>
__global__ void __launch_bounds__(256, KT == 256 ? 1 : (KT == 64 && BN <= 64) ? 3 : 2) conv1_kernel(ConvArgs a, int groups) {
  conv1_body<BN, MODE, KT>(a, groups);
}
template <int BN, int KT>
__global__ void __launch_bounds__(256, KT == 256 ? 1 : (KT == 64 && BN <= 64) ? 3 : 2) conv1_act_kernel(ConvArgs a, int groups) {
  conv1_body<BN, CV_FWD, KT, true>(a, groups);
}
template <int BN, int KT>
__global__ void __launch_bounds__(256, KT == 256 ? 1 : (KT == 64 && BN <= 64) ? 3 : 2) conv1_xf_kernel(ConvArgs a, int groups) {
  conv1_body<BN, CV_FWD, KT, false, XF_FWD>(a, groups);
}
template <int BN>
__global__ void __launch_bounds__(256, BN <= 64 ? 4 : 2) conv_bf16_act_kernel(ConvArgs a) { conv_bf16_body<BN, CV_FWD, true>(a); }
template <int TW, bool DG, int BN>
__global__ void __launch_bounds__(256, 3) conv3_kernel(ConvArgs a) { conv3_body<TW, DG, BN, false>(a); }
template <int TW, int BN>
__global__ void __launch_bounds__(256, 3) conv3_act_kernel(ConvArgs a) { conv3_body<TW, false, BN, true>(a); }
template <bool DG, bool EPI>
__global__ void __launch_bounds__(512, 1) conv3w_kernel(ConvArgs a) { conv3_body<16, DG, 128, EPI, XF_NONE, 2>(a); }
// training Conv-BN-act fusion: the A operand is the producer BatchNorm's input (FWD) or the gradient of its output
// (DGRAD) and the BN-act (backward) is applied while staging it (XF_FWD / XF_BWD); the coefficient table and the
// second operand cost LDS and registers, so these run at 3 (2 for the 3x3 halo tiles) workgroups per CU
template <int BN, int MODE, int XF>
__global__ void __launch_bounds__(256, (XF == XF_BWD && BN == 64) ? 2 : 3) conv_bf16_xf_kernel(ConvArgs a) {
  conv_bf16_body<BN, MODE, false, XF>(a);
}
template <int TW, bool DG, int BN, int XF>
__global__ void __launch_bounds__(256, 2) conv3_xf_kernel(ConvArgs a) { conv3_body<TW, DG, BN, false, XF>(a); }
// stride-2 3x3 data gradient on super-pixel halo tiles (plain / XF backward operand / BSTAT epilogue)
template <int TJ, int BN, int XF, bool BST>
__global__ void __launch_bounds__(32 * TJ, (XF == XF_BWD && BN == 64) ? 2 : 3) dg2_kernel(ConvArgs a) {
  dg2_body<TJ, BN, XF, BST>(a);
}
// BSTAT data gradients (adr_conv2d_dgrad_bf16_bstat): the same bodies with the BN-backward statistics epilogue, as
// separate symbols so the plain kernels keep their code and register allocation
template <int BN, int MODE, int XF>
__global__ void __launch_bounds__(256, XF == XF_BWD ? ((BN == 64) ? 2 : 3) : (BN <= 64 ? 4 : 2))
    conv_bf16_bst_kernel(ConvArgs a) {
  conv_bf16_body<BN, MODE, false, XF, true>(a);
}
template <int BN, int KT>
__global__ void __launch_bounds__(256, KT == 256 ? 1 : (KT == 64 && BN <= 64) ? 3 : 2) conv1_bst_kernel(ConvArgs a, int groups) {
  conv1_body<BN, CV_DGRAD, KT, false, XF_NONE, true>(a, groups);
}
template <int TW, int BN, int XF>
__global__ void __launch_bounds__(256, XF == XF_NONE ? 3 : 2) conv3_bst_kernel(ConvArgs a) {
  conv3_body<TW, true, BN, false, XF, 1, true>(a);
}
__global__ void __launch_bounds__(512, 1) conv3w_bst_kernel(ConvArgs a) { conv3_body<16, true, 128, false, XF_NONE, 2, true>(a); }

// tile width of the 3x3 path for this geometry, or 0 when it does not apply
static int conv3_tw(const adr_conv_desc* d, int red_ch, int out_ch) {
  if (d->r != 3 || d->s != 3 || d->stride_h != 1 || d->pad_h != 1 || red_ch % C3_CK || out_ch % 32) return 0;
  if (d->w % 16 == 0 && d->h >= 8) return 16;
  if (d->w % 8 == 0) return 8;
  return 0;
}
static int conv3_bn(int out_ch) { return out_ch % 64 == 0 ? 64 : 32; }
static int conv3_tiles(const adr_conv_desc* d, int tw, int pix = 128) {
  return d->n * ((d->h + pix / tw - 1) / (pix / tw)) * (d->w / tw);
}
// the wide 256-pixel x 128-channel tile (conv3w_kernel, one 512-thread block per CU) for big-channel 3x3 convs with
// enough tiles to fill the chip twice over
static bool conv3_wide(const adr_conv_desc* d, int tw, int red_ch, int out_ch) {
  static const int on = getenv("ADR_CONV3W") ? atoi(getenv("ADR_CONV3W")) : 1;  // A/B
  return on && tw == 16 && d->h >= 16 && red_ch >= 128 && out_ch % 128 == 0 &&
         (long)conv3_tiles(d, 16, 256) * (out_ch / 128) >= 512;
}
template <bool DG>
static void launch_conv3(int tw, int bn, const adr_conv_desc* d, ConvArgs& g, hipStream_t st, bool wide = false) {
  if (DG && g.by) {  // BSTAT data gradient
    if constexpr (!DG) return;
    if (wide) {
      g.ntiles = g.N / 128;
      hipLaunchKernelGGL(conv3w_bst_kernel, dim3(conv3_tiles(d, 16, 256) * g.ntiles), dim3(512), 0, st, g);
      return;
    }
    g.ntiles = g.N / bn;
    dim3 grid(conv3_tiles(d, tw) * g.ntiles);
#define ADR_C3B(TW_, BN_)                                                                                   \
  do {                                                                                                      \
    if (g.xs) hipLaunchKernelGGL((conv3_bst_kernel<TW_, BN_, XF_BWD>), grid, dim3(256), 0, st, g);          \
    else hipLaunchKernelGGL((conv3_bst_kernel<TW_, BN_, XF_NONE>), grid, dim3(256), 0, st, g);              \
  } while (0)
    if (bn == 64) {
      if (tw == 16) ADR_C3B(16, 64);
      else ADR_C3B(8, 64);
    } else {
      if (tw == 16) ADR_C3B(16, 32);
      else ADR_C3B(8, 32);
    }
#undef ADR_C3B
    return;
  }
  if (wide) {
    g.ntiles = g.N / 128;
    dim3 grid(conv3_tiles(d, 16, 256) * g.ntiles);
    if (!DG && g.escale) hipLaunchKernelGGL((conv3w_kernel<false, true>), grid, dim3(512), 0, st, g);
    else hipLaunchKernelGGL((conv3w_kernel<DG, false>), grid, dim3(512), 0, st, g);
    return;
  }
  g.ntiles = g.N / bn;
  dim3 grid(conv3_tiles(d, tw) * g.ntiles);
  if (g.xs) {  // XF: FWD applies the producer's BN-act, DGRAD its backward
    constexpr int XF = DG ? XF_BWD : XF_FWD;
    if (bn == 64) {
      if (tw == 16) hipLaunchKernelGGL((conv3_xf_kernel<16, DG, 64, XF>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((conv3_xf_kernel<8, DG, 64, XF>), grid, dim3(256), 0, st, g);
    } else {
      if (tw == 16) hipLaunchKernelGGL((conv3_xf_kernel<16, DG, 32, XF>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((conv3_xf_kernel<8, DG, 32, XF>), grid, dim3(256), 0, st, g);
    }
    return;
  }
  if (!DG && g.escale) {
    if (bn == 64) {
      if (tw == 16) hipLaunchKernelGGL((conv3_act_kernel<16, 64>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((conv3_act_kernel<8, 64>), grid, dim3(256), 0, st, g);
    } else {
      if (tw == 16) hipLaunchKernelGGL((conv3_act_kernel<16, 32>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((conv3_act_kernel<8, 32>), grid, dim3(256), 0, st, g);
    }
    return;
  }
  if (bn == 64) {
    if (tw == 16) hipLaunchKernelGGL((conv3_kernel<16, DG, 64>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((conv3_kernel<8, DG, 64>), grid, dim3(256), 0, st, g);
  } else {
    if (tw == 16) hipLaunchKernelGGL((conv3_kernel<16, DG, 32>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((conv3_kernel<8, DG, 32>), grid, dim3(256), 0, st, g);
  }
}

static int dg2_tiles(const adr_conv_desc* d) {
  return d->n * ((d->ho + G2_TI - 1) / G2_TI) * ((d->wo + G2_TJ - 1) / G2_TJ);
}
static void launch_dg2(int bn, const adr_conv_desc* d, ConvArgs& g, hipStream_t st) {
  g.ntiles = g.N / bn;
  const dim3 grid(dg2_tiles(d) * g.ntiles), blk(32 * G2_TJ);
#define ADR_G2(BN_)                                                                                            \
  do {                                                                                                         \
    if (g.xs && g.by) hipLaunchKernelGGL((dg2_kernel<G2_TJ, BN_, XF_BWD, true>), grid, blk, 0, st, g);         \
    else if (g.xs) hipLaunchKernelGGL((dg2_kernel<G2_TJ, BN_, XF_BWD, false>), grid, blk, 0, st, g);           \
    else if (g.by) hipLaunchKernelGGL((dg2_kernel<G2_TJ, BN_, XF_NONE, true>), grid, blk, 0, st, g);           \
    else hipLaunchKernelGGL((dg2_kernel<G2_TJ, BN_, XF_NONE, false>), grid, blk, 0, st, g);                    \
  } while (0)
  if (bn == 64) ADR_G2(64);
  else if (bn == 32) ADR_G2(32);
  else ADR_G2(16);
#undef ADR_G2
}

template <int MODE>
static void launch_conv(int bn, dim3 grid, const ConvArgs& g, hipStream_t st) {
  if constexpr (MODE != CV_FWD) {
    if (g.by) {  // BSTAT data gradient (XF: bn <= 64)
#define ADR_CB(BN_)                                                                                         \
  do {                                                                                                      \
    if (g.xs) hipLaunchKernelGGL((conv_bf16_bst_kernel<BN_, MODE, XF_BWD>), grid, dim3(256), 0, st, g);     \
    else hipLaunchKernelGGL((conv_bf16_bst_kernel<BN_, MODE, XF_NONE>), grid, dim3(256), 0, st, g);         \
  } while (0)
      switch (bn) {
        case 16: ADR_CB(16); break;
        case 32: ADR_CB(32); break;
        case 64: ADR_CB(64); break;
        default: hipLaunchKernelGGL((conv_bf16_bst_kernel<128, MODE, XF_NONE>), grid, dim3(256), 0, st, g); break;
      }
#undef ADR_CB
      return;
    }
  }
  if (g.xs) {  // XF (bn <= 64)
    constexpr int XF = MODE == CV_FWD ? XF_FWD : XF_BWD;
    switch (bn) {
      case 16: hipLaunchKernelGGL((conv_bf16_xf_kernel<16, MODE, XF>), grid, dim3(256), 0, st, g); break;
      case 32: hipLaunchKernelGGL((conv_bf16_xf_kernel<32, MODE, XF>), grid, dim3(256), 0, st, g); break;
      default: hipLaunchKernelGGL((conv_bf16_xf_kernel<64, MODE, XF>), grid, dim3(256), 0, st, g); break;
    }
    return;
  }
  if (MODE == CV_FWD && g.escale) {
    switch (bn) {
      case 16: hipLaunchKernelGGL((conv_bf16_act_kernel<16>), grid, dim3(256), 0, st, g); break;
      case 32: hipLaunchKernelGGL((conv_bf16_act_kernel<32>), grid, dim3(256), 0, st, g); break;
      case 64: hipLaunchKernelGGL((conv_bf16_act_kernel<64>), grid, dim3(256), 0, st, g); break;
      default: hipLaunchKernelGGL((conv_bf16_act_kernel<128>), grid, dim3(256), 0, st, g); break;
    }
    return;
  }
  switch (bn) {
    case 16: hipLaunchKernelGGL((conv_bf16_kernel<16, MODE>), grid, dim3(256), 0, st, g); break;
    case 32: hipLaunchKernelGGL((conv_bf16_kernel<32, MODE>), grid, dim3(256), 0, st, g); break;
    case 64: hipLaunchKernelGGL((conv_bf16_kernel<64, MODE>), grid, dim3(256), 0, st, g); break;
    default: hipLaunchKernelGGL((conv_bf16_kernel<128, MODE>), grid, dim3(256), 0, st, g); break;
  }
}

static int conv1_enabled() {
  static const int on = getenv("ADR_CONV1") ? atoi(getenv("ADR_CONV1")) : 1;  // A/B: 0 = per-tile kernel
  return on;
}
// column-tile count and block groups of a conv1 launch: about one resident wave of blocks (3 or 2 per CU)
static int conv1_groups(long rows, int ntiles, int kt, int bn) {
  const int mtiles = cdiv(rows, CBM);
  // resident blocks per CU (LDS: 27 / 33 / 46 / 72 KB at KT 64, 45 / 54 / 71 / 104 KB at KT 128)
  const int occ = kt == 256 ? 1 : kt == 64 ? (bn <= 32 ? 4 : bn == 64 ? 3 : 2) : (bn <= 32 ? 3 : bn == 64 ? 2 : 1);
  const int target = 256 * occ;
  int g = target / ntiles;
  if (g < 1) g = 1;
  return g < mtiles ? g : mtiles;
}

template <int MODE>
static void launch_conv1(int bn, int kt, long rows, ConvArgs& g, hipStream_t st) {
  const int groups = conv1_groups(rows, g.ntiles, kt, bn);
  const dim3 grid(groups * g.ntiles);
#define ADR_C1(BN, KT)                                                                                     \
  do {                                                                                                     \
    if (MODE == CV_DGRAD && g.by)                                                                          \
      hipLaunchKernelGGL((conv1_bst_kernel<BN, KT>), grid, dim3(256), 0, st, g, groups);                   \
    else if (MODE == CV_FWD && g.escale)                                                                   \
      hipLaunchKernelGGL((conv1_act_kernel<BN, KT>), grid, dim3(256), 0, st, g, groups);                   \
    else if (MODE == CV_FWD && g.xs)                                                                       \
      hipLaunchKernelGGL((conv1_xf_kernel<BN, KT>), grid, dim3(256), 0, st, g, groups);                    \
    else                                                                                                   \
      hipLaunchKernelGGL((conv1_kernel<BN, MODE, KT>), grid, dim3(256), 0, st, g, groups);                 \
  } while (0)
  if (kt == 64) {
    switch (bn) {
      case 16: ADR_C1(16, 64); break;
      case 32: ADR_C1(32, 64); break;
      case 64: ADR_C1(64, 64); break;
      default: ADR_C1(128, 64); break;
    }
  } else if (kt == 128) {
    switch (bn) {
      case 16: ADR_C1(16, 128); break;
      case 32: ADR_C1(32, 128); break;
      case 64: ADR_C1(64, 128); break;
      default: ADR_C1(128, 128); break;
    }
  } else {  // KT 256: column tiles of at most 64 (LDS)
    switch (bn) {
      case 16: ADR_C1(16, 256); break;
      case 32: ADR_C1(32, 256); break;
      default: ADR_C1(64, 256); break;
    }
  }
#undef ADR_C1
}

static int conv_pick_bn(int n) { return n <= 16 ? 16 : n <= 32 ? 32 : n <= 64 ? 64 : 128; }

static int conv_check(const adr_conv_desc* d) {
  ADR_REQUIRE(d && d->n > 0 && d->h > 0 && d->w > 0 && d->c > 0 && d->k > 0 && d->r > 0 && d->s > 0,
              "conv: bad geometry");
  ADR_REQUIRE(d->dtype == ADR_BF16, "conv (bf16 engine): dtype %d", d->dtype);
  ADR_REQUIRE(d->c % 8 == 0 && d->k % 8 == 0, "conv: C (%d) and K (%d) must be multiples of 8", d->c, d->k);
  ADR_REQUIRE(d->x_cstride % 8 == 0 && d->x_coff % 8 == 0 && d->y_cstride % 8 == 0 && d->y_coff % 8 == 0,
              "conv: channel views must be 16-byte aligned");
  ADR_REQUIRE(d->x_cstride >= d->x_coff + d->c && d->y_cstride >= d->y_coff + d->k, "conv: view exceeds stride");
  // the row decoder keeps one stride but separate paddings (ELA_HSFPN's 7x1 Conv1d pads (3, 0))
  ADR_REQUIRE(d->stride_h == d->stride_w, "conv: anisotropic stride");
  const int ho = (d->h + 2 * d->pad_h - d->r) / d->stride_h + 1, wo = (d->w + 2 * d->pad_w - d->s) / d->stride_w + 1;
  ADR_REQUIRE(ho == d->ho && wo == d->wo, "conv: output size mismatch (%dx%d vs %dx%d)", d->ho, d->wo, ho, wo);
  ADR_REQUIRE((long)d->n * d->h * d->w * d->x_cstride < (1l << 30) && (long)d->n * d->ho * d->wo * d->y_cstride < (1l << 30)
              && (long)d->k * d->c * d->r * d->s < (1l << 30), "conv: tensor exceeds 2^30 elements (32-bit buffer offsets)");
  return ADR_OK;
}

// The kernel a bf16 contraction runs on — shared by the launchers and adr_conv2d_bf16_kernel_symbol, so the
// roofline labels cannot drift from the dispatch.
struct ConvPlan {
  int tw;    // > 0: conv3_kernel<tw, dgrad> (3x3 stride-1 halo tiles)
  int wide;  // with tw: the 256 x 128 tile (conv3w_kernel)
  int bn;    // else conv_bf16_kernel<bn, mode>
  int mode;  // CV_FWD / CV_DGRAD / CV_DGRAD2
  int kt;    // > 0: conv1_kernel<bn, mode, kt> (streaming 1x1, reduction <= kt)
  int dg2;   // > 0 (stride-2 DGRAD): dg2_kernel<dg2 = TJ, bn> (super-pixel halo tiles, all parity classes at once)
};
// ADR_DG2H: 0 = per-class implicit GEMM only (A/B), 1 = DG2H where it pays (default), 2 = DG2H wherever it applies
// (tests: ragged super-pixel tiles). Read per plan, so a test can switch it in-process.
static int dg2_mode() {
  const char* e = getenv("ADR_DG2H");
  return e ? atoi(e) : 1;
}
static ConvPlan conv_plan(const adr_conv_desc* d, bool dgrad, bool xf = false) {
  ConvPlan p{0, 0, 0, dgrad ? (d->stride_h == 2 ? CV_DGRAD2 : CV_DGRAD) : CV_FWD};
  const int red = dgrad ? d->k : d->c, out = dgrad ? d->c : d->k;
  // DG2H where its 8 x 8 super-pixel tiles cover the dy grid with <= 15 % padding (the 20 x 20 grids of the P5
  // layers would run 44 % empty rows: the per-class implicit GEMM is faster there, 27 vs 32 us)
  const long g2_area = (long)((d->ho + G2_TI - 1) / G2_TI * G2_TI) * ((d->wo + G2_TJ - 1) / G2_TJ * G2_TJ);
  if (p.mode == CV_DGRAD2 && d->r == 3 && d->s == 3 && d->pad_h == 1 && d->pad_w == 1 && red % C3_CK == 0 &&
      out % 16 == 0 && (out <= 64 || out % 64 == 0) && dg2_mode() &&
      (dg2_mode() == 2 || g2_area * 100 <= 115l * d->ho * d->wo)) {
    p.dg2 = G2_TJ;
    p.bn = out % 64 == 0 ? 64 : out % 32 == 0 ? 32 : 16;
    p.kt = 0;
    return p;
  }
  if (p.mode != CV_DGRAD2) p.tw = conv3_tw(d, red, out);
  p.wide = p.tw && !xf && conv3_wide(d, p.tw, red, out);
  // 1x1 contractions are two or three K-steps long: 64-wide column tiles (4 waves/SIMD) hide their load latency
  // better than 128-wide ones (2 waves/SIMD), at the cost of reading the A rows once per column tile (L2 hits).
  // XF kernels are single-buffered: at most 64 columns.
  p.bn = p.tw ? conv3_bn(out) : ((d->r * d->s == 1 || xf) && out > 64) ? 64 : conv_pick_bn(out);
  {
    // the 128-wide double-buffered tile runs two workgroups per CU; when its grid is under two such rounds of the
    // chip (the n-scale 80^2 -> 40^2 / 40^2 -> 20^2 stride-2 convs: 800 / 200 workgroups), the 64-wide tile's
    // four per CU fill it better. ADR_CONV_BN_MAX: A/B override (128 = never narrow, 64 = always)
    const char* e = getenv("ADR_CONV_BN_MAX");
    const int cap = e ? atoi(e) : 0;
    const long rows = dgrad ? (long)d->n * d->h * d->w : (long)d->n * d->ho * d->wo;
    const long grid128 = (rows + CBM - 1) / CBM * ((out + 127) / 128);
    if (!p.tw && p.bn == 128 && (cap ? cap < 128 : grid128 < 1024)) p.bn = cap ? (cap >= 16 ? cap : 64) : 64;
  }
  p.kt = 0;
  const bool c1 = !p.tw && p.mode != CV_DGRAD2 && d->r == 1 && d->s == 1 && d->stride_h == 1 && d->pad_h == 0 &&
                  d->pad_w == 0 && conv1_enabled();
  // forward XF runs on the streaming kernel with the plain forward's tiling (so its output and statistics rows are
  // bitwise the unfused pair's); the data-gradient XF keeps the per-tile kernel
  // KT 256 (1 block per CU) measured a gain for DGRAD only (forward at l-scale 1280^2: 126.5 vs 126.4 ms/step)
  if (c1 && (!xf || !dgrad) && red <= (dgrad && p.bn <= 64 ? 256 : 128))
    p.kt = red <= 64 ? 64 : red <= 128 ? 128 : 256;
  return p;
}

// XF arguments (adr_bnact_xf) into the kernel arguments; `red` = reduction channels, the source grid sh x sw
static int xf_args(const adr_bnact_xf* xf, bool bwd, int red, int n, int sh, int sw, ConvArgs& g) {
  ADR_REQUIRE(xf && xf->scale && xf->shift && xf->out && (xf->act == ACT_NONE || xf->act == ACT_SILU),
              "conv bnact: scale / shift / side output / act (none or silu)");
  ADR_REQUIRE(red <= XMAXC, "conv bnact: %d reduction channels (table holds %d)", red, XMAXC);
  ADR_REQUIRE(xf->out_cstride >= red && xf->out_cstride % 8 == 0 && ((uintptr_t)xf->out & 15) == 0,
              "conv bnact: side output view");
  g.xs = xf->scale; g.xt = xf->shift; g.xact = xf->act;
  g.xo = (__bf16*)xf->out; g.xocs = xf->out_cstride;
  if (bwd) {
    ADR_REQUIRE(xf->y && xf->A && xf->B && xf->Cc && xf->y_cstride >= red && xf->y_cstride % 8 == 0 &&
                    ((uintptr_t)xf->y & 15) == 0,
                "conv bnact (dgrad): y view and A / B / Cc coefficients");
    ADR_REQUIRE((long)n * sh * sw * xf->y_cstride < (1l << 30), "conv bnact: y exceeds 2^30 elements");
    g.xy = (const __bf16*)xf->y; g.xycs = xf->y_cstride; g.xy_bytes = (int)(2l * n * sh * sw * xf->y_cstride);
    g.xA = xf->A; g.xB = xf->B; g.xC = xf->Cc;
  }
  return ADR_OK;
}

}  // namespace adr

using namespace adr;

static int conv_fwd_impl(const adr_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                         float* stats, int accumulate, const float* escale, const float* eshift, int eact,
                         void* stream, const adr_bnact_xf* xf = nullptr) {
  int rc = conv_check(d);
  if (rc) return rc;
  ConvArgs g{};
  if (xf) {
    ADR_REQUIRE(!escale, "conv fwd bnact: no eval epilogue");
    rc = xf_args(xf, false, d->c, d->n, d->h, d->w, g);
    if (rc) return rc;
  }
  g.src = (const __bf16*)x; g.wt = (const __bf16*)w; g.out = (__bf16*)y; g.bias = bias; g.stats = stats;
  g.escale = escale; g.eshift = eshift; g.eact = escale ? eact : 0;
  g.n = d->n; g.sh_ = d->h; g.sw_ = d->w; g.scs = d->x_cstride; g.sco = d->x_coff; g.sc = d->c;
  g.rh = d->ho; g.rw = d->wo; g.ocs = d->y_cstride; g.oco = d->y_coff;
  g.r = d->r; g.s = d->s; g.str = d->stride_h; g.ph = d->pad_h; g.pw = d->pad_w;
  g.N = d->k; g.ktot = d->r * d->s * d->c; g.accumulate = accumulate;
  g.src_bytes = (int)(2l * d->n * d->h * d->w * d->x_cstride);
  g.wt_bytes = (int)(2l * g.N * g.ktot);
  const ConvPlan pl = conv_plan(d, false, xf != nullptr);
  if (pl.tw) {
    launch_conv3<false>(pl.tw, pl.bn, d, g, (hipStream_t)stream, pl.wide);
    return check_launch("adr_conv2d_fwd_bf16");
  }
  const int bn = pl.bn;
  g.ntiles = cdiv(g.N, bn);
  if (pl.kt) {  // (escale: eval Conv-BN-act epilogue; xs: the XF forward)
    launch_conv1<CV_FWD>(bn, pl.kt, (long)d->n * d->ho * d->wo, g, (hipStream_t)stream);
    return check_launch("adr_conv2d_fwd_bf16");
  }
  dim3 grid(cdiv((long)d->n * d->ho * d->wo, CBM) * g.ntiles);
  launch_conv<CV_FWD>(bn, grid, g, (hipStream_t)stream);
  return check_launch("adr_conv2d_fwd_bf16");
}

extern "C" int adr_conv2d_fwd_bf16(const adr_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                                   float* stats, int accumulate, void* stream) {
  return conv_fwd_impl(d, x, w, bias, y, stats, accumulate, nullptr, nullptr, 0, stream);
}

// Eval Conv-BN-act (reference: the predictor's fused Conv.forward_fuse, nn/modules/conv.py:52-54 after
// fuse_conv_and_bn): y = act(conv(x, w) * scale + shift) in one launch, scale/shift from adr_bn_finalize with
// training = 0. Same dispatch as adr_conv2d_fwd_bf16 (bias-free, no statistics, no accumulation).
extern "C" int adr_conv2d_fwd_bf16_act(const adr_conv_desc* d, const void* x, const void* w, const float* scale,
                                       const float* shift, int act, void* y, void* stream) {
  ADR_REQUIRE(scale && shift && act >= ACT_NONE && act <= ACT_HSWISH, "conv fwd act: scale/shift/act");
  return conv_fwd_impl(d, x, w, nullptr, y, nullptr, 0, scale, shift, act, stream);
}

static int conv_dgrad_impl(const adr_conv_desc* d, const void* dy, const void* w_crsk, const float* bias, void* dx,
                           int accumulate, const void* addend, int adcs, void* stream,
                           const adr_bnact_xf* xf = nullptr, const adr_bn_bstat* bst = nullptr,
                           float* stats = nullptr) {
  int rc = conv_check(d);
  if (rc) return rc;
  ConvArgs g{};
  if (xf) {
    rc = xf_args(xf, true, d->k, d->n, d->ho, d->wo, g);
    if (rc) return rc;
  }
  if (bst) {
    ADR_REQUIRE(stats && bst->y && bst->scale && bst->shift && (bst->act == ACT_NONE || bst->act == ACT_SILU),
                "conv dgrad bstat: stats / y / scale / shift / act (none or silu)");
    ADR_REQUIRE(bst->y_cstride >= d->c && bst->y_cstride % 8 == 0 && ((uintptr_t)bst->y & 15) == 0 &&
                    ((uintptr_t)bst->scale & 15) == 0 && ((uintptr_t)bst->shift & 15) == 0,
                "conv dgrad bstat: 16-byte aligned y view / coefficients");
    ADR_REQUIRE((long)d->n * d->h * d->w * bst->y_cstride < (1l << 30), "conv dgrad bstat: y exceeds 2^30 elements");
    g.by = (const __bf16*)bst->y; g.bycs = bst->y_cstride; g.bact = bst->act; g.bs = bst->scale; g.bt = bst->shift;
  }
  g.src = (const __bf16*)dy; g.wt = (const __bf16*)w_crsk; g.out = (__bf16*)dx; g.bias = bias;
  g.stats = bst ? stats : nullptr;
  g.addend = (const __bf16*)addend; g.adcs = adcs;
  g.n = d->n; g.sh_ = d->ho; g.sw_ = d->wo; g.scs = d->y_cstride; g.sco = d->y_coff; g.sc = d->k;
  g.rh = d->h; g.rw = d->w; g.ocs = d->x_cstride; g.oco = d->x_coff;
  g.r = d->r; g.s = d->s; g.str = d->stride_h; g.ph = d->pad_h; g.pw = d->pad_w;
  g.N = d->c; g.ktot = d->r * d->s * d->k; g.accumulate = accumulate;
  g.src_bytes = (int)(2l * d->n * d->ho * d->wo * d->y_cstride);
  g.wt_bytes = (int)(2l * g.N * g.ktot);
  ADR_REQUIRE(d->stride_h == 1 || d->stride_h == 2, "conv dgrad (bf16 engine): stride %d", d->stride_h);
  const ConvPlan pl = conv_plan(d, true, xf != nullptr);
  const int bn = pl.bn;
  g.ntiles = cdiv(g.N, bn);
  hipStream_t st = (hipStream_t)stream;
  if (pl.dg2) {  // stride-2 3x3: all parity classes on super-pixel halo tiles
    launch_dg2(bn, d, g, st);
  } else if (pl.mode == CV_DGRAD2) {  // parity classes; the largest (even, even) class sizes the grid
    dim3 grid(cdiv((long)d->n * ((d->h + 1) / 2) * ((d->w + 1) / 2), CBM) * g.ntiles, 1, 4);
    launch_conv<CV_DGRAD2>(bn, grid, g, st);
  } else if (pl.tw) {
    launch_conv3<true>(pl.tw, pl.bn, d, g, st, pl.wide);
  } else if (pl.kt) {
    launch_conv1<CV_DGRAD>(bn, pl.kt, (long)d->n * d->h * d->w, g, st);
  } else {
    dim3 grid(cdiv((long)d->n * d->h * d->w, CBM) * g.ntiles);
    launch_conv<CV_DGRAD>(bn, grid, g, st);
  }
  return check_launch("adr_conv2d_dgrad_bf16");
}

extern "C" int adr_conv2d_dgrad_bf16(const adr_conv_desc* d, const void* dy, const void* w_crsk, const float* bias,
                                     void* dx, int accumulate, void* stream) {
  return conv_dgrad_impl(d, dy, w_crsk, bias, dx, accumulate, nullptr, 0, stream);
}

// dx (+)= dgrad(dy) + addend in one launch: the fan-out gradient sink's first conv consumer folds in a pass-through
// gradient (a residual add's) that FanOutFn would otherwise add with its own elementwise launch
extern "C" int adr_conv2d_dgrad_bf16_add(const adr_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                                         int accumulate, const void* addend, int addend_cstride, void* stream) {
  ADR_REQUIRE(addend && addend_cstride >= d->c && addend_cstride % 8 == 0 && ((uintptr_t)addend & 15) == 0,
              "conv dgrad add: addend must be a 16-byte aligned NHWC view with channel stride >= C");
  return conv_dgrad_impl(d, dy, w_crsk, nullptr, dx, accumulate, addend, addend_cstride, stream);
}

// Training Conv-BN-act fusion (XF kernels): the data gradient of a conv whose output y went through a training
// BatchNorm + activation, taking dz (the gradient of the activation output) and applying the BN-act backward
// dy = A * dz * act'(y * scale + shift) + B * y + C while staging the operand; dy is side-written once to xf->out
// (for the weight gradient). Replaces adr_affine_act_bwd + adr_conv2d_dgrad_bf16.
extern "C" int adr_conv2d_dgrad_bf16_bnact(const adr_conv_desc* d, const void* dz, const void* w_crsk, void* dx,
                                           int accumulate, const void* addend, int addend_cstride,
                                           const adr_bnact_xf* xf, void* stream) {
  ADR_REQUIRE(xf, "conv dgrad bnact: xf");
  if (addend)
    ADR_REQUIRE(addend_cstride >= d->c && addend_cstride % 8 == 0 && ((uintptr_t)addend & 15) == 0,
                "conv dgrad bnact: addend view");
  return conv_dgrad_impl(d, dz, w_crsk, nullptr, dx, accumulate, addend, addend_cstride, stream, xf);
}

// Any of the data gradients above (plain / + addend / XF), whose stored dx is the final gradient dz of a training
// BatchNorm-act (the conv's input was that BN's output, with no other reader): the epilogue also reads the BN input y
// and writes per-tile (sum g, sum g * y) partials — adr_nc_reduce's backward statistics — to stats
// ([adr_conv2d_dgrad_bf16_stat_tiles][2][C]), so adr_bn_bwd_finalize runs on them without a pass over dz and y.
extern "C" int adr_conv2d_dgrad_bf16_bstat(const adr_conv_desc* d, const void* dy, const void* w_crsk, void* dx,
                                           int accumulate, const void* addend, int addend_cstride,
                                           const adr_bnact_xf* xf, const adr_bn_bstat* bs, float* stats,
                                           void* stream) {
  ADR_REQUIRE(bs, "conv dgrad bstat: bs");
  if (addend)
    ADR_REQUIRE(addend_cstride >= d->c && addend_cstride % 8 == 0 && ((uintptr_t)addend & 15) == 0,
                "conv dgrad bstat: addend view");
  return conv_dgrad_impl(d, dy, w_crsk, nullptr, dx, accumulate, addend, addend_cstride, stream, xf, bs, stats);
}

// The forward counterpart: the conv's input is a training BatchNorm's input y; z = act(y * scale + shift) is
// applied while staging (0 in the zero padding) and side-written once to xf->out. Replaces adr_affine_act +
// adr_conv2d_fwd_bf16 (stats as adr_conv2d_fwd_bf16).
extern "C" int adr_conv2d_fwd_bf16_bnact(const adr_conv_desc* d, const void* y, const void* w, void* out,
                                         float* stats, const adr_bnact_xf* xf, void* stream) {
  ADR_REQUIRE(xf, "conv fwd bnact: xf");
  return conv_fwd_impl(d, y, w, nullptr, out, stats, 0, nullptr, nullptr, 0, stream, xf);
}

// How many times the XF kernel would stage (and transform) each source element, x100: column tiles x gathers per
// element (taps / stride^2 for FWD implicit GEMM, all taps for DGRAD, the halo overlap for the 3x3 tiles). The XF
// transform is VALU work per staged element (a sigmoid per element for SiLU); it pays for the elementwise pass it
// replaces only when each element is staged about once (adr_conv2d_{fwd,dgrad}_bf16_bnact callers test this).
extern "C" int adr_conv2d_bf16_xf_reuse(const adr_conv_desc* d, int dgrad) {
  const ConvPlan pl = conv_plan(d, dgrad != 0, true);
  if (dgrad) {
    // an XF data gradient that would leave the streaming 1x1 kernel for the per-tile engine is latency-bound on the
    // large thin maps (e.g. 160^2 x 32 -> 48: 187 us fused against ~70 us for the BN-act pass + streaming dgrad)
    // and so is the stride-2 halo-tile one on the stem-side maps (320^2 x 16 <- 160^2 x 32: 291 us fused, the BN-act
    // pass + plain DG2H are faster; same-box step A/B 20.93 -> 20.83 ms), and since round 6 the 3x3 halo-tile one too
    // (l-scale 111.2 -> 110.6 ms same box, n-scale neutral). ADR_XF_STREAM / ADR_XF_DG2 / ADR_XF_CONV3 = 1 keep the
    // fusion there (A/B, tests).
    const char* es = getenv("ADR_XF_STREAM");
    const char* eg = getenv("ADR_XF_DG2");
    const char* e3 = getenv("ADR_XF_CONV3");
    if (!(es && atoi(es)) && conv_plan(d, true, false).kt > 0 && pl.kt == 0) return 1 << 20;
    if (!(eg && atoi(eg)) && pl.dg2) return 1 << 20;
    if (!(e3 && atoi(e3)) && pl.tw) return 1 << 20;
  }
  const int out = dgrad ? d->c : d->k;
  const int nt = pl.tw ? out / pl.bn : cdiv(out, pl.bn);
  if (pl.dg2) return nt * 100 * (G2_TI + 1) * (pl.dg2 + 1) / (G2_TI * pl.dg2);
  if (pl.tw) return nt * 100 * (128 / pl.tw + 2) * (pl.tw + 2) / 128;
  const int taps = d->r * d->s;
  if (!dgrad) return nt * 100 * taps / (d->stride_h * d->stride_w);
  return nt * 100 * taps;
}

static int fwd_stat_tiles(const adr_conv_desc* d, bool xf) {
  const ConvPlan pl = conv_plan(d, false, xf);
  if (pl.tw) return pl.wide ? conv3_tiles(d, 16, 256) : conv3_tiles(d, pl.tw);
  if (pl.kt) return conv1_groups((long)d->n * d->ho * d->wo, cdiv(d->k, pl.bn), pl.kt, pl.bn);
  return cdiv((long)d->n * d->ho * d->wo, CBM);
}

extern "C" int adr_conv2d_fwd_bf16_stat_tiles(const adr_conv_desc* d) { return fwd_stat_tiles(d, false); }

// statistics rows of adr_conv2d_dgrad_bf16_bstat (xf: with the XF operand transform)
extern "C" int adr_conv2d_dgrad_bf16_stat_tiles(const adr_conv_desc* d, int xf) {
  const ConvPlan pl = conv_plan(d, true, xf != 0);
  if (pl.dg2) return dg2_tiles(d);
  if (pl.mode == CV_DGRAD2) return 4 * cdiv((long)d->n * ((d->h + 1) / 2) * ((d->w + 1) / 2), CBM);
  if (pl.tw) return pl.wide ? conv3_tiles(d, 16, 256) : conv3_tiles(d, pl.tw);
  if (pl.kt) return conv1_groups((long)d->n * d->h * d->w, cdiv(d->c, pl.bn), pl.kt, pl.bn);
  return cdiv((long)d->n * d->h * d->w, CBM);
}

// statistics rows of adr_conv2d_fwd_bf16_bnact (its kernel choice can differ from the plain forward's)
extern "C" int adr_conv2d_fwd_bf16_bnact_stat_tiles(const adr_conv_desc* d) { return fwd_stat_tiles(d, true); }

extern "C" int adr_conv2d_bf16_kernel_symbol(const adr_conv_desc* d, int dgrad, char* buf, int len) {
  ADR_REQUIRE(d && buf && len >= 64, "conv kernel symbol: bad arguments");
  const bool dg = (dgrad & 1) != 0, xf = (dgrad & 2) != 0;  // bit 1: the BN-act (XF) variant
  const bool bst = dg && (dgrad & 4) != 0;                     // bit 2: the BSTAT data gradient
  const ConvPlan pl = conv_plan(d, dg, xf);
  if (pl.dg2) {
    snprintf(buf, len, "_ZN3adr10dg2_kernelILi%dELi%dELi%dELb%dEEEvNS_8ConvArgsE", pl.dg2, pl.bn, xf ? XF_BWD : XF_NONE,
             bst ? 1 : 0);
    return ADR_OK;
  }
  if (bst) {
    if (pl.tw && pl.wide && !xf)
      snprintf(buf, len, "_ZN3adr17conv3w_bst_kernelENS_8ConvArgsE");
    else if (pl.tw)
      snprintf(buf, len, "_ZN3adr16conv3_bst_kernelILi%dELi%dELi%dEEEvNS_8ConvArgsE", pl.tw, pl.bn, xf ? XF_BWD : XF_NONE);
    else if (pl.kt && !xf)
      snprintf(buf, len, "_ZN3adr16conv1_bst_kernelILi%dELi%dEEEvNS_8ConvArgsEi", pl.bn, pl.kt);
    else
      snprintf(buf, len, "_ZN3adr20conv_bf16_bst_kernelILi%dELi%dELi%dEEEvNS_8ConvArgsE", pl.bn, pl.mode,
               xf ? XF_BWD : XF_NONE);
    return ADR_OK;
  }
  if (xf && pl.tw)
    snprintf(buf, len, "_ZN3adr15conv3_xf_kernelILi%dELb%dELi%dELi%dEEEvNS_8ConvArgsE", pl.tw, dg ? 1 : 0, pl.bn,
             dg ? XF_BWD : XF_FWD);
  else if (xf)
    snprintf(buf, len, "_ZN3adr19conv_bf16_xf_kernelILi%dELi%dELi%dEEEvNS_8ConvArgsE", pl.bn, pl.mode,
             dg ? XF_BWD : XF_FWD);
  else if (pl.tw && pl.wide)
    snprintf(buf, len, "_ZN3adr13conv3w_kernelILb%dELb0EEEvNS_8ConvArgsE", dg ? 1 : 0);
  else if (pl.tw)
    snprintf(buf, len, "_ZN3adr12conv3_kernelILi%dELb%dELi%dEEEvNS_8ConvArgsE", pl.tw, dg ? 1 : 0, pl.bn);
  else if (pl.kt && xf)
    snprintf(buf, len, "_ZN3adr15conv1_xf_kernelILi%dELi%dEEEvNS_8ConvArgsEi", pl.bn, pl.kt);
  else if (pl.kt)
    snprintf(buf, len, "_ZN3adr12conv1_kernelILi%dELi%dELi%dEEEvNS_8ConvArgsEi", pl.bn, pl.mode, pl.kt);
  else
    snprintf(buf, len, "_ZN3adr16conv_bf16_kernelILi%dELi%dEEEvNS_8ConvArgsE", pl.bn, pl.mode);
  return ADR_OK;
}
