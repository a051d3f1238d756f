// The network stem — model.0 Conv(3, c2, 3, 2) (reference nn/modules/conv.py:36-54, first row of the yaml
// backbone) — read straight from the preprocessed fp32 NCHW image batch (detect/train.py:57-59), bf16 compute:
//   * forward: y (16 pixels x 16 channels) = im2col (16 x 27->32) x W^T per v_mfma_f32_16x16x32_bf16 from the
//     image rows staged in LDS (bf16), fp32 accumulation, bf16 NHWC output, plus the per-block BatchNorm
//     partial statistics of the stored values (the same contract as the conv epilogue).
//   * weight gradient: dw[k][j] = sum_pixels dy[p][k] * im2col(img)[p][j] (j = c*9 + ky*3 + kx) on MFMA
//     v_mfma_f32_16x16x32_bf16: A = dy^T (16 output channels x 32 pixels), B = im2col (32 pixels x 2 x 16
//     columns), accumulated per wave over a pixel range, block partials summed in a fixed order.
// Both replace image_to_nhwc + the generic implicit GEMM on a channel-padded copy of the image (420 MB of
// bf16 written and read twice per bs64 step) with one read of the image per pass. The _u8 entry points read the
// dataloader's uint8 batch and apply preprocess_batch's /255 (detect/train.py:57-59) while staging: the
// float image never exists (79 MB read per pass at bs 64 instead of 315 MB).
#include "adr_common.h"

namespace adr {

typedef __attribute__((ext_vector_type(8))) short s16x8;

constexpr int STEM_ROWS = 2;

// image element -> the reference's preprocessed value: fp32 as is; uint8 as .float() / 255 (detect/train.py:57-59,
// the dataloader's uint8 batch normalised on the device). torch evaluates a division by a scalar on the device as
// a multiplication by the fp32 reciprocal (BinaryDivTrueKernel), so this does too — bitwise the reference's input
__device__ __forceinline__ float img_val(float v) { return v; }
__device__ __forceinline__ float img_val(uint8_t v) { return (float)v * (1.f / 255.f); }
// word of 4 image pixels, pixel e of it, two values as a packed bf16 pair
template <typename TI> struct StemQWord { typedef unsigned T; };  // 4 uint8 pixels
template <> struct StemQWord<float> { typedef f32x4 T; };
__device__ __forceinline__ float stem_w(unsigned v, int e) { return img_val((uint8_t)(v >> (8 * e))); }
__device__ __forceinline__ float stem_w(f32x4 v, int e) { return v[e]; }
typedef __attribute__((ext_vector_type(2))) unsigned u32x2s;
typedef __attribute__((ext_vector_type(2))) float stem_f2;
typedef __attribute__((ext_vector_type(2))) __bf16 stem_bf2;
__device__ __forceinline__ unsigned pack_bf2(float a, float b) {  // one v_cvt_pk_bf16_f32
  const stem_bf2 r = __builtin_convertvector((stem_f2){a, b}, stem_bf2);
  return *reinterpret_cast<const unsigned*>(&r);
}

// stage image rows iy0 .. iy0+IR-1 of the 3 channels of image n into LDS as bf16 [3][IR][W+2] with zero
// columns at -1 and W (and zero rows outside the image); 16-byte (fp32) / 4-byte (uint8) loads when W % 4 == 0
template <int IR>
__device__ __forceinline__ void stage_rows(const uint8_t* __restrict__ img, int n, int H, int W, int iy0, __bf16* xs) {
  constexpr int NR = 3 * IR;
  const int Wp = W + 2;
  if ((W & 3) == 0) {
    for (int q = threadIdx.x; q < W / 4; q += blockDim.x) {
      unsigned v[NR];
#pragma unroll
      for (int row = 0; row < NR; ++row) {
        const int c = row / IR, iy = iy0 + row % IR;
        const bool rok = iy >= 0 && iy < H;
        v[row] = rok ? *reinterpret_cast<const unsigned*>(img + (((long)n * 3 + c) * H + iy) * W + 4 * q) : 0u;
      }
#pragma unroll
      for (int row = 0; row < NR; ++row)
#pragma unroll
        for (int e = 0; e < 4; ++e) xs[row * Wp + 1 + 4 * q + e] = (__bf16)img_val((uint8_t)(v[row] >> (8 * e)));
    }
  } else {
    for (int row = 0; row < NR; ++row) {
      const int c = row / IR, iy = iy0 + row % IR;
      const bool rok = iy >= 0 && iy < H;
      for (int q = threadIdx.x; q < W; q += blockDim.x)
        xs[row * Wp + 1 + q] = (__bf16)(rok ? img_val(img[(((long)n * 3 + c) * H + iy) * W + q]) : 0.f);
    }
  }
  if (threadIdx.x < NR) {
    xs[threadIdx.x * Wp] = (__bf16)0.f;
    xs[threadIdx.x * Wp + W + 1] = (__bf16)0.f;
  }
}

template <int IR>
__device__ __forceinline__ void stage_rows(const float* __restrict__ img, int n, int H, int W, int iy0, __bf16* xs) {
  constexpr int NR = 3 * IR;
  const int Wp = W + 2;
  if ((W & 3) == 0) {
    // every row's 16-byte load issued before any LDS store: NR loads in flight per thread
    for (int q = threadIdx.x; q < W / 4; q += blockDim.x) {
      f32x4 v[NR];
#pragma unroll
      for (int row = 0; row < NR; ++row) {
        const int c = row / IR, iy = iy0 + row % IR;
        const bool rok = iy >= 0 && iy < H;
        v[row] = rok ? *reinterpret_cast<const f32x4*>(img + (((long)n * 3 + c) * H + iy) * W + 4 * q)
                     : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int row = 0; row < NR; ++row)
#pragma unroll
        for (int e = 0; e < 4; ++e) xs[row * Wp + 1 + 4 * q + e] = (__bf16)v[row][e];
    }
  } else {
    for (int row = 0; row < NR; ++row) {
      const int c = row / IR, iy = iy0 + row % IR;
      const bool rok = iy >= 0 && iy < H;
      for (int q = threadIdx.x; q < W; q += blockDim.x)
        xs[row * Wp + 1 + q] = (__bf16)(rok ? img[(((long)n * 3 + c) * H + iy) * W + q] : 0.f);
    }
  }
  if (threadIdx.x < NR) {
    xs[threadIdx.x * Wp] = (__bf16)0.f;
    xs[threadIdx.x * Wp + W + 1] = (__bf16)0.f;
  }
}

// weight gradient partials: block per (image, pair of output rows); the 5 input rows it needs (3 channels,
// columns -1..W zero-padded) and its dy rows are staged in LDS as bf16, then 4 waves run the MFMA steps over
// the block's 2*Wo pixels (32 per step). part[block][KT*16][32].
// Wide images (the l-scale 1280^2 configuration) split each row pair into column segments of wseg output columns
// (segs per row pair) so the staged rows fit the LDS plan; segs == 1 is the whole row.
template <int IR, typename TI>
__device__ __forceinline__ void stage_cols(const TI* __restrict__ img, int n, int H, int W, int iy0, int ix0, int Wc,
                                           int Wp, __bf16* xs) {
  for (int q = threadIdx.x; q < 3 * IR * Wc; q += blockDim.x) {
    const int row = q / Wc, col = q - row * Wc;
    const int c = row / IR, iy = iy0 + row % IR, ix = ix0 + col;
    const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
    xs[row * Wp + col] = (__bf16)(ok ? img_val(img[(((long)n * 3 + c) * H + iy) * W + ix]) : 0.f);
  }
}

template <int KT, typename TI>
__global__ void __launch_bounds__(256) stem_wgrad_kernel(const TI* __restrict__ img, int H, int W,
                                                         const __bf16* __restrict__ dy, int dcs, int Ho, int Wo,
                                                         int segs, int wseg, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
  constexpr int IR = 2 * STEM_ROWS + 1;  // input rows
  const int Wp = segs == 1 ? W + 2 : 2 * wseg + 2;
  __bf16* xs = reinterpret_cast<__bf16*>(smraw);                 // [3][IR][Wp]
  __bf16* ds = xs + ((3 * IR * Wp + 7) & ~7);                    // [STEM_ROWS * wseg][KT * 16]
  float* red = reinterpret_cast<float*>(ds + (long)STEM_ROWS * wseg * KT * 16);  // [4][KT*16][32]
  const int nrb = (Ho + STEM_ROWS - 1) / STEM_ROWS;
  const int seg = blockIdx.x % segs, rb = (blockIdx.x / segs) % nrb, n = blockIdx.x / segs / nrb;
  const int oy0 = rb * STEM_ROWS, nrow = min(STEM_ROWS, Ho - oy0), iy0 = 2 * oy0 - 1;
  const int ox0 = seg * wseg, nox = min(wseg, Wo - ox0);
  if (segs == 1) stage_rows<IR>(img, n, H, W, iy0, xs);
  else stage_cols<IR>(img, n, H, W, iy0, 2 * ox0 - 1, 2 * nox + 1, Wp, xs);
  const int npx = nrow * nox;
  const __bf16* dyb = dy + (((long)n * Ho + oy0) * Wo + ox0) * (long)dcs;
  {  // 16-byte chunks of 8 channels, four loads in flight per thread
    const int nch = npx * KT * 2;
    for (int i0 = threadIdx.x; i0 < nch; i0 += 4 * 256) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        const int px = i / (KT * 2), pr = px / nox;  // segment pixel -> (row, column) of the dy image
        if (i < nch) v[u] = ld16(dyb + ((long)pr * Wo + (px - pr * nox)) * dcs + (i % (KT * 2)) * 8);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        if (i < nch) *reinterpret_cast<u32x4*>(ds + (long)(i / (KT * 2)) * KT * 16 + (i % (KT * 2)) * 8) = v[u];
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  int cj[2], kyj[2], kxj[2];
  bool jok[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int j = jt * 16 + i;
    jok[jt] = j < 27;
    const int jj = jok[jt] ? j : 0;
    cj[jt] = jj / 9;
    kyj[jt] = (jj % 9) / 3;
    kxj[jt] = jj % 3;
  }
  f32x4 acc[KT][2];
#pragma unroll
  for (int t = 0; t < KT; ++t) acc[t][0] = acc[t][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int nsteps = (npx + 31) / 32;
  for (int s = wave; s < nsteps; s += 4) {
    const int pbase = s * 32 + 8 * g;
    int r = pbase / nox, ox = pbase - r * nox;
    s16x8 a[KT], b[2];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool pok = pbase + e < npx;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const __bf16 v = pok ? ds[(long)(pbase + e) * KT * 16 + t * 16 + i] : (__bf16)0.f;
        a[t][e] = *reinterpret_cast<const short*>(&v);
      }
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        const __bf16 v = (pok && jok[jt]) ? xs[(cj[jt] * IR + 2 * r + kyj[jt]) * Wp + 2 * ox + kxj[jt]]
                                          : (__bf16)0.f;
        b[jt][e] = *reinterpret_cast<const short*>(&v);
      }
      if (++ox == nox) {
        ox = 0;
        ++r;
      }
    }
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
        acc[t][jt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&a[t]),
                                                             *reinterpret_cast<bf16x8*>(&b[jt]), acc[t][jt], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) red[(wave * KT * 16 + t * 16 + 4 * g + rr) * 32 + jt * 16 + i] = acc[t][jt][rr];
  __syncthreads();
  for (int idx = threadIdx.x; idx < KT * 16 * 32; idx += 256) {
    const int M = KT * 16 * 32;
    part[(long)blockIdx.x * M + idx] = (red[idx] + red[M + idx]) + (red[2 * M + idx] + red[3 * M + idx]);
  }
}

// weight gradient, persistent form (rows of the image fit one LDS plan: W <= STEM_LOOP_W, W % 4 == 0): a block walks
// a contiguous range of (image, output-row-pair) tiles, accumulating in registers, and the next tile's image words
// and dy chunks are loaded into registers while the current one runs its MFMA steps — the per-tile kernel above
// exposed a full load latency per tile at 3 blocks per CU and wrote one partial slab per tile (10 240 at bs 64,
// 640^2), which the reduce then gathered. Same MFMA steps per tile as above; partials [block][KT*16][32].
constexpr int STEM_LOOP_W = 640;
template <typename TI> struct StemWord { typedef unsigned T; };            // 4 uint8 pixels
template <> struct StemWord<float> { typedef f32x4 T; };                   // 4 fp32 pixels
__device__ __forceinline__ void stem_put4(__bf16* d, unsigned v) {
#pragma unroll
  for (int e = 0; e < 4; ++e) d[e] = (__bf16)img_val((uint8_t)(v >> (8 * e)));
}
__device__ __forceinline__ void stem_put4(__bf16* d, f32x4 v) {
#pragma unroll
  for (int e = 0; e < 4; ++e) d[e] = (__bf16)v[e];
}

template <int KT, typename TI>
__global__ void __launch_bounds__(256) stem_wgrad_loop_kernel(const TI* __restrict__ img, int H, int W,
                                                              const __bf16* __restrict__ dy, int dcs, int Ho, int Wo,
                                                              int ntiles, int per, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
  constexpr int IR = 2 * STEM_ROWS + 1, NR = 3 * IR;
  constexpr int DCH = STEM_ROWS * (STEM_LOOP_W / 2) * KT * 2 / 256;  // 16-byte dy chunks per thread
  typedef typename StemWord<TI>::T Word;
  const int Wp = W + 2;
  __bf16* xs = reinterpret_cast<__bf16*>(smraw);                 // [3][IR][Wp]
  __bf16* ds = xs + ((3 * IR * Wp + 7) & ~7);                    // [STEM_ROWS * Wo][KT * 16]
  float* red = reinterpret_cast<float*>(smraw);                  // [4][KT*16][32], after the last tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nrb = (Ho + STEM_ROWS - 1) / STEM_ROWS;
  const int t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  const int W4 = W / 4;
  if (tid < NR) {  // zero columns -1 and W (never written by the row stores)
    xs[tid * Wp] = (__bf16)0.f;
    xs[tid * Wp + W + 1] = (__bf16)0.f;
  }
  Word iv[NR];
  u32x4 dv[DCH];
  auto load = [&](int tile) {
    const int rb = tile % nrb, n = tile / nrb;
    const int oy0 = rb * STEM_ROWS, iy0 = 2 * oy0 - 1, npx = min(STEM_ROWS, Ho - oy0) * Wo;
#pragma unroll
    for (int row = 0; row < NR; ++row) {
      const int c = row / IR, iy = iy0 + row % IR;
      const bool ok = tid < W4 && iy >= 0 && iy < H;
      if constexpr (sizeof(Word) == 4) iv[row] = ok ? *reinterpret_cast<const unsigned*>(img + (((long)n * 3 + c) * H + iy) * W + 4 * tid) : 0u;
      else iv[row] = ok ? *reinterpret_cast<const f32x4*>(img + (((long)n * 3 + c) * H + iy) * W + 4 * tid) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    const __bf16* dyb = dy + ((long)n * Ho + oy0) * Wo * (long)dcs;
    const int nch = npx * KT * 2;
#pragma unroll
    for (int u = 0; u < DCH; ++u) {
      const int i = tid + 256 * u;
      if (i < nch) dv[u] = ld16(dyb + (long)(i / (KT * 2)) * dcs + (i % (KT * 2)) * 8);
    }
  };
  auto store = [&](int tile) {
    const int rb = tile % nrb;
    const int npx = min(STEM_ROWS, Ho - rb * STEM_ROWS) * Wo, nch = npx * KT * 2;
    if (tid < W4) {
#pragma unroll
      for (int row = 0; row < NR; ++row) stem_put4(xs + row * Wp + 1 + 4 * tid, iv[row]);
    }
#pragma unroll
    for (int u = 0; u < DCH; ++u) {
      const int i = tid + 256 * u;
      if (i < nch) *reinterpret_cast<u32x4*>(ds + (long)(i / (KT * 2)) * KT * 16 + (i % (KT * 2)) * 8) = dv[u];
    }
  };
  const int g = lane >> 4, i = lane & 15;
  int cj[2], kyj[2], kxj[2];
  bool jok[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int j = jt * 16 + i;
    jok[jt] = j < 27;
    const int jj = jok[jt] ? j : 0;
    cj[jt] = jj / 9;
    kyj[jt] = (jj % 9) / 3;
    kxj[jt] = jj % 3;
  }
  f32x4 acc[KT][2];
#pragma unroll
  for (int t = 0; t < KT; ++t) acc[t][0] = acc[t][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (t0 < t1) load(t0);
  for (int tile = t0; tile < t1; ++tile) {
    store(tile);
    __syncthreads();
    if (tile + 1 < t1) load(tile + 1);
    const int npx = min(STEM_ROWS, Ho - (tile % nrb) * STEM_ROWS) * Wo;
    const int nsteps = (npx + 31) / 32;
    for (int s = wave; s < nsteps; s += 4) {
      const int pbase = s * 32 + 8 * g;
      int r = pbase / Wo, ox = pbase - r * Wo;
      s16x8 a[KT], b[2];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool pok = pbase + e < npx;
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const __bf16 v = pok ? ds[(long)(pbase + e) * KT * 16 + t * 16 + i] : (__bf16)0.f;
          a[t][e] = *reinterpret_cast<const short*>(&v);
        }
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
          const __bf16 v = (pok && jok[jt]) ? xs[(cj[jt] * IR + 2 * r + kyj[jt]) * Wp + 2 * ox + kxj[jt]]
                                            : (__bf16)0.f;
          b[jt][e] = *reinterpret_cast<const short*>(&v);
        }
        if (++ox == Wo) {
          ox = 0;
          ++r;
        }
      }
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
          acc[t][jt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&a[t]),
                                                               *reinterpret_cast<bf16x8*>(&b[jt]), acc[t][jt], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) red[(wave * KT * 16 + t * 16 + 4 * g + rr) * 32 + jt * 16 + i] = acc[t][jt][rr];
  __syncthreads();
  for (int idx = tid; idx < KT * 16 * 32; idx += 256) {
    const int M = KT * 16 * 32;
    part[(long)blockIdx.x * M + idx] = (red[idx] + red[M + idx]) + (red[2 * M + idx] + red[3 * M + idx]);
  }
}

// weight gradient, persistent, on deinterleaved rows (W % 4 == 0, tiles of two output rows x stem_wq_seg columns
// dividing the row into multiples of 16). The kernel above feeds
// each 16x16x32 step with 24 two-byte LDS reads per lane (eight dy values of one channel, sixteen im2col taps of
// eight pixels); here both operands come from 8-byte reads:
//   * dy^T (A: output channel x 32 pixels) by ds_read_b64_tr_b16 from the natural [pixel][K] dy image: lane group g
//     takes pixels 4g .. 4g+3 and 16 + 4g .. 16 + 4g + 3 of the step (two transposed 4 x 16 blocks; the two groups of
//     a 32-lane half read 256 contiguous bytes, no bank conflict);
//   * im2col (B: 32 pixels x tap) from the staged input rows split by column parity — E[m] = x[2m], O[m] = x[2m+1],
//     O'[m] = x[2m-1] — where tap kx of output columns ox .. ox+3 is the aligned 8-byte run E / O / O' [ox .. ox+3]
//     (kx = 1 / 2 / 0), the same pixels as the dy block.
// The reduction slots of a step are permuted against the kernel above (the MFMA sums the same 32 products), so the
// partials agree to fp32 rounding. Next-tile prefetch into registers and partials [block][KT*16][32] as above.
constexpr int STEM_PP_PAD = 8;  // plane pitch wseg + 8: the 16 taps of a lane group spread over the banks
// output columns per tile: the whole row at K 16 (n-scale 640^2: 320), 160-column segments at K 32 / 64 (the dy
// slab of two rows x 160 columns x 64 channels is 40 KB)
__host__ __device__ constexpr int stem_wq_seg(int KT) { return KT == 1 ? 320 : 160; }
template <int KT, typename TI>
__global__ void __launch_bounds__(256) stem_wgrad_q_kernel(const TI* __restrict__ img, int H, int W,
                                                           const __bf16* __restrict__ dy, int dcs, int Ho, int Wo,
                                                           int ntiles, int per, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
  constexpr int IR = 2 * STEM_ROWS + 1, NR = 3 * IR, KC = KT * 16, WSEG = stem_wq_seg(KT);
  constexpr int DCH = STEM_ROWS * WSEG * KT * 2 / 256;  // 16-byte dy chunks per thread
  typedef typename StemWord<TI>::T Word;
  const int wseg = Wo < WSEG ? Wo : WSEG, segs = (Wo + wseg - 1) / wseg;  // the host checks Wo % wseg == 0
  const int PP = wseg + STEM_PP_PAD;
  __bf16* pl = reinterpret_cast<__bf16*>(smraw);                          // [NR][3: E, O, O'][PP]
  __bf16* ds = pl + ((NR * 3 * PP + 7) & ~7);                             // [STEM_ROWS * wseg][KC]
  float* red = reinterpret_cast<float*>(smraw);                           // [4][KC][32], after the last tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nrb = (Ho + STEM_ROWS - 1) / STEM_ROWS;
  const int t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
  const int W4 = wseg / 2;  // image words (4 pixels) per staged row of a segment
  Word iv[NR];
  float lpx = 0.f;  // thread row < NR: the pixel left of the segment, x = 2 ox0 - 1 (O'[0])
  u32x4 dv[DCH];
  // tile -> (image, row pair, column segment)
  auto geo = [&](int tile, int& n, int& oy0, int& ox0) {
    const int seg = tile % segs, rt = tile / segs;
    n = rt / nrb;
    oy0 = (rt - n * nrb) * STEM_ROWS;
    ox0 = seg * wseg;
  };
  auto load = [&](int tile) {
    int n, oy0, ox0;
    geo(tile, n, oy0, ox0);
    const int iy0 = 2 * oy0 - 1, nrow = min(STEM_ROWS, Ho - oy0);
    const TI* imn = img + (long)n * 3 * H * W + 2 * ox0;
#pragma unroll
    for (int row = 0; row < NR; ++row) {
      const int c = row / IR, iy = iy0 + row % IR;
      const bool ok = tid < W4 && iy >= 0 && iy < H;
      if constexpr (sizeof(Word) == 4) iv[row] = ok ? *reinterpret_cast<const unsigned*>(imn + ((long)c * H + iy) * W + 4 * tid) : 0u;
      else iv[row] = ok ? *reinterpret_cast<const f32x4*>(imn + ((long)c * H + iy) * W + 4 * tid) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    if (tid < NR) {
      const int c = tid / IR, iy = iy0 + tid % IR;
      lpx = (ox0 > 0 && iy >= 0 && iy < H) ? img_val(imn[((long)c * H + iy) * W - 1]) : 0.f;
    }
    const __bf16* dyb = dy + (((long)n * Ho + oy0) * Wo + ox0) * (long)dcs;
    const int nch = nrow * wseg * KT * 2;
#pragma unroll
    for (int u = 0; u < DCH; ++u) {
      const int i = tid + 256 * u, px = i / (KT * 2), pr = px / wseg;  // segment pixel -> (row, column)
      dv[u] = i < nch ? ld16(dyb + ((long)pr * Wo + (px - pr * wseg)) * dcs + (i % (KT * 2)) * 8)
                      : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&]() {
    if (tid < W4) {
#pragma unroll
      for (int row = 0; row < NR; ++row) {
        const float x0 = stem_w(iv[row], 0), x1 = stem_w(iv[row], 1), x2 = stem_w(iv[row], 2), x3 = stem_w(iv[row], 3);
        __bf16* b = pl + row * 3 * PP;
        *reinterpret_cast<unsigned*>(b + 2 * tid) = pack_bf2(x0, x2);           // E[2q], E[2q+1]
        *reinterpret_cast<unsigned*>(b + PP + 2 * tid) = pack_bf2(x1, x3);      // O[2q], O[2q+1]
        b[2 * PP + 2 * tid + 1] = (__bf16)x1;                                   // O'[2q+1]
        if (2 * tid + 2 < PP) b[2 * PP + 2 * tid + 2] = (__bf16)x3;             // O'[2q+2]
      }
    }
    if (tid < NR) pl[(tid * 3 + 2) * PP] = (__bf16)lpx;  // O'[0]
#pragma unroll
    for (int u = 0; u < DCH; ++u) {
      const int i = tid + 256 * u;
      if (i < STEM_ROWS * wseg * KT * 2) *reinterpret_cast<u32x4*>(ds + (long)(i / (KT * 2)) * KC + (i % (KT * 2)) * 8) = dv[u];
    }
  };
  const int g = lane >> 4, i = lane & 15, q4 = (lane & 15) >> 2, p4 = lane & 3;
  // this lane's taps (B columns jt*16 + i): staged plane (row c*IR + ky, parity array) and validity
  int jpl[2];
  bool jok[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int j = jt * 16 + i;
    jok[jt] = j < 27;
    const int jj = jok[jt] ? j : 0, c = jj / 9, ky = (jj % 9) / 3, kx = jj % 3;
    jpl[jt] = (c * IR + ky) * 3 + (kx == 1 ? 0 : kx == 2 ? 1 : 2);
  }
  f32x4 acc[KT][2];
#pragma unroll
  for (int t = 0; t < KT; ++t) acc[t][0] = acc[t][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  typedef __attribute__((ext_vector_type(4))) short s16x4;
  if (t0 < t1) load(t0);
  for (int tile = t0; tile < t1; ++tile) {
    store();
    __syncthreads();
    if (tile + 1 < t1) load(tile + 1);
    const int nsteps = STEM_ROWS * wseg / 32;  // a short last row pair reads zero dy rows
    for (int s = wave; s < nsteps; s += 4) {
      s16x4 a[KT][2];
      uint2 b[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = s * 32 + 16 * h + 4 * g;  // first pixel of this lane group's block
        // dy^T block: lane 4q + p4 addresses pixel p + q4, channels t*16 + 4 p4 .. +3
#pragma unroll
        for (int t = 0; t < KT; ++t)
          a[t][h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(ds + (long)(p + q4) * KC + t * 16 + 4 * p4));
        const int r = p / wseg, ox = p - r * wseg;
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
          b[jt][h] = jok[jt] ? *reinterpret_cast<const uint2*>(pl + (jpl[jt] + 6 * r) * PP + ox) : uint2{0u, 0u};
      }
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const s16x4 a0 = a[t][0], a1 = a[t][1];
        const s16x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
          const uint4 bv = {b[jt][0].x, b[jt][0].y, b[jt][1].x, b[jt][1].y};
          acc[t][jt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&av),
                                                               *reinterpret_cast<const bf16x8*>(&bv), acc[t][jt], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) red[(wave * KC + t * 16 + 4 * g + rr) * 32 + jt * 16 + i] = acc[t][jt][rr];
  __syncthreads();
  for (int idx = tid; idx < KC * 32; idx += 256) {
    const int M = KC * 32;
    part[(long)blockIdx.x * M + idx] = (red[idx] + red[M + idx]) + (red[2 * M + idx] + red[3 * M + idx]);
  }
}

static size_t stem_wgrad_smem(int Wp, int wseg, int KT) {
  const int IR = 2 * STEM_ROWS + 1;
  return (((size_t)3 * IR * Wp + 7) & ~(size_t)7) * 2 + (size_t)STEM_ROWS * wseg * KT * 16 * 2 +
         (size_t)4 * KT * 16 * 32 * 4;
}

// column plan of the weight gradient: (segments per row pair, output columns per segment) within 64 KB of LDS
static void stem_wgrad_plan(int W, int Wo, int KT, int* segs, int* wseg) {
  if (stem_wgrad_smem(W + 2, Wo, KT) <= 64 * 1024) {
    *segs = 1;
    *wseg = Wo;
    return;
  }
  int ws = (Wo + 15) / 16 * 16;
  while (ws > 16 && stem_wgrad_smem(2 * ws + 2, ws, KT) > 64 * 1024) ws -= 16;
  *wseg = ws;
  *segs = (Wo + ws - 1) / ws;
}

// forward on MFMA: block per (image, pair of output rows), image rows staged in LDS exactly as for the weight
// gradient; y[16 pixels][16 k] = im2col (16 x 32) * W^T (32 x 16) per v_mfma_f32_16x16x32_bf16. The W^T
// fragment is the same for every step (preloaded); stats = per-block sums of the stored bf16 values.
template <int KT, typename TI>
__global__ void __launch_bounds__(256) stem_fwd_kernel(const TI* __restrict__ img, int H, int W,
                                                       const float* __restrict__ w, __bf16* __restrict__ y, int ycs,
                                                       int Ho, int Wo, float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
  constexpr int IR = 2 * STEM_ROWS + 1;
  const int Wp = W + 2;
  __bf16* xs = reinterpret_cast<__bf16*>(smraw);  // [3][IR][Wp]
  __shared__ float red[4][2][KT * 16];
  const int nrb = (Ho + STEM_ROWS - 1) / STEM_ROWS;
  const int rb = blockIdx.x % nrb, n = blockIdx.x / nrb;
  const int oy0 = rb * STEM_ROWS, nrow = min(STEM_ROWS, Ho - oy0), iy0 = 2 * oy0 - 1;
  stage_rows<IR>(img, n, H, W, iy0, xs);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  // B = W^T: lane supplies B[j = 8g + e][k = t*16 + i] = w[k][j]
  s16x8 bw[KT];
  int jc[8], jky[8], jkx[8];
  bool jok[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int j = 8 * g + e;
    jok[e] = j < 27;
    const int jj = jok[e] ? j : 0;
    jc[e] = jj / 9;
    jky[e] = (jj % 9) / 3;
    jkx[e] = jj % 3;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const __bf16 v = (__bf16)(jok[e] ? w[(t * 16 + i) * 27 + j] : 0.f);
      bw[t][e] = *reinterpret_cast<const short*>(&v);
    }
  }
  __syncthreads();
  // D^T[k][pixel] = W (16 k x 32 j) * im2col^T (32 j x 16 pixels): the same two register operands as
  // im2col * W^T with the roles swapped, so lane (g, i) holds output channels t*16 + 4g .. +3 of pixel i — one
  // 8-byte store per lane, 512 contiguous bytes per wave when ycs == 16 (the D[pixel][k] orientation stored
  // 2-byte values, four partial 32-byte pieces per cache line per instruction)
  float s1[KT][4], s2[KT][4];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s1[t][rr] = s2[t][rr] = 0.f;
  const int npx = nrow * Wo;
  __bf16* yb = y + ((long)n * Ho + oy0) * Wo * (long)ycs;
  for (int st = wave; st * 16 < npx; st += 4) {
    // B = im2col^T: lane supplies B[j = 8g + e][pixel i]
    const int p = st * 16 + i;
    const bool pok = p < npx;
    const int r = pok ? p / Wo : 0, ox = pok ? p - r * Wo : 0;
    s16x8 a;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const __bf16 v = (pok && jok[e]) ? xs[(jc[e] * IR + 2 * r + jky[e]) * Wp + 2 * ox + jkx[e]] : (__bf16)0.f;
      a[e] = *reinterpret_cast<const short*>(&v);
    }
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      f32x4 d = {0.f, 0.f, 0.f, 0.f};
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&bw[t]), *reinterpret_cast<bf16x8*>(&a),
                                                  d, 0, 0, 0);
      // D[k = t*16 + 4g + rr][pixel i]
      if (pok) {
        __bf16 v[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          v[rr] = (__bf16)d[rr];
          const float f = (float)v[rr];
          s1[t][rr] += f;
          s2[t][rr] += f * f;
        }
        *reinterpret_cast<uint2*>(yb + (long)p * ycs + t * 16 + 4 * g) = *reinterpret_cast<const uint2*>(v);
      }
    }
  }
  if (!stats) return;
#pragma unroll
  for (int t = 0; t < KT; ++t)  // combine the 16 pixel lanes of each channel group, then the waves
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[t][rr] += __shfl_xor(s1[t][rr], o, 64);
        s2[t][rr] += __shfl_xor(s2[t][rr], o, 64);
      }
      if (i == 0) {
        red[wave][0][t * 16 + 4 * g + rr] = s1[t][rr];
        red[wave][1][t * 16 + 4 * g + rr] = s2[t][rr];
      }
    }
  __syncthreads();
  if (threadIdx.x < 2 * KT * 16) {
    const int q = threadIdx.x / (KT * 16), k = threadIdx.x % (KT * 16);
    stats[(long)blockIdx.x * 2 * KT * 16 + threadIdx.x] = (red[0][q][k] + red[1][q][k]) + (red[2][q][k] + red[3][q][k]);
  }
}

// Forward on quad images (W % 4 == 0). The kernel above gathers the im2col operand from the staged bf16 rows with
// eight 2-byte LDS reads per lane per 16 pixels and stages the rows with 2-byte writes: on the bs 64, 640^2 stem a
// third of its wave cycles were LDS issue stalls (SQ_WAIT_INST_LDS, scripts/stem_micro.py). Here each staged input
// row (c, iy) is stored as quads Q[row][ox] = (x = 2ox-1, 2ox, 2ox+1, 0): the three taps of output column ox in one
// aligned 8-byte word, so the 27 (-> 32) reduction slots of a pixel are 9 quads (c, ky). A 16x16x32 step takes
// quads (g, g+4) in lane group g (two 8-byte reads) and a second step quad 8 (lane group 0), so a lane reads 2-3
// LDS words per 16 pixels; the staging writes 16 bytes per (row, output column pair). Rows of the quad image are
// QP = 16 (mod 32) quads apart, so the two lane groups of each 32-lane half (rows an odd number apart) hit disjoint
// banks. Wide images are walked in column segments of STEM_QSEG output columns. Output contract as above; the
// statistics rows (adr_stem_fwd_tiles) hold per-block sums (see the end of the kernel), whose total is the same.
constexpr int STEM_QSEG = 320;  // <= 512: one column pair per thread in the staging
__host__ __device__ constexpr int stem_qp(int nox) { return (nox + 15) / 32 * 32 + 16; }

// persistent: a block walks a contiguous range of units (tile = (image, output-row pair), column segment) — the
// W^T fragments are built once per block, the next unit's image words are in flight (registers) while the current
// one runs its MFMA steps, and consecutive tiles share their boundary input row in L2. The kernel is bound by
// instruction issue (SQ_ACTIVE_INST_ANY ~ the wave lifetime: bs 64, 640^2, 91.6 M wave instructions for the row
// kernel above, 61 M here at per-tile statistics), hence buffer loads / stores with out-of-range zeros instead of
// branches, scalar step geometry, packed conversions, and one statistics reduction per block.
template <int KT, typename TI>
__global__ void __launch_bounds__(256) stem_fwd_q_kernel(const TI* __restrict__ img, int H, int W,
                                                         const float* __restrict__ w, __bf16* __restrict__ y, int ycs,
                                                         int Ho, int Wo, float* __restrict__ stats, int nunits, int per,
                                                         int probe, int N) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smraw[];
  constexpr int IR = 2 * STEM_ROWS + 1, NR = 3 * IR;
  typedef typename StemQWord<TI>::T Word;
  const int segs = (Wo + STEM_QSEG - 1) / STEM_QSEG;
  const int QP = stem_qp(Wo < STEM_QSEG ? Wo : STEM_QSEG);
  uint2* Q = reinterpret_cast<uint2*>(smraw);  // [NR][QP]
  __shared__ float red[4][2][KT * 16];
  const int nrb = (Ho + STEM_ROWS - 1) / STEM_ROWS;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i = lane & 15;
  const int u0 = blockIdx.x * per, u1 = min(nunits, u0 + per);
  // A = W (16 k x 32 slots): lane (g, i) supplies output channel t*16 + i at slots 8g + e: quad g (e < 4) or g + 4
  // (e >= 4), tap kx = e & 3 (kx 3 is the zero pad); the second step holds quad 8 in lane group 0
  s16x8 bw[2][KT];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = h == 0 ? (e < 4 ? g : g + 4) : (g == 0 && e < 4 ? 8 : -1), kx = e & 3;
      const bool ok = q >= 0 && kx < 3;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const __bf16 v = (__bf16)(ok ? w[(t * 16 + i) * 27 + (q / 3) * 9 + (q % 3) * 3 + kx] : 0.f);
        bw[h][t][e] = *reinterpret_cast<const short*>(&v);
      }
    }
  // quad q = (c, ky) -> staged row c * IR + ky (+ 2 r for output row r of the pair)
  auto qrow = [](int q) { return (q / 3) * IR + q % 3; };
  const int rA = qrow(g) * QP, rB = qrow(g + 4) * QP, rC = qrow(8) * QP;
  const __amdgpu_buffer_rsrc_t yrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, N * Ho * Wo * ycs * 2, 0x00020000);
  Word v[NR];
  float lv[NR];  // the pixel at x - 1 of each row
  // unit -> (image, first output row, column segment)
  auto unit_geo = [&](int u, int& n, int& oy0, int& ox0) {
    const int tile = u / segs;
    ox0 = (u - tile * segs) * STEM_QSEG;
    n = tile / nrb;
    oy0 = (tile - n * nrb) * STEM_ROWS;
  };
  auto load = [&](int u) {
    int n, oy0, ox0;
    unit_geo(u, n, oy0, ox0);
    const int x = 2 * (ox0 + 2 * tid), iy0 = 2 * oy0 - 1;
    const bool tok = 2 * tid < min(STEM_QSEG, Wo - ox0) && !(probe & 2);
    // buffer loads over image n: rows above / below the image, columns past the segment and x - 1 = -1 read
    // out of range, which the hardware returns as zeros (no branch, no select)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(img + (long)n * 3 * H * W), (short)0, 3 * H * W * (int)sizeof(TI),
                                          0x00020000);
    constexpr unsigned OOR = 0x7FFFFFF0u;
#pragma unroll
    for (int row = 0; row < NR; ++row) {
      const int iy = iy0 + row % IR;
      const bool rok = tok && (unsigned)iy < (unsigned)H;
      const unsigned off = ((row / IR) * H + iy) * W + x;
      const unsigned ob = rok ? off * (unsigned)sizeof(TI) : OOR;
      const unsigned lb = rok && x > 0 ? (off - 1) * (unsigned)sizeof(TI) : OOR;
      if constexpr (sizeof(Word) == 4) {
        v[row] = __builtin_amdgcn_raw_buffer_load_b32(rs, ob, 0, 0);
        lv[row] = img_val((uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rs, lb, 0, 0));
      } else {
        const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, ob, 0, 0);
        v[row] = *reinterpret_cast<const f32x4*>(&b);
        lv[row] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lb, 0, 0));
      }
    }
  };
  auto store = [&](int u) {
    int n, oy0, ox0;
    unit_geo(u, n, oy0, ox0);
    if (2 * tid < min(STEM_QSEG, Wo - ox0)) {
#pragma unroll
      for (int row = 0; row < NR; ++row) {
        const float x1 = stem_w(v[row], 1);
        uint4 q;
        q.x = pack_bf2(lv[row], stem_w(v[row], 0));
        q.y = pack_bf2(x1, 0.f);
        q.z = pack_bf2(x1, stem_w(v[row], 2));
        q.w = pack_bf2(stem_w(v[row], 3), 0.f);
        *reinterpret_cast<uint4*>(Q + row * QP + 2 * tid) = q;
      }
    }
  };
  float s1[KT][4], s2[KT][4];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s1[t][rr] = s2[t][rr] = 0.f;
  if (u0 < u1) load(u0);
  for (int u = u0; u < u1; ++u) {
    int n, oy0, ox0;
    unit_geo(u, n, oy0, ox0);
    store(u);
    __syncthreads();
    if (u + 1 < u1) load(u + 1);
    const int nrow = min(STEM_ROWS, Ho - oy0), nox = min(STEM_QSEG, Wo - ox0), npx = nrow * nox;
    const int ybase = (((n * Ho + oy0) * Wo + ox0) * ycs + 4 * g) * 2;  // bytes, < 2^31 (checked by the launcher)
    // fast path (every row a multiple of 64 columns, all pixels valid): blocks of 64 pixels of one row per wave,
    // four 16-pixel steps whose LDS and store addresses differ by immediates, no validity masks
    const int nb64 = (nox & 63) || (probe & 1) ? 0 : npx / 64;
    for (int blk = wave; blk < nb64; blk += 4) {
      const int pb = blk * 64, r = pb / nox, oxb = pb - r * nox;  // scalar
      const uint2* qb = Q + 2 * r * QP + oxb + i;
      const unsigned yo = ybase + ((r * Wo + oxb + i) * ycs) * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint2 a0 = qb[rA + 16 * j], a1 = qb[rB + 16 * j];
        uint2 a2 = {0u, 0u};
        if (g == 0) a2 = qb[rC + 16 * j];
        const uint4 b01 = {a0.x, a0.y, a1.x, a1.y}, b2 = {a2.x, a2.y, 0u, 0u};
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          f32x4 d = {0.f, 0.f, 0.f, 0.f};
          d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&bw[0][t]),
                                                      *reinterpret_cast<const bf16x8*>(&b01), d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&bw[1][t]),
                                                      *reinterpret_cast<const bf16x8*>(&b2), d, 0, 0, 0);
          const unsigned lo = pack_bf2(d[0], d[1]), hi = pack_bf2(d[2], d[3]);
          const float f0 = __uint_as_float(lo << 16), f1 = __uint_as_float(lo & 0xFFFF0000u);
          const float f2 = __uint_as_float(hi << 16), f3 = __uint_as_float(hi & 0xFFFF0000u);
          s1[t][0] += f0; s1[t][1] += f1; s1[t][2] += f2; s1[t][3] += f3;
          s2[t][0] += f0 * f0; s2[t][1] += f1 * f1; s2[t][2] += f2 * f2; s2[t][3] += f3 * f3;
          __builtin_amdgcn_raw_buffer_store_b64((u32x2s){lo, hi}, yrs, yo, 16 * j * ycs * 2 + t * 32, 0);
        }
      }
    }
    for (int st = nb64 ? npx / 16 : wave; st * 16 < npx; st += 4) {
      // the step's first pixel, row and column in scalar registers; a step crosses into the next row only when
      // nox is not a multiple of 16
      const int pb = st * 16, rs = pb / nox, os = pb - rs * nox;
      int r = rs, ox = os + i;
      if (nox & 15) {
        if (ox >= nox) {
          ox -= nox;
          ++r;
        }
      }
      const bool pok = pb + i < npx;
      if (!pok) r = ox = 0;
      const uint2* qb = Q + 2 * r * QP + ox;
      const uint2 a0 = qb[rA], a1 = qb[rB];
      uint2 a2 = {0u, 0u};
      if (g == 0) a2 = qb[rC];
      const uint4 b01 = {a0.x, a0.y, a1.x, a1.y}, b2 = {a2.x, a2.y, 0u, 0u};
      const unsigned yo = pok && !(probe & 1) ? ybase + (r * Wo + ox) * ycs * 2 : 0x7FFFFFF0u;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&bw[0][t]),
                                                    *reinterpret_cast<const bf16x8*>(&b01), d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&bw[1][t]),
                                                    *reinterpret_cast<const bf16x8*>(&b2), d, 0, 0, 0);
        const unsigned lo = pack_bf2(d[0], d[1]), hi = pack_bf2(d[2], d[3]);
        const float m = pok ? 1.f : 0.f;  // statistics of the stored pixels only
        const float f0 = __uint_as_float(lo << 16) * m, f1 = __uint_as_float(lo & 0xFFFF0000u) * m;
        const float f2 = __uint_as_float(hi << 16) * m, f3 = __uint_as_float(hi & 0xFFFF0000u) * m;
        s1[t][0] += f0; s1[t][1] += f1; s1[t][2] += f2; s1[t][3] += f3;
        s2[t][0] += f0 * f0; s2[t][1] += f1 * f1; s2[t][2] += f2 * f2; s2[t][3] += f3 * f3;
        __builtin_amdgcn_raw_buffer_store_b64((u32x2s){lo, hi}, yrs, yo + t * 32, 0, 0);
      }
    }
    __syncthreads();  // the quads are read before the next unit's store
  }
  // statistics: the block's sums (over all its tiles) in the row of its first tile, zeros in its other tiles' rows
  // (the BatchNorm finalize sums every row of adr_stem_fwd_tiles)
  if (!stats || u0 >= u1) return;
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[t][rr] += __shfl_xor(s1[t][rr], o, 64);
        s2[t][rr] += __shfl_xor(s2[t][rr], o, 64);
      }
      if (i == 0) {
        red[wave][0][t * 16 + 4 * g + rr] = s1[t][rr];
        red[wave][1][t * 16 + 4 * g + rr] = s2[t][rr];
      }
    }
  __syncthreads();
  const int tile0 = u0 / segs, tile1 = (u1 + segs - 1) / segs;
  for (int idx = tid; idx < (tile1 - tile0) * 2 * KT * 16; idx += 256) {
    float v = 0.f;
    if (idx < 2 * KT * 16) {
      const int q = idx / (KT * 16), k = idx % (KT * 16);
      v = (red[0][q][k] + red[1][q][k]) + (red[2][q][k] + red[3][q][k]);
    }
    stats[(long)tile0 * 2 * KT * 16 + idx] = v;
  }
}

// dw[k][j] (+)= sum_blocks part[b][k][j], j < 27 (the (K, 3, 3, 3) parameter layout)
__global__ void __launch_bounds__(256) stem_wgrad_reduce_kernel(const float* __restrict__ part, int nblk, int K,
                                                                float* dw, int accumulate) {
  __shared__ float sh[256];
  const int k = blockIdx.x / 27, j = blockIdx.x % 27;
  float s = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 256) s += part[((long)b * K + k) * 32 + j];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) dw[k * 27 + j] = accumulate ? dw[k * 27 + j] + sh[0] : sh[0];
}


}  // namespace adr

using namespace adr;

// forward tiles = blocks (image, pair of output rows); npix = N * Ho * Wo with Ho, Wo of the stem
extern "C" int adr_stem_fwd_tiles(int N, int Ho) { return N * ((Ho + STEM_ROWS - 1) / STEM_ROWS); }

template <typename TI>
static int stem_fwd(const TI* img, int N, int H, int W, const float* w, int K, void* y, int ycs, float* stats,
                    void* stream) {
  ADR_REQUIRE(N > 0 && H > 1 && W > 1 && (K == 16 || K == 32 || K == 64) && ycs >= K && ycs % 4 == 0 &&
                  ((uintptr_t)y & 7) == 0,
              "stem_conv_fwd: N=%d H=%d W=%d K=%d ycs=%d (8-byte aligned rows)", N, H, W, K, ycs);
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  ADR_REQUIRE((long)N * Ho * Wo < (1l << 31), "stem_conv_fwd: too many pixels");
  const size_t sm = (((size_t)3 * (2 * STEM_ROWS + 1) * (W + 2) + 7) & ~(size_t)7) * 2;
  ADR_REQUIRE(sm <= 64 * 1024, "stem_conv_fwd: W=%d too wide for the LDS plan", W);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(adr_stem_fwd_tiles(N, Ho));
  const char* qe = getenv("ADR_STEM_FWD_Q");  // A/B, read per call: 0 = the row-gather kernel
  const char* pe = getenv("ADR_STEM_PROBE");  // diagnostics: 1 = no y stores, 2 = no image loads
  const int probe = pe ? atoi(pe) : 0;
  if (W % 4 == 0 && (!qe || atoi(qe))) {
    const size_t qsm = (size_t)3 * (2 * STEM_ROWS + 1) * stem_qp(Wo < STEM_QSEG ? Wo : STEM_QSEG) * 8;
    ADR_REQUIRE(qsm <= 64 * 1024 && 3l * H * W * (long)sizeof(TI) < (1l << 31) && 2l * N * Ho * Wo * ycs < (1l << 31),
                "stem_conv_fwd: quad image %zu bytes / 32-bit buffer offsets", qsm);
    const int nunits = (int)grid.x * ((Wo + STEM_QSEG - 1) / STEM_QSEG);
    auto kern = K == 16 ? (const void*)stem_fwd_q_kernel<1, TI>
                        : K == 32 ? (const void*)stem_fwd_q_kernel<2, TI> : (const void*)stem_fwd_q_kernel<4, TI>;
    int occ = 1, dev = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 256, qsm) != hipSuccess || occ < 1) occ = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    // one resident round of blocks; whole tiles per block (a tile's statistics row sums all its column segments)
    const int segs = (Wo + STEM_QSEG - 1) / STEM_QSEG;
    const int per = ((int)grid.x + cus * occ - 1) / (cus * occ) * segs;
    const dim3 qgrid((nunits + per - 1) / per);
    if (K == 16)
      hipLaunchKernelGGL((stem_fwd_q_kernel<1, TI>), qgrid, dim3(256), qsm, st, img, H, W, w, (__bf16*)y, ycs, Ho, Wo, stats, nunits, per, probe, N);
    else if (K == 32)
      hipLaunchKernelGGL((stem_fwd_q_kernel<2, TI>), qgrid, dim3(256), qsm, st, img, H, W, w, (__bf16*)y, ycs, Ho, Wo, stats, nunits, per, probe, N);
    else
      hipLaunchKernelGGL((stem_fwd_q_kernel<4, TI>), qgrid, dim3(256), qsm, st, img, H, W, w, (__bf16*)y, ycs, Ho, Wo, stats, nunits, per, probe, N);
    return check_launch("adr_stem_conv_fwd");
  }
  if (K == 16)
    hipLaunchKernelGGL((stem_fwd_kernel<1, TI>), grid, dim3(256), sm, st, img, H, W, w, (__bf16*)y, ycs, Ho, Wo, stats);
  else if (K == 32)
    hipLaunchKernelGGL((stem_fwd_kernel<2, TI>), grid, dim3(256), sm, st, img, H, W, w, (__bf16*)y, ycs, Ho, Wo, stats);
  else
    hipLaunchKernelGGL((stem_fwd_kernel<4, TI>), grid, dim3(256), sm, st, img, H, W, w, (__bf16*)y, ycs, Ho, Wo, stats);
  return check_launch("adr_stem_conv_fwd");
}

extern "C" int adr_stem_conv_fwd(const float* img, int N, int H, int W, const float* w, int K, void* y, int ycs,
                                 float* stats, void* stream) {
  return stem_fwd(img, N, H, W, w, K, y, ycs, stats, stream);
}

extern "C" int adr_stem_conv_fwd_u8(const uint8_t* img, int N, int H, int W, const float* w, int K, void* y, int ycs,
                                    float* stats, void* stream) {
  return stem_fwd(img, N, H, W, w, K, y, ycs, stats, stream);
}

extern "C" size_t adr_stem_wgrad_workspace(int N, int H, int W, int K) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  int segs, wseg;
  stem_wgrad_plan(W, Wo, K / 16 > 0 ? K / 16 : 1, &segs, &wseg);
  const long blocks = (long)N * ((Ho + STEM_ROWS - 1) / STEM_ROWS) * segs;
  return (size_t)blocks * K * 32 * sizeof(float);
}

template <typename TI>
static int stem_wgrad(const TI* img, int N, int H, int W, const void* dy, int dcs, int K, float* dw, int accumulate,
                      float* ws, size_t ws_bytes, void* stream) {
  ADR_REQUIRE(N > 0 && H > 1 && W > 1 && (K == 16 || K == 32 || K == 64) && dcs >= K,
              "stem_conv_wgrad: N=%d H=%d W=%d K=%d", N, H, W, K);
  ADR_REQUIRE(ws_bytes >= adr_stem_wgrad_workspace(N, H, W, K), "stem_conv_wgrad: workspace");
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int KT = K / 16;
  int segs, wseg;
  stem_wgrad_plan(W, Wo, KT, &segs, &wseg);
  const int blocks = N * ((Ho + STEM_ROWS - 1) / STEM_ROWS) * segs;
  const size_t sm = stem_wgrad_smem(segs == 1 ? W + 2 : 2 * wseg + 2, wseg, KT);
  ADR_REQUIRE(sm <= 64 * 1024 && dcs % 8 == 0, "stem_conv_wgrad: W=%d too wide for the LDS plan", W);
  hipStream_t st = (hipStream_t)stream;
  int nblk = blocks;
  const char* qe = getenv("ADR_STEM_WG_Q");  // A/B, read per call: 0 = the row-gather kernels
  const int qseg = Wo < stem_wq_seg(KT) ? Wo : stem_wq_seg(KT);
  const size_t qsm_rows = (((size_t)3 * 3 * (2 * STEM_ROWS + 1) * (qseg + STEM_PP_PAD) + 7) & ~(size_t)7) * 2 +
                          (size_t)STEM_ROWS * qseg * KT * 16 * 2;
  const size_t qsm_red = (size_t)4 * KT * 16 * 32 * 4;
  const size_t qsm = qsm_rows > qsm_red ? qsm_rows : qsm_red;
  // whole 32-pixel steps per tile, 4-pixel runs within a row, 16-byte image words per thread pair
  if (W % 4 == 0 && Wo % qseg == 0 && qseg % 16 == 0 && qsm <= 64 * 1024 && (!qe || atoi(qe))) {
    const int qtiles = N * ((Ho + STEM_ROWS - 1) / STEM_ROWS) * (Wo / qseg);
    auto kern = K == 16 ? (const void*)stem_wgrad_q_kernel<1, TI>
                        : K == 32 ? (const void*)stem_wgrad_q_kernel<2, TI> : (const void*)stem_wgrad_q_kernel<4, TI>;
    int occ = 1, dev = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 256, qsm) != hipSuccess || occ < 1) occ = 1;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int want = cus * (occ < 4 ? occ : 4);
    const int per = (qtiles + want - 1) / want;
    nblk = (qtiles + per - 1) / per;
    ADR_REQUIRE((size_t)nblk * K * 32 * sizeof(float) <= ws_bytes, "stem_conv_wgrad: workspace");
    if (K == 16)
      hipLaunchKernelGGL((stem_wgrad_q_kernel<1, TI>), dim3(nblk), dim3(256), qsm, st, img, H, W, (const __bf16*)dy,
                         dcs, Ho, Wo, qtiles, per, ws);
    else if (K == 32)
      hipLaunchKernelGGL((stem_wgrad_q_kernel<2, TI>), dim3(nblk), dim3(256), qsm, st, img, H, W, (const __bf16*)dy,
                         dcs, Ho, Wo, qtiles, per, ws);
    else
      hipLaunchKernelGGL((stem_wgrad_q_kernel<4, TI>), dim3(nblk), dim3(256), qsm, st, img, H, W, (const __bf16*)dy,
                         dcs, Ho, Wo, qtiles, per, ws);
  } else if (segs == 1 && W % 4 == 0 && W <= STEM_LOOP_W) {  // persistent form: ~4 blocks per CU, contiguous tile ranges
    const size_t lsm = (((size_t)3 * (2 * STEM_ROWS + 1) * (W + 2) + 7) & ~(size_t)7) * 2 +
                       (size_t)STEM_ROWS * Wo * KT * 16 * 2;
    const size_t lsm_red = (size_t)4 * KT * 16 * 32 * 4;
    const size_t lsmem = lsm > lsm_red ? lsm : lsm_red;
    auto kern = K == 16 ? (const void*)stem_wgrad_loop_kernel<1, TI>
                        : K == 32 ? (const void*)stem_wgrad_loop_kernel<2, TI> : (const void*)stem_wgrad_loop_kernel<4, TI>;
    int occ = 1, dev = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 256, lsmem) != hipSuccess || occ < 1) occ = 1;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int want = cus * (occ < 4 ? occ : 4);  // one resident round of blocks
    const int per = (blocks + want - 1) / want;
    nblk = (blocks + per - 1) / per;
    if (K == 16)
      hipLaunchKernelGGL((stem_wgrad_loop_kernel<1, TI>), dim3(nblk), dim3(256), lsmem, st, img, H, W, (const __bf16*)dy,
                         dcs, Ho, Wo, blocks, per, ws);
    else if (K == 32)
      hipLaunchKernelGGL((stem_wgrad_loop_kernel<2, TI>), dim3(nblk), dim3(256), lsmem, st, img, H, W, (const __bf16*)dy,
                         dcs, Ho, Wo, blocks, per, ws);
    else
      hipLaunchKernelGGL((stem_wgrad_loop_kernel<4, TI>), dim3(nblk), dim3(256), lsmem, st, img, H, W, (const __bf16*)dy,
                         dcs, Ho, Wo, blocks, per, ws);
  } else if (K == 16)
    hipLaunchKernelGGL((stem_wgrad_kernel<1, TI>), dim3(blocks), dim3(256), sm, st, img, H, W, (const __bf16*)dy, dcs,
                       Ho, Wo, segs, wseg, ws);
  else if (K == 32)
    hipLaunchKernelGGL((stem_wgrad_kernel<2, TI>), dim3(blocks), dim3(256), sm, st, img, H, W, (const __bf16*)dy, dcs,
                       Ho, Wo, segs, wseg, ws);
  else
    hipLaunchKernelGGL((stem_wgrad_kernel<4, TI>), dim3(blocks), dim3(256), sm, st, img, H, W, (const __bf16*)dy, dcs,
                       Ho, Wo, segs, wseg, ws);
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(K * 27), dim3(256), 0, st, ws, nblk, K, dw, accumulate);
  return check_launch("adr_stem_conv_wgrad");
}

extern "C" int adr_stem_conv_wgrad(const float* img, int N, int H, int W, const void* dy, int dcs, int K, float* dw,
                                   int accumulate, float* ws, size_t ws_bytes, void* stream) {
  return stem_wgrad(img, N, H, W, dy, dcs, K, dw, accumulate, ws, ws_bytes, stream);
}

extern "C" int adr_stem_conv_wgrad_u8(const uint8_t* img, int N, int H, int W, const void* dy, int dcs, int K,
                                      float* dw, int accumulate, float* ws, size_t ws_bytes, void* stream) {
  return stem_wgrad(img, N, H, W, dy, dcs, K, dw, accumulate, ws, ws_bytes, stream);
}
