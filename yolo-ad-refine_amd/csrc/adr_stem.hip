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
  if (segs == 1 && W % 4 == 0 && W <= STEM_LOOP_W) {  // persistent form: ~4 blocks per CU, contiguous tile ranges
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
