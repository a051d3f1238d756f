// Implicit-GEMM convolution engine for NHWC activations on CDNA4 MFMA.
//
// One kernel template serves the three contractions of a dense 2-D convolution (and everything that is
// one: 1x1 projections / nn.Linear, the ELA 7x1 Conv1d, ConvTranspose2d which is the dgrad of a conv):
//   FWD   y [m=(n,oh,ow)][k]          = sum_{tap,c}  x[n, oh*s-p+kh, ow*s-p+kw, c] * w[k][tap][c]
//   DGRAD dx[m=(n,ih,iw)][c]          = sum_{tap,k}  dy[n, (ih+p-kh)/s, (iw+p-kw)/s, k] * w[k][tap][c]
//   WGRAD dw[k][tap][c] (split-K)     = sum_{m}      dy[m][k] * x[n, oh*s-p+kh, ow*s-p+kw, c]
// Weights are KRSC (= a PyTorch (K,C,R,S) parameter stored channels_last), activations NHWC with an
// arbitrary per-pixel channel stride + channel offset, so channel slices (C2f chunk/cat) are free views.
//
// Tiling: 256 threads (4 waves), BM = 128 rows x BN (16..128) cols x BK (32 bf16 / 16 f32) per K-step.
// Operands are staged global -> registers (16-byte loads) -> LDS images [row][k] (k contiguous, rows padded
// to 80 B so the 16-lane ds_read_b128 groups are conflict-free), then read as MFMA fragments:
//   bf16: v_mfma_f32_16x16x32_bf16  (lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], j<8)
//   f32 : v_mfma_f32_16x16x4_f32    (lane l: A[l&15][l>>4],      B[l>>4][l&15])  -- exact fp32 parity mode
// The next K-tile's global loads are issued before the current tile's MFMAs (register double buffer).
// FWD epilogue optionally adds a bias and emits per-(row-tile, channel) partial sum / sum-of-squares of the
// stored values for a following train-mode BatchNorm (deterministic: fixed-order reduction later).
#include "adr_common.h"
#include "adr_wgrad.h"

namespace adr {

enum GemmMode { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2, MODE_DGRAD2 = 3 };  // DGRAD2: stride-2 parity classes

struct GemmArgs {
  const void* x;    // conv input  (FWD, WGRAD)
  const void* w;    // weights KRSC (FWD, DGRAD)
  const void* dy;   // conv output gradient (DGRAD, WGRAD)
  void* out;        // FWD: y ; DGRAD: dx ; WGRAD: fp32 partials [split][K][R*S*C]
  const float* bias;
  float* stats;     // FWD: [mtiles][2][N] partial sums (may be null)
  int n, h, w_, c, xcs, xco;          // conv input geometry and view
  int k, r, s, sh, sw, ph, pw, ho, wo;  // conv output channels, kernel, stride, pad, output size
  int ycs, yco;                        // conv output (y or dy) view: channel stride / offset
  int M, N;                            // GEMM rows / cols
  int cblocks;                         // reduction-channel blocks per tap
  int ktiles;                          // K-steps per block
  int ntiles;                          // column tiles
  int accumulate;                      // out += result
  int par;                             // DGRAD stride-2: blockIdx.z = output parity class (see below)
  int red_per_split;                   // WGRAD: reduction rows per split (multiple of BK)
  long red_total;                      // WGRAD: total reduction rows (n*ho*wo)
};

template <typename T> struct Cfg;
template <> struct Cfg<__bf16> { static constexpr int BK = 32, VEC = 8, LDA = 40; };
template <> struct Cfg<float> { static constexpr int BK = 16, VEC = 4, LDA = 20; };

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
__device__ __forceinline__ v4s tr_read16(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}
// reduction index kk = 8g + 4h + q (MFMA k-slot of lane group g, element 4h + q) -> LDS row: the two groups of
// each 32-lane half read 8 consecutive rows per transposed read (conflict-free with an odd-32-byte pitch)
__device__ __forceinline__ int trb_row(int kk) {
  return (kk & 3) + 4 * ((kk >> 3) & 1) + 8 * ((kk >> 2) & 1) + 16 * (kk >> 4);
}

template <typename T, int BN, int MODE_>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs a) {
  constexpr bool PAR = MODE_ == MODE_DGRAD2;
  constexpr int MODE = PAR ? MODE_DGRAD : MODE_;
  constexpr int BM = 128, BK = Cfg<T>::BK, VEC = Cfg<T>::VEC, LDA = Cfg<T>::LDA;
  constexpr int WAVES_N = (BN >= 128) ? 2 : 1;
  constexpr int WAVES_M = 4 / WAVES_N;
  constexpr int WROWS = BM / WAVES_M, WCOLS = BN / WAVES_N;
  constexpr int TM = WROWS / 16, TN = WCOLS / 16;
  constexpr int KCH = BK / VEC;  // 16-byte chunks per LDS row (=4)
  // chunks each thread moves per K-step
  constexpr int A_CH = (MODE == MODE_WGRAD) ? (BK * (BM / VEC)) / 256 : (BM * KCH) / 256;
  constexpr int B_TOT = (MODE == MODE_FWD) ? BN * KCH : BK * (BN / VEC);
  constexpr int B_CH = (B_TOT + 255) / 256;

  // bf16 DGRAD: the weight tile arrives as [co = reduction][ci = column] rows; it is stored row-for-row (no
  // scalar transposition) at permuted rows and read back with ds_read_b64_tr_b16 (see adr_wgrad.hip)
  constexpr bool TRB = (MODE == MODE_DGRAD) && (sizeof(T) == 2);
  constexpr int PB = ((BN / 16) % 2 == 1) ? BN : BN + 16;  // TRB row pitch: odd multiple of 32 bytes
  constexpr int BS_SIZE = (TRB && BK * PB > BN * LDA) ? BK * PB : BN * LDA;
  __shared__ __attribute__((aligned(16))) T As[BM * LDA];
  __shared__ __attribute__((aligned(16))) T Bs[BS_SIZE];
  __shared__ float red[2][WAVES_M][BN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  int bid = blockIdx.x;
  const int mt = bid / a.ntiles, nt = bid % a.ntiles;
  const int split = blockIdx.y;
  const int m0 = mt * BM;
  const int RS = a.r * a.s;

  // ---- DGRAD of a stride-2 conv by output parity class (py, px) = blockIdx.z: the rows are the dx pixels
  //      (2i + py, 2j + px) and the reduction runs only over the taps whose (pixel + pad - tap) is even, i.e.
  //      kh = kh0, kh0 + 2, ... — a quarter of the taps on average instead of masking 3/4 of them to zero ----
  int cls_y = 0, cls_x = 0, rows_h = (MODE == MODE_FWD) ? a.ho : a.h, rows_w = (MODE == MODE_FWD) ? a.wo : a.w_;
  int kh0 = 0, kw0 = 0, nkw = a.s, tstep = 1;
  long Mrows = a.M;
  int ktiles = a.ktiles;
  if constexpr (PAR) {
    {
      cls_y = blockIdx.z >> 1;
      cls_x = blockIdx.z & 1;
      rows_h = (a.h - cls_y + 1) >> 1;
      rows_w = (a.w_ - cls_x + 1) >> 1;
      Mrows = (long)a.n * rows_h * rows_w;
      kh0 = (cls_y + a.ph) & 1;
      kw0 = (cls_x + a.pw) & 1;
      const int nkh = (a.r - kh0 + 1) >> 1;
      nkw = (a.s - kw0 + 1) >> 1;
      tstep = 2;
      ktiles = nkh * nkw * a.cblocks;
      if ((long)m0 >= Mrows) return;  // this class has fewer rows than the grid's largest
    }
  }
  constexpr int ystep = PAR ? 2 : 1;
  // output pixel (linear NHWC row) of GEMM row m
  auto pixel_of = [&](long m) -> long {
    if constexpr (PAR) {
      const long hw = (long)rows_h * rows_w;
      const long img = m / hw;
      const int rem = (int)(m % hw);
      return (img * a.h + (rem / rows_w) * 2 + cls_y) * a.w_ + (rem % rows_w) * 2 + cls_x;
    }
    return m;
  };

  // ---- per-thread row decode for the A operand (FWD / DGRAD: output pixels) ----
  int a_img[A_CH], a_y[A_CH], a_x[A_CH];
  bool a_ok[A_CH];
  if constexpr (MODE != MODE_WGRAD) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int row = (tid + 256 * i) / KCH;
      long m = (long)m0 + row;
      a_ok[i] = m < Mrows;
      const int hw = rows_h * rows_w;
      long mm = a_ok[i] ? m : 0;
      a_img[i] = (int)(mm / hw);
      int rem = (int)(mm % hw);
      a_y[i] = (rem / rows_w) * ystep + cls_y;
      a_x[i] = (rem % rows_w) * ystep + cls_x;
    }
  }
  // column tile -> tap / channel block for WGRAD
  int wg_tap = 0, wg_c0 = 0;
  const int n0 = nt * BN;
  if constexpr (MODE == MODE_WGRAD) {
    int cbn = (a.c + BN - 1) / BN;
    wg_tap = nt / cbn;
    wg_c0 = (nt % cbn) * BN;
  }
  const long red_begin = (MODE == MODE_WGRAD) ? (long)split * a.red_per_split : 0;

  u32x4 ra[A_CH], rb[B_CH > 0 ? B_CH : 1];
  const u32x4 zero = {0u, 0u, 0u, 0u};

  auto load_tile = [&](int t) {
    if constexpr (MODE == MODE_FWD) {
      const int tap = t / a.cblocks, cb = t % a.cblocks;
      const int kh = tap / a.s, kw = tap % a.s;
      const int kc = tid % KCH;
      const int c = cb * BK + kc * VEC;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        int ih = a_y[i] * a.sh - a.ph + kh, iw = a_x[i] * a.sw - a.pw + kw;
        bool ok = a_ok[i] && c < a.c && ih >= 0 && ih < a.h && iw >= 0 && iw < a.w_;
        const T* p = (const T*)a.x + ((long)(a_img[i] * a.h + ih) * a.w_ + iw) * a.xcs + a.xco + c;
        ra[i] = ok ? ld16(p) : zero;
      }
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        int q = tid + 256 * i;
        int row = q / KCH, kcb = q % KCH;
        int n = n0 + row;
        int cc = cb * BK + kcb * VEC;
        bool ok = (q < B_TOT) && n < a.N && cc < a.c;
        const T* p = (const T*)a.w + ((long)n * RS + tap) * a.c + cc;
        rb[i] = ok ? ld16(p) : zero;
      }
    } else if constexpr (MODE == MODE_DGRAD) {
      const int ti = t / a.cblocks, cb = t % a.cblocks;
      const int kh = kh0 + tstep * (ti / nkw), kw = kw0 + tstep * (ti % nkw);
      const int tap = kh * a.s + kw;
      const int kc = tid % KCH;
      const int co = cb * BK + kc * VEC;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        int ny = a_y[i] + a.ph - kh, nx = a_x[i] + a.pw - kw;
        bool ok = a_ok[i] && co < a.k && ny >= 0 && nx >= 0;
        int oy = ny / a.sh, ox = nx / a.sw;
        ok = ok && (oy * a.sh == ny) && (ox * a.sw == nx) && oy < a.ho && ox < a.wo;
        const T* p = (const T*)a.dy + ((long)(a_img[i] * a.ho + oy) * a.wo + ox) * a.ycs + a.yco + co;
        ra[i] = ok ? ld16(p) : zero;
      }
      // B image Bs[ci][co] from w[co][tap][ci]: chunk = (co_local, ci chunk)
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        int q = tid + 256 * i;
        int col = q / (BN / VEC), cch = q % (BN / VEC);
        int coo = cb * BK + col;
        int ci = n0 + cch * VEC;
        bool ok = (q < B_TOT) && coo < a.k && ci < a.c;
        const T* p = (const T*)a.w + ((long)coo * RS + tap) * a.c + ci;
        rb[i] = ok ? ld16(p) : zero;
      }
    } else {  // WGRAD
      const long p0 = red_begin + (long)t * BK;
      // A image As[co][p] from dy[p][co]: chunk = (p_local, co chunk)
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        int q = tid + 256 * i;
        int pl = q / (BM / VEC), cch = q % (BM / VEC);
        long p = p0 + pl;
        int co = m0 + cch * VEC;
        bool ok = p < a.red_total && p < red_begin + a.red_per_split && co < a.k;
        const T* ptr = (const T*)a.dy + p * a.ycs + a.yco + co;
        ra[i] = ok ? ld16(ptr) : zero;
      }
      const int kh = wg_tap / a.s, kw = wg_tap % a.s;
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        int q = tid + 256 * i;
        int pl = q / (BN / VEC), cch = q % (BN / VEC);
        long p = p0 + pl;
        int ci = wg_c0 + cch * VEC;
        bool ok = (q < B_TOT) && p < a.red_total && p < red_begin + a.red_per_split && ci < a.c;
        long pp = ok ? p : 0;
        int hw = a.ho * a.wo;
        int img = (int)(pp / hw), rem = (int)(pp % hw);
        int oy = rem / a.wo, ox = rem % a.wo;
        int iy = oy * a.sh - a.ph + kh, ix = ox * a.sw - a.pw + kw;
        ok = ok && iy >= 0 && iy < a.h && ix >= 0 && ix < a.w_;
        const T* ptr = (const T*)a.x + ((long)(img * a.h + iy) * a.w_ + ix) * a.xcs + a.xco + ci;
        rb[i] = ok ? ld16(ptr) : zero;
      }
    }
  };

  auto store_tile = [&]() {
    if constexpr (MODE == MODE_WGRAD) {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        int q = tid + 256 * i;
        int pl = q / (BM / VEC), cch = q % (BM / VEC);
        const T* v = reinterpret_cast<const T*>(&ra[i]);
#pragma unroll
        for (int e = 0; e < VEC; ++e) As[(cch * VEC + e) * LDA + pl] = v[e];
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        int q = tid + 256 * i;
        int row = q / KCH, kc = q % KCH;
        st16(&As[row * LDA + kc * VEC], ra[i]);
      }
    }
    if constexpr (MODE == MODE_FWD) {
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        int q = tid + 256 * i;
        if (q < B_TOT) {
          int row = q / KCH, kc = q % KCH;
          st16(&Bs[row * LDA + kc * VEC], rb[i]);
        }
      }
    } else if constexpr (TRB) {
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        int q = tid + 256 * i;
        if (q < B_TOT) {
          int kl = q / (BN / VEC), cch = q % (BN / VEC);
          st16(&Bs[trb_row(kl) * PB + cch * VEC], rb[i]);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < B_CH; ++i) {
        int q = tid + 256 * i;
        if (q < B_TOT) {
          int kl = q / (BN / VEC), cch = q % (BN / VEC);
          const T* v = reinterpret_cast<const T*>(&rb[i]);
#pragma unroll
          for (int e = 0; e < VEC; ++e) Bs[(cch * VEC + e) * LDA + kl] = v[e];
        }
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int wr0 = wm * WROWS, wc0 = wn * WCOLS;
  if (ktiles > 0) {
    load_tile(0);
    store_tile();
    __syncthreads();
  }
  for (int t = 0; t < ktiles; ++t) {
    if (t + 1 < ktiles) load_tile(t + 1);
    if constexpr (sizeof(T) == 2) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(&As[(wr0 + i * 16 + (lane & 15)) * LDA + 8 * (lane >> 4)]);
      if constexpr (TRB) {
        // lane (g, q4, p4): k-slot (g, 4h + q4) lives at LDS row trb_row(8g + 4h + q4), column 4*p4
        const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
        const T* b0 = &Bs[trb_row(8 * g + q4) * PB + wc0 + 4 * p4];
        const T* b1 = &Bs[trb_row(8 * g + 4 + q4) * PB + wc0 + 4 * p4];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          v4s both[2] = {tr_read16(b0 + j * 16), tr_read16(b1 + j * 16)};
          fb[j] = *reinterpret_cast<bf16x8*>(both);
        }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wc0 + j * 16 + (lane & 15)) * LDA + 8 * (lane >> 4)]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int sub = 0; sub < BK / 4; ++sub) {
        float fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = (float)As[(wr0 + i * 16 + (lane & 15)) * LDA + 4 * sub + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = (float)Bs[(wc0 + j * 16 + (lane & 15)) * LDA + 4 * sub + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
    if (t + 1 < ktiles) {
      store_tile();
      __syncthreads();
    }
  }

  // ---- epilogue ----
  if constexpr (MODE == MODE_WGRAD) {
    float* part = (float*)a.out + (long)split * a.k * ((long)RS * a.c);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int ci = wg_c0 + wc0 + j * 16 + (lane & 15);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int co = m0 + wr0 + i * 16 + 4 * (lane >> 4) + e;
          if (co < a.k && ci < a.c) part[((long)co * RS + wg_tap) * a.c + ci] = acc[i][j][e];
        }
      }
  } else {
    T* out = (T*)a.out;
    const int ocs = (MODE == MODE_FWD) ? a.ycs : a.xcs, oco = (MODE == MODE_FWD) ? a.yco : a.xco;
    float csum[TN], csq[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) { csum[j] = 0.f; csq[j] = 0.f; }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int n = n0 + wc0 + j * 16 + (lane & 15);
        float b = (a.bias && n < a.N) ? a.bias[n] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          long m = (long)m0 + wr0 + i * 16 + 4 * (lane >> 4) + e;
          if (m < Mrows && n < a.N) {
            T* p = out + pixel_of(m) * ocs + oco + n;
            float v = acc[i][j][e] + b;
            if (a.accumulate) v += to_f(*p);
            T tv = from_f<T>(v);
            *p = tv;
            float vr = to_f(tv);
            csum[j] += vr;
            csq[j] += vr * vr;
          }
        }
      }
    if (a.stats) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float s = csum[j], q = csq[j];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        if (lane < 16) {
          red[0][wm][wc0 + j * 16 + lane] = s;
          red[1][wm][wc0 + j * 16 + lane] = q;
        }
      }
      __syncthreads();
      if (tid < BN) {
        int n = n0 + tid;
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < WAVES_M; ++w) { s += red[0][w][tid]; q += red[1][w][tid]; }
        if (n < a.N) {
          a.stats[(long)mt * 2 * a.N + n] = s;
          a.stats[(long)mt * 2 * a.N + a.N + n] = q;
        }
      }
    }
  }
}

// deterministic reduction of WGRAD split partials: dw[i] (+)= sum_s part[s][i]. A block owns 32 consecutive
// outputs; its 8 slices of 32 threads each sum every 8th split (coalesced 128-byte rows, 4 loads in flight),
// then the slices are combined in LDS in a fixed order — parallel over splits as well as outputs, so a
// small-output / many-split reduction still fills the chip.
struct Unpack {  // UNPACK: output i = (k*RS + t)*Cp + c of the KRSC partials lands at the (K,C,RS) parameter slot
  int K, C, Cp, RS, transpose_kc;
};
// OUT outputs x SL split slices per 256-thread block; many-split reductions use 16 x 16 so that each thread sums
// fewer splits, with 8 loads in flight (fixed order per configuration: deterministic)
template <bool UNPACK, int OUT, int SL>
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ part, long stride,
                                                           float* __restrict__ dw, long n, int splits, int accumulate,
                                                           Unpack u) {
  __shared__ float sh[SL][OUT];
  const int o = threadIdx.x % OUT, sl = threadIdx.x / OUT;
  const long i = (long)blockIdx.x * OUT + o;
  constexpr int U = 8;
  float acc[U];
#pragma unroll
  for (int v = 0; v < U; ++v) acc[v] = 0.f;
  if (i < n) {
    int k = sl;
    for (; k + (U - 1) * SL < splits; k += U * SL) {
#pragma unroll
      for (int v = 0; v < U; ++v) acc[v] += part[(long)(k + v * SL) * stride + i];
    }
#pragma unroll
    for (int v = 0; v < U; ++v)
      if (k + v * SL < splits) acc[v] += part[(long)(k + v * SL) * stride + i];
  }
  sh[sl][o] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (sl == 0 && i < n) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < SL; ++q) s += sh[q][o];
    long di = i;
    if constexpr (UNPACK) {
      const int c = (int)(i % u.Cp);
      const long r = i / u.Cp;
      const int t = (int)(r % u.RS), k = (int)(r / u.RS);
      if (c >= u.C) return;
      di = u.transpose_kc ? ((long)c * u.K + k) * u.RS + t : ((long)k * u.C + c) * u.RS + t;
    }
    dw[di] = accumulate ? dw[di] + s : s;
  }
}

// Many WGRAD reductions in one launch (the trainer defers them to the end of the backward pass; the immediate
// adr_wgrad_reduce_unpack is a batch of one, so deferring changes no result). The entries ride in the kernel
// arguments; a block's entry is found from the per-entry block offsets. A thread owns 4 consecutive outputs (one
// 16-byte load per split slab: the partial rows are channel-contiguous) and a split lane; `SL` lanes per output quad
// (per entry, from the host: small outputs with many splits still spread over the chip) each sum their splits in
// order, 4 slabs in flight, and the lanes are combined in lane order through LDS — a fixed order per entry
// (deterministic). The sum then lands at its (K, C, RS) parameter slot (or (C, K, RS) with transpose_kc).
// Round 4: replaces a 32-output x 8-lane scalar version that read 4-byte words (l-scale: 800 us per launch).
constexpr int RB_MAX = 56;
struct RedBatch {
  adr_wgrad_reduce_entry e[RB_MAX];  // e[j].pad_ carries the entry's split lanes (SL)
  int start[RB_MAX + 1];
  int count;
};
__global__ void __launch_bounds__(256) wgrad_reduce_batched_kernel(RedBatch b) {
  int j = 0;
  while (j + 1 < b.count && (int)blockIdx.x >= b.start[j + 1]) ++j;
  const adr_wgrad_reduce_entry& en = b.e[j];
  const int SL = en.pad_, QPB = 256 / SL;
  const int q = threadIdx.x % QPB, lane = threadIdx.x / QPB;
  const long i0 = ((long)(blockIdx.x - b.start[j]) * QPB + q) * 4;
  const long n = (long)en.K * en.RS * en.Cp;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i0 < n) {
    const float* p = en.part + i0;
    int s = lane;
    for (; s + 3 * SL < en.splits; s += 4 * SL) {
      const float4 v0 = *reinterpret_cast<const float4*>(p + (long)s * en.split_stride);
      const float4 v1 = *reinterpret_cast<const float4*>(p + (long)(s + SL) * en.split_stride);
      const float4 v2 = *reinterpret_cast<const float4*>(p + (long)(s + 2 * SL) * en.split_stride);
      const float4 v3 = *reinterpret_cast<const float4*>(p + (long)(s + 3 * SL) * en.split_stride);
      acc.x += v0.x; acc.y += v0.y; acc.z += v0.z; acc.w += v0.w;
      acc.x += v1.x; acc.y += v1.y; acc.z += v1.z; acc.w += v1.w;
      acc.x += v2.x; acc.y += v2.y; acc.z += v2.z; acc.w += v2.w;
      acc.x += v3.x; acc.y += v3.y; acc.z += v3.z; acc.w += v3.w;
    }
    for (; s < en.splits; s += SL) {
      const float4 v = *reinterpret_cast<const float4*>(p + (long)s * en.split_stride);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  __shared__ float4 sh[256];
  if (SL > 1) {
    sh[threadIdx.x] = acc;
    __syncthreads();
    if (lane != 0) return;
    for (int l = 1; l < SL; ++l) {
      const float4 v = sh[l * QPB + q];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  if (i0 >= n) return;
  const float r4[4] = {acc.x, acc.y, acc.z, acc.w};
  const int c0 = (int)(i0 % en.Cp);  // Cp % 4 == 0: the quad shares (k, t)
  const long r = i0 / en.Cp;
  const int t = (int)(r % en.RS), kk = (int)(r / en.RS);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c0 + e;
    if (c >= en.C) break;
    const long di = en.transpose_kc ? ((long)c * en.K + kk) * en.RS + t : ((long)kk * en.C + c) * en.RS + t;
    en.dst[di] = en.accumulate ? en.dst[di] + r4[e] : r4[e];
  }
}

static int reduce_lanes(long n, int splits) {  // split lanes: enough blocks to spread a small output over the chip
  int sl = 1;
  while (sl < 32 && sl < splits && cdiv(n / 4, 256 / sl) < 512) sl *= 2;
  return sl;
}

// ------------------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------------------

static int pick_bn(int n) {
  if (n <= 16) return 16;
  if (n <= 32) return 32;
  if (n <= 64) return 64;
  return 128;
}

template <typename T, int MODE>
static void launch_bn(int bn, dim3 grid, const GemmArgs& g, hipStream_t st) {
  switch (bn) {
    case 16: hipLaunchKernelGGL((gemm_kernel<T, 16, MODE>), grid, dim3(256), 0, st, g); break;
    case 32: hipLaunchKernelGGL((gemm_kernel<T, 32, MODE>), grid, dim3(256), 0, st, g); break;
    case 64: hipLaunchKernelGGL((gemm_kernel<T, 64, MODE>), grid, dim3(256), 0, st, g); break;
    default: hipLaunchKernelGGL((gemm_kernel<T, 128, MODE>), grid, dim3(256), 0, st, g); break;
  }
}

static int fill_common(const adr_conv_desc* d, GemmArgs& g) {
  ADR_REQUIRE(d && d->n > 0 && d->h > 0 && d->w > 0 && d->c > 0 && d->k > 0 && d->r > 0 && d->s > 0,
              "conv: bad geometry");
  ADR_REQUIRE(d->dtype == ADR_F32 || d->dtype == ADR_BF16, "conv: unsupported dtype %d", d->dtype);
  int vec = d->dtype == ADR_BF16 ? 8 : 4;
  ADR_REQUIRE(d->c % vec == 0 && d->k % vec == 0, "conv: C (%d) and K (%d) must be multiples of %d", d->c, d->k, vec);
  ADR_REQUIRE(d->x_cstride % vec == 0 && d->x_coff % vec == 0 && d->y_cstride % vec == 0 && d->y_coff % vec == 0,
              "conv: channel views must be 16-byte aligned");
  ADR_REQUIRE(d->x_cstride >= d->x_coff + d->c && d->y_cstride >= d->y_coff + d->k, "conv: view exceeds stride");
  int ho = (d->h + 2 * d->pad_h - d->r) / d->stride_h + 1;
  int wo = (d->w + 2 * d->pad_w - d->s) / d->stride_w + 1;
  ADR_REQUIRE(ho == d->ho && wo == d->wo, "conv: output size mismatch (%dx%d vs %dx%d)", d->ho, d->wo, ho, wo);
  g.n = d->n; g.h = d->h; g.w_ = d->w; g.c = d->c; g.xcs = d->x_cstride; g.xco = d->x_coff;
  g.k = d->k; g.r = d->r; g.s = d->s; g.sh = d->stride_h; g.sw = d->stride_w; g.ph = d->pad_h; g.pw = d->pad_w;
  g.ho = d->ho; g.wo = d->wo; g.ycs = d->y_cstride; g.yco = d->y_coff;
  return ADR_OK;
}

static int bk_of(int dtype) { return dtype == ADR_BF16 ? 32 : 16; }

}  // namespace adr

using namespace adr;

extern "C" int adr_conv2d_fwd(const adr_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                              float* stats, int accumulate, void* stream) {
  GemmArgs g{};
  int rc = fill_common(d, g);
  if (rc) return rc;
  g.x = x; g.w = w; g.out = y; g.bias = bias; g.stats = stats; g.accumulate = accumulate;
  g.M = d->n * d->ho * d->wo;
  g.N = d->k;
  int BK = bk_of(d->dtype);
  g.cblocks = cdiv(d->c, BK);
  g.ktiles = d->r * d->s * g.cblocks;
  int bn = pick_bn(g.N);
  g.ntiles = cdiv(g.N, bn);
  int mtiles = cdiv(g.M, 128);
  dim3 grid(mtiles * g.ntiles, 1);
  hipStream_t st = (hipStream_t)stream;
  if (d->dtype == ADR_BF16) launch_bn<__bf16, MODE_FWD>(bn, grid, g, st);
  else launch_bn<float, MODE_FWD>(bn, grid, g, st);
  return check_launch("adr_conv2d_fwd");
}

extern "C" int adr_conv2d_fwd_stat_tiles(const adr_conv_desc* d) { return cdiv((long)d->n * d->ho * d->wo, 128); }

extern "C" int adr_conv2d_dgrad(const adr_conv_desc* d, const void* dy, const void* w, const float* bias, void* dx,
                                int accumulate, void* stream) {
  GemmArgs g{};
  int rc = fill_common(d, g);
  if (rc) return rc;
  // reads dy through the y view (y_cstride, y_coff); writes dx through the x view (x_cstride, x_coff)
  g.dy = dy; g.w = w; g.out = dx; g.bias = bias; g.accumulate = accumulate;
  g.M = d->n * d->h * d->w;
  g.N = d->c;
  int BK = bk_of(d->dtype);
  g.cblocks = cdiv(d->k, BK);
  g.ktiles = d->r * d->s * g.cblocks;
  int bn = pick_bn(g.N);
  g.ntiles = cdiv(g.N, bn);
  dim3 grid(cdiv(g.M, 128) * g.ntiles, 1);
  hipStream_t st = (hipStream_t)stream;
  if (d->stride_h == 2 && d->stride_w == 2) {  // parity classes: the largest one sizes the grid
    g.par = 1;
    grid = dim3(cdiv((long)d->n * ((d->h + 1) / 2) * ((d->w + 1) / 2), 128) * g.ntiles, 1, 4);
    if (d->dtype == ADR_BF16) launch_bn<__bf16, MODE_DGRAD2>(bn, grid, g, st);
    else launch_bn<float, MODE_DGRAD2>(bn, grid, g, st);
    return check_launch("adr_conv2d_dgrad");
  }
  if (d->dtype == ADR_BF16) launch_bn<__bf16, MODE_DGRAD>(bn, grid, g, st);
  else launch_bn<float, MODE_DGRAD>(bn, grid, g, st);
  return check_launch("adr_conv2d_dgrad");
}

static int wgrad_splits(const adr_conv_desc* d, int* bn_out, int* ntiles_out) {
  long red = (long)d->n * d->ho * d->wo;
  int BK = bk_of(d->dtype);
  int bn = pick_bn(d->c);
  int ntiles = d->r * d->s * cdiv(d->c, bn);
  int mtiles = cdiv(d->k, 128);
  long tiles = (long)ntiles * mtiles;
  long want = (2048 + tiles - 1) / tiles;
  long maxs = (red + BK * 8 - 1) / (BK * 8);  // at least 8 K-steps per split
  long s = want < maxs ? want : maxs;
  if (s < 1) s = 1;
  if (s > 65535) s = 65535;
  *bn_out = bn;
  *ntiles_out = ntiles;
  return (int)s;
}

extern "C" size_t adr_conv2d_wgrad_workspace(const adr_conv_desc* d) {
  int bn, nt;
  const int splits = d->dtype == ADR_BF16 ? wgrad_bf16_plan(d).splits : wgrad_splits(d, &bn, &nt);
  return (size_t)splits * d->k * d->r * d->s * d->c * sizeof(float);
}

extern "C" int adr_conv2d_wgrad_splits(const adr_conv_desc* d) {
  if (d->dtype == ADR_BF16) return wgrad_bf16_plan(d).splits;
  int bn, nt;
  return wgrad_splits(d, &bn, &nt);
}

extern "C" int adr_conv2d_wgrad_partials(const adr_conv_desc* d, const void* x, const void* dy, float* out,
                                         int accumulate, void* stream) {
  GemmArgs g{};
  int rc = fill_common(d, g);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (d->dtype == ADR_BF16) {
    WgPlan p = wgrad_bf16_plan(d);
    ADR_REQUIRE(!accumulate || p.splits == 1, "conv wgrad partials: accumulate needs a single split");
    return wgrad_bf16_launch(d, x, dy, out, accumulate, p, st);
  }
  int bn, ntiles;
  int splits = wgrad_splits(d, &bn, &ntiles);
  ADR_REQUIRE(!accumulate, "conv wgrad partials: fp32 path writes (no accumulate)");
  int BK = bk_of(d->dtype);
  long red = (long)d->n * d->ho * d->wo;
  long per = (red + splits - 1) / splits;
  per = (per + BK - 1) / BK * BK;
  g.x = x; g.dy = dy; g.out = out;
  g.M = d->k; g.N = d->r * d->s * d->c;
  g.red_total = red;
  g.red_per_split = (int)per;
  g.ktiles = (int)(per / BK);
  g.ntiles = ntiles;
  // every (co, tap, ci) inside [K x RSC] is written by exactly one block per split
  launch_bn<float, MODE_WGRAD>(bn, dim3(cdiv(d->k, 128) * ntiles, splits), g, st);
  return check_launch("adr_conv2d_wgrad_partials");
}

extern "C" int adr_wgrad_reduce(const float* part, float* dw, long n, int splits, int accumulate, void* stream) {
  ADR_REQUIRE(n > 0 && splits >= 1, "wgrad_reduce: n=%ld splits=%d", n, splits);
  if (splits >= 256)
    hipLaunchKernelGGL((wgrad_reduce_kernel<false, 16, 16>), dim3(cdiv(n, 16)), dim3(256), 0, (hipStream_t)stream, part,
                       n, dw, n, splits, accumulate, Unpack{});
  else
    hipLaunchKernelGGL((wgrad_reduce_kernel<false, 32, 8>), dim3(cdiv(n, 32)), dim3(256), 0, (hipStream_t)stream, part,
                       n, dw, n, splits, accumulate, Unpack{});
  return check_launch("adr_wgrad_reduce");
}

extern "C" int adr_wgrad_reduce_batched(const adr_wgrad_reduce_entry* entries, int count, void* stream);

extern "C" int adr_wgrad_reduce_unpack(const float* part, long split_stride, int splits, float* dst, int K, int C,
                                       int Cp, int RS, int transpose_kc, int accumulate, void* stream) {
  adr_wgrad_reduce_entry en{part, dst, split_stride, splits, K, C, Cp, RS, transpose_kc, accumulate, 0};
  return adr_wgrad_reduce_batched(&en, 1, stream);
}

extern "C" int adr_wgrad_reduce_batched(const adr_wgrad_reduce_entry* entries, int count, void* stream) {
  ADR_REQUIRE(count >= 0 && (count == 0 || entries), "wgrad_reduce_batched: count=%d", count);
  for (int b0 = 0; b0 < count; b0 += RB_MAX) {
    RedBatch rb{};
    rb.count = count - b0 < RB_MAX ? count - b0 : RB_MAX;
    int blocks = 0;
    for (int j = 0; j < rb.count; ++j) {
      const adr_wgrad_reduce_entry& en = entries[b0 + j];
      const long n = (long)en.K * en.RS * en.Cp;
      ADR_REQUIRE(en.part && en.dst && n > 0 && en.splits >= 1 && en.C <= en.Cp && en.split_stride >= n &&
                      en.Cp % 4 == 0 && en.split_stride % 4 == 0 && ((uintptr_t)en.part & 15) == 0,
                  "wgrad_reduce_batched: entry %d (K=%d C=%d Cp=%d RS=%d splits=%d)", b0 + j, en.K, en.C, en.Cp,
                  en.RS, en.splits);
      for (int q = 0; q < j; ++q)  // same destination twice in one launch would race: the caller must split
        ADR_REQUIRE(rb.e[q].dst != en.dst, "wgrad_reduce_batched: entries %d and %d share a destination", b0 + q,
                    b0 + j);
      rb.e[j] = en;
      rb.e[j].pad_ = reduce_lanes(n, en.splits);
      rb.start[j] = blocks;
      blocks += (int)cdiv(n / 4, 256 / rb.e[j].pad_);
    }
    rb.start[rb.count] = blocks;
    hipLaunchKernelGGL(wgrad_reduce_batched_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, rb);
  }
  return check_launch("adr_wgrad_reduce_batched");
}

extern "C" int adr_conv2d_wgrad(const adr_conv_desc* d, const void* x, const void* dy, float* dw, int accumulate,
                                void* ws, size_t ws_bytes, void* stream) {
  const int splits = adr_conv2d_wgrad_splits(d);
  const long nout = (long)d->k * d->r * d->s * d->c;
  if (splits == 1 && (d->dtype == ADR_BF16 || !accumulate))
    return adr_conv2d_wgrad_partials(d, x, dy, dw, accumulate, stream);
  size_t need = (size_t)splits * nout * sizeof(float);
  ADR_REQUIRE(ws && ws_bytes >= need, "conv wgrad: workspace %zu < %zu bytes", ws_bytes, need);
  int rc = adr_conv2d_wgrad_partials(d, x, dy, (float*)ws, 0, stream);
  if (rc) return rc;
  return adr_wgrad_reduce((const float*)ws, dw, nout, splits, accumulate, stream);
}
