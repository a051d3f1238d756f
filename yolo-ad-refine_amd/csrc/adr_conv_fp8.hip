// fp8 (OCP e4m3) forward convolution for the l-scale configuration (BASELINE.json configs[4]: "fp8 MFMA conv
// path"): the implicit GEMM of adr_conv.hip's forward on v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales),
// twice the bf16 MFMA rate per clock.
//
// Recipe ("fp8 forward", delayed scaling): activations stay bf16 in HBM and are quantised while they are staged
// into LDS, q(x) = e4m3(x / 2^e) with 2^e the power of two that maps amax|x| of the SAME conv's input at the
// previous step to <= 28 (16x headroom: the hardware conversion does not saturate)
// (per tensor; the kernel collects this step's amax as it stages x: per-wave maxima -> an atomicMax on the bits of
// a non-negative float into one of 256 slots, order-independent; the weight-pack launch rotates the slots before
// the conv; the first call seeds them with one adr_amax_bf16 pass);
// weights are quantised once per step at pack time per output channel, sw[k] = 448 / amax|w[k, :]|. The fp32
// accumulator is rescaled by 1 / (sa * sw[k]) in the epilogue, which then matches the bf16 engine's (bias, bf16
// rounding, BatchNorm partial statistics of the stored values). The backward (dgrad / wgrad) stays on the bf16
// engine with the bf16 activations saved by the forward.
//
// Tile: 256 threads, BM = 128 rows x BN (64 / 128) columns, BK = 128 reduction elements per step. Each thread owns
// one 8-element position of the 128-wide step for 8 rows (16-byte bf16 gathers through buffer descriptors, as the
// bf16 engine), converts them with v_cvt_pk_fp8_f32 and stores 8 bytes into a 144-byte LDS row. The MFMA fragment
// of lane l is bytes [32 (l >> 4), +32) of row l & 15 for both operands (a shared k permutation within the step;
// scripts/probes/fp8_mfma_probe.hip checks it on exact integer data).
#include "adr_common.h"

namespace adr {

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

struct Fp8Args {
  const __bf16* src;      // x (NHWC view)
  const uint8_t* wt;      // fp8 KRSC rows, reduction-contiguous (ktot bytes per output channel)
  const float* wscale;    // [N] 1 / sw[k]
  const float* amax_part; // [AMAX_BLOCKS] |x| maxima of this conv's input at the previous step (sa from their max)
  float* amax_next;       // [AMAX_BLOCKS] this step's maxima (atomicMax on the float bits; zeroed by the pack)
  __bf16* out;
  const float* bias;
  float* stats;           // [mtiles][2][N] or null
  int n;
  int sh_, sw_, scs, sco, sc;
  int rh, rw, ocs, oco;
  int r, s, str, ph, pw;
  int N, ktot, ntiles;
  int src_bytes, wt_bytes;
};

constexpr int F8BM = 128, F8BK = 128, F8P = 144;  // LDS row pitch in bytes
constexpr int AMAX_BLOCKS = 256;

__device__ __forceinline__ int xcd_block8(int b, int nb) { return xcd_remap(b, nb); }

// per-block max |x| over an NHWC channel view (C channels at offset co of stride cs), 8 channels per lane
__global__ void __launch_bounds__(256) amax_bf16_kernel(const __bf16* x, int cs, int co, long npix, int C, float* part) {
  const int G = C / 8;
  float m = 0.f;
  const long total = npix * G;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long p = i / G;
    const int g = (int)(i - p * G);
    const u32x4 v = ld16(x + p * cs + co + g * 8);
    const __bf16* e = reinterpret_cast<const __bf16*>(&v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // finite values only (as the conv's own amax collection)
      const float f = fabsf((float)e[k]);
      m = f < INFINITY ? fmaxf(m, f) : m;
    }
  }
  __shared__ float sh[256];
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] = fmaxf(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

// fp32 (K, C, R, S) weights -> fp8 KRSC rows (channels padded to Cp with zeros) + 1 / sw[k]; block per k. Block 0
// also rotates the activation amax slots of this conv: prev <- cur (last step's maxima), cur <- 0.
__global__ void __launch_bounds__(256) pack_fp8_kernel(const float* w, int C, int Cp, int RS, uint8_t* out,
                                                       float* inv_scale, float* amax_cur, float* amax_prev) {
  const int k = blockIdx.x;
  if (k == 0 && amax_cur) {
    amax_prev[threadIdx.x] = amax_cur[threadIdx.x];
    amax_cur[threadIdx.x] = 0.f;
  }
  const float* wk = w + (long)k * C * RS;
  float m = 0.f;
  for (int i = threadIdx.x; i < C * RS; i += 256) m = fmaxf(m, fabsf(wk[i]));
  __shared__ float sh[256];
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] = fmaxf(sh[threadIdx.x], sh[threadIdx.x + o]);
    __syncthreads();
  }
  const float amax = sh[0];
  const float sc = amax > 0.f ? 448.f / amax : 1.f;
  if (threadIdx.x == 0) inv_scale[k] = 1.f / sc;
  uint8_t* ok = out + (long)k * RS * Cp;
  for (int i = threadIdx.x; i < RS * Cp; i += 256) {
    const int t = i / Cp, c = i - t * Cp;
    const float v = c < C ? wk[(long)c * RS + t] * sc : 0.f;
    ok[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 255);
  }
}

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) short s16x2;
typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;

// 8 bf16 (one 16-byte chunk) -> 8 e4m3 bytes as x / scale (scale a power of two: v_cvt_scalef32_pk_fp8_bf16, two
// elements per instruction, straight from the bf16 pairs); m tracks max |x| of the FINITE inputs as bf16 bit
// patterns (non-negative floats order like their bits) with packed 16-bit maxima. The conversion does not
// saturate, so finite magnitudes are first clamped to lim2 (both halves = the bf16 bits of 448 * scale): an input
// past the delayed scale's 16x headroom becomes +-448, not NaN. Inf / NaN inputs pass through (NaN out, visible)
// and are left out of the maximum, so one bad value cannot poison the next steps' scale.
__device__ __forceinline__ u32x2 to_fp8x8(u32x4 v, float scale, unsigned lim2, u16x2& m) {
  u32x4 c;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned a = v[q] & 0x7FFF7FFFu;
    // per 16-bit half: all ones where |x| >= 0x7F80 (Inf / NaN); a half + 0x80 stays below 0x10000
    const unsigned hb = (a + 0x00800080u) & 0x80008000u;
    const unsigned nf = hb | (hb - (hb >> 15));
    const unsigned fin = a & ~nf;
    m = __builtin_elementwise_max(m, *reinterpret_cast<const u16x2*>(&fin));
    const u16x2 cl = __builtin_elementwise_min(*reinterpret_cast<const u16x2*>(&fin),
                                               *reinterpret_cast<const u16x2*>(&lim2));
    c[q] = (*reinterpret_cast<const unsigned*>(&cl) | (a & nf)) | (v[q] & 0x80008000u);
  }
  const bf16x2* e = reinterpret_cast<const bf16x2*>(&c);
  s16x2 lo = {0, 0}, hi = {0, 0};
  lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(lo, e[0], scale, false);
  lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(lo, e[1], scale, true);
  hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(hi, e[2], scale, false);
  hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(hi, e[3], scale, true);
  return (u32x2){*reinterpret_cast<const unsigned*>(&lo), *reinterpret_cast<const unsigned*>(&hi)};
}

// activation scale (a power of two) from last step's maximum: amax maps to <= 28, so values up to 16x last step's
// maximum still fit e4m3's 448 (the conversion does not saturate); e4m3's normal range keeps 3 mantissa bits down
// to amax / 2^11
__device__ __forceinline__ float act_scale_pow2(float amax) {
  return amax > 0.f ? exp2f(ceilf(log2f(amax / 28.f))) : 1.f;
}

template <int BN>
__global__ void __launch_bounds__(256, 2) conv_fp8_kernel(Fp8Args a) {
  constexpr int WAVES_N = BN >= 128 ? 2 : 1, WAVES_M = 4 / WAVES_N;
  constexpr int WROWS = F8BM / WAVES_M, WCOLS = BN / WAVES_N;
  constexpr int TM = WROWS / 16, TN = WCOLS / 16;
  constexpr int A_CH = F8BM * (F8BK / 8) / 256;        // 8 bf16 chunks per thread
  constexpr int B_TOT = BN * (F8BK / 16), B_CH = (B_TOT + 255) / 256;
  constexpr int OPITCH = BN + 8;
  constexpr int SMEM_AB = (F8BM + BN) * F8P;
  constexpr int SMEM_O = F8BM * OPITCH * 2;
  constexpr int RG = 256 / (BN / 8);
  constexpr int SMEM0 = SMEM_AB > SMEM_O ? SMEM_AB : SMEM_O;
  constexpr int SMEM = SMEM0 > 2 * RG * BN * 4 ? SMEM0 : 2 * RG * BN * 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds[SMEM];
  __shared__ float s_inv;
  uint8_t* As = lds;
  uint8_t* Bs = lds + F8BM * F8P;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bid = xcd_block8(blockIdx.x, gridDim.x);
  const int mt = bid / a.ntiles, nt = bid % a.ntiles;
  const int m0 = mt * F8BM, n0 = nt * BN;
  const long Mrows = (long)a.n * a.rh * a.rw;
  if ((long)m0 >= Mrows) return;

  // activation scale from the amax partials (every block reduces the same 256 values in the same order)
  {
    float m = a.amax_part[tid];
    __shared__ float sm[256];
    sm[tid] = m;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (tid < o) sm[tid] = fmaxf(sm[tid], sm[tid + o]);
      __syncthreads();
    }
    if (tid == 0) s_inv = act_scale_pow2(sm[0]);
    __syncthreads();
  }
  const float inv_sa = s_inv;  // q = x / inv_sa, dequantised by inv_sa in the epilogue
  // bf16 bits of 448 * inv_sa (exact: inv_sa is a power of two), in both halves: the saturation bound
  const unsigned lim = __float_as_uint(fminf(448.f * inv_sa, 3.0e38f)) >> 16, lim2 = lim | (lim << 16);

  const int hw = a.rh * a.rw;
  const int kc = tid & 15;  // this thread's 8-element position within the 128-wide step
  int r_y[A_CH], r_x[A_CH], r_off[A_CH];
  bool r_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const long m = (long)m0 + (tid >> 4) + 16 * i;
    r_ok[i] = m < Mrows;
    const long mm = r_ok[i] ? m : 0;
    const int img = (int)(mm / hw);
    const int rem = (int)(mm - (long)img * hw);
    r_y[i] = (rem / a.rw) * a.str - a.ph;
    r_x[i] = (rem % a.rw) * a.str - a.pw;
    r_off[i] = ((img * a.sh_ + r_y[i]) * a.sw_ + r_x[i]) * a.scs + a.sco;
  }
  const int ksteps = (a.ktot + F8BK - 1) / F8BK;
  const int ntaps = a.ktot / a.sc;
  int ta = (kc * 8) / a.sc, ca = kc * 8 - ta * a.sc;
  int kh = ta / a.s, kw = ta - kh * a.s;
  auto advance = [&]() {
    ca += F8BK;
    while (ca >= a.sc) {
      ca -= a.sc;
      ++ta;
      if (++kw >= a.s) {
        kw = 0;
        ++kh;
      }
    }
  };
  constexpr unsigned OOR = 0x7FFFFFF0u;
  const __amdgpu_buffer_rsrc_t src_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, a.src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wt_rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, a.wt_bytes, 0x00020000);
  // B chunks (16 fp8 = 16 reduction elements): chunk q = tid + 256 i -> row q >> 3, position (q & 7) * 16
  const int b_row = tid >> 3, b_pos = (tid & 7) * 16;
  u32x4 ra[A_CH], rb[B_CH];
  auto load = [&](int t) {
    const bool kok = ta < ntaps;
    const int toff = (kh * a.sw_ + kw) * a.scs + ca;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const bool ok = kok && r_ok[i] && (unsigned)(r_y[i] + kh) < (unsigned)a.sh_ &&
                      (unsigned)(r_x[i] + kw) < (unsigned)a.sw_;
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(src_rs, ok ? (unsigned)(r_off[i] + toff) * 2u : OOR, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = n0 + b_row + 32 * i, kp = t * F8BK + b_pos;
      const bool ok = tid + 256 * i < B_TOT && row < a.N && kp < a.ktot;
      rb[i] = __builtin_amdgcn_raw_buffer_load_b128(wt_rs, ok ? (unsigned)((long)row * a.ktot + kp) : OOR, 0, 0);
    }
    advance();
  };
  u16x2 xbits = {0, 0};
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      *reinterpret_cast<u32x2*>(&As[((tid >> 4) + 16 * i) * F8P + kc * 8]) = to_fp8x8(ra[i], inv_sa, lim2, xbits);
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      if (tid + 256 * i < B_TOT) *reinterpret_cast<u32x4*>(&Bs[(b_row + 32 * i) * F8P + b_pos]) = rb[i];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int wr0 = wm * WROWS, wc0 = wn * WCOLS;
  auto frag = [&](const uint8_t* base, int row) {
    const u32x4 lo = *reinterpret_cast<const u32x4*>(base + row * F8P + 32 * (lane >> 4));
    const u32x4 hi = *reinterpret_cast<const u32x4*>(base + row * F8P + 32 * (lane >> 4) + 16);
    i32x8 f;
    f[0] = (int)lo[0]; f[1] = (int)lo[1]; f[2] = (int)lo[2]; f[3] = (int)lo[3];
    f[4] = (int)hi[0]; f[5] = (int)hi[1]; f[6] = (int)hi[2]; f[7] = (int)hi[3];
    return f;
  };
  auto compute = [&]() {
    i32x8 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[i] = frag(As, wr0 + i * 16 + (lane & 15));
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = frag(Bs, wc0 + j * 16 + (lane & 15));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[i], fb[j], acc[i][j], 0, 0, 0, 127, 0, 127);
  };
  if (ksteps > 0) {
    load(0);
    store();
    __syncthreads();
  }
  for (int t = 0; t < ksteps; ++t) {
    if (t + 1 < ksteps) load(t + 1);
    compute();
    __syncthreads();
    if (t + 1 < ksteps) {
      store();
      __syncthreads();
    }
  }

  if (a.amax_next) {  // this step's input maximum for the next step's scale: one atomic per wave
    float xmax = __uint_as_float((unsigned)(xbits[0] > xbits[1] ? xbits[0] : xbits[1]) << 16);
    for (int o = 32; o > 0; o >>= 1) xmax = fmaxf(xmax, __shfl_xor(xmax, o, 64));
    if (lane == 0 && xmax > 0.f)
      atomicMax(reinterpret_cast<unsigned*>(a.amax_next) + (blockIdx.x & (AMAX_BLOCKS - 1)), __float_as_uint(xmax));
  }
  // ---- epilogue: rescale, bias, bf16 image of the tile in LDS, 16-byte row stores, BN partial statistics ----
  __bf16* Os = reinterpret_cast<__bf16*>(lds);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wc0 + j * 16 + (lane & 15);
    const bool cok = n0 + col < a.N;
    const float b = (a.bias && cok) ? a.bias[n0 + col] : 0.f;
    const float rs = cok ? inv_sa * a.wscale[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Os[(wr0 + i * 16 + 4 * (lane >> 4) + e) * OPITCH + col] = (__bf16)(acc[i][j][e] * rs + b);
  }
  __syncthreads();
  constexpr int CPR = BN / 8, RPP = 256 / CPR;
  const int oc = tid % CPR, orow = tid / CPR;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  const bool col_ok = n0 + oc * 8 < a.N;
  for (int r = orow; r < F8BM; r += RPP) {
    const long m = (long)m0 + r;
    if (m >= Mrows || !col_ok) continue;
    const u32x4 v = *reinterpret_cast<const u32x4*>(&Os[r * OPITCH + oc * 8]);
    st16(a.out + m * a.ocs + a.oco + n0 + oc * 8, v);
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
  if (a.stats) {
    float (*red)[RG][BN] = reinterpret_cast<float (*)[RG][BN]>(lds);
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
      a.stats[(long)mt * 2 * a.N + n0 + tid] = x1;
      a.stats[(long)mt * 2 * a.N + a.N + n0 + tid] = x2;
    }
  }
}

}  // namespace adr

using namespace adr;

extern "C" int adr_fp8_amax_blocks(void) { return AMAX_BLOCKS; }

extern "C" int adr_conv2d_fwd_fp8_stat_tiles(const adr_conv_desc* d) { return cdiv((long)d->n * d->ho * d->wo, F8BM); }

extern "C" int adr_amax_bf16(const void* x, int cs, int co, long npix, int C, float* part, void* stream) {
  ADR_REQUIRE(C % 8 == 0 && cs % 8 == 0 && co % 8 == 0 && npix > 0, "amax_bf16: C=%d cs=%d co=%d", C, cs, co);
  hipLaunchKernelGGL(amax_bf16_kernel, dim3(AMAX_BLOCKS), dim3(256), 0, (hipStream_t)stream, (const __bf16*)x, cs, co,
                     npix, C, part);
  return check_launch("adr_amax_bf16");
}

extern "C" int adr_pack_weight_fp8(const float* w, int K, int C, int Cp, int RS, uint8_t* out, float* inv_scale,
                                   float* amax_cur, float* amax_prev, void* stream) {
  ADR_REQUIRE(K > 0 && C > 0 && Cp >= C && RS > 0 && (!amax_cur == !amax_prev), "pack_weight_fp8: K=%d C=%d Cp=%d RS=%d",
              K, C, Cp, RS);
  hipLaunchKernelGGL(pack_fp8_kernel, dim3(K), dim3(256), 0, (hipStream_t)stream, w, C, Cp, RS, out, inv_scale,
                     amax_cur, amax_prev);
  return check_launch("adr_pack_weight_fp8");
}

// 1 when the fp8 forward engine takes this contraction (stride 1 or 2, C a multiple of 16, K >= 64)
extern "C" int adr_conv2d_fp8_supported(const adr_conv_desc* d) {
  return d && d->dtype == ADR_BF16 && d->stride_h == d->stride_w && d->c % 16 == 0 && d->k % 8 == 0 && d->k >= 64 &&
         d->x_cstride % 8 == 0 && d->x_coff % 8 == 0 && d->y_cstride % 8 == 0 && d->y_coff % 8 == 0 &&
         (long)d->n * d->h * d->w * d->x_cstride < (1l << 30) && (long)d->k * d->c * d->r * d->s < (1l << 31);
}

extern "C" int adr_conv2d_fwd_fp8(const adr_conv_desc* d, const void* x, const uint8_t* w_fp8, const float* w_inv_scale,
                                  const float* amax_part, float* amax_next, const float* bias, void* y, float* stats,
                                  void* stream) {
  ADR_REQUIRE(adr_conv2d_fp8_supported(d), "conv fwd (fp8): unsupported contraction (C=%d K=%d)", d ? d->c : 0,
              d ? d->k : 0);
  const int ho = (d->h + 2 * d->pad_h - d->r) / d->stride_h + 1, wo = (d->w + 2 * d->pad_w - d->s) / d->stride_w + 1;
  ADR_REQUIRE(ho == d->ho && wo == d->wo, "conv fwd (fp8): output size mismatch");
  Fp8Args g{};
  g.src = (const __bf16*)x; g.wt = w_fp8; g.wscale = w_inv_scale; g.amax_part = amax_part; g.amax_next = amax_next;
  g.out = (__bf16*)y; g.bias = bias; g.stats = stats;
  g.n = d->n; g.sh_ = d->h; g.sw_ = d->w; g.scs = d->x_cstride; g.sco = d->x_coff; g.sc = d->c;
  g.rh = d->ho; g.rw = d->wo; g.ocs = d->y_cstride; g.oco = d->y_coff;
  g.r = d->r; g.s = d->s; g.str = d->stride_h; g.ph = d->pad_h; g.pw = d->pad_w;
  g.N = d->k; g.ktot = d->r * d->s * d->c;
  g.src_bytes = (int)(2l * d->n * d->h * d->w * d->x_cstride);
  g.wt_bytes = (int)((long)g.N * g.ktot);
  const int bn = d->k > 64 ? 128 : 64;
  g.ntiles = cdiv(g.N, bn);
  dim3 grid(cdiv((long)d->n * d->ho * d->wo, F8BM) * g.ntiles);
  hipStream_t st = (hipStream_t)stream;
  if (bn == 128) hipLaunchKernelGGL((conv_fp8_kernel<128>), grid, dim3(256), 0, st, g);
  else hipLaunchKernelGGL((conv_fp8_kernel<64>), grid, dim3(256), 0, st, g);
  return check_launch("adr_conv2d_fwd_fp8");
}
