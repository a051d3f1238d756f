/* libadr_hip — C ABI of the MI355X-native YOLO-AD-Refine hot path (gfx950 / CDNA4).
 *
 * Conventions (all entry points):
 *   - Return ADR_OK (0) on success, a non-zero adr_status otherwise; adr_last_error() (thread-local) has text.
 *     The Python shim raises RuntimeError, as the reference's native ops do (AT_ASSERTM -> RuntimeError,
 *     reference ultralytics/nn/modules/ops_dscn/src/cuda/dscn_cuda.cu).
 *   - The caller owns every buffer (outputs and workspaces included); the library never allocates device
 *     memory and keeps no mutable global state. Every launch is ordered on the `stream` argument
 *     (a hipStream_t passed as void*), normally PyTorch's current stream.
 *   - Activations are NHWC ("channels_last"): pixel-major, channels contiguous, with a per-pixel channel
 *     stride and a channel offset so channel slices of concat buffers are zero-copy views.
 *   - Weights of dense convolutions are KRSC (a PyTorch (K, C, R, S) parameter in channels_last memory).
 *   - dtype: ADR_F32 (exact-fp32 parity mode, MFMA 16x16x4 f32) or ADR_BF16 (bf16 storage, fp32 accumulate).
 * Each declaration names the reference interface it replaces (file:line, paths relative to the reference).
 */
#ifndef ADR_H_
#define ADR_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADR_ABI_VERSION 1

enum adr_status { ADR_OK = 0, ADR_ERR_BAD_ARG = 1, ADR_ERR_UNSUPPORTED = 2, ADR_ERR_LAUNCH = 3 };
enum adr_dtype { ADR_F32 = 0, ADR_BF16 = 1 };
enum adr_act { ADR_ACT_NONE = 0, ADR_ACT_SILU = 1, ADR_ACT_GELU = 2, ADR_ACT_RELU = 3, ADR_ACT_SIGMOID = 4,
               ADR_ACT_HSWISH = 5 };

int adr_abi_version(void);
const char* adr_last_error(void);
/* hipMemsetAsync(ptr, 0, bytes) on `stream` (zero-initialised gradient / accumulation buffers). */
int adr_memset_zero(void* ptr, size_t bytes, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * Dense convolution as implicit GEMM on MFMA.
 * Replaces: nn.Conv2d inside Conv (nn/modules/conv.py:44-50), Conv_GN (nn/modules/head.py:607-620),
 * nn.Conv2d / nn.ConvTranspose2d yaml rows (nn/tasks.py:1005-1016), nn.Linear in CrossScaleAttentionTSSA
 * (nn/modules/block.py:2426-2446) and the ELA Conv1d (block.py:1413). */
typedef struct adr_conv_desc {
  int n, h, w, c;           /* input batch, height, width, channels */
  int x_cstride, x_coff;    /* input view: elements between pixels, first channel */
  int k, r, s;              /* output channels, kernel height, kernel width */
  int stride_h, stride_w, pad_h, pad_w;
  int ho, wo;               /* output height/width (validated) */
  int y_cstride, y_coff;    /* output view */
  int dtype;                /* adr_dtype */
} adr_conv_desc;

/* y = conv(x, w) (+ bias[k]) (+ y if accumulate). If stats != NULL it receives per-row-tile partial
 * [tiles][2][k] (sum, sum of squares) of the stored outputs, tiles = adr_conv2d_fwd_stat_tiles(d). */
int adr_conv2d_fwd(const adr_conv_desc* d, const void* x, const void* w, const float* bias, void* y,
                   float* stats, int accumulate, void* stream);
int adr_conv2d_fwd_stat_tiles(const adr_conv_desc* d);
/* bf16 engine (adr_conv.hip): the same contractions with BK = 64 steps, tap-packed reductions for channel
 * counts below 64, LDS-staged 16-byte output rows and stride-2 DGRAD by output parity class. The forward takes
 * the KRSC weight; the data gradient takes the CRSK weight (adr_pack_weight2). 3x3 / stride-1 / pad-1 shapes with
 * reduction channels % 32 == 0, output channels % 32 == 0 and W % 8 == 0 run on 2-D output tiles with an LDS
 * halo tile (all nine taps from one staging). Stats tiles: adr_conv2d_fwd_bf16_stat_tiles(d) (tile geometry
 * depends on the path). */
int adr_conv2d_fwd_bf16(const adr_conv_desc* d, const void* x, const void* w_krsc, const float* bias, void* y,
                        float* stats, int accumulate, void* stream);
int adr_conv2d_dgrad_bf16(const adr_conv_desc* d, const void* dy, const void* w_crsk, const float* bias, void* dx,
                          int accumulate, void* stream);
int adr_conv2d_fwd_bf16_stat_tiles(const adr_conv_desc* d);
/* dx (+)= dgrad(dy, w_crsk) + addend in one launch (bf16 engine): `addend` is an NHWC view shaped like dx with
 * channel stride addend_cstride, added in the epilogue with a single rounding. Used by the fan-out gradient sink:
 * a residual add's pass-through gradient (nn/modules/block.py:354 `x + self.cv2(self.cv1(x))`, autograd's
 * gradient accumulation for a tensor read twice) folds into the first conv consumer's data gradient instead of
 * an elementwise add of its own. */
int adr_conv2d_dgrad_bf16_add(const adr_conv_desc* d, const void* dy, const void* w_crsk, void* dx, int accumulate,
                              const void* addend, int addend_cstride, void* stream);
/* Eval Conv-BN-act in one launch: y = act(conv(x, w_krsc) * scale + shift) on the bf16 engine, the BatchNorm's
 * running-statistics affine (scale/shift from adr_bn_finalize with training = 0) and the activation applied to the
 * fp32 accumulator before the bf16 store. Replaces the reference predictor's fused Conv.forward_fuse
 * (nn/modules/conv.py:52-54, after utils/torch_utils.py:fuse_conv_and_bn); no bias, statistics or accumulation. */
int adr_conv2d_fwd_bf16_act(const adr_conv_desc* d, const void* x, const void* w_krsc, const float* scale,
                            const float* shift, int act, void* y, void* stream);
/* fp8 (OCP e4m3) forward conv for BASELINE.json configs[4] (l-scale "fp8 MFMA conv path"), replacing the same
 * nn.Conv2d forward as adr_conv2d_fwd_bf16 (nn/modules/conv.py:44-50) on v_mfma_scale_f32_16x16x128_f8f6f4.
 * Delayed per-tensor activation scaling: sa = 448 / max(amax_part[0 .. adr_fp8_amax_blocks())) — last step's
 * |x| maxima of this conv's input, collected by the previous launch into amax_next (atomicMax slots, zeroed
 * and rotated by adr_pack_weight_fp8: prev <- cur, cur <- 0; seed both once with adr_amax_bf16). Weights per
 * output channel (adr_pack_weight_fp8: fp8 KRSC rows + 1/sw[k]). Output bf16 + optional BN partial statistics
 * per 128-row tile (adr_conv2d_fwd_fp8_stat_tiles). Backward stays on the bf16 engine. */
int adr_fp8_amax_blocks(void);
int adr_amax_bf16(const void* x, int cs, int co, long npix, int C, float* part, void* stream);
int adr_pack_weight_fp8(const float* w, int K, int C, int Cp, int RS, uint8_t* out, float* inv_scale,
                        float* amax_cur, float* amax_prev, void* stream);
int adr_conv2d_fp8_supported(const adr_conv_desc* d);
int adr_conv2d_fwd_fp8_stat_tiles(const adr_conv_desc* d);
int adr_conv2d_fwd_fp8(const adr_conv_desc* d, const void* x, const uint8_t* w_fp8, const float* w_inv_scale,
                       const float* amax_part, float* amax_next, const float* bias, void* y, float* stats,
                       void* stream);
/* Training Conv-BN-act fusion on the bf16 engine (the XF kernels): the operand of a conv is staged through a
 * training BatchNorm's affine + activation (forward) or its backward, so the elementwise pass and its launch
 * disappear. Reference: Conv.forward = act(bn(conv(x))) (nn/modules/conv.py:48-50) and its autograd backward.
 *   forward  (adr_conv2d_fwd_bf16_bnact): the conv input x is the producer's pre-BN output y (desc x view);
 *            the operand is z = act(y * scale + shift) (0 in the zero padding); z is side-written to `out`
 *            (every element exactly once) for the layer's other readers and the weight gradient.
 *   backward (adr_conv2d_dgrad_bf16_bnact): the data gradient of the conv that produced y, fed dz (the gradient of
 *            z = act(bn(y))); the operand is dy = A * g + B * y + C, g = dz * act'(y * scale + shift) (A / B / Cc
 *            from adr_bn_bwd_finalize), side-written to `out` for the weight gradient.
 * The operand values are bitwise those adr_affine_act / adr_affine_act_bwd store (same bf16 arithmetic).
 * act: ADR_ACT_NONE or ADR_ACT_SILU; at most 512 reduction channels. */
typedef struct adr_bnact_xf {
  const void* y;        /* backward: the BN input y (NHWC bf16 over the dz grid, channel stride y_cstride) */
  const float* scale;
  const float* shift;
  const float* A;       /* backward coefficients */
  const float* B;
  const float* Cc;
  void* out;            /* side output (z / dy), NHWC bf16, channel stride out_cstride */
  int y_cstride, out_cstride, act, pad_;
} adr_bnact_xf;
int adr_conv2d_fwd_bf16_bnact(const adr_conv_desc* d, const void* y, const void* w_krsc, void* out, float* stats,
                              const adr_bnact_xf* xf, void* stream);
/* Rows of its BatchNorm partial statistics (stats holds rows x 2 x K floats). */
int adr_conv2d_fwd_bf16_bnact_stat_tiles(const adr_conv_desc* d);
int adr_conv2d_dgrad_bf16_bnact(const adr_conv_desc* d, const void* dz, const void* w_crsk, void* dx, int accumulate,
                                const void* addend, int addend_cstride, const adr_bnact_xf* xf, void* stream);
/* BN-backward statistics in the data gradient's epilogue (BSTAT). When the conv's input x was the output
 * z = act(bn(y)) of a training BatchNorm-act and this conv was its only reader, the stored dx IS that BN's complete
 * dz: the epilogue reads y at the same pixel / channel and writes per-tile partials (sum g, sum g * y),
 * g = dz * act'(y * scale + shift) (bf16 arithmetic of adr_nc_reduce's backward mode), as [tiles][2][C] with
 * tiles = adr_conv2d_dgrad_bf16_stat_tiles(d, xf != NULL); adr_bn_bwd_finalize takes them in place of the
 * adr_nc_reduce pass. Replaces the statistics half of the BatchNorm2d backward of Conv (nn/modules/conv.py:48-50).
 * Column c of dx is BN channel c (y, scale, shift point at channel 0); act: ADR_ACT_NONE or ADR_ACT_SILU. */
typedef struct adr_bn_bstat {
  const void* y;        /* the BN input, NHWC bf16 over the dx grid, channel stride y_cstride */
  const float* scale;   /* the BN-act forward affine (adr_bn_finalize) */
  const float* shift;
  int y_cstride, act;
} adr_bn_bstat;
int adr_conv2d_dgrad_bf16_bstat(const adr_conv_desc* d, const void* dy, const void* w_crsk, void* dx, int accumulate,
                                const void* addend, int addend_cstride, const adr_bnact_xf* xf,
                                const adr_bn_bstat* bs, float* stats, void* stream);
int adr_conv2d_dgrad_bf16_stat_tiles(const adr_conv_desc* d, int xf);
/* Times x100 the XF kernel for this contraction stages each source element (column tiles x gathers per element):
 * the transform is per-staged-element VALU work, so the fusion pays only near 100. */
int adr_conv2d_bf16_xf_reuse(const adr_conv_desc* d, int dgrad);
/* Mangled name of the kernel the bf16 engine launches for this contraction (dgrad bit 0: the data gradient; bit 1:
 * the XF Conv-BN-act variant), written to buf (len >= 64) — the label the bench's roofline and rocprofv3 share. */
int adr_conv2d_bf16_kernel_symbol(const adr_conv_desc* d, int dgrad, char* buf, int len);
/* dx = conv_transpose(dy, w) (+ bias[c]) (+ dx if accumulate).  Also ConvTranspose2d forward
 * (nn.ConvTranspose2d weight (Cin_T, Cout_T, R, S) channels_last == KRSC of the equivalent conv). */
int adr_conv2d_dgrad(const adr_conv_desc* d, const void* dy, const void* w, const float* bias, void* dx,
                     int accumulate, void* stream);
/* dw[k][r][s][c] (fp32, += if accumulate) = sum over output pixels dy * im2col(x); split-K workspace. */
size_t adr_conv2d_wgrad_workspace(const adr_conv_desc* d);
int adr_conv2d_wgrad(const adr_conv_desc* d, const void* x, const void* dy, float* dw, int accumulate,
                     void* ws, size_t ws_bytes, void* stream);
/* The two phases of adr_conv2d_wgrad, for callers that schedule (or time) them separately:
 * partials writes [splits][k][r][s][c] fp32 slabs to `out` (splits = adr_conv2d_wgrad_splits(d); with one
 * split `out` may be dw itself, accumulate allowed for bf16), adr_wgrad_reduce sums the slabs in a fixed
 * order into dw (+= if accumulate). */
int adr_conv2d_wgrad_splits(const adr_conv_desc* d);
/* Many WGRAD partial launches in one call (bf16 engine): each job writes exactly what adr_conv2d_wgrad_partials(
 * &job->d, x, dy, out, accumulate) writes (same splits and tiles, bitwise), but the jobs on the generic tile kernel
 * are grouped by tile shape into one launch per shape. The trainer defers the weight gradients of a backward stage
 * and issues them here at the stage's end (reference: the per-conv weight gradients of nn.Conv2d's backward). */
typedef struct adr_wgrad_job {
  adr_conv_desc d;
  const void* x;
  const void* dy;
  float* out;
  int accumulate, pad_;
  float* bias;  /* NULL, or [splits][2][K] rows whose half 0 receives sum_p dy[p][k] per split (fused bias gradient:
                   the column sums nn.Conv2d's bias backward takes, reference nn/modules/conv.py:36-54 / head.py) */
} adr_wgrad_job;
int adr_conv2d_wgrad_partials_batched(const adr_wgrad_job* jobs, int count, void* stream);
/* The tile kernel a job of adr_conv2d_wgrad_partials_batched goes to: bm * 256 + bn of the grouped
 * wgrad_bf16_batched_kernel<bm, bn>, or 0 when the job runs its own thin / 3x3-halo kernel (bench timing labels). */
int adr_conv2d_wgrad_batched_tile(const adr_conv_desc* d);
int adr_conv2d_wgrad_partials(const adr_conv_desc* d, const void* x, const void* dy, float* out, int accumulate,
                              void* stream);
/* The bias gradient's column sums of dy computed by the weight-gradient GEMM that already holds dy in registers
 * (one extra MFMA per row tile against ones) instead of a separate pass over dy (adr_nc_reduce / the batched column
 * sums): fusable when the plan is the generic bf16 tile kernel with bm, bn >= 32 (adr_conv2d_wgrad_bias_fusable).
 * bias_part: [splits][2][K] floats, half 0 of each row written (reduce with adr_partial_sum, which = 0). */
int adr_conv2d_wgrad_bias_fusable(const adr_conv_desc* d);
int adr_conv2d_wgrad_partials_bias(const adr_conv_desc* d, const void* x, const void* dy, float* out, float* bias_part,
                                   void* stream);
int adr_wgrad_reduce(const float* part, float* dw, long n, int splits, int accumulate, void* stream);
/* The split sum fused with the KRSC -> (K, C, R, S) parameter layout (adr_unpack_weight_grad): part holds
 * `splits` slabs of split_stride floats whose first K*RS*Cp entries are [k][rs][c]; dst (+)= their sum at
 * (k, c, rs) (or (c, k, rs) with transpose_kc), padded channels c >= C dropped. */
int adr_wgrad_reduce_unpack(const float* part, long split_stride, int splits, float* dst, int K, int C, int Cp,
                            int RS, int transpose_kc, int accumulate, void* stream);
/* Deferred WGRAD reductions, many per launch (<= 56 entries each; more are split into several launches): each
 * entry is reduced and unpacked in the split order adr_wgrad_reduce_unpack uses below 256 splits.
 * `entries` is a host array (its contents travel in the kernel arguments). Two entries of one call must not
 * share a destination. */
typedef struct {
  const float* part;   /* [splits][K*RS*Cp] partials */
  float* dst;          /* (K, C, RS) parameter gradient (or (C, K, RS) with transpose_kc) */
  long split_stride;   /* floats between consecutive splits' slabs */
  int splits, K, C, Cp, RS, transpose_kc, accumulate, pad_;
} adr_wgrad_reduce_entry;
int adr_wgrad_reduce_batched(const adr_wgrad_reduce_entry* entries, int count, void* stream);


/* ---------------------------------------------------------------------------------------------------------
 * Normalisation + activation (NHWC). Replaces nn.BatchNorm2d+SiLU in Conv (nn/modules/conv.py:44-50),
 * nn.GroupNorm(16)+SiLU in Conv_GN / TaskDecomposition / DyDCNv2 (nn/modules/head.py:607-669, 751-782),
 * GroupNorm+Sigmoid in ELA_HSFPN (nn/modules/block.py:1413-1416), BN+GELU in ProgressiveFeatureFusion
 * (block.py:2589-2593), BN+Hardswish in CoordAtt (head.py:684-686).
 * Partial-statistics rows are [P][2][C] floats (sum, sum of squares — or sum g, sum g*x in backward). */
int adr_nc_reduce_chunks(int HW, int rows_per_chunk);
/* mode 0: stats of x;  mode 1: g = dz * act'(x*scale+shift) -> (sum g, sum g*x).  Output [N*chunks][2][C]. */
int adr_nc_reduce(int dtype, int mode, const void* x, int xcs, int xco, const void* dz, int dcs, int dco,
                  const float* scale, const float* shift, int per_sample, int act, int N, int HW, int C,
                  int rows_per_chunk, float* partial, void* stream);
int adr_bn_finalize(const float* partial, int P, int C, double count, const float* gamma, const float* beta,
                    float* running_mean, float* running_var, float momentum, float eps, int training,
                    float* scale, float* shift, float* mean, float* rstd, void* stream);
int adr_bn_bwd_finalize(const float* partial, int P, int C, double count, const float* mean, const float* rstd,
                        const float* gamma, float* dgamma, float* dbeta, float* A, float* B, float* Cc,
                        int training, int accumulate, void* stream);
int adr_gn_finalize(const float* partial, int N, int chunks, int C, int G, double count, const float* gamma,
                    const float* beta, float eps, float* scale, float* shift, float* mean, float* rstd,
                    void* stream);
int adr_gn_bwd_finalize(const float* partial, int N, int chunks, int C, int G, double count, const float* mean,
                        const float* rstd, const float* gamma, float* dgamma, float* dbeta, float* A, float* B,
                        float* Cc, int accumulate, void* stream);
/* GroupNorm(G) + activation fused per image (one 1024-thread workgroup per image: channel sums -> group
 * statistics -> z = act(x*scale + shift)); writes scale/shift per (image, channel) and mean/rstd per
 * (image, group) for the backward. Replaces adr_nc_reduce + adr_gn_finalize + adr_affine_act when
 * adr_gn_fused_supported(dtype, C, G) (the LDS plan fits). Conv_GN / TaskDecomposition / DyDCNv2
 * (nn/modules/head.py:607-669, 751-782), ELA_HSFPN's GroupNorm+Sigmoid (block.py:1413-1416). */
int adr_gn_fused_supported(int dtype, int C, int G);
int adr_gn_act_fused(int dtype, const void* x, int xcs, int xco, void* z, int zcs, int zco, const float* gamma,
                     const float* beta, float eps, int N, int HW, int C, int G, int act, float* scale,
                     float* shift, float* mean, float* rstd, void* stream);
/* Backward of adr_gn_act_fused per image: dx = A*g + B*x + C (g = dz * act'(x*scale+shift)), and the
 * per-image rows (sum g, sum g*x) -> partial[N][2][C] for adr_gn_param_grad. */
int adr_gn_act_bwd_fused(int dtype, const void* x, int xcs, int xco, const void* dz, int dcs, int dco, void* dx,
                         int ocs, int oco, const float* scale, const float* shift, const float* mean,
                         const float* rstd, const float* gamma, int N, int HW, int C, int G, int act,
                         float* partial, void* stream);
/* Level-packed GroupNorm (AYHead1.forward's per-level loop, nn/modules/head.py:1132-1176, run once over the three
 * levels): the levels' NHWC rows are stored back to back (level 0's N images, then level 1's, ...) and cut into
 * sub-images of `sub_rows` rows; an image of level l is k[l] consecutive sub-images (k: host array of `levels`
 * ints). partial is adr_nc_reduce's [N' sub-images][chunks][2][C] over that row space. Per (level, image):
 * group statistics over its k[l]*chunks rows, written replicated to each of its sub-images — mean/rstd
 * [N'][G], scale/shift [N'][C] with level l's gamma/beta (host arrays of `levels` device pointers, entries may
 * be NULL; the head's shared convs pass the same pointer for every level) — so adr_affine_act(per_sample) and
 * adr_gn_param_grad(_batched) over the N' sub-images give the per-image GroupNorm of each level. */
int adr_gn_finalize_packed(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows, int C,
                           int G, const void* const* gamma, const void* const* beta, float eps, float* scale,
                           float* shift, float* mean, float* rstd, void* stream);
/* Backward coefficients of the level-packed GroupNorm (partial from adr_nc_reduce RED_BWD over the sub-images):
 * dx = A*g + B*x + C with A, B, C [N'][C] replicated per sub-image (adr_gn_bwd_finalize's gn_bwd_coef per image). */
/* Gradient of per-image gates s feeding a GroupNorm (TaskDecomposition, nn/modules/head.py:651-667 — replaces the
 * autograd of `weight * conv_weight` -> bmm -> gn for its gate): dL/ds = sum(dZ * Z) / s, computed as the exact
 * eps-residue eps * rstd^2 * sum(dY' * Zhat) per group from the backward's fp32 partial rows (sum g, sum g*x) and the
 * forward's mean / rstd (level-packed layout as adr_gn_bwd_coef_packed; an unpacked GN is levels 1, k {1}). gate /
 * dgate per sub-image [N']: the segment's value goes to its first sub-image, 0 to the others. */
int adr_gn_gate_grad(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows, int C, int G,
                     const void* const* gamma, const float* mean, const float* rstd, float eps, const float* gate,
                     float* dgate, void* stream);
int adr_gn_bwd_coef_packed(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows, int C,
                           int G, const void* const* gamma, const float* mean, const float* rstd, float* A, float* B,
                           float* Cc, void* stream);
/* Per (level, image) segment of the packed row space (segments level-major: s = l * N + n), rows of C fp32:
 * v = in[s] (in_per_seg) or the sum of in[j] over the segment's sub-images j (in: [N'][C]), times
 * 1 / (k[l] * sub_rows) when `mean`; written to out[s] (out_per_seg, out: [levels * N][C]) or to every sub-image
 * row of the segment. With `in` the per-sub-image pixel sums and (0, 1, 1) this is the head's global average pool
 * (head.py:1142) for every level at once; (1, 0, 0) expands a per-image gate (TaskDecomposition's layer attention,
 * head.py:655-662) to the sub-images; (0, 1, 0) is that expansion's backward, (1, 0, 1) the pool's. */
int adr_seg_reduce_packed(const float* in, int in_per_seg, int out_per_seg, int mean, int levels, const int* k, int N,
                          int sub_rows, int C, float* out, void* stream);
/* Level-packed training BatchNorm (CoordAtt's bn1 on the pooled planes of the three head levels,
 * nn/modules/head.py:684-700, one call instead of one per level): rows of level l are the N * k[l] sub-images
 * starting at sub-image N * (k[0] + ... + k[l-1]); partial from adr_nc_reduce over the sub-images. Statistics per
 * level, running statistics updated level by level in order (the reference's per-level calls); scale / shift
 * [N'][C] per sub-image, mean / rstd [levels][C]. The backward writes A / B / C per sub-image and dgamma / dbeta
 * summed over the levels (+= with accumulate). */
int adr_bn_finalize_packed(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows, int C,
                           const float* gamma, const float* beta, float* running_mean, float* running_var,
                           float momentum, float eps, float* scale, float* shift, float* mean, float* rstd,
                           void* stream);
int adr_bn_bwd_finalize_packed(const float* partial, int levels, const int* k, int N, int chunks, int sub_rows, int C,
                               const float* mean, const float* rstd, const float* gamma, float* dgamma, float* dbeta,
                               float* A, float* B, float* Cc, int accumulate, void* stream);
/* dgamma / dbeta (+)= column sums over images of the adr_gn_act_bwd_fused rows. */
int adr_gn_param_grad(const float* partial, int N, int C, int G, const float* mean, const float* rstd,
                      float* dgamma, float* dbeta, int accumulate, void* stream);
/* z = act(x * scale + shift), scale/shift per channel or (per_sample) per (image, channel). */
int adr_affine_act(int dtype, const void* x, int xcs, int xco, void* z, int zcs, int zco, const float* scale,
                   const float* shift, int per_sample, int act, int N, int HW, int C, void* stream);
/* z = act(x*scale+shift) + res, bitwise the adr_affine_act + adr_ew add pair (BN-act ending a residual branch:
 * Bottleneck's x + cv2(cv1(x)), nn/modules/block.py:341-354). */
int adr_affine_act_res(int dtype, const void* x, int xcs, int xco, const void* res, int rcs, void* z, int zcs, int zco,
                       const float* scale, const float* shift, int per_sample, int act, int N, int HW, int C,
                       void* stream);
/* dx (+)= A*g + B*x + C, g = dz * act'(x*scale+shift). */
int adr_affine_act_bwd(int dtype, const void* x, int xcs, int xco, const void* dz, int dcs, int dco, void* dx,
                       int ocs, int oco, const float* scale, const float* shift, const float* A, const float* B,
                       const float* Cc, int per_sample, int coef_per_sample, int act, int N, int HW, int C,
                       int accumulate, void* stream);
/* out[c] (+)= sum_p partial[p][which][c] */
int adr_partial_sum(const float* partial, int P, int C, int which, float* out, int accumulate, void* stream);
/* Many adr_partial_sum reductions in one launch (<= 80 entries each; more are split), each reduced in the same
 * order as adr_partial_sum. `entries` is a host array (kernel arguments); destinations must be distinct. */
typedef struct {
  const float* partial;
  float* out;
  int P, C, which, accumulate;
} adr_psum_entry;
int adr_partial_sum_batched(const adr_psum_entry* entries, int count, void* stream);
/* Many bf16 adr_nc_reduce(RED_STATS) column-sum reductions in one launch (the bias gradients of every biased conv,
 * nn.Conv2d(bias=True) rows, nn/tasks.py:1005-1016, deferred to the end of backward): entry e reads x (NHWC,
 * channel stride xcs, N images of HW pixels, C channels) in chunks of rows_per_chunk pixels and writes
 * partial[(n * chunks + chunk)][2][C] exactly as adr_nc_reduce does (chunks = ceil(HW / rows_per_chunk)). */
typedef struct adr_colsum_entry {
  const void* x;
  float* partial;
  int xcs, N, HW, C, rows_per_chunk, chunks;
} adr_colsum_entry;
int adr_nc_reduce_batched(const adr_colsum_entry* entries, int count, void* stream);
/* Many GroupNorm dgamma / dbeta reductions (the gn_bwd_param part of adr_gn_bwd_finalize / adr_gn_param_grad,
 * nn.GroupNorm in Conv_GN, nn/modules/head.py:607-620) in as few launches as the destinations allow: entries
 * with a destination already in the current launch go to the next one, so repeated modules (the AYHead's shared
 * per-level convs) accumulate in entry order. partial is [N][chunks][2][C] (sum g, sum g*x). */
typedef struct adr_gnparam_entry {
  const float* partial;
  const float* mean;
  const float* rstd;
  float* dgamma;
  float* dbeta;
  int N, chunks, C, G, accumulate, pad_;
} adr_gnparam_entry;
int adr_gn_param_grad_batched(const adr_gnparam_entry* entries, int count, void* stream);
/* Deferred scalar parameter gradients, batched: out[0] = sum over all pixels and channels of x * dz for each entry
 * (bf16 NHWC views) — the Scale (nn/modules/head.py:783 Scale, `x * self.scale`) and weighted-sum weight gradients,
 * i.e. adr_dot_reduce + adr_nc_collapse(sum_n = sum_c = 1) for many tensors in two launches. partial is the
 * caller's [N][chunks][2][C] workspace per entry. */
typedef struct adr_dotsum_entry {
  const void* x;
  const void* dz;
  float* partial;
  float* out;
  int xcs, dcs, N, HW, C, rows_per_chunk, chunks, pad_;
} adr_dotsum_entry;
int adr_dotsum_batched(const adr_dotsum_entry* entries, int count, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * Parameter plumbing: (K, C, R*S) fp32 <-> KRSC operand (compute dtype); transpose_kc=1 reads a
 * ConvTranspose2d weight (C_in_T=K, C_out_T=C, R, S) as the equivalent conv's KRSC weight. */
int adr_pack_weight(int dtype, const float* src, void* dst, int K, int C, int Cp, int RS, int transpose_kc,
                    void* stream);
/* Both GEMM operand layouts of one weight in one pass: KRSC [Kp][RS][Cp] (forward rows) and CRSK [Cp][RS][Kp]
 * (data-gradient rows), zero-padded for k >= K / c >= C; transpose_kc as adr_pack_weight. */
int adr_pack_weight2(int dtype, const float* src, void* krsc, void* crsk, int K, int Kp, int C, int Cp, int RS,
                     int transpose_kc, void* stream);
/* Many adr_pack_weight2 calls in one launch: table = nchunks device rows {const float* src; void* krsc;
 * void* crsk; int K, Kp, C, Cp, RS, transpose_kc; long start, len;} (adr_pack_chunk_size() bytes each), each row
 * packing elements [start, start+len) of one weight (the trainer packs every conv weight once per step). */
int adr_pack_chunk_size(void);
int adr_pack_weight2_batched(int dtype, const void* table, int nchunks, void* stream);
/* The same packing by 64 x 64 tiles (what the trainer launches once per step): table = ntiles device rows
 * {const float* src; void* krsc; void* crsk; int K, Kp, C, Cp, RS, transpose_kc; int t, k0, c0, pad;}
 * (adr_pack_tile_size() bytes each), each row packing tap t, rows [k0, k0+64) x columns [c0, c0+64) of one weight
 * (clipped to Kp x Cp; zeros beyond K / C) into both layouts with coalesced stores. */
int adr_pack_tile_size(void);
int adr_pack_weight2_tiled(int dtype, const void* table, int ntiles, void* stream);
int adr_unpack_weight_grad(const float* src, float* dst, int K, int C, int Cp, int RS, int transpose_kc,
                           int accumulate, void* stream);
/* Stem: model.0 Conv(3, K, 3, 2) (nn/modules/conv.py:36-54, the first yaml row) straight from the fp32 NCHW
 * image batch (detect/train.py:57-59), bf16 compute (adr_stem.hip). Forward writes y (N, H/2, W/2, K) NHWC bf16
 * and, when stats != NULL, [adr_stem_fwd_tiles(N, Ho)][2][K] BatchNorm partial sums of the stored values.
 * The weight gradient writes dw (K, 3, 3, 3) fp32 (+= if accumulate). K in {16, 32, 64}. */
int adr_stem_fwd_tiles(int N, int Ho);
int adr_stem_conv_fwd(const float* img, int N, int H, int W, const float* w, int K, void* y, int ycs, float* stats,
                      void* stream);
size_t adr_stem_wgrad_workspace(int N, int H, int W, int K);
int adr_stem_conv_wgrad(const float* img, int N, int H, int W, const void* dy, int dcs, int K, float* dw,
                        int accumulate, float* ws, size_t ws_bytes, void* stream);
/* The same on the dataloader's uint8 NCHW batch: preprocess_batch's .float() / 255 (detect/train.py:57-59) is
 * applied while the rows are staged, so the float image never exists in HBM. */
int adr_stem_conv_fwd_u8(const uint8_t* img, int N, int H, int W, const float* w, int K, void* y, int ycs,
                         float* stats, void* stream);
int adr_stem_conv_wgrad_u8(const uint8_t* img, int N, int H, int W, const void* dy, int dcs, int K, float* dw,
                           int accumulate, float* ws, size_t ws_bytes, void* stream);
/* NCHW fp32 images (detect/train.py:57-59 preprocess output) -> NHWC compute dtype, channels padded to Cp. */
int adr_image_to_nhwc(int dtype, const float* src, void* dst, int N, int C, int H, int W, int Cp, void* stream);
/* uint8 NCHW images -> NHWC compute dtype, value / 255 (preprocess_batch), channels padded to Cp. */
int adr_image_u8_to_nhwc(int dtype, const uint8_t* src, void* dst, int N, int C, int H, int W, int Cp, void* stream);
int adr_cast(int src_dtype, const void* src, int dst_dtype, void* dst, long n, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * Elementwise glue on NHWC views (npix pixels x C channels, per-pixel channel strides).
 * op: 0 copy (torch.cat pieces, block.py:244-247) | 1 o = ca*a + cb*b (Fusion bifpn block.py:1532-1535,
 * residual adds block.py:353, Add :1448-1453) | 2 o = a*b (Multiply :1442-1447) | 3 o = a + b*c
 * (CrossTaskInteraction head.py:744-745) | 4 o = act(a) | 5 o = b*act'(a) | 6 o = a+b+c | 8 o = T(a*b) + c (the
 * product rounded to the dtype first: Add(Multiply(a, b), c), bitwise the op-2 + op-1 pair).
 * ca / cb are device scalars (null = 1). accumulate: o += result. */
int adr_ew(int dtype, int op, int act, const void* a, int acs, const void* b, int bcs, const void* c, int ccs,
           void* o, int ocs, long npix, int C, const float* ca, const float* cb, int accumulate, void* stream);
/* o (+)= x * g[n*gns + c*gcs] (+ res): per-image / per-channel broadcast scale (TaskDecomposition
 * head.py:657-664, Scale head.py:797, residual_weight block.py:2680). */
int adr_bcast_mul(int dtype, const void* x, int xcs, const float* g, int gns, int gcs, const void* res, int rcs,
                  void* o, int ocs, int N, int HW, int C, int accumulate, void* stream);
/* partial[n][chunk][0][c] = sum x*dz, [1][c] = sum dz (x may be NULL); then collapse over chunks (+n, +c). */
int adr_dot_reduce(int dtype, const void* x, int xcs, const void* dz, int dcs, int N, int HW, int C,
                   int rows_per_chunk, float* partial, void* stream);
int adr_nc_collapse(const float* partial, int N, int chunks, int C, int which, float* out, int sum_n, int sum_c,
                    int accumulate, void* stream);
/* y += a*x over n fp32 values (gradient accumulation into the trainer's flat gradient arena). */
int adr_axpy(long n, float a, const float* x, float* y, void* stream);
/* y_i += x_i for many (x, y, n) in one launch (<= 96 entries each; more are split); destinations distinct.
 * `entries` is a host array (kernel arguments). */
typedef struct {
  const float* x;
  float* y;
  long n;
} adr_axpy_entry;
int adr_axpy_batched(const adr_axpy_entry* entries, int count, void* stream);
/* The pieces of one torch.cat(dim=1) that their producers did not write in place, copied in ONE launch (bf16 NHWC,
 * 16-byte channel rows): dst[p][c] = src[p][c] for p < npix, c < C of each piece (reference torch.cat in Concat,
 * nn/modules/conv.py:322-335, and the neck / head concats); bitwise the per-piece adr_ew copies. */
typedef struct adr_copy_piece {
  const void* src;
  void* dst;
  int scs, dcs, C, pad_;
} adr_copy_piece;
int adr_copy_pieces(const adr_copy_piece* pieces, int count, long npix, void* stream);
/* BiFPN weights w = relu(fw)/(sum relu(fw)+eps) and backward (block.py:1532-1535). */
int adr_fusion_weights(const float* fw, int n, float eps, float* w, void* stream);
int adr_fusion_weights_bwd(const float* fw, int n, float eps, const float* dw, float* dfw, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * Pooling / resampling (NHWC). Max pool k x k stride 1 pad k/2 with uint8 argmax (SPPF block.py:177-196);
 * axis means + separable gate (ELA_HSFPN block.py:1408-1424, CoordAtt head.py:671-707); adaptive average
 * pooling (block.py:1558-1581, 2455); bilinear resize align_corners=False (block.py:2459-2462).
 * Axis-mean outputs / gate inputs are [n][l][c] planes addressed as base + n*stride_n + l*C + c. adr_gate_bwd's
 * zero_other (CoordAtt: both gate gradients span H + W rows): also write zeros to the rows the gate does not read
 * (dah rows H.., daw rows ..H of the (H + W)-row tensors; daw passed at row H as usual). */
int adr_maxpool(int dtype, const void* x, int xcs, void* y, int ycs, uint8_t* arg, int N, int H, int W, int C, int k,
                void* stream);
int adr_maxpool_bwd(int dtype, const void* dy, int dcs, const uint8_t* arg, void* dx, int ocs, int N, int H, int W,
                    int C, int k, int accumulate, void* stream);
int adr_axis_mean(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* oh, long ohn, void* ow,
                  long own, void* stream);
int adr_axis_mean_bwd(int dtype, const void* dh, long dhn, const void* dw, long dwn, void* dx, int ocs, int N, int H,
                      int W, int C, int accumulate, void* stream);
int adr_gate(int dtype, const void* x, int xcs, const void* ah, long ahn, const void* aw, long awn, void* o, int ocs,
             int N, int H, int W, int C, void* stream);
int adr_gate_bwd(int dtype, const void* x, int xcs, const void* ah, long ahn, const void* aw, long awn,
                 const void* dout, int dcs, void* dx, int ocs, void* dah, long dahn, void* daw, long dawn, int N,
                 int H, int W, int C, int accumulate, int zero_other, void* stream);
int adr_adapool(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* y, int ycs, int OH, int OW,
                void* stream);
int adr_adapool_bwd(int dtype, const void* dy, int dcs, int N, int H, int W, int C, void* dx, int ocs, int OH, int OW,
                    int accumulate, void* stream);
int adr_bilinear(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* y, int ycs, int OH, int OW,
                 void* stream);
int adr_bilinear_bwd(int dtype, const void* dy, int dcs, int N, int H, int W, int C, void* dx, int ocs, int OH,
                     int OW, int accumulate, void* stream);
/* nn.Upsample(scale_factor=s, mode='nearest') (yolo11.yaml head rows; torch upsample_nearest2d with an
 * integer factor: out[oh][ow] = x[oh/s][ow/s]). y may be a channel slice of a concat buffer (ycs). Backward
 * gathers the s x s block of dy per input pixel (no atomics). */
int adr_upsample_nearest(int dtype, const void* x, int xcs, int N, int H, int W, int C, void* y, int ycs, int s,
                         void* stream);
int adr_upsample_nearest_bwd(int dtype, const void* dy, int dcs, int N, int H, int W, int C, void* dx, int ocs, int s,
                             int accumulate, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * MLCA (block.py:1540-1584) fused: out = res + y * up(att(y)).  Saved tensors (fp32, caller-owned):
 * local [N][25][C], att [N][25][C], sig_l [N][25*C], sig_g [N][C]. */
int adr_mlca_fwd(int dtype, const void* y, int ycs, const void* res, int rcs, void* out, int ocs, int N, int H, int W,
                 int C, const float* wl, const float* wg, int k, float local_weight, float* local, float* att,
                 float* sig_l, float* sig_g, void* stream);
/* adr_mlca_bwd: dwl / dwg (k floats each) receive the two Conv1d weight gradients; with both NULL they are left as
 * per-image rows [N][2][k] (local conv in half 0, global in half 1) at float offset 2 * N * 25 * C of ws, for the
 * caller to reduce (adr_partial_sum(_batched) with P = N, C = k, which = 0 / 1: the trainer's deferred flush). */
size_t adr_mlca_bwd_workspace(int N, int C, int k);
int adr_mlca_bwd(int dtype, const void* y, int ycs, const void* dout, int dcs, void* dy, int ocs, int N, int H, int W,
                 int C, const float* wl, const float* wg, int k, float local_weight, const float* local,
                 const float* att, const float* sig_l, const float* sig_g, float* dwl, float* dwg, float* ws,
                 size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * AYHead (nn/modules/head.py:1049-1252).
 * DyDCNv2 / mmcv ModulatedDeformConv2d (head.py:751-782), 3x3, stride 1, pad 1, deform_groups 1. `om` holds
 * the spatial_conv_offset output: channels [0,18) offsets (2k = dy, 2k+1 = dx), [18,27) mask LOGITS (the
 * sigmoid of head.py:1156 is applied inside). cols: [N*H*W][9][C]. dx32: fp32 NHWC accumulation buffer
 * (zeroed by the caller). dom receives d(offset) and d(mask logit) in the om layout.
 * adr_dcn_col2im: deterministic = 0 accumulates dx32 with float atomics (mmcv's own col2im order-freedom);
 * deterministic != 0 (fp32 parity mode) accumulates it with one thread per (image, channel) in a fixed order:
 * bitwise repeatable. */
int adr_dcn_im2col(int dtype, const void* x, int xcs, const void* om, int omcs, void* cols, int N, int H, int W,
                   int C, void* stream);
int adr_dcn_col2im(int dtype, const void* x, int xcs, const void* om, int omcs, const void* dcols, float* dx32,
                   void* dom, int domcs, int N, int H, int W, int C, int deterministic, void* stream);
/* Fused bf16 DCNv2 (adr_dcn.hip; replaces im2col + GEMMs + col2im on the performance path; no column matrix in
 * HBM). C % 64 == 0, Cout % 64 == 0 (<= 256), omcs % 8 == 0 and >= 32.
 * adr_dcn_fwd_bf16: y[p][co] = sum W_krsc[co][t][c] * m * bilinear(x)  (w_krsc: bf16 [Cout][9][C]).
 * adr_dcn_wgrad_bf16: split-K partials part[split][Cout][9][C] (fp32) of dW, `splits` from
 *   adr_dcn_wgrad_bf16_splits; reduce with adr_wgrad_reduce_unpack(K=Cout, C=C, RS=9).
 * adr_dcn_bwd_bf16 (C == Cout in {64, 128, 256}): dx = input gradient (bf16, every element written once, gathered
 *   by destination tile), dom = offset / mask-logit gradient (channels [0,27), [27,32) written as zeros; domcs >=
 *   32); w_t: bf16 [9][C][Cout] (adr_dcn_weight_t). dxf (fp32, N*H*W*C) and tile_flags (adr_dcn_bwd_tiles ints)
 *   are persistent scratch that must be zero on entry and are zero again on return: corners whose source lies more
 *   than ~2 px outside the destination tile are added to dxf with float atomics and folded into dx by a second
 *   launch (with |offsets| < 2 px there are none and dx is bitwise repeatable). */
int adr_dcn_fwd_bf16(const void* x, int xcs, const void* om, int omcs, const void* w_krsc, void* y, int ycs, int N,
                     int H, int W, int C, int Cout, void* stream);
int adr_dcn_wgrad_bf16_splits(int N, int H, int W, int C, int Cout);
int adr_dcn_wgrad_bf16(const void* x, int xcs, const void* om, int omcs, const void* dy, int dycs, float* part,
                       int splits, int N, int H, int W, int C, int Cout, void* stream);
int adr_dcn_bwd_bf16(const void* x, int xcs, const void* om, int omcs, const void* dy, int dycs, const void* w_t,
                     void* dx, int dxcs, void* dom, int domcs, float* dxf, int* tile_flags, int N, int H, int W, int C,
                     int Cout, void* stream);
int adr_dcn_bwd_tiles(int N, int H, int W);
/* The AYHead's pyramid levels of one DyDCNv2 call per launch (LevelDCNFn; reference head.py:751-782 runs the module
 * per level): each writes, for every level, exactly what adr_dcn_{fwd,wgrad,bwd}_bf16 write for that level alone
 * (same blocks and arithmetic: bitwise), one launch for all levels (bwd: plus one far-corner launch). Per level:
 * pointers into the level-packed activations, its H x W, the wgrad partial slab and split count, the bwd far-corner
 * scratch (dxf: N*H*W*C fp32, flags: adr_dcn_bwd_tiles ints; zero on first use, left zero). Up to 3 levels. */
typedef struct adr_dcn_level {
  const void* x;
  const void* om;
  const void* dy;
  void* y;
  void* dx;
  void* dom;
  float* dxf;
  int* flags;
  float* part;
  int H, W, splits, pad_;
} adr_dcn_level;
int adr_dcn_fwd_bf16_levels(const adr_dcn_level* lv, int levels, int xcs, int omcs, const void* w_krsc, int ycs,
                            int N, int C, int Cout, void* stream);
int adr_dcn_wgrad_bf16_levels(const adr_dcn_level* lv, int levels, int xcs, int omcs, int dycs, int N, int C,
                              int Cout, void* stream);
int adr_dcn_bwd_bf16_levels(const adr_dcn_level* lv, int levels, int xcs, int omcs, int dycs, const void* w_t,
                            int dxcs, int domcs, int N, int C, int Cout, void* stream);
/* ---------------------------------------------------------------------------------------------------------
 * Training augmentation pixels (data/augment.py v8_transforms :2273-2335, through Format :2072-2100 and
 * YOLODataset.collate_fn, data/dataset.py:230-246): Mosaic canvas -> warpAffine (RandomPerspective) -> RandomHSV
 * -> RandomFlip -> CHW RGB, fused, one thread per output pixel, into out (B, 3, H, W) uint8. pool: the batch's
 * source images (HWC BGR uint8, resized as BaseDataset.load_image leaves them); descs: B device adr_aug_desc
 * records (4 tiles {int64 byte offset; int sw, x1a, y1a, x2a, y2a, x1b, y1b}, then int ntile, cw, ch, warp,
 * tab_off, lut_off, flip_ud, flip_lr, rgb, pad; size adr_augment_desc_size()); tables: per warped image adelta[W],
 * bdelta[W], X0[H], Y0[H] (cv::warpAffine fixed point, from the host); luts: 768 bytes (hue, sat, val) per image
 * with HSV (lut_off -1: none). Random draws, matrices and labels stay on the host (adrefine/data/augment.py). */
int adr_augment_u8(const void* pool, const void* descs, int B, const int* tables, const void* luts, void* out, int H,
                   int W, void* stream);
int adr_augment_desc_size(void);
/* W (Cout, C, 3, 3) fp32 -> [(tap*C + c)][Cout] operand for dcols = dy x W. */
int adr_dcn_weight_t(int dtype, const float* w, void* out, int Cout, int C, void* stream);
/* Per-image 2-layer gate MLP on pooled vectors: out = act2(W2 act1(W1 (in*in_scale) + b1) + b2);
 * act: 0 none, 3 relu, 4 sigmoid, 6 softmax. TaskDecomposition la_conv1/2 (head.py:633-650),
 * AdaptiveDynamicTanh importance_gate (block.py:2521-2531). */
int adr_gate_mlp(const float* in, float in_scale, int N, int Cin, const float* W1, const float* b1, int H1, int act1,
                 const float* W2, const float* b2, int H2, int act2, float* hidden, float* out, void* stream);
int adr_gate_mlp_bwd(const float* in, float in_scale, int N, int Cin, const float* W1, int H1, int act1,
                     const float* W2, int H2, int act2, const float* hidden, const float* out, const float* dout,
                     float* din, float* dW1, float* db1, float* dW2, float* db2, int accumulate, void* stream);
/* o (+)= g[n*gns + c*gcs] * s broadcast over pixels (adjoint of a global average pool). */
int adr_bcast_fill(int dtype, const float* g, int gns, int gcs, float s, void* o, int ocs, int N, int HW, int C,
                   int accumulate, void* stream);
/* o = x * p[pixel] (cls_prob gate, head.py:1172) and its backward (dx, dp = sum_c dout*x). */
int adr_mul_pixel(int dtype, const void* x, int xcs, const void* p, int pcs, void* o, int ocs, long npix, int C,
                  void* stream);
int adr_mul_pixel_bwd(int dtype, const void* x, int xcs, const void* p, int pcs, const void* dout, int dcs, void* dx,
                      int ocs, void* dp, int dpcs, long npix, int C, void* stream);
/* Eval decode (head.py:1181-1204): 3 level outputs (B, 4*reg_max+nc, Hi, Wi) NHWC -> y (B, 4+nc, A) fp32
 * = [xywh * stride (DFL expectation, dist2bbox), sigmoid(cls)]. */
int adr_detect_decode(int dtype, const void* f0, const void* f1, const void* f2, int cs0, int cs1, int cs2, int H0,
                      int W0, int H1, int W1, int H2, int W2, float s0, float s1, float s2, int B, int nc, int reg_max,
                      float* y, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * C2PTSSA (nn/modules/block.py:2376-2710).
 * Depthwise k x k conv + bias, stride 1, pad k/2 (ProgressiveFeatureFusion :2589-2593, EDFFN :2387);
 * weights (C, 1, k, k) fp32. dw / dx may be NULL to skip. */
int adr_dwconv_fwd(int dtype, const void* x, int xcs, const float* w, const float* b, void* y, int ycs, int N, int H,
                   int W, int C, int k, void* stream);
/* Eval DWConv-BN-act in one launch (bf16, whole-image kernel; adr_dwconv_fwd_act_supported says whether the shape
 * fits it): y = act(dwconv(x, w * scale) + shift), scale/shift from adr_bn_finalize with training = 0. Replaces
 * Conv.forward_fuse after fuse_conv_and_bn on a depthwise Conv (nn/modules/conv.py:52-54, 101-106). */
int adr_dwconv_fwd_act_supported(int H, int W, int C, int k);
int adr_dwconv_fwd_act(const void* x, int xcs, const float* w, const float* scale, const float* shift, int act,
                       void* y, int ycs, int N, int H, int W, int C, int k, void* stream);
size_t adr_dwconv_wgrad_workspace(int N, int H, int W, int C, int k);
int adr_dwconv_bwd(int dtype, const void* x, int xcs, const void* dy, int dcs, const float* w, void* dx, int ocs,
                   float* dw, int N, int H, int W, int C, int k, int accumulate, int dw_accumulate, float* ws,
                   size_t ws_bytes, void* stream);
/* The weight gradient's partial rows only ([*chunks][k*k][C] floats in ws); the trainer reduces them at its
 * deferred flush through adr_wgrad_reduce_batched (K = 1, RS = k*k, the [C][k*k] parameter layout). */
int adr_dwconv_wgrad_partials(int dtype, const void* x, int xcs, const void* dy, int dcs, int N, int H, int W, int C,
                              int k, float* ws, size_t ws_bytes, int* chunks, void* stream);
/* The same partial rows plus the depthwise conv's bias gradient (column sums of dy per image, from the staged dy
 * slab the weight gradient already holds): bias_part [N][2][C], half 0 written (adr_partial_sum, which = 0).
 * Only on the whole-image kernels (adr_dwconv_wgrad_bias_fusable). Reference: nn.Conv2d(groups=C, bias=True)'s bias
 * backward in the C2PTSSA / EDFFN / Mona depthwise convs (block.py:2376-2710). */
int adr_dwconv_wgrad_bias_fusable(int dtype, int H, int W, int C, int k, int xcs, int dcs);
int adr_dwconv_wgrad_partials_bias(int dtype, const void* x, int xcs, const void* dy, int dcs, int N, int H, int W,
                                   int C, int k, float* ws, size_t ws_bytes, float* bias_part, int* chunks,
                                   void* stream);
/* AdaptiveDynamicTanh (:2493-2577): y = (sum_i tanh(alpha_i x) imp[n,i]) * w[c] + b[c]; imp from adr_gate_mlp. */
int adr_adyt_fwd(int dtype, const void* x, int xcs, const float* alphas, const float* imp, const float* w,
                 const float* b, void* y, int ycs, int N, int HW, int C, void* stream);
size_t adr_adyt_bwd_workspace(int N, int HW, int C);
int adr_adyt_bwd(int dtype, const void* x, int xcs, const void* dout, int dcs, const float* alphas, const float* imp,
                 const float* w, void* dx, int ocs, float* dimp, float* dalpha, float* dw, float* db, int N, int HW,
                 int C, float* ws, size_t ws_bytes, void* stream);
/* TSSA token statistics for one scale (:2465-2477): q/k/v rows [b*Ntok + n] with channel stride cs, head h at
 * channels [h*D, (h+1)*D); out row of (b, n) is b*oimg + n (so the 3 scales stack into one buffer as
 * torch.stack(dim=1) does). Saves Pi/ss [B][heads][Ntok], attn [B][heads][D]. */
int adr_tssa_fwd(int dtype, const void* q, const void* k, const void* v, int cs, int B, int Ntok, int heads, int D,
                 const float* temp, void* out, int ocs, int oimg, float* Pi, float* ss, float* attn, void* stream);
int adr_tssa_bwd(int dtype, const void* q, const void* k, const void* v, int cs, int B, int Ntok, int heads, int D,
                 const float* temp, const void* dout, int dcs, int dimg, const float* Pi, const float* ss,
                 const float* attn, void* dq, void* dk, void* dv, int gcs, float* dtemp, float* ws, void* stream);
/* mean over S stacked token groups (fused_features.view(B, S, HW, C).mean(1), :2484-2486); backward spreads. */
int adr_group_mean(int dtype, const void* x, int xcs, int S, int HW, void* y, int ycs, int B, int C, int backward,
                   void* stream);
/* EDFFN 8x8-patch rfft2 * fft -> irfft2 (:2399-2413) as M_c = sum_uv fft[c,uv] basis[uv] (64x64, fp32). */
int adr_edffn_build(const float* w, const float* basis, int C, int nuv, float* M, void* stream);
int adr_edffn_fwd(int dtype, const void* x, int xcs, const float* M, void* y, int ycs, int N, int H, int W, int C,
                  void* stream);
size_t adr_edffn_bwd_workspace(int N, int H, int W, int C);
int adr_edffn_bwd(int dtype, const void* x, int xcs, const void* dy, int dcs, const float* M, const float* basis,
                  int nuv, void* dx, int ocs, float* dw, int N, int H, int W, int C, int dw_accumulate, float* ws,
                  size_t ws_bytes, void* stream);
/* Flash attention (no mask): o = softmax(q k^T * scale) v per (image, head); token rows [b*L + l], channel
 * strides cs / ocs. Head h's q / k / v start at channel qo / ko / vo + h*hs (hs = head stride); q/k width
 * qk_dim in {32, 64}, v / o width v_dim = 64 (o and dO hold head h at [h*64, h*64+64)).
 * Replaces: nn.MultiheadAttention core in CrossScaleAttentionTSSA (block.py:2432/:2484; qk 64, hs 64) and
 * Attention.forward of C2PSA/PSABlock (block.py:906-927, `(q^T k) * key_dim^-0.5`, softmax, `v @ attn^T`;
 * qk 32, hs 128). lse [B][heads][L] (natural log) is saved for the backward; dq/dk/dv use the same head
 * stride at offsets gqo/gko/gvo of a gcs-strided gradient buffer. */
int adr_attn_fwd(int dtype, const void* q, const void* k, const void* v, int cs, int qo, int ko, int vo, int hs,
                 void* o, int ocs, int B, int L, int heads, int qk_dim, int v_dim, float scale, float* lse,
                 void* stream);
int adr_attn_bwd(int dtype, const void* q, const void* k, const void* v, int cs, int qo, int ko, int vo, int hs,
                 const void* o, int ocs, const void* dout, int dcs, const float* lse, void* dq, void* dk, void* dv,
                 int gcs, int gqo, int gko, int gvo, int B, int L, int heads, int qk_dim, int v_dim, float scale,
                 float* dvec_ws, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * v8DetectionLoss (utils/loss.py:355-520) + TaskAlignedAssigner(topk 10, alpha 0.5, beta 6) (utils/tal.py)
 * + BboxLoss 0.5 CIoU + 0.5 NWD, DFLoss, SlideLoss BCE — value and gradient in one call, no host sync.
 * f0..f2: the three AYHead train outputs (B, 4*16+nc, Hi, Wi) NHWC; gt: (B, nmax, 5) fp32 device rows
 * [cls, x1, y1, x2, y2] in pixels (the reference's preprocess output, loss.py:392-408; zero rows = padding);
 * g0..g2 receive d(out[3]) / d(f) * grad_scale / B (dense NHWC, row stride 4*16+nc).
 * out (5 floats): box*7.5, cls*0.5, dfl*1.5 (the reference's loss.detach()), (sum)*B, number of positives. */
size_t adr_det_loss_workspace(int B, int nmax, int A);
int adr_det_loss(int dtype, const void* f0, const void* f1, const void* f2, int cs0, int cs1, int cs2, int H0, int W0,
                 int H1, int W1, int H2, int W2, float s0, float s1, float s2, int B, int nc, const float* gt,
                 int nmax, void* g0, void* g1, void* g2, float grad_scale, float box_gain, float cls_gain,
                 float dfl_gain, float* out, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * Trainer tail (engine/trainer.py:580-588, 753-813; utils/torch_utils.py:521-546) over a chunk table:
 * entry = {float* p; float* g; float* momentum_buf; float* ema; int64 n; int group; int pad}
 * (group 0 decayed weights, 1 norm weights, 2 biases, 3 buffers / frozen: EMA only);
 * chunk = {int entry; int pad; int64 start; int64 len}. Both tables live in device memory.
 * adr_opt_step: clip_grad_norm_(10) + SGD(momentum, nesterov, per-group lr / weight decay) + EMA
 * (ema = d*ema + (1-d)*p after the update) + optimizer.zero_grad() (trainer.py:586: each updated entry's
 * gradient is zeroed after it is consumed); norm_out (optional) receives the pre-clip total norm.
 * hyper is DEVICE memory: [lr0, lr1, lr2, wd0, wd1, wd2, momentum, nesterov, first, ema_decay] (first != 0:
 * momentum buffer initialised to the gradient), so a captured hipGraph of the step follows the schedule. */
int adr_opt_entry_size(void);
int adr_opt_chunk_size(void);
int adr_opt_step(const void* tab, const void* chunks, int nchunks, float* partial, float max_norm,
                 const float* hyper, float* norm_out, void* stream);
/* dst[0..n) = vals[0..n) (host array, n <= 16) as a stream-ordered kernel (values travel as kernel
 * arguments: no host buffer lifetime to manage, safe to enqueue ahead of a graph replay). */
int adr_set_f32(float* dst, const float* vals, int n, void* stream);
/* gradient (or, when g == NULL, value) gather into / scatter from a flat fp32 buffer at per-entry offsets
 * (the DDP all-reduce bucket). */
int adr_flat_copy(const void* tab, const void* chunks, int nchunks, float* flat, const int64_t* offsets,
                  int to_flat, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * 697 L10 variant C2TSSA_DYT_Mona_EDFFN (nn/modules/block.py:1624-1709, nn/modules/mona.py) — adr_mona.hip.
 * DynamicTanh (block.py:1624-1641): y = tanh(alpha x) w[c] + b[c]; backward writes dx and (+)= dalpha (scalar),
 * dw, db (accumulate) through a fixed-order two-stage reduction in ws. */
int adr_dyt_fwd(int dtype, const void* x, int xcs, const float* alpha, const float* w, const float* b, void* y,
                int ycs, long npix, int C, void* stream);
size_t adr_dyt_bwd_workspace(long npix, int C);
int adr_dyt_bwd(int dtype, const void* x, int xcs, const void* dy, int dcs, const float* alpha, const float* w,
                void* dx, int ocs, float* dalpha, float* dw, float* db, int accumulate, long npix, int C, float* ws,
                size_t ws_bytes, void* stream);
/* Mona prologue (mona.py:5-10, 55-58): y = LayerNorm_C(x; lw, lb, eps) * gamma[c] + x * gammax[c] per pixel;
 * saves per-pixel mean / rstd. C / (8 bf16 | 4 fp32) must be 8, 16, 32 or 64. */
int adr_ln_mix_fwd(int dtype, const void* x, int xcs, const float* lw, const float* lb, const float* gamma,
                   const float* gammax, void* y, int ycs, float* mean, float* rstd, long npix, int C, float eps,
                   void* stream);
size_t adr_ln_mix_bwd_workspace(long npix, int C);
int adr_ln_mix_bwd(int dtype, const void* x, int xcs, const void* dz, int dcs, const float* lw, const float* lb,
                   const float* gamma, const float* gammax, const float* mean, const float* rstd, void* dx, int ocs,
                   float* dlw, float* dlb, float* dgamma, float* dgammax, int accumulate, long npix, int C, float* ws,
                   size_t ws_bytes, void* stream);
/* AttentionTSSA core (block.py:1646-1683) on the qkv-linear output tokens w (B, N, H*D), token stride cs:
 * F.normalize over tokens, softmax over HEADS, out = -w * Pi * attn. state = adr_tssa1_state_floats floats
 * saved by the forward for the backward. D = 64. */
size_t adr_tssa1_state_floats(int B, int N, int H, int D);
int adr_tssa1_fwd(int dtype, const void* w, int cs, int B, int N, int H, int D, const float* temp, void* out, int ocs,
                  float* state, void* stream);
size_t adr_tssa1_bwd_workspace(int B, int N, int H, int D);
int adr_tssa1_bwd(int dtype, const void* w, int cs, int B, int N, int H, int D, const float* temp,
                  const float* state, const void* g, int gcs, void* dw, int dwcs, float* dtemp, int accumulate,
                  float* ws, size_t ws_bytes, void* stream);
/* Dropout (Mona.dropout, mona.py:44/63) with a counter-based hash mask keyed by the DEVICE seed (so a captured
 * graph draws a fresh mask per replay once adr_seed_advance is captured with it); the backward is the same
 * call on the gradient with the same seed. */
int adr_dropout(int dtype, const void* x, int xcs, void* y, int ycs, long npix, int C, float p, const int64_t* seed,
                void* stream);
int adr_seed_advance(int64_t* seed, void* stream);

/* ---------------------------------------------------------------------------------------------------------
 * Batched NMS: replaces utils/ops.py:163-312 non_max_suppression (agnostic=False, classes=None, nm=0,
 * labels=()) with its torchvision.ops.nms call. y = decoded head output (B, 4+nc, A) fp32, rows xywh then class
 * scores. multi != 0: every (anchor, class) with score > conf (multi_label=True, the val path); else best class.
 * agnostic: one NMS over all classes (single-label only); class_mask[nc] (nullable): the `classes` filter.
 * out (B, max_det, 6) rows x1 y1 x2 y2 conf cls in the reference's output order; nout[B] valid rows per image.
 * Requires A <= 16384, nc <= 1024, max_det <= 300. One persistent launch (one 1024-thread workgroup per CU, grid
 * barriers); ws (adr_nms_workspace bytes) must be zero-filled when first used and not shared by concurrent calls. */
/* Pairwise IoU of xyxy boxes a (N,4) and b (M,4) -> out (N,M), eps added to the union (utils/metrics.py:52-72);
 * the validator's TP matching (models/yolo/detect/val.py:213-214). */
int adr_box_iou(const float* a, int N, const float* b, int M, float eps, float* out, void* stream);
/* Validator TP matching of one image (replaces engine/validator.py:221-261 match_predictions, use_scipy=False):
 * iou (G, P) fp32 from adr_box_iou (labels x detections); a pair counts only when gt_cls[g] == pred_cls[p].
 * For each detection its best label (largest IoU; on exact ties the larger label index, as the reference's reversed
 * ascending sort orders small inputs); for each threshold thr[t] (fp32, compared as the reference's float32
 * `iou >= threshold`) a label is credited to the lowest-index detection whose best it is with IoU >= thr[t].
 * correct (P, T) uint8. P <= 2048, T <= 16; G unbounded. One workgroup, no atomics outside LDS (atomicMin order-free). */
int adr_match_predictions(const float* iou, int G, int P, const float* gt_cls, const float* pred_cls, const float* thr,
                          int T, unsigned char* correct, void* stream);
size_t adr_nms_workspace(int B, int nc, int A, int multi, int max_det);
int adr_nms(const float* y, int B, int nc, int A, float conf, float iou, int multi, int agnostic,
            const unsigned char* class_mask, int max_det, int max_nms, float max_wh, float* out, int* nout, void* ws,
            size_t ws_bytes, void* stream);
/* Return an adr_nms workspace to its first-use state in place (zero its control words on the stream) after a call
 * reported a grid-barrier timeout (nout < 0). The buffer is not freed, so a hipGraph that captured adr_nms on it
 * stays valid. */
int adr_nms_reset(void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ADR_H_ */
