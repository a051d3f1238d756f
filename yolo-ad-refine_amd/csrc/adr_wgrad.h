// bf16 WGRAD planner / launcher shared by adr_gemm.hip (ABI entry) and adr_wgrad.hip (kernel)
#pragma once
#include "adr_common.h"

namespace adr {
// sub-steps per WGRAD k-step for a BM x BN tile: enough that a wave issues ~32 MFMAs between barriers, at
// most 128 reduction rows per step
__host__ __device__ constexpr int wg_ku(int bm, int bn) {
  const int wm = bm / 16 < 2 ? bm / 16 : 2, wn = bn / 16 < 2 ? bn / 16 : 2;
  const int wk = 4 / (wm * wn), tm = bm / wm / 16, tn = bn / wn / 16;
  (void)tm;
  (void)tn;
  (void)wk;
  return 1;  // measured: deeper k-steps (2-4 sub-steps) are neutral on the 80x80 shapes and cost splits on 20x20
}
struct WgPlan {
  int bm, bn, R, tiles, splits;
  long per;  // reduction rows per split (multiple of R); for the 3x3 halo kernel: output tiles per split
  int tw3;   // > 0: 3x3 stride-1 halo-tile kernel (wgrad3_kernel<tw3>) with `per` 128-pixel tiles per split
  int thin;  // > 0: thin-channel 3x3 halo kernel (wgrad3t_kernel, stride `thin`), `per` tiles per split
};
WgPlan wgrad_bf16_plan(const adr_conv_desc* d);
int wgrad_bf16_launch(const adr_conv_desc* d, const void* x, const void* dy, float* out, int accumulate,
                      const WgPlan& p, hipStream_t st, float* bias = nullptr);
}  // namespace adr
