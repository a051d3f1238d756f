// bf16 WGRAD planner / launcher shared by adr_gemm.hip (ABI entry) and adr_wgrad.hip (kernel)
#pragma once
#include "adr_common.h"

namespace adr {
struct WgPlan {
  int bm, bn, R, tiles, splits;
  long per;  // reduction rows per split (multiple of R)
};
WgPlan wgrad_bf16_plan(const adr_conv_desc* d);
int wgrad_bf16_launch(const adr_conv_desc* d, const void* x, const void* dy, float* out, int accumulate,
                      const WgPlan& p, hipStream_t st);
}  // namespace adr
