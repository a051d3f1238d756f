// Probe (GPU): semantics of v_cvt_scalef32_pk_fp8_bf16 (gfx950): fp8 = e4m3(x * scale)? x / scale? saturation?
// build: hipcc --offload-arch=gfx950 -O2 scripts/probes/fp8_cvt_probe.hip -o scripts/probes/fp8cvt
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) short s16x2;

__global__ void k(const float* x, const float* sc, int* o, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  bf16x2 v = {(__bf16)x[i], (__bf16)x[i]};
  s16x2 r = {0, 0};
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, v, sc[i], false);
  o[i] = *(int*)&r & 0xffff;
}

int main() {
  const int n = 8;
  float hx[n] = {1.f, 1.f, 1.f, 3.f, 300.f, 1000.f, -1000.f, 1.f};
  float hs[n] = {1.f, 2.f, 0.5f, 4.f, 1.f, 1.f, 1.f, 3.f};
  float *dx, *ds;
  int* dout;
  (void)hipMalloc(&dx, sizeof hx);
  (void)hipMalloc(&ds, sizeof hs);
  (void)hipMalloc(&dout, n * 4);
  (void)hipMemcpy(dx, hx, sizeof hx, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice);
  k<<<1, 64>>>(dx, ds, dout, n);
  int ho[n];
  (void)hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) printf("x=%g scale=%g -> %02x %02x\n", hx[i], hs[i], ho[i] & 255, (ho[i] >> 8) & 255);
  printf("(e4m3fn: 1->38 2->40 0.5->30 4->48 12->54 0.25->28 0.333->2d 448->7e nan->7f)\n");
  return 0;
}
