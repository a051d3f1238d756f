// Probe (GPU): lane maps of v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 operands (unit E8M0 scales) and the
// encoding of v_cvt_pk_fp8_f32, checked against host arithmetic on exact small-integer data.
// build: hipcc --offload-arch=gfx950 -O2 scripts/probes/fp8_mfma_probe.hip -o /tmp/fp8probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void mfma_k(const uint8_t* a, const uint8_t* b, float* d) {
  const int l = threadIdx.x;
  i32x8 av, bv;
  for (int q = 0; q < 8; ++q) {
    av[q] = *reinterpret_cast<const int*>(a + l * 32 + 4 * q);
    bv[q] = *reinterpret_cast<const int*>(b + l * 32 + 4 * q);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, acc, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

__global__ void cvt_k(const float* f, int* o, int n) {
  const int i = threadIdx.x;
  if (2 * i + 1 < n) o[i] = __builtin_amdgcn_cvt_pk_fp8_f32(f[2 * i], f[2 * i + 1], 0, false);
}

// OCP e4m3fn encode for small integers / simple values (exact)
static uint8_t enc(int v) {
  if (v == 0) return 0;
  const int s = v < 0 ? 0x80 : 0;
  int m = abs(v), e = 0;
  while (m >= 2 << e) ++e;  // 2^e <= m < 2^(e+1)
  const int frac = (m - (1 << e)) << 3 >> e;  // 3 mantissa bits (exact for |v| <= 15)
  return (uint8_t)(s | ((e + 7) << 3) | frac);
}

int main() {
  uint8_t ha[64 * 32], hb[64 * 32];
  int av[64][32], bv[64][32];
  srand(1);
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 32; ++j) {
      av[l][j] = rand() % 7 - 3;
      bv[l][j] = rand() % 7 - 3;
      ha[l * 32 + j] = enc(av[l][j]);
      hb[l * 32 + j] = enc(bv[l][j]);
    }
  uint8_t *da, *db;
  float* dd;
  hipMalloc(&da, sizeof ha);
  hipMalloc(&db, sizeof hb);
  hipMalloc(&dd, 64 * 4 * 4);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  mfma_k<<<1, 64>>>(da, db, dd);
  float hd[64 * 4];
  hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
  // candidate maps (lane l, byte j) -> k index (row / column = l & 15)
  const char* names[3] = {"k = 32*(l>>4) + j", "k = 16*(l>>4) + (j&15) + 64*(j>>4)", "k = 8*(l>>4) + (j&7) + 32*(j>>3)"};
  for (int cand = 0; cand < 3; ++cand) {
    int A[16][128] = {}, B[128][16] = {};
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int g = l >> 4;
        const int k = cand == 0 ? 32 * g + j : cand == 1 ? 16 * g + (j & 15) + 64 * (j >> 4) : 8 * g + (j & 7) + 32 * (j >> 3);
        A[l & 15][k] = av[l][j];
        B[k][l & 15] = bv[l][j];
      }
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        const int row = (l >> 4) * 4 + r, col = l & 15;
        long s = 0;
        for (int k = 0; k < 128; ++k) s += (long)A[row][k] * B[k][col];
        if ((float)s != hd[l * 4 + r]) ++bad;
      }
    printf("candidate %d (%s): %d of 256 outputs differ\n", cand, names[cand], bad);
  }
  const float fv[8] = {1.f, -2.f, 448.f, 0.5f, 3.f, -0.015625f, 0.f, 15.f};
  float* df;
  int* dcv;
  hipMalloc(&df, sizeof fv);
  hipMalloc(&dcv, 16);
  hipMemcpy(df, fv, sizeof fv, hipMemcpyHostToDevice);
  cvt_k<<<1, 4>>>(df, dcv, 8);
  int hc[4];
  hipMemcpy(hc, dcv, 16, hipMemcpyDeviceToHost);
  printf("cvt_pk_fp8: ");
  for (int i = 0; i < 4; ++i) printf("%02x %02x ", hc[i] & 255, (hc[i] >> 8) & 255);
  printf(" (OCP e4m3fn expects 38 c0 7e 30 44 a8 00 57)\n");
  return 0;
}
