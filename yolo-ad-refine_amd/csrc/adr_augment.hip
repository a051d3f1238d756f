// Training augmentation pixels in one launch (reference data/augment.py v8_transforms :2273-2335): for every output
// pixel of every image of the batch, the fused chain
//
//   Mosaic canvas (four resized sources placed around the mosaic centre, 114 elsewhere; augment.py:657-713)
//   -> RandomPerspective's cv2.warpAffine (INTER_LINEAR, border 114; augment.py:1016-1077)
//   -> RandomHSV (BGR -> HSV, per-channel LUTs, HSV -> BGR; augment.py:1344-1378)
//   -> RandomFlip up-down / left-right (index mirrors; augment.py:1429-1472)
//   -> Format's HWC BGR -> CHW RGB (augment.py:2072-2100) into the collated uint8 (B, 3, H, W) batch
//
// is evaluated directly: the 2s x 2s mosaic canvas, the warped image and the HSV image are never materialised.
// Canvas pixels are looked up in the tile table (source pixel or 114) when the warp's bilinear taps read them.
// The host draws every random parameter in the reference's order and supplies the integer tables of the chain:
// the warp's fixed-point source coordinates (cv::warpAffine's AB_BITS 10 / INTER_BITS 5 arithmetic, computed in
// double on the host exactly as OpenCV does) and the three HSV LUTs; the kernel is integer arithmetic plus the
// float32 HSV -> BGR of OpenCV's 8U path (contraction off, round half to even). One thread per output pixel: the
// three plane stores are coalesced, the bilinear taps read neighbouring source pixels (L2 hits).
#include "adr_common.h"

#include <cstdint>

#pragma clang fp contract(off)

namespace adr {

struct AugTile {
  long long off;  // byte offset of the source image (HWC BGR uint8) in the pool
  int sw;         // source width (row pitch / 3)
  int x1a, y1a, x2a, y2a, x1b, y1b;  // canvas rectangle and its top-left in the source
};

struct AugDesc {
  AugTile tile[4];
  int ntile;
  int cw, ch;       // canvas size
  int warp;         // 1: warpAffine tables at tab_off (adelta[W], bdelta[W], X0[H], Y0[H])
  int tab_off;
  int lut_off;      // -1: no HSV; else 768 bytes (hue, sat, val)
  int flip_ud, flip_lr, rgb;
  int pad_;
};

namespace {

__device__ __forceinline__ void canvas_px(const uint8_t* pool, const AugDesc& d, int x, int y, int v[3]) {
  v[0] = v[1] = v[2] = 114;
  if (x < 0 || y < 0 || x >= d.cw || y >= d.ch) return;
  for (int i = 0; i < d.ntile; ++i) {
    const AugTile& t = d.tile[i];
    if (x >= t.x1a && x < t.x2a && y >= t.y1a && y < t.y2a) {
      const uint8_t* p = pool + t.off + ((long long)(y - t.y1a + t.y1b) * t.sw + (x - t.x1a + t.x1b)) * 3;
      v[0] = p[0];
      v[1] = p[1];
      v[2] = p[2];
    }
  }
}

// OpenCV RGB2HSV_b (hsv_shift 12, hrange 180) on one BGR pixel; sdiv_table[v] / hdiv_table180[diff] are the
// cvRound'ed double quotients, evaluated here (IEEE double division and rint) instead of read from a table
__device__ __forceinline__ void bgr2hsv(int b, int g, int r, int& h, int& s, int& v) {
  v = max(max(b, g), r);
  const int vmin = min(min(b, g), r);
  const int diff = v - vmin;
  const int sdiv = v ? (int)__builtin_rint((double)(255 << 12) / (1. * v)) : 0;
  const int hdiv = diff ? (int)__builtin_rint((double)(180 << 12) / (6. * diff)) : 0;
  s = (diff * sdiv + (1 << 11)) >> 12;
  h = v == r ? g - b : (v == g ? b - r + 2 * diff : r - g + 4 * diff);
  h = (h * hdiv + (1 << 11)) >> 12;
  if (h < 0) h += 180;
}

// OpenCV HSV2RGB_b: u8 -> float (h, s/255, v/255), HSV2RGB_native, saturate_cast<uchar>(x * 255.f)
__device__ __forceinline__ void hsv2bgr(int hi, int si, int vi, int out[3]) {
  const float s = (float)si * (1.f / 255.f), v = (float)vi * (1.f / 255.f);
  float b, g, r;
  if (s == 0.f) {
    b = g = r = v;
  } else {
    float h = (float)hi * (6.f / 180.f);
    h = fmodf(h, 6.f);
    int sector = (int)floorf(h);
    h -= (float)sector;
    if ((unsigned)sector >= 6u) {
      sector = 0;
      h = 0.f;
    }
    float tab[4];
    tab[0] = v;
    tab[1] = v * (1.f - s);
    tab[2] = v * (1.f - s * h);
    tab[3] = v * (1.f - s * (1.f - h));
    const int sd[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
    b = tab[sd[sector][0]];
    g = tab[sd[sector][1]];
    r = tab[sd[sector][2]];
  }
  const float f[3] = {b, g, r};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int q = (int)__builtin_rintf(f[k] * 255.f);
    out[k] = q < 0 ? 0 : (q > 255 ? 255 : q);
  }
}

}  // namespace

__global__ void __launch_bounds__(256) augment_u8_kernel(const uint8_t* pool, const AugDesc* descs, const int* tabs,
                                                          const uint8_t* luts, uint8_t* out, int H, int W) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= H * W) return;
  const AugDesc& d = descs[b];
  const int y = p / W, x = p - y * W;
  const int ys = d.flip_ud ? H - 1 - y : y, xs = d.flip_lr ? W - 1 - x : x;
  int bgr[3];
  if (d.warp) {
    const int* t = tabs + d.tab_off;
    const int X = (t[2 * W + ys] + t[xs]) >> 5, Y = (t[2 * W + H + ys] + t[W + xs]) >> 5;
    const int sx = X >> 5, sy = Y >> 5, fx = X & 31, fy = Y & 31;
    int v00[3], v01[3], v10[3], v11[3];
    canvas_px(pool, d, sx, sy, v00);
    canvas_px(pool, d, sx + 1, sy, v01);
    canvas_px(pool, d, sx, sy + 1, v10);
    canvas_px(pool, d, sx + 1, sy + 1, v11);
    const int w00 = (32 - fx) * (32 - fy) * 32, w01 = fx * (32 - fy) * 32, w10 = (32 - fx) * fy * 32,
              w11 = fx * fy * 32;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int a = (v00[k] * w00 + v01[k] * w01 + v10[k] * w10 + v11[k] * w11 + (1 << 14)) >> 15;
      bgr[k] = a < 0 ? 0 : (a > 255 ? 255 : a);
    }
  } else {
    canvas_px(pool, d, xs, ys, bgr);
  }
  if (d.lut_off >= 0) {
    const uint8_t* L = luts + d.lut_off;
    int h, s, v;
    bgr2hsv(bgr[0], bgr[1], bgr[2], h, s, v);
    hsv2bgr(L[h], L[256 + s], L[512 + v], bgr);
  }
  const long plane = (long)H * W;
  uint8_t* o = out + (long)b * 3 * plane + p;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[c * plane] = (uint8_t)bgr[d.rgb ? 2 - c : c];
}

}  // namespace adr

using namespace adr;

extern "C" int adr_augment_u8(const void* pool, const void* descs, int B, const int* tables, const void* luts,
                              void* out, int H, int W, void* stream) {
  ADR_REQUIRE(B > 0 && H > 0 && W > 0 && (long)H * W < (1l << 30), "augment: B=%d H=%d W=%d", B, H, W);
  hipLaunchKernelGGL(augment_u8_kernel, dim3(cdiv((long)H * W, 256), B), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)pool, (const AugDesc*)descs, tables, (const uint8_t*)luts, (uint8_t*)out, H, W);
  return check_launch("adr_augment_u8");
}

extern "C" int adr_augment_desc_size(void) { return (int)sizeof(AugDesc); }
