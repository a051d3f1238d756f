// Batched NMS (reference utils/ops.py:163-312 non_max_suppression -> torchvision.ops.nms), per image:
//   candidates: xywh -> xyxy; single-label: best class (first max) with conf > thr; multi-label: every
//               (anchor, class) with score > thr, in torch.where row-major order (anchor, class)
//   max_nms:    keep the max_nms highest scores (ties: lower candidate order first)
//   greedy NMS: boxes offset by class * max_wh (computed in fp32 exactly as the reference, so IoUs round the
//               same way), stable descending-score order, suppress IoU > iou_thres, keep <= max_det.
// Because offset boxes of different classes never overlap, greedy NMS decomposes per class: one workgroup per
// (image, class) sorts its bucket (bitonic, LDS) and runs the greedy scan with wave ballots; a final merge
// takes the best max_det survivors per image in (score desc, candidate order asc) order.
// Compiled with -ffp-contract=off (Makefile) so no FMA changes IoU rounding.
#include "adr_common.h"

namespace adr {

static constexpr int NMS_SORT_CAP = 16384;  // per-(image, class) bucket capacity (A <= 16384, i.e. <= 896^2 input)

struct NmsArgs {
  const float* y;   // (B, 4+nc, A)
  int B, nc, A;
  float conf, iou;
  int multi, max_det, max_nms;
  float max_wh;
  int agnostic;                 // one NMS group for all classes (offset 0); single-label only
  int ng;                       // groups: agnostic ? 1 : nc
  const unsigned char* cmask;   // [nc] class filter (classes=...), null = all
  // workspace
  int* counts;      // [B][ng]
  int* offs;        // [B][ng]
  int* ccnt;        // [B][chunks][ng] per-chunk counts, then start slots
  float* cscore;    // [B][cap]   candidate scores
  int* ckey;        // [B][cap]   candidate order key (anchor*nc + class for multi, anchor for single)
  int* ccls;        // [B][cap]   candidate class
  int cap;          // per-image candidate capacity (A * nc or A)
  unsigned* thr;    // [B][2] radix-select threshold (score bits, tie key)
  int* kept;        // [B][ng][max_det] candidate index (into the image's arrays)
  int* nkept;       // [B][ng]
  float* out;       // (B, max_det, 6)
  int* nout;        // [B]
};

__device__ __forceinline__ float ycoord(const NmsArgs& a, int b, int ch, int an) {
  return a.y[((long)b * (4 + a.nc) + ch) * a.A + an];
}

// Candidate collection, per image in anchor order within each group (deterministic), over a (chunk, image) grid
// of 256-anchor chunks so the class-score reads of the whole batch are in flight at once:
//   count: every wave records one ballot mask per group in LDS; the block writes its per-group counts;
//   scan:  per image, group totals -> group offsets (counts/offs) and each (chunk, group)'s start slot;
//   fill:  the same ballots again; a candidate's slot = its chunk's start + earlier waves' popcounts + lane rank.
__device__ __forceinline__ void nms_chunk_masks(const NmsArgs& a, int b, int an, unsigned long long (*wm)[1024],
                                                float& bs, int& best) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool valid = an < a.A;
  const int nc = a.nc, ng = a.ng;
  best = 0;
  bs = -INFINITY;
  bool ok = false;
  if (!a.multi) {
    if (valid) {
      float s[8];
      for (int c0 = 0; c0 < nc; c0 += 8) {  // 8 class rows in flight per thread
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] = c0 + j < nc ? ycoord(a, b, 4 + c0 + j, an) : -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (s[j] > bs) {  // first maximum, as torch.max(1)
            bs = s[j];
            best = c0 + j;
          }
      }
    }
    ok = valid && bs > a.conf && (!a.cmask || a.cmask[best]);
  }
#pragma unroll 8
  for (int g = 0; g < ng; ++g) {
    bool take;
    if (a.multi) {
      const float sc = valid ? ycoord(a, b, 4 + g, an) : 0.f;
      take = valid && sc > a.conf && (!a.cmask || a.cmask[g]);
    } else {
      take = ok && (a.agnostic || best == g);
    }
    const unsigned long long m = __ballot(take);
    if (lane == 0) wm[wave][g] = m;
  }
}

__global__ void __launch_bounds__(256) nms_count_kernel(NmsArgs a) {
  const int chunk = blockIdx.x, b = blockIdx.y, nch = gridDim.x;
  __shared__ unsigned long long wm[4][1024];
  float bs;
  int best;
  nms_chunk_masks(a, b, chunk * 256 + threadIdx.x, wm, bs, best);
  __syncthreads();
  for (int g = threadIdx.x; g < a.ng; g += 256)
    a.ccnt[((long)b * nch + chunk) * a.ng + g] =
        __popcll(wm[0][g]) + __popcll(wm[1][g]) + __popcll(wm[2][g]) + __popcll(wm[3][g]);
}

__global__ void __launch_bounds__(256) nms_scan_kernel(NmsArgs a, int nch) {
  const int b = blockIdx.x, ng = a.ng;
  __shared__ int tot[1024];
  for (int g = threadIdx.x; g < ng; g += 256) {
    int t = 0;
    for (int ch = 0; ch < nch; ++ch) t += a.ccnt[((long)b * nch + ch) * ng + g];
    tot[g] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int g = 0; g < ng; ++g) {
      a.counts[b * ng + g] = tot[g];
      a.offs[b * ng + g] = run;
      run += tot[g];
    }
  }
  __syncthreads();
  for (int g = threadIdx.x; g < ng; g += 256) {
    int run = a.offs[b * ng + g];
    for (int ch = 0; ch < nch; ++ch) {
      const long i = ((long)b * nch + ch) * ng + g;
      const int c = a.ccnt[i];
      a.ccnt[i] = run;  // count -> start slot of (chunk, group)
      run += c;
    }
  }
}

__global__ void __launch_bounds__(256) nms_fill_kernel(NmsArgs a) {
  const int chunk = blockIdx.x, b = blockIdx.y, nch = gridDim.x;
  __shared__ unsigned long long wm[4][1024];
  const int an = chunk * 256 + threadIdx.x;
  float bs;
  int best;
  nms_chunk_masks(a, b, an, wm, bs, best);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  const int nc = a.nc;
  for (int g = 0; g < a.ng; ++g) {
    const unsigned long long m = wm[wave][g];
    if (!((m >> lane) & 1ull)) continue;
    int base = a.ccnt[((long)b * nch + chunk) * a.ng + g];
    for (int w = 0; w < wave; ++w) base += __popcll(wm[w][g]);
    const long pos = (long)b * a.cap + base + __popcll(m & below);
    a.cscore[pos] = a.multi ? ycoord(a, b, 4 + g, an) : bs;
    a.ckey[pos] = a.multi ? an * nc + g : an;
    a.ccls[pos] = a.multi ? g : best;
  }
}

// max_nms: radix-select the max_nms-th largest (score bits, then order key) per image; one block per image
__global__ void __launch_bounds__(256) nms_select_kernel(NmsArgs a) {
  int b = blockIdx.x;
  const int ng = a.ng;
  int total = a.offs[b * ng + ng - 1] + a.counts[b * ng + ng - 1];
  if (total <= a.max_nms) {
    if (threadIdx.x == 0) {
      a.thr[b * 2] = 0u;
      a.thr[b * 2 + 1] = 0x7fffffffu;
    }
    return;
  }
  __shared__ int hist[256];
  __shared__ unsigned prefix_s;
  __shared__ int need_s;
  const float* sc = a.cscore + (long)b * a.cap;
  const int* ky = a.ckey + (long)b * a.cap;
  unsigned prefix = 0u, mask = 0u;
  int need = a.max_nms;  // how many we still need among candidates matching prefix
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += 256) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += 256) {
      unsigned bits = __float_as_uint(sc[i]);
      if ((bits & mask) == prefix) atomicAdd(&hist[(bits >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0, d = 255;
      for (; d >= 0; --d) {
        if (acc + hist[d] >= need) break;
        acc += hist[d];
      }
      prefix_s = prefix | ((unsigned)d << shift);
      need_s = need - acc;
    }
    __syncthreads();
    prefix = prefix_s;
    need = need_s;
    mask |= 255u << shift;
  }
  // prefix = exact threshold score bits; keep all > prefix, and the `need` lowest keys among == prefix
  // tie keys: select the need-th smallest key among ties by a second radix pass on the key
  unsigned kprefix = 0u, kmask = 0u;
  int kneed = need;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += 256) hist[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += 256) {
      if (__float_as_uint(sc[i]) != prefix) continue;
      unsigned k = (unsigned)ky[i];
      if ((k & kmask) == kprefix) atomicAdd(&hist[(k >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0, d = 0;
      for (; d < 256; ++d) {
        if (acc + hist[d] >= kneed) break;
        acc += hist[d];
      }
      prefix_s = kprefix | ((unsigned)d << shift);
      need_s = kneed - acc;
    }
    __syncthreads();
    kprefix = prefix_s;
    kneed = need_s;
    kmask |= 255u << shift;
  }
  if (threadIdx.x == 0) {
    a.thr[b * 2] = prefix;
    a.thr[b * 2 + 1] = kprefix;
  }
}

__device__ __forceinline__ bool keep_after_select(unsigned bits, unsigned key, unsigned tb, unsigned tk) {
  return bits > tb || (bits == tb && key <= tk);
}

__device__ __forceinline__ void box_of(const NmsArgs& a, int b, int key, float* bx) {
  int an = a.multi ? key / a.nc : key;
  float x = ycoord(a, b, 0, an), yy = ycoord(a, b, 1, an), w = ycoord(a, b, 2, an), h = ycoord(a, b, 3, an);
  float hw = w / 2.f, hh = h / 2.f;  // xywh2xyxy (ops.py:412-429)
  bx[0] = x - hw;
  bx[1] = yy - hh;
  bx[2] = x + hw;
  bx[3] = yy + hh;
}

// per (image, class): sort bucket (score desc, key asc), greedy NMS, kept list (<= max_det)
__global__ void __launch_bounds__(256) nms_class_kernel(NmsArgs a) {
  int b = blockIdx.x / a.ng, c = blockIdx.x % a.ng;  // c: group (class, or 0 when agnostic)
  int n0 = a.counts[b * a.ng + c], off = a.offs[b * a.ng + c];
  if (n0 == 0) {
    if (threadIdx.x == 0) a.nkept[b * a.ng + c] = 0;
    return;
  }
  __shared__ unsigned long long sk[NMS_SORT_CAP];  // sort keys (128 KiB; one workgroup per CU at full size)
  __shared__ float kb[300][4];
  __shared__ float ka[300];
  const float* sc = a.cscore + (long)b * a.cap + off;
  const int* ky = a.ckey + (long)b * a.cap + off;
  unsigned tb = a.thr[b * 2], tk = a.thr[b * 2 + 1];
  // keys: (~score_bits << 32) | bucket index -> ascending = score desc, candidate order asc; dropped -> ~0
  int n = 1;
  while (n < n0) n <<= 1;
  for (int i = threadIdx.x; i < n; i += 256) {
    unsigned long long v = ~0ull;
    if (i < n0) {
      unsigned bits = __float_as_uint(sc[i]);
      if (keep_after_select(bits, (unsigned)ky[i], tb, tk))
        v = ((unsigned long long)(~bits) << 32) | (unsigned long long)i;
    }
    sk[i] = v;
  }
  __syncthreads();
  for (int size = 2; size <= n; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n; i += 256) {
        int j = i ^ stride;
        if (j > i) {
          bool up = (i & size) == 0;
          unsigned long long x = sk[i], y = sk[j];
          if ((x > y) == up) {
            sk[i] = y;
            sk[j] = x;
          }
        }
      }
      __syncthreads();
    }
  if (threadIdx.x >= 64) return;
  // greedy scan by one wave: candidates fetched 64 at a time (one per lane), then visited in order with the
  // kept list tested 64 boxes per ballot
  const int lane = threadIdx.x;
  const float offc = a.agnostic ? 0.f : (float)c * a.max_wh;  // x[:, 5:6] * (0 if agnostic else max_wh)
  int nk = 0;
  bool done = false;
  for (int t0 = 0; t0 < n && !done; t0 += 64) {
    unsigned long long v = t0 + lane < n ? sk[t0 + lane] : ~0ull;
    int idx = (int)(v & 0xffffffffu);
    float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;
    if (v != ~0ull) {
      float bx[4];
      box_of(a, b, ky[idx], bx);
      q0 = bx[0] + offc;
      q1 = bx[1] + offc;
      q2 = bx[2] + offc;
      q3 = bx[3] + offc;
    }
    unsigned long long live = __ballot(v != ~0ull);
    for (int j = 0; j < 64; ++j) {
      if (!((live >> j) & 1ull) || nk >= a.max_det) {
        done = true;
        break;
      }
      float o0 = __shfl(q0, j, 64), o1 = __shfl(q1, j, 64), o2 = __shfl(q2, j, 64), o3 = __shfl(q3, j, 64);
      int cand = __shfl(idx, j, 64);
      float area = (o2 - o0) * (o3 - o1);
      bool sup = false;
      for (int k0 = 0; k0 < nk && !sup; k0 += 64) {
        int k = k0 + lane;
        bool s = false;
        if (k < nk) {
          float xx1 = fmaxf(kb[k][0], o0), yy1 = fmaxf(kb[k][1], o1);
          float xx2 = fminf(kb[k][2], o2), yy2 = fminf(kb[k][3], o3);
          float w = fmaxf(0.f, xx2 - xx1), h = fmaxf(0.f, yy2 - yy1);
          float inter = w * h;
          float ovr = inter / (ka[k] + area - inter);  // torchvision: inter / (iarea + areas[j] - inter)
          s = ovr > a.iou;
        }
        sup = __ballot(s) != 0ull;
      }
      if (!sup) {
        if (lane == 0) {
          kb[nk][0] = o0;
          kb[nk][1] = o1;
          kb[nk][2] = o2;
          kb[nk][3] = o3;
          ka[nk] = area;
          a.kept[((long)b * a.ng + c) * a.max_det + nk] = off + cand;
        }
        __builtin_amdgcn_wave_barrier();
        nk++;
      }
    }
  }
  if (lane == 0) a.nkept[b * a.ng + c] = nk;
}

// per image: merge per-class kept lists by (score desc, candidate order asc); write up to max_det rows
__global__ void __launch_bounds__(64) nms_merge_kernel(NmsArgs a) {
  int b = blockIdx.x;
  int lane = threadIdx.x;
  __shared__ int head[1024];
  for (int c = lane; c < a.ng; c += 64) head[c] = 0;
  __syncthreads();
  const float* sc = a.cscore + (long)b * a.cap;
  const int* ky = a.ckey + (long)b * a.cap;
  int nout = 0;
  for (; nout < a.max_det; ++nout) {
    // each lane scans its classes for the best head
    unsigned long long best = ~0ull;
    int bc = -1;
    for (int c = lane; c < a.ng; c += 64) {
      int h = head[c];
      if (h >= a.nkept[b * a.ng + c]) continue;
      int ci = a.kept[((long)b * a.ng + c) * a.max_det + h];
      unsigned long long v = ((unsigned long long)(~__float_as_uint(sc[ci])) << 32) | (unsigned)ky[ci];
      if (v < best) {
        best = v;
        bc = c;
      }
    }
    // wave argmin over (best, bc)
    for (int o = 32; o > 0; o >>= 1) {
      unsigned long long ov = __shfl_xor(best, o, 64);
      int oc = __shfl_xor(bc, o, 64);
      if (ov < best) {
        best = ov;
        bc = oc;
      }
    }
    if (bc < 0) break;
    if (lane == 0) {
      int ci = a.kept[((long)b * a.ng + bc) * a.max_det + head[bc]];
      float bx[4];
      box_of(a, b, ky[ci], bx);
      float* o = a.out + ((long)b * a.max_det + nout) * 6;
      o[0] = bx[0];
      o[1] = bx[1];
      o[2] = bx[2];
      o[3] = bx[3];
      o[4] = sc[ci];
      o[5] = (float)a.ccls[(long)b * a.cap + ci];
      head[bc]++;
    }
    __syncthreads();
  }
  if (lane == 0) a.nout[b] = nout;
}

}  // namespace adr

using namespace adr;

extern "C" size_t adr_nms_workspace(int B, int nc, int A, int multi, int max_det) {
  size_t cap = (size_t)A * (multi ? nc : 1);
  return (size_t)B * nc * 4 * 2 + (size_t)B * cap * 12 + (size_t)B * 8 + (size_t)B * nc * max_det * 4 +
         (size_t)B * nc * 4 + (size_t)B * cdiv(A, 256) * nc * 4 + 256;
}

extern "C" int adr_nms(const float* y, int B, int nc, int A, float conf, float iou, int multi, int agnostic,
                       const unsigned char* class_mask, int max_det, int max_nms, float max_wh, float* out, int* nout,
                       void* ws, size_t ws_bytes, void* stream) {
  ADR_REQUIRE(B > 0 && nc >= 1 && nc <= 1024 && max_det >= 1 && max_det <= 300 && A >= 1 && A <= NMS_SORT_CAP &&
                  max_nms >= 1,
              "nms: B=%d nc=%d max_det=%d A=%d max_nms=%d unsupported", B, nc, max_det, A, max_nms);
  ADR_REQUIRE(!(agnostic && multi), "nms: agnostic multi-label groups exceed the per-group sort capacity");
  ADR_REQUIRE(ws_bytes >= adr_nms_workspace(B, nc, A, multi, max_det), "nms: workspace");
  NmsArgs a;
  a.y = y; a.B = B; a.nc = nc; a.A = A; a.conf = conf; a.iou = iou; a.multi = multi; a.max_det = max_det;
  a.max_nms = max_nms; a.max_wh = max_wh;
  a.agnostic = agnostic; a.ng = agnostic ? 1 : nc; a.cmask = class_mask;
  char* w = (char*)ws;
  a.counts = (int*)w; w += (size_t)B * nc * 4;
  a.offs = (int*)w; w += (size_t)B * nc * 4;
  a.cap = A * (multi ? nc : 1);
  a.cscore = (float*)w; w += (size_t)B * a.cap * 4;
  a.ckey = (int*)w; w += (size_t)B * a.cap * 4;
  a.ccls = (int*)w; w += (size_t)B * a.cap * 4;
  a.thr = (unsigned*)w; w += (size_t)B * 8;
  a.kept = (int*)w; w += (size_t)B * nc * max_det * 4;
  a.nkept = (int*)w; w += (size_t)B * nc * 4;
  a.ccnt = (int*)w;
  const int nch = cdiv(A, 256);
  a.out = out;
  a.nout = nout;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(nms_count_kernel, dim3(nch, B), dim3(256), 0, st, a);
  hipLaunchKernelGGL(nms_scan_kernel, dim3(B), dim3(256), 0, st, a, nch);
  hipLaunchKernelGGL(nms_fill_kernel, dim3(nch, B), dim3(256), 0, st, a);
  hipLaunchKernelGGL(nms_select_kernel, dim3(B), dim3(256), 0, st, a);
  hipLaunchKernelGGL(nms_class_kernel, dim3(B * a.ng), dim3(256), 0, st, a);
  hipLaunchKernelGGL(nms_merge_kernel, dim3(B), dim3(64), 0, st, a);
  return check_launch("adr_nms");
}

// ---------------- box IoU matrix for the validator's TP matching (models/yolo/detect/val.py:213-214) ----------------
// out[i][j] = inter / (area_a + area_b - inter + eps), xyxy boxes, the reference's utils/metrics.py:52-72 arithmetic
// order (compiled without FMA contraction, like the rest of this file).
__global__ void __launch_bounds__(256) box_iou_kernel(const float* __restrict__ a, int N, const float* __restrict__ b,
                                                      int M, float eps, float* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * M) return;
  const int r = (int)(i / M), c = (int)(i % M);
  const float ax1 = a[4 * r], ay1 = a[4 * r + 1], ax2 = a[4 * r + 2], ay2 = a[4 * r + 3];
  const float bx1 = b[4 * c], by1 = b[4 * c + 1], bx2 = b[4 * c + 2], by2 = b[4 * c + 3];
  const float iw = fmaxf(fminf(ax2, bx2) - fmaxf(ax1, bx1), 0.f);
  const float ih = fmaxf(fminf(ay2, by2) - fmaxf(ay1, by1), 0.f);
  const float inter = iw * ih;
  const float area_a = (ax2 - ax1) * (ay2 - ay1), area_b = (bx2 - bx1) * (by2 - by1);
  out[i] = inter / (area_a + area_b - inter + eps);
}

extern "C" int adr_box_iou(const float* a, int N, const float* b, int M, float eps, float* out, void* stream) {
  ADR_REQUIRE(N >= 0 && M >= 0, "box_iou: N=%d M=%d", N, M);
  if ((long)N * M == 0) return 0;
  hipLaunchKernelGGL(box_iou_kernel, dim3(cdiv((long)N * M, 256)), dim3(256), 0, (hipStream_t)stream, a, N, b, M, eps,
                     out);
  return check_launch("adr_box_iou");
}
