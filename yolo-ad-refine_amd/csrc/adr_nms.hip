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

#include <algorithm>
#include <cstdlib>
#include <cstring>

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
  unsigned* rec_ok; // the persistent kernel's "cursors left zero" record: cleared by this pipeline (it reuses them)
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
  if (chunk == 0 && b == 0 && threadIdx.x == 0) *a.rec_ok = 0u;
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

// ---------------- persistent single-launch variant (the default) ----------------
// One launch of gridDim = resident capacity (one workgroup of 1024 threads per CU, so every workgroup is resident
// and grid barriers are safe); phases are separated by grid barriers and each is a grid-stride loop over its items.
//
// Bucket layouts. direct (the default while B * nc * A keys fit in 1 GiB): bucket (b, g) is a fixed A-key slot
// array, so candidates go straight to their bucket in one pass over the head output. scanned (larger shapes):
// a count pass, an offset scan and the fill pass pack the buckets densely (cap keys per image).
//   P0 fill    one wave per 64 anchors of one image: every candidate to a slot of its (image, group) bucket; the
//              slot cursors are claimed with one atomic per group and batch of 16 class rows, issued by different
//              lanes at once. scanned: P0a count (caching each anchor's key / the per-group ballots), P0b offsets.
//   P1 select  (only when some image has more than max_nms candidates) radix select of the max_nms-th smallest key
//   P2 class   one workgroup per (image, group): the bucket's keys compacted into LDS, bitonic sort, greedy NMS in
//              tiles of 64 candidates (below)
//   P3 merge   one wave per image: the per-group kept lists -> max_det rows in key order.
// The slot order inside a bucket is arbitrary (atomics). Every step after the fill orders candidates by the 64-bit
// key (~score_bits << 32 | anchor * nc + class), unique per image and equal to the reference's order (score
// descending, then torch.where / argmax row order), so the result does not depend on the slot order.
//
// The cursors must be zero when the fill starts. A launch zeroes them itself (one more barrier) unless the record
// in the control words says the previous launch left exactly these words zero (direct layout, same workspace and
// size): steady-state batches skip that pass. Only the control words (the first NMSP_CTL_BYTES of the workspace)
// must be zero when a workspace is first used; every launch leaves the barrier words as it found them.
static constexpr int NMSP_THREADS = 1024;
static constexpr int NMSP_WAVES = NMSP_THREADS / 64;
static constexpr int NMSP_MAX_GRID = 1024;
static constexpr long NMSP_SPIN_LIMIT = 1l << 25;  // ~2 s of s_sleep: a barrier that never completes sets CTL_ERR
static constexpr int NMSP_GB = 16;                 // class rows per batch of loads
static constexpr int SEL_W = 12, SEL_BINS = 1 << SEL_W;        // radix-select digit width / bins
static constexpr int SEL_CAP = NMS_SORT_CAP - SEL_BINS / 2;   // keys an LDS select holds (u64 slots after the histogram)
static constexpr int SEL_U = 8, SEL_CH = 64 * SEL_U;
static constexpr int HIST_W = 16, HIST_BINS = 1 << HIST_W;     // fill-time top-digit histogram (distributed select)
enum : int {
  CTL_GEN = 1,      // barrier generation
  CTL_ERR = 2,      // a barrier wait timed out
  CTL_REC_LO = 3,   // record: cursor words left zero by the last launch (address lo / hi, count, valid)
  CTL_REC_HI = 4,
  CTL_REC_N = 5,
  CTL_REC_OK = 6,
  CTL_FLAGS = 64,   // arrival flag per workgroup
  CTL_WORDS = CTL_FLAGS + NMSP_MAX_GRID,
};
static constexpr size_t NMSP_CTL_BYTES = CTL_WORDS * 4;

struct NmsP {
  NmsArgs a;
  unsigned* ctl;
  int* cur;                       // [B][ng] bucket fill cursors, then tot = cur + B * ng: [B] candidates per image,
  int* tot;                       // ccur: [B] select compaction cursors, hist: [B][SEL_BINS] top-digit histograms
  int* ccur;
  int* hist;
  int sel_hist;                   // an image may exceed max_nms: the fill builds the top-digit histograms
  int* seld;                      // [B][3] select: first digit, rank within it, keys under it (-1: no select)
  unsigned long long* comp;       // [B][SEL_CAP] keys under the first digit (distributed select)
  int* gcnt;                      // scanned: [B][ng] count cursors
  unsigned long long* cand;       // direct: [B][ng][A]; scanned: [B][cap] (bucket at offs)
  unsigned long long* thr;        // [B] max_nms threshold key (keep key <= thr)
  unsigned long long* kept;       // [B][ng][max_det] kept keys per group, in order
  unsigned long long* best;       // scanned single-label: [B][A] the anchor's key, ~0 if not a candidate
  unsigned long long* masks;      // scanned multi-label: [B][A/64][ng] candidate ballots per 64 anchors and group
  int direct;
  int stop;                       // ADR_NMS_STOP (phase timing): return after this phase, 0 = run all
};

__device__ __forceinline__ unsigned long long nms_key(float s, int key) {
  return ((unsigned long long)(~__float_as_uint(s)) << 32) | (unsigned)key;
}
__device__ __forceinline__ float key_score(unsigned long long v) { return __uint_as_float(~(unsigned)(v >> 32)); }
__device__ __forceinline__ int cdiv_d(int a, int b) { return (a + b - 1) / b; }
__device__ __forceinline__ unsigned ld_rlx(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_rlx(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Grid barrier over all (co-resident) workgroups, bounded wait. Each workgroup raises its own arrival flag to the
// next generation; workgroup 0 polls all flags at once (one per thread) and then publishes the generation. No
// serialised atomics on one line, and flags need no reset (they only ever move to the next generation).
__device__ void nmsp_grid_sync(unsigned* ctl) {
  __syncthreads();
  const unsigned gen = ld_rlx(&ctl[CTL_GEN]);
  __syncthreads();  // every thread read the generation before this workgroup arrives
  if (blockIdx.x == 0) {
    for (int t = threadIdx.x; t < (int)gridDim.x; t += NMSP_THREADS) {
      if (t == 0) continue;
      long spins = 0;
      while (ld_rlx(&ctl[CTL_FLAGS + t]) != gen + 1u) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > NMSP_SPIN_LIMIT) {
          st_rlx(&ctl[CTL_ERR], 1u);
          break;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
      __hip_atomic_store(&ctl[CTL_GEN], gen + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    st_rlx(&ctl[CTL_FLAGS + blockIdx.x], gen + 1u);
    long spins = 0;
    while (ld_rlx(&ctl[CTL_GEN]) == gen) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > NMSP_SPIN_LIMIT) {
        st_rlx(&ctl[CTL_ERR], 1u);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// best class of one anchor (first maximum, as torch.max(1)), 16 class rows in flight per lane
__device__ __forceinline__ void nmsp_best(const NmsArgs& a, int b, int an, bool valid, float& bs, int& best) {
  bs = -INFINITY;
  best = 0;
  if (!valid) return;
  float s[NMSP_GB];
  for (int c0 = 0; c0 < a.nc; c0 += NMSP_GB) {
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j) s[j] = c0 + j < a.nc ? ycoord(a, b, 4 + c0 + j, an) : -INFINITY;
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j)
      if (s[j] > bs) {
        bs = s[j];
        best = c0 + j;
      }
  }
}

// top-digit histogram of the wave's candidate keys (one atomic per distinct digit); the whole wave calls it
__device__ __forceinline__ void nmsp_hist_add(const NmsP& p, int b, bool on, unsigned long long key) {
  if (!p.sel_hist) return;
  const int lane = threadIdx.x & 63;
  const int d = (int)(key >> (64 - HIST_W));
  unsigned long long left = __ballot(on);
  while (left) {
    const int lead = __builtin_ctzll(left);
    const int d0 = __shfl(d, lead, 64);
    const unsigned long long mm = __ballot(on && d == d0);
    if (lane == lead) atomicAdd(&p.hist[(long)b * HIST_BINS + d0], __popcll(mm));
    left &= ~mm;
  }
}

// single-label: slot claim for the candidates of one wave (one atomic per distinct group, all issued at once)
__device__ __forceinline__ void nmsp_put_single(const NmsP& p, int b, bool ok, int g, unsigned long long key,
                                                unsigned long long* bucket0, long gstride, const int* offs) {
  const int lane = threadIdx.x & 63, ng = p.a.ng;
  const unsigned long long below = (1ull << lane) - 1ull;
  unsigned long long left = __ballot(ok);
  if (!left) return;
  nmsp_hist_add(p, b, ok, key);
  const int total = __popcll(left);
  int myl = 0, myr = 0, lcnt = 0;
  while (left) {
    const int lead = __builtin_ctzll(left);
    const int g0 = __shfl(g, lead, 64);
    const unsigned long long mm = __ballot(ok && g == g0);
    if (ok && g == g0) {
      myl = lead;
      myr = __popcll(mm & below);
    }
    if (lane == lead) lcnt = __popcll(mm);
    left &= ~mm;
  }
  long base = 0;
  if (lcnt) base = (offs ? offs[b * ng + g] : g * gstride) + atomicAdd(&p.cur[b * ng + g], lcnt);
  base = __shfl(base, myl, 64);
  if (ok) bucket0[base + myr] = key;
  if (p.direct && lane == 0) atomicAdd(&p.tot[b], total);
}

// direct fill of the 64 anchors of chunk ch of image b
__device__ __forceinline__ void nmsp_fill_direct(const NmsP& p, int b, int ch) {
  const NmsArgs& a = p.a;
  const int lane = threadIdx.x & 63, an = ch * 64 + lane;
  const unsigned long long below = (1ull << lane) - 1ull;
  const bool valid = an < a.A;
  const int nc = a.nc, ng = a.ng, A = a.A;
  unsigned long long* bucket0 = p.cand + (long)b * ng * A;  // bucket g at bucket0 + g * A
  if (!a.multi) {
    float bs;
    int best;
    nmsp_best(a, b, an, valid, bs, best);
    const bool ok = valid && bs > a.conf && (!a.cmask || a.cmask[best]);
    nmsp_put_single(p, b, ok, a.agnostic ? 0 : best, nms_key(bs, an * nc + best), bucket0, A, nullptr);
    return;
  }
  int acc = 0;
  for (int g0 = 0; g0 < ng; g0 += NMSP_GB) {
    float s[NMSP_GB];
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j) s[j] = valid && g0 + j < ng ? ycoord(a, b, 4 + g0 + j, an) : 0.f;
    unsigned long long mine = 0ull;
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j) {
      const bool take = valid && g0 + j < ng && s[j] > a.conf && (!a.cmask || a.cmask[g0 + j]);
      const unsigned long long m = __ballot(take);
      if (lane == j) mine = m;
    }
    if (!__ballot(mine != 0ull)) continue;
    int base = 0;
    if (mine) {
      base = atomicAdd(&p.cur[b * ng + g0 + lane], __popcll(mine));
      acc += __popcll(mine);
    }
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j) {
      const unsigned long long m = __shfl(mine, j, 64);
      const int bj = __shfl(base, j, 64);
      const bool on = (m >> lane) & 1ull;
      const unsigned long long key = nms_key(s[j], an * nc + g0 + j);
      if (on) bucket0[(long)(g0 + j) * A + bj + __popcll(m & below)] = key;
      if (m) nmsp_hist_add(p, b, on, key);
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);  // lanes 0..15 hold the counts
  if (lane == 0 && acc) atomicAdd(&p.tot[b], acc);
}

// scanned P0a: counts per (image, group); caches the anchor keys (single) or the per-group ballots (multi)
__device__ __forceinline__ void nmsp_count_scanned(const NmsP& p, int b, int ch) {
  const NmsArgs& a = p.a;
  const int lane = threadIdx.x & 63, an = ch * 64 + lane;
  const bool valid = an < a.A;
  const int nc = a.nc, ng = a.ng;
  if (!a.multi) {
    float bs;
    int best;
    nmsp_best(a, b, an, valid, bs, best);
    const bool ok = valid && bs > a.conf && (!a.cmask || a.cmask[best]);
    if (valid) p.best[(long)b * a.A + an] = ok ? nms_key(bs, an * nc + best) : ~0ull;
    const int g = a.agnostic ? 0 : best;
    unsigned long long left = __ballot(ok);
    while (left) {
      const int lead = __builtin_ctzll(left);
      const int g0 = __shfl(g, lead, 64);
      const unsigned long long mm = __ballot(ok && g == g0);
      if (lane == lead) atomicAdd(&p.gcnt[b * ng + g0], __popcll(mm));
      left &= ~mm;
    }
    return;
  }
  unsigned long long* mk = p.masks + ((long)b * cdiv_d(a.A, 64) + ch) * ng;
  for (int g0 = 0; g0 < ng; g0 += NMSP_GB) {
    float s[NMSP_GB];
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j) s[j] = valid && g0 + j < ng ? ycoord(a, b, 4 + g0 + j, an) : 0.f;
    unsigned long long mine = 0ull;
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j) {
      const bool take = valid && g0 + j < ng && s[j] > a.conf && (!a.cmask || a.cmask[g0 + j]);
      const unsigned long long m = __ballot(take);
      if (lane == j) mine = m;
    }
    if (lane < NMSP_GB && g0 + lane < ng) {
      mk[g0 + lane] = mine;
      if (mine) atomicAdd(&p.gcnt[b * ng + g0 + lane], __popcll(mine));
    }
  }
}

// scanned fill from the cached keys / ballots
__device__ __forceinline__ void nmsp_fill_scanned(const NmsP& p, int b, int ch) {
  const NmsArgs& a = p.a;
  const int lane = threadIdx.x & 63, an = ch * 64 + lane;
  const unsigned long long below = (1ull << lane) - 1ull;
  const bool valid = an < a.A;
  const int nc = a.nc, ng = a.ng;
  unsigned long long* cv = p.cand + (long)b * a.cap;
  if (!a.multi) {
    const unsigned long long key = valid ? p.best[(long)b * a.A + an] : ~0ull;
    const bool ok = key != ~0ull;
    nmsp_put_single(p, b, ok, a.agnostic ? 0 : (int)((unsigned)key % (unsigned)nc), key, cv, 0, a.offs);
    return;
  }
  const unsigned long long* mk = p.masks + ((long)b * cdiv_d(a.A, 64) + ch) * ng;
  for (int g0 = 0; g0 < ng; g0 += NMSP_GB) {
    const unsigned long long mine = lane < NMSP_GB && g0 + lane < ng ? mk[g0 + lane] : 0ull;
    if (!__ballot(mine != 0ull)) continue;
    int base = 0;
    if (mine) base = a.offs[b * ng + g0 + lane] + atomicAdd(&p.cur[b * ng + g0 + lane], __popcll(mine));
    float s[NMSP_GB];
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j) s[j] = valid && g0 + j < ng ? ycoord(a, b, 4 + g0 + j, an) : 0.f;
#pragma unroll
    for (int j = 0; j < NMSP_GB; ++j) {
      const unsigned long long m = __shfl(mine, j, 64);
      const int bj = __shfl(base, j, 64);
      const bool on = (m >> lane) & 1ull;
      const unsigned long long key = nms_key(s[j], an * nc + g0 + j);
      if (on) cv[bj + __popcll(m & below)] = key;
      if (m) nmsp_hist_add(p, b, on, key);
    }
  }
}

// exclusive scan of one int per thread over the workgroup (NMSP_THREADS); returns the exclusive prefix
__device__ __forceinline__ int nmsp_block_scan(int v, int* wsum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int pre = 0;
  for (int w = 0; w < wave; ++w) pre += wsum[w];
  __syncthreads();
  return pre + x - v;
}

__device__ __forceinline__ void box_of_anchor(const NmsArgs& a, int b, int an, float* bx) {
  const float x = ycoord(a, b, 0, an), yy = ycoord(a, b, 1, an), w = ycoord(a, b, 2, an), h = ycoord(a, b, 3, an);
  const float hw = w / 2.f, hh = h / 2.f;  // xywh2xyxy (ops.py:412-429)
  bx[0] = x - hw;
  bx[1] = yy - hh;
  bx[2] = x + hw;
  bx[3] = yy + hh;
}

struct NmspLds {
  unsigned long long sk[NMS_SORT_CAP];  // P2 sort keys; the P1 histogram and compaction buffer alias it
  float kb[300][4];                     // kept boxes (class-offset) and areas of the current group
  float ka[300];
  int head[1025];                       // P1 (direct) chunk prefix per bucket; P3 kept-list offsets / cursors
  int gc[1024];                         // P1 (direct) keys per bucket
  int wsum[NMSP_WAVES];
  unsigned long long bcast;
  unsigned long long supw;              // P2 tile: candidates suppressed by earlier tiles' kept boxes
  unsigned long long mt[64];            // P2 tile: per candidate, the earlier in-tile candidates overlapping it
  int sel[2];
  int cnt;
};

// ascending bitonic sort of sk[0..n) (n a power of two) by the workgroup, one compare-exchange pair per thread and
// step; up to 128 keys wave 0 sorts alone (no workgroup barriers between steps)
__device__ void nmsp_bitonic(unsigned long long* sk, int n) {
  if (n <= 128) {
    if (threadIdx.x < 64) {
      const int t = threadIdx.x;
      for (int size = 2; size <= n; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          const int i = (t / stride) * 2 * stride + (t % stride), j = i + stride;
          if (j < n) {
            const bool up = (i & size) == 0;
            const unsigned long long x = sk[i], y = sk[j];
            if ((x > y) == up) {
              sk[i] = y;
              sk[j] = x;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();
    return;
  }
  for (int size = 2; size <= n; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < n / 2; t += NMSP_THREADS) {
        const int i = (t / stride) * 2 * stride + (t % stride), j = i + stride;
        const bool up = (i & size) == 0;
        const unsigned long long x = sk[i], y = sk[j];
        if ((x > y) == up) {
          sk[i] = y;
          sk[j] = x;
        }
      }
      __syncthreads();
    }
}

// max_nms threshold of image b: the max_nms-th smallest key (keys are unique, so exactly max_nms keys are <= it).
// Radix select on 12-bit digits from the top; histogram atomics aggregated per wave (one LDS atomic per distinct
// digit in the wave), SEL_U keys per lane in flight. Once the keys matching the prefix fit in LDS they are
// compacted there and the remaining digits are resolved without touching HBM.

__device__ __forceinline__ void nmsp_select(const NmsP& p, NmspLds& L, int b, int total) {
  const NmsArgs& a = p.a;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, ng = a.ng;
  int* hist = reinterpret_cast<int*>(L.sk);
  unsigned long long* buf = L.sk + SEL_BINS / 2;
  const unsigned long long* gv = p.direct ? p.cand + (long)b * ng * a.A : p.cand + (long)b * a.cap;
  // the keys are read in chunks of SEL_CH (one chunk per wave and step); direct: bucket g holds the chunks
  // head[g] <= chunk < head[g + 1], its key count in gc[g]
  int gchunks = 0;
  if (p.direct) {
    const int c = tid < ng ? p.cur[b * ng + tid] : 0;
    const int nchk = (c + SEL_CH - 1) / SEL_CH;
    const int off = nmsp_block_scan(nchk, L.wsum);
    if (tid < ng) {
      L.head[tid] = off;
      L.gc[tid] = c;
    }
    if (tid == ng - 1) L.sel[0] = off + nchk;
    __syncthreads();
    gchunks = L.sel[0];
    __syncthreads();
  }
  unsigned long long prefix = 0ull, mask = 0ull;
  int need = a.max_nms;  // rank (1-based) of the threshold among the keys matching prefix
  int m = total;         // keys matching prefix
  int nbuf = 0;          // keys compacted into buf (those matching the prefix of the compacting pass)
  bool inlds = false;
  for (int hi = 64; hi > 0;) {
    const int w = hi < SEL_W ? hi : SEL_W, shift = hi - w;
    const bool compact = !inlds && m <= SEL_CAP;
    for (int i = tid; i < SEL_BINS; i += NMSP_THREADS) hist[i] = 0;
    if (tid == 0) L.cnt = 0;
    __syncthreads();
    const int nchunks = inlds ? (nbuf + SEL_CH - 1) / SEL_CH : p.direct ? gchunks : (total + SEL_CH - 1) / SEL_CH;
    for (int ck = wave; ck < nchunks; ck += NMSP_WAVES) {
      const unsigned long long* src;
      int lim;
      if (inlds) {
        src = buf + ck * SEL_CH;
        lim = nbuf - ck * SEL_CH;
      } else if (p.direct) {
        int lo = 0, hb = ng;  // bucket of this chunk: head[lo] <= ck < head[lo + 1]
        while (hb - lo > 1) {
          const int mid = (lo + hb) >> 1;
          if (L.head[mid] <= ck) lo = mid; else hb = mid;
        }
        const int first = (ck - L.head[lo]) * SEL_CH;
        src = gv + (long)lo * a.A + first;
        lim = L.gc[lo] - first;
      } else {
        src = gv + (long)ck * SEL_CH;
        lim = total - ck * SEL_CH;
      }
      unsigned long long vv[SEL_U];
#pragma unroll
      for (int u = 0; u < SEL_U; ++u) vv[u] = u * 64 + lane < lim ? src[u * 64 + lane] : ~0ull;
#pragma unroll
      for (int u = 0; u < SEL_U; ++u) {
        const unsigned long long v = vv[u];
        const bool in = u * 64 + lane < lim && (v & mask) == prefix;
        const int d = (int)(v >> shift) & ((1 << w) - 1);
        unsigned long long left = __ballot(in);
        if (compact && left) {
          int base = 0;
          if (lane == 0) base = atomicAdd(&L.cnt, __popcll(left));
          base = __shfl(base, 0, 64);
          if (in) buf[base + __popcll(left & ((1ull << lane) - 1ull))] = v;
        }
        while (left) {
          const int lead = __builtin_ctzll(left);
          const int d0 = __shfl(d, lead, 64);
          const unsigned long long mm = __ballot(in && d == d0);
          if (lane == lead) atomicAdd(&hist[d0], __popcll(mm));
          left &= ~mm;
        }
      }
    }
    __syncthreads();
    // digit holding the need-th key: 4 bins per thread, block scan of the per-thread sums
    int loc[SEL_BINS / NMSP_THREADS], sum = 0;
#pragma unroll
    for (int k = 0; k < SEL_BINS / NMSP_THREADS; ++k) sum += loc[k] = hist[tid * (SEL_BINS / NMSP_THREADS) + k];
    int acc = nmsp_block_scan(sum, L.wsum);
    if (acc < need && need <= acc + sum) {
#pragma unroll
      for (int k = 0; k < SEL_BINS / NMSP_THREADS; ++k) {
        if (need <= acc + loc[k]) {
          L.bcast = prefix | ((unsigned long long)(tid * (SEL_BINS / NMSP_THREADS) + k) << shift);
          L.sel[0] = need - acc;
          L.sel[1] = loc[k];
          break;
        }
        acc += loc[k];
      }
    }
    __syncthreads();
    prefix = L.bcast;
    need = L.sel[0];
    m = L.sel[1];
    if (compact) nbuf = L.cnt;
    mask |= (unsigned long long)((1 << w) - 1) << shift;
    inlds = inlds || compact;
    hi = shift;
    __syncthreads();
  }
  if (tid == 0) p.thr[b] = prefix;
}

// the k-th smallest of the n (> k) distinct keys keys[0..n) in LDS (outside the histogram's first 16 KiB of L.sk)
__device__ unsigned long long nmsp_kth_lds(const unsigned long long* keys, int n, int k, NmspLds& L) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int* hist = reinterpret_cast<int*>(L.sk);
  unsigned long long prefix = 0ull, mask = 0ull;
  int need = k;
  for (int hi = 64; hi > 0;) {
    const int w = hi < SEL_W ? hi : SEL_W, shift = hi - w;
    for (int i = tid; i < SEL_BINS; i += NMSP_THREADS) hist[i] = 0;
    __syncthreads();
    for (int i0 = wave * 64; i0 < n; i0 += NMSP_THREADS) {
      const int i = i0 + lane;
      const unsigned long long v = i < n ? keys[i] : ~0ull;
      const bool in = i < n && (v & mask) == prefix;
      const int d = (int)(v >> shift) & ((1 << w) - 1);
      unsigned long long left = __ballot(in);
      while (left) {
        const int lead = __builtin_ctzll(left);
        const int d0 = __shfl(d, lead, 64);
        const unsigned long long mm = __ballot(in && d == d0);
        if (lane == lead) atomicAdd(&hist[d0], __popcll(mm));
        left &= ~mm;
      }
    }
    __syncthreads();
    int loc[SEL_BINS / NMSP_THREADS], sum = 0;
#pragma unroll
    for (int q = 0; q < SEL_BINS / NMSP_THREADS; ++q) sum += loc[q] = hist[tid * (SEL_BINS / NMSP_THREADS) + q];
    int acc = nmsp_block_scan(sum, L.wsum);
    if (acc < need && need <= acc + sum) {
#pragma unroll
      for (int q = 0; q < SEL_BINS / NMSP_THREADS; ++q) {
        if (need <= acc + loc[q]) {
          L.bcast = prefix | ((unsigned long long)(tid * (SEL_BINS / NMSP_THREADS) + q) << shift);
          L.sel[0] = need - acc;
          break;
        }
        acc += loc[q];
      }
    }
    __syncthreads();
    prefix = L.bcast;
    need = L.sel[0];
    mask |= (unsigned long long)((1 << w) - 1) << shift;
    hi = shift;
    __syncthreads();
  }
  return prefix;
}

// Greedy NMS over the sorted bucket L.sk[0..n) by the whole workgroup, 64 candidates (one per lane) per tile, with
// the same survivors as torchvision's sequential scan: a candidate is dropped iff an earlier KEPT box overlaps it
// by more than iou. Per tile: (1) every wave tests the tile against its share of the kept boxes of earlier tiles;
// (2) wave 0 computes the in-tile overlap bits (bit j of lane l: candidate j < l overlaps l) and (3) resolves the
// tile in order with one ballot per kept candidate; kept boxes are appended in order. IoU arithmetic as the
// reference: inter / (area_kept + area_candidate - inter). Returns the kept count.
__device__ __forceinline__ int nmsp_greedy(const NmsP& p, NmspLds& L, int b, int c, int item, int n) {
  const NmsArgs& a = p.a;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nc = a.nc;
  const unsigned long long below = (1ull << lane) - 1ull;
  const float offc = a.agnostic ? 0.f : (float)c * a.max_wh;  // x[:, 5:6] * (0 if agnostic else max_wh)
  int nk = 0;
  for (int t0 = 0; t0 < n; t0 += 64) {
    const unsigned long long v = t0 + lane < n ? L.sk[t0 + lane] : ~0ull;
    const bool live = v != ~0ull;
    if (!__ballot(live)) break;  // block-uniform: every wave reads the same tile
    float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;
    if (live) {
      float bx[4];
      box_of_anchor(a, b, (int)(unsigned)v / nc, bx);
      q0 = bx[0] + offc;
      q1 = bx[1] + offc;
      q2 = bx[2] + offc;
      q3 = bx[3] + offc;
    }
    const float area = (q2 - q0) * (q3 - q1);
    if (tid == 0) L.supw = 0ull;
    if (tid < 64) L.mt[tid] = 0ull;
    __syncthreads();
    bool sup = !live;
    for (int k = wave; k < nk; k += NMSP_WAVES) {
      if (!sup) {
        const float xx1 = fmaxf(L.kb[k][0], q0), yy1 = fmaxf(L.kb[k][1], q1);
        const float xx2 = fminf(L.kb[k][2], q2), yy2 = fminf(L.kb[k][3], q3);
        const float w = fmaxf(0.f, xx2 - xx1), h = fmaxf(0.f, yy2 - yy1);
        const float inter = w * h;
        const float ovr = inter / (L.ka[k] + area - inter);  // torchvision: inter / (iarea + areas[j] - inter)
        sup = ovr > a.iou;
      }
    }
    const unsigned long long sm = __ballot(sup);
    if (lane == 0 && sm) atomicOr(&L.supw, sm);
    {  // in-tile overlap bits: wave w tests the earlier candidates j = w, w + 16, ...
      unsigned long long M = 0ull;
      for (int j = wave; j < 63; j += NMSP_WAVES) {
        const float o0 = __shfl(q0, j, 64), o1 = __shfl(q1, j, 64), o2 = __shfl(q2, j, 64), o3 = __shfl(q3, j, 64);
        const float aj = __shfl(area, j, 64);
        if (j < lane && live) {
          const float xx1 = fmaxf(o0, q0), yy1 = fmaxf(o1, q1);
          const float xx2 = fminf(o2, q2), yy2 = fminf(o3, q3);
          const float w = fmaxf(0.f, xx2 - xx1), h = fmaxf(0.f, yy2 - yy1);
          const float inter = w * h;
          const float ovr = inter / (aj + area - inter);
          if (ovr > a.iou) M |= 1ull << j;
        }
      }
      if (M) atomicOr(&L.mt[lane], M);
    }
    __syncthreads();
    if (wave == 0) {
      const unsigned long long M = L.mt[lane];  // earlier in-tile candidates overlapping this one
      unsigned long long alive = ~L.supw & __ballot(live), keptm = 0ull;
      int room = a.max_det - nk;
      while (alive && room > 0) {
        const int j = __builtin_ctzll(alive);
        keptm |= 1ull << j;
        --room;
        alive &= ~(1ull << j);
        alive &= ~__ballot((M >> j) & 1ull);
      }
      if ((keptm >> lane) & 1ull) {
        const int r = nk + __popcll(keptm & below);
        L.kb[r][0] = q0;
        L.kb[r][1] = q1;
        L.kb[r][2] = q2;
        L.kb[r][3] = q3;
        L.ka[r] = area;
        p.kept[(long)item * a.max_det + r] = v;
      }
      if (lane == 0) L.sel[0] = nk + __popcll(keptm);
    }
    __syncthreads();
    nk = L.sel[0];
    if (nk >= a.max_det) break;
  }
  return nk;
}

__global__ void __launch_bounds__(NMSP_THREADS) nms_persistent_kernel(NmsP p) {
  const NmsArgs& a = p.a;
  __shared__ NmspLds L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int B = a.B, ng = a.ng, nc = a.nc;
  const int nch64 = cdiv_d(a.A, 64);
  const long nwaves = (long)gridDim.x * NMSP_WAVES;
  const long wave0 = (long)blockIdx.x * NMSP_WAVES + (tid >> 6);
  const int ncur = B * ng + 2 * B + (p.sel_hist ? B * HIST_BINS : 0);  // cursors, totals, compaction, histograms
  unsigned* ctl = p.ctl;

  // cursors: zero unless the previous launch recorded that it left exactly these words zero
  const unsigned long long cp = (unsigned long long)p.cur;
  const bool rec = ld_rlx(&ctl[CTL_REC_OK]) == 1u && ld_rlx(&ctl[CTL_REC_LO]) == (unsigned)cp &&
                   ld_rlx(&ctl[CTL_REC_HI]) == (unsigned)(cp >> 32) && ld_rlx(&ctl[CTL_REC_N]) == (unsigned)ncur;
  const bool zero_pass = !(p.direct && rec);
  if (zero_pass) {
    for (long i = (long)blockIdx.x * NMSP_THREADS + tid; i < ncur; i += (long)gridDim.x * NMSP_THREADS) p.cur[i] = 0;
    if (!p.direct)
      for (long i = (long)blockIdx.x * NMSP_THREADS + tid; i < (long)B * ng; i += (long)gridDim.x * NMSP_THREADS)
        p.gcnt[i] = 0;
    nmsp_grid_sync(ctl);
    if (blockIdx.x == 0 && tid == 0) st_rlx(&ctl[CTL_REC_OK], 0u);  // every workgroup has read the record
  }
  if (p.stop == 10) return;

  // P0 fill
  if (p.direct) {
    for (long it = wave0; it < (long)B * nch64; it += nwaves) nmsp_fill_direct(p, (int)(it / nch64), (int)(it % nch64));
    nmsp_grid_sync(ctl);
    if (!zero_pass && blockIdx.x == 0 && tid == 0) st_rlx(&ctl[CTL_REC_OK], 0u);
  } else {
    for (long it = wave0; it < (long)B * nch64; it += nwaves)
      nmsp_count_scanned(p, (int)(it / nch64), (int)(it % nch64));
    nmsp_grid_sync(ctl);
    for (int b = blockIdx.x; b < B; b += gridDim.x) {  // bucket offsets per image (ng <= 1024: one group per thread)
      const int c = tid < ng ? ld_rlx(&p.gcnt[b * ng + tid]) : 0;
      const int off = nmsp_block_scan(c, L.wsum);
      if (tid < ng) {
        a.offs[b * ng + tid] = off;
        a.counts[b * ng + tid] = c;
        if (tid == ng - 1) p.tot[b] = off + c;
      }
    }
    nmsp_grid_sync(ctl);
    for (long it = wave0; it < (long)B * nch64; it += nwaves)
      nmsp_fill_scanned(p, (int)(it / nch64), (int)(it % nch64));
    nmsp_grid_sync(ctl);
  }
  if (p.stop == 1) return;

  // P1 max_nms select (uniform decision: every workgroup reads the same totals)
  bool any_sel = false;
  for (int b = 0; b < B; ++b) any_sel |= ld_rlx(&p.tot[b]) > a.max_nms;
  if (any_sel && p.sel_hist) {
    // distributed select: (1) per image, the digit of the max_nms-th key from the fill-time histogram
    for (int b = blockIdx.x; b < B; b += gridDim.x) {
      const int total = ld_rlx(&p.tot[b]);
      if (total <= a.max_nms) {  // block-uniform
        if (tid == 0) p.seld[3 * b] = -1;
        continue;
      }
      constexpr int PER = HIST_BINS / NMSP_THREADS;  // 64 consecutive bins per thread
      const int* hb = p.hist + (long)b * HIST_BINS + tid * PER;
      int sum = 0;
      for (int k = 0; k < PER; ++k) sum += ld_rlx(&hb[k]);
      int acc = nmsp_block_scan(sum, L.wsum);
      const int need = a.max_nms;
      if (acc < need && need <= acc + sum) {
        for (int k = 0; k < PER; ++k) {
          const int c = ld_rlx(&hb[k]);
          if (need <= acc + c) {
            p.seld[3 * b] = tid * PER + k;
            p.seld[3 * b + 1] = need - acc;
            p.seld[3 * b + 2] = c;
            break;
          }
          acc += c;
        }
      }
    }
    nmsp_grid_sync(ctl);
    // (2) every wave compacts the keys under its bucket's image digit (images whose digit holds <= SEL_CAP keys)
    for (long it = wave0; it < (long)B * ng; it += nwaves) {
      const int b = (int)(it / ng);
      const int d1 = ld_rlx(&p.seld[3 * b]);
      if (d1 < 0 || ld_rlx(&p.seld[3 * b + 2]) > SEL_CAP) continue;  // wave-uniform
      const int n = p.direct ? p.cur[it] : a.counts[it];
      const unsigned long long* cv = p.direct ? p.cand + it * a.A : p.cand + (long)b * a.cap + a.offs[it];
      for (int i0 = 0; i0 < n; i0 += SEL_CH) {
        unsigned long long vv[SEL_U];
#pragma unroll
        for (int u = 0; u < SEL_U; ++u) vv[u] = i0 + u * 64 + lane < n ? cv[i0 + u * 64 + lane] : ~0ull;
#pragma unroll
        for (int u = 0; u < SEL_U; ++u) {
          const bool in = i0 + u * 64 + lane < n && (int)(vv[u] >> (64 - HIST_W)) == d1;
          const unsigned long long m = __ballot(in);
          if (!m) continue;
          int base = 0;
          if (lane == 0) base = atomicAdd(&p.ccur[b], __popcll(m));
          base = __shfl(base, 0, 64);
          if (in) p.comp[(long)b * SEL_CAP + base + __popcll(m & ((1ull << lane) - 1ull))] = vv[u];
        }
      }
    }
    nmsp_grid_sync(ctl);
    // (3) per image: the rank-th key among the compacted ones (LDS radix select); too many under the digit: the
    // per-image select over all keys
    for (int b = blockIdx.x; b < B; b += gridDim.x) {
      const int d1 = ld_rlx(&p.seld[3 * b]);
      if (d1 < 0) continue;  // block-uniform
      const int m1 = ld_rlx(&p.seld[3 * b + 2]);
      if (m1 > SEL_CAP) {
        nmsp_select(p, L, b, ld_rlx(&p.tot[b]));
        continue;
      }
      unsigned long long* buf = L.sk + SEL_BINS / 2;
      for (int i = tid; i < m1; i += NMSP_THREADS) buf[i] = p.comp[(long)b * SEL_CAP + i];
      __syncthreads();
      const unsigned long long T = nmsp_kth_lds(buf, m1, ld_rlx(&p.seld[3 * b + 1]), L);
      if (tid == 0) p.thr[b] = T;
      __syncthreads();
    }
    nmsp_grid_sync(ctl);
  } else if (any_sel) {
    for (int b = blockIdx.x; b < B; b += gridDim.x) {
      const int total = ld_rlx(&p.tot[b]);
      if (total > a.max_nms) nmsp_select(p, L, b, total);  // block-uniform
    }
    nmsp_grid_sync(ctl);
  }
  if (p.stop == 2) return;

  // P2 per (image, group): compact (keys <= threshold), sort, greedy
  for (int item = blockIdx.x; item < B * ng; item += gridDim.x) {
    const int b = item / ng, c = item - b * ng;
    const int n0 = p.direct ? p.cur[item] : a.counts[item];
    const unsigned long long* cv = p.direct ? p.cand + (long)item * a.A : p.cand + (long)b * a.cap + a.offs[item];
    const unsigned long long T = any_sel && ld_rlx(&p.tot[b]) > a.max_nms ? p.thr[b] : ~0ull;
    int nk = 0;
    if (n0 > 0) {
      if (tid == 0) L.cnt = 0;
      __syncthreads();
      for (int i0 = (tid >> 6) * 256; i0 < n0; i0 += NMSP_THREADS * 4) {  // 4 loads per lane in flight
        unsigned long long vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) vv[u] = i0 + u * 64 + lane < n0 ? cv[i0 + u * 64 + lane] : ~0ull;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool keep = vv[u] <= T && vv[u] != ~0ull;
          const unsigned long long m = __ballot(keep);
          if (!m) continue;
          int base = 0;
          if (lane == 0) base = atomicAdd(&L.cnt, __popcll(m));
          base = __shfl(base, 0, 64);
          if (keep) L.sk[base + __popcll(m & ((1ull << lane) - 1ull))] = vv[u];
        }
      }
      __syncthreads();
      const int nn = L.cnt;
      int n = 1;
      while (n < nn) n <<= 1;
      for (int i = nn + tid; i < n; i += NMSP_THREADS) L.sk[i] = ~0ull;
      __syncthreads();
      if (p.stop != 21) nmsp_bitonic(L.sk, n);
      if (nn > 0 && p.stop != 20 && p.stop != 21) nk = nmsp_greedy(p, L, b, c, item, nn);
    }
    if (tid == 0) a.nkept[item] = nk;
    __syncthreads();
  }
  nmsp_grid_sync(ctl);
  if (p.stop == 3) return;

  // P3 merge per image (workgroup b): the groups' kept lists are gathered into LDS in batches that fit; whenever
  // more than max_det keys are held, an LDS radix select keeps the max_det smallest. The survivors, sorted, are the
  // output rows (the max_det smallest keys over all kept lists, i.e. the reference's final order and cut).
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const long kb0 = (long)b * ng * a.max_det;
    unsigned long long* buf = L.sk + SEL_BINS / 2;  // SEL_CAP keys after the select histogram
    unsigned long long* tmp = L.sk;                 // <= max_det survivors (histogram space, free after a select)
    const int c = tid < ng ? a.nkept[b * ng + tid] : 0;
    const int off = nmsp_block_scan(c, L.wsum);
    if (tid < ng) L.head[tid] = off;
    if (tid == ng - 1) L.head[ng] = off + c;
    __syncthreads();
    int run = 0;
    for (int g = 0; g < ng;) {
      int g2 = g + 1;  // groups [g, g2) fit after the run (one group holds <= max_det <= SEL_CAP - max_det keys)
      while (g2 < ng && run + L.head[g2 + 1] - L.head[g] <= SEL_CAP) ++g2;
      for (int gg = g + (tid >> 6); gg < g2; gg += NMSP_WAVES) {
        const int nk = L.head[gg + 1] - L.head[gg];
        unsigned long long* dst = buf + run + L.head[gg] - L.head[g];
        for (int i = lane; i < nk; i += 64) dst[i] = p.kept[kb0 + (long)gg * a.max_det + i];
      }
      int n = run + L.head[g2] - L.head[g];
      __syncthreads();
      if (n > a.max_det) {
        const unsigned long long T = nmsp_kth_lds(buf, n, a.max_det, L);
        if (tid == 0) L.cnt = 0;
        __syncthreads();
        for (int i0 = (tid >> 6) * 64; i0 < n; i0 += NMSP_THREADS) {
          const int i = i0 + lane;
          const bool keep = i < n && buf[i] <= T;
          const unsigned long long m = __ballot(keep);
          if (!m) continue;
          int base = 0;
          if (lane == 0) base = atomicAdd(&L.cnt, __popcll(m));
          base = __shfl(base, 0, 64);
          if (keep) tmp[base + __popcll(m & ((1ull << lane) - 1ull))] = buf[i];
        }
        __syncthreads();
        for (int i = tid; i < a.max_det; i += NMSP_THREADS) buf[i] = tmp[i];
        n = a.max_det;
        __syncthreads();
      }
      run = n;
      g = g2;
    }
    int n = 1;
    while (n < run) n <<= 1;
    for (int i = run + tid; i < n; i += NMSP_THREADS) buf[i] = ~0ull;
    __syncthreads();
    nmsp_bitonic(buf, n);
    const int nout = run;
    for (int r = tid; r < nout; r += NMSP_THREADS) {
      const unsigned long long v = buf[r];
      const int key = (int)(unsigned)v;
      float bx[4];
      box_of_anchor(a, b, key / nc, bx);
      float* o = a.out + ((long)b * a.max_det + r) * 6;
      o[0] = bx[0];
      o[1] = bx[1];
      o[2] = bx[2];
      o[3] = bx[3];
      o[4] = key_score(v);
      o[5] = (float)(key % nc);
    }
    // a grid barrier that timed out (CTL_ERR, set before this phase's last barrier released) leaves the phases
    // unordered: report -1 detections so the host fails loudly instead of reading a wrong selection
    if (tid == 0) a.nout[b] = ld_rlx(&ctl[CTL_ERR]) ? -1 : nout;
    __syncthreads();
  }
  if (p.direct) {  // leave the cursors zero for the next launch, and say so
    for (long i = (long)blockIdx.x * NMSP_THREADS + tid; i < ncur; i += (long)gridDim.x * NMSP_THREADS) p.cur[i] = 0;
    if (blockIdx.x == 0 && tid == 0) {
      st_rlx(&ctl[CTL_REC_LO], (unsigned)cp);
      st_rlx(&ctl[CTL_REC_HI], (unsigned)(cp >> 32));
      st_rlx(&ctl[CTL_REC_N], (unsigned)ncur);
      st_rlx(&ctl[CTL_REC_OK], 1u);
    }
  }
}

}  // namespace adr

using namespace adr;

namespace {

struct WsCarve {
  char* p;
  size_t used = 0;
  template <class T>
  T* take(size_t n) {
    used = (used + 255) & ~(size_t)255;
    T* r = reinterpret_cast<T*>(p ? p + used : nullptr);
    used += n * sizeof(T);
    return r;
  }
};

// chain layout (ADR_NMS_MODE=chain: the six-kernel pipeline), after the zero region
void carve_chain(NmsArgs& a, WsCarve& w, int B, int nc, int A, int multi, int max_det) {
  const size_t cap = (size_t)A * (multi ? nc : 1);
  a.counts = w.take<int>((size_t)B * nc);
  a.offs = w.take<int>((size_t)B * nc);
  a.cscore = w.take<float>(B * cap);
  a.ckey = w.take<int>(B * cap);
  a.ccls = w.take<int>(B * cap);
  a.thr = w.take<unsigned>((size_t)B * 2);
  a.kept = w.take<int>((size_t)B * nc * max_det);
  a.nkept = w.take<int>((size_t)B * nc);
  a.ccnt = w.take<int>((size_t)B * cdiv(A, 256) * nc);
}

void carve_persistent(NmsP& p, WsCarve& w, int B, int nc, int A, int multi, int max_det, bool direct) {
  const size_t cap = (size_t)A * (multi ? nc : 1);
  // fill cursors, per-image totals, select compaction cursors, top-digit histograms (contiguous: one record)
  p.cur = w.take<int>((size_t)B * nc + 2 * B + (size_t)B * HIST_BINS);
  p.seld = w.take<int>((size_t)B * 3);
  p.comp = w.take<unsigned long long>((size_t)B * SEL_CAP);
  p.a.nkept = w.take<int>((size_t)B * nc);
  p.thr = w.take<unsigned long long>(B);
  p.kept = w.take<unsigned long long>((size_t)B * nc * max_det);
  if (direct) {
    p.cand = w.take<unsigned long long>((size_t)B * nc * A);
    return;
  }
  p.a.counts = w.take<int>((size_t)B * nc);
  p.a.offs = w.take<int>((size_t)B * nc);
  p.gcnt = w.take<int>((size_t)B * nc);
  p.cand = w.take<unsigned long long>(B * cap);
  if (multi)
    p.masks = w.take<unsigned long long>((size_t)B * cdiv(A, 64) * nc);
  else
    p.best = w.take<unsigned long long>((size_t)B * A);
}

// control words: a fixed NMSP_CTL_BYTES at the start of the workspace (zero on first use)
void carve_zero(NmsP& p, WsCarve& w) {
  p.ctl = w.take<unsigned>(CTL_WORDS);
  w.used = (w.used + 255) & ~(size_t)255;
}

// direct bucket layout while the B * nc * A slot array stays within 1 GiB (ADR_NMS_DIRECT=0 forces the scanned one)
bool nms_direct(int B, int nc, int A) {
  const char* e = getenv("ADR_NMS_DIRECT");
  if (e && !strcmp(e, "0")) return false;
  return (size_t)B * nc * A * 8 <= ((size_t)1 << 30);
}

int nmsp_grid(int want) {
  static int dev_cached = -1, cap = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != dev_cached) {
    int cus = 0, per = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)nms_persistent_kernel, NMSP_THREADS, 0);
    cap = cus * per;
    dev_cached = dev;
  }
  return cap < want ? cap : want;
}

bool getenv_is(const char* k, const char* v) {
  const char* e = getenv(k);
  return e && !strcmp(e, v);
}

bool nms_chain_mode() {
  const char* e = getenv("ADR_NMS_MODE");
  return e && !strcmp(e, "chain");
}

}  // namespace

extern "C" size_t adr_nms_workspace(int B, int nc, int A, int multi, int max_det) {
  NmsP p{};
  WsCarve z{nullptr};
  carve_zero(p, z);
  WsCarve c{nullptr, z.used}, q{nullptr, z.used};
  carve_chain(p.a, c, B, nc, A, multi, max_det);
  carve_persistent(p, q, B, nc, A, multi, max_det, nms_direct(B, nc, A));
  return (c.used > q.used ? c.used : q.used) + 256;
}

// After a barrier timeout (counts of -1) the control words are in an unknown state: CTL_ERR is sticky and the
// arrival flags may be a generation apart. Zeroing them in place, on the stream, returns the workspace to its
// first-use state without freeing it, so a hipGraph that captured adr_nms on this workspace stays valid (the next
// launch also re-zeroes its cursors: the record word is cleared).
extern "C" int adr_nms_reset(void* ws, size_t ws_bytes, void* stream) {
  ADR_REQUIRE(ws && ws_bytes >= NMSP_CTL_BYTES, "nms_reset: workspace of %zu bytes", ws_bytes);
  if (hipMemsetAsync(ws, 0, NMSP_CTL_BYTES, (hipStream_t)stream) != hipSuccess) {
    set_error("nms_reset: hipMemsetAsync failed");
    return ADR_ERR_LAUNCH;
  }
  return ADR_OK;
}

extern "C" int adr_nms(const float* y, int B, int nc, int A, float conf, float iou, int multi, int agnostic,
                       const unsigned char* class_mask, int max_det, int max_nms, float max_wh, float* out, int* nout,
                       void* ws, size_t ws_bytes, void* stream) {
  ADR_REQUIRE(B > 0 && nc >= 1 && nc <= 1024 && max_det >= 1 && max_det <= 300 && A >= 1 && A <= NMS_SORT_CAP &&
                  max_nms >= 1,
              "nms: B=%d nc=%d max_det=%d A=%d max_nms=%d unsupported", B, nc, max_det, A, max_nms);
  ADR_REQUIRE(!(agnostic && multi), "nms: agnostic multi-label groups exceed the per-group sort capacity");
  ADR_REQUIRE(ws_bytes >= adr_nms_workspace(B, nc, A, multi, max_det), "nms: workspace");
  NmsP p{};
  NmsArgs& a = p.a;
  a.y = y; a.B = B; a.nc = nc; a.A = A; a.conf = conf; a.iou = iou; a.multi = multi; a.max_det = max_det;
  a.max_nms = max_nms; a.max_wh = max_wh;
  a.agnostic = agnostic; a.ng = agnostic ? 1 : nc; a.cmask = class_mask;
  a.cap = A * (multi ? nc : 1);
  a.out = out;
  a.nout = nout;
  WsCarve w{(char*)ws};
  carve_zero(p, w);
  hipStream_t st = (hipStream_t)stream;
  if (nms_chain_mode()) {
    a.rec_ok = p.ctl + CTL_REC_OK;
    carve_chain(a, w, B, nc, A, multi, max_det);
    const int nch = cdiv(A, 256);
    hipLaunchKernelGGL(nms_count_kernel, dim3(nch, B), dim3(256), 0, st, a);
    hipLaunchKernelGGL(nms_scan_kernel, dim3(B), dim3(256), 0, st, a, nch);
    hipLaunchKernelGGL(nms_fill_kernel, dim3(nch, B), dim3(256), 0, st, a);
    hipLaunchKernelGGL(nms_select_kernel, dim3(B), dim3(256), 0, st, a);
    hipLaunchKernelGGL(nms_class_kernel, dim3(B * a.ng), dim3(256), 0, st, a);
    hipLaunchKernelGGL(nms_merge_kernel, dim3(B), dim3(64), 0, st, a);
    return check_launch("adr_nms");
  }
  p.direct = nms_direct(B, nc, A);
  carve_persistent(p, w, B, nc, A, multi, max_det, p.direct);
  p.tot = p.cur + (size_t)B * a.ng;
  p.ccur = p.tot + B;
  p.hist = p.ccur + B;
  p.sel_hist = (long)A * (multi ? a.ng : 1) > max_nms && !getenv_is("ADR_NMS_DSEL", "0");
  const long waves = (long)B * cdiv(A, 64);
  const long want = std::max<long>(cdiv(waves, NMSP_WAVES), (long)B * a.ng);
  const int grid = nmsp_grid((int)std::min<long>(want, NMSP_MAX_GRID));
  ADR_REQUIRE(grid >= 1, "nms: persistent kernel has no resident capacity");
  const char* st_env = getenv("ADR_NMS_STOP");
  p.stop = st_env ? atoi(st_env) : 0;
  hipLaunchKernelGGL(nms_persistent_kernel, dim3(grid), dim3(NMSP_THREADS), 0, st, p);
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

// ---------------- validator TP matching (engine/validator.py:221-261, greedy branch) ----------------
// The reference sorts every (label, detection) pair with IoU >= t by IoU, keeps each detection's best pair, then
// keeps, per label, the surviving pair of the lowest detection index. Restated per detection: best label b(p) =
// argmax_g iou'[g][p] (iou' = iou masked to 0 on class mismatch); at threshold t, p is correct iff iou'[b(p)][p] >= t
// and p is the smallest such detection with that best label. One 1024-thread workgroup per image: the best labels in
// LDS, then, per chunk of labels, first[t][g] = min p by LDS atomicMin (order-independent) and the read-back.
static constexpr int MATCH_THREADS = 1024, MATCH_PMAX = 2048, MATCH_TMAX = 16, MATCH_GCHUNK = 512;

__global__ void __launch_bounds__(MATCH_THREADS)
match_predictions_kernel(const float* __restrict__ iou, int G, int P, const float* __restrict__ gt_cls,
                         const float* __restrict__ pred_cls, const float* __restrict__ thr, int T,
                         unsigned char* __restrict__ correct) {
  __shared__ int bg[MATCH_PMAX];
  __shared__ float bv[MATCH_PMAX];
  __shared__ int first[MATCH_TMAX * MATCH_GCHUNK];
  __shared__ float th[MATCH_TMAX];
  const int tid = threadIdx.x;
  if (tid < T) th[tid] = thr[tid];
  for (int p = tid; p < P; p += MATCH_THREADS) {  // coalesced over p: iou rows are labels
    const float pc = pred_cls[p];
    float best = -1.f;
    int g_best = 0;
    for (int g = 0; g < G; ++g) {
      const float v = gt_cls[g] == pc ? iou[(long)g * P + p] : 0.f;
      if (v >= best) {  // ties: the larger label index
        best = v;
        g_best = g;
      }
    }
    bg[p] = g_best;
    bv[p] = best;
  }
  __syncthreads();
  for (int g0 = 0; g0 < G; g0 += MATCH_GCHUNK) {
    const int gn = min(MATCH_GCHUNK, G - g0);
    for (int i = tid; i < T * MATCH_GCHUNK; i += MATCH_THREADS) first[i] = 0x7fffffff;
    __syncthreads();
    for (int p = tid; p < P; p += MATCH_THREADS) {
      const int g = bg[p] - g0;
      if (g < 0 || g >= gn) continue;
      for (int t = 0; t < T; ++t)
        if (bv[p] >= th[t]) atomicMin(&first[t * MATCH_GCHUNK + g], p);
    }
    __syncthreads();
    for (int p = tid; p < P; p += MATCH_THREADS) {
      const int g = bg[p] - g0;
      if (g < 0 || g >= gn) continue;
      for (int t = 0; t < T; ++t)
        correct[(long)p * T + t] = (unsigned char)(bv[p] >= th[t] && first[t * MATCH_GCHUNK + g] == p);
    }
    __syncthreads();
  }
}

extern "C" int adr_match_predictions(const float* iou, int G, int P, const float* gt_cls, const float* pred_cls,
                                     const float* thr, int T, unsigned char* correct, void* stream) {
  ADR_REQUIRE(G >= 1 && P >= 0 && P <= MATCH_PMAX && T >= 1 && T <= MATCH_TMAX,
              "match_predictions: G=%d P=%d T=%d unsupported (G >= 1, P <= %d, T <= %d)", G, P, T, MATCH_PMAX,
              MATCH_TMAX);
  if (P == 0) return 0;
  hipLaunchKernelGGL(match_predictions_kernel, dim3(1), dim3(MATCH_THREADS), 0, (hipStream_t)stream, iou, G, P, gt_cls,
                     pred_cls, thr, T, correct);
  return check_launch("adr_match_predictions");
}
