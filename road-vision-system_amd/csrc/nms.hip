// Batched Ultralytics non_max_suppression + scale_boxes + class filter on
// gfx950: one workgroup per image.
//
// Reference: src/detect/yolo_ultralytics.py:28-53 -> Ultralytics
// non_max_suppression(conf, iou, max_det, max_nms=30000, max_wh=7680,
// agnostic=False) -> torchvision.ops.nms (CPU kernel semantics: stable
// descending score sort, greedy suppression of later boxes whose IoU with a
// kept box is `> iou_threshold` compared in double, IoU on class-offset
// f32 boxes) -> i[:max_det] -> scale_boxes (subtract pad, divide by gain,
// clip) -> the reference's own post-NMS class filter (classes_keep,
// yolo_ultralytics.py:49-50).
//
// Sort: 64-bit keys (~score_bits, anchor, slot) bitonic-sorted in LDS
// (score desc, anchor asc == the stable order of rows in anchor order).
// One launch: an image with up to 4096 candidates sorts its keys in ~41 KB
// of LDS (so conv blocks still fit beside it when the track stage overlaps
// the next forward); an image with more keeps them in the caller's
// workspace (global memory) -- the same code on either pointer (nms_body).
// kSortCap = 65536 covers every slot of the candidate layout (cap <= 65536),
// so no candidate is ever dropped before the sort.  (r04 ran the overflow
// images in a second launch, one more dependent launch per call.)  max_nms: after the sort only the first max_nms
// keys take part in the greedy pass -- Ultralytics' `if n > max_nms: x =
// x[x[:, 4].argsort(descending=True)[:max_nms]]` (top max_nms by score; ties
// resolved in anchor order like the stable sort of the oracle).
// Greedy: wave 0 walks the sorted list in chunks of 64; each lane tests its
// candidate against every kept box, builds the 64-bit mask of later chunk
// members it would suppress, and a uniform scalar loop resolves the chunk.
#include "conv.h"

namespace rv {

constexpr int kSortCap = 65536;  // candidates per image (overflow pass, keys in global memory)
constexpr int kSortSmall = 4096;  // first pass (32 KB of keys)
constexpr int kMaxDet = 1024;
constexpr int kMaxSeg = 1024;    // 64-candidate segments per image (<= 65536 slots)

struct ScaleArgs {
  float gain;   // f32(gain) as torch divides by the python-float gain
  float pad_x, pad_y;
  float clip_w, clip_h;
};

// compiler-level ordering of LDS accesses between lanes of one wave (the
// hardware executes a wave's LDS ops in order)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float4 offset_box(const Cand& c, float max_wh) {
  const float off = (float)c.cls * max_wh;
  return make_float4(c.x1 + off, c.y1 + off, c.x2 + off, c.y2 + off);
}

// torchvision nms_kernel_impl IoU test: i kept (earlier), j later.
__device__ __forceinline__ bool suppresses(float4 bi, float ai, float4 bj, float aj, double thr) {
  const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
  const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
  const float w = fmaxf(0.f, xx2 - xx1), h = fmaxf(0.f, yy2 - yy1);
  const float inter = w * h;
  const float ovr = inter / (ai + aj - inter);
  return (double)ovr > thr;
}

// LDS bytes of nms_kernel<CAP> for max_det kept boxes (the segment prefix
// region is padded to 16 B so the float4 arrays after it stay aligned)
constexpr int kSegBytes = ((kMaxSeg + 1) * 4 + 15) & ~15;
static size_t nms_smem(int cap_keys, int max_det) {
  const size_t lds_keys = cap_keys > kSortSmall ? 0 : (size_t)cap_keys * 8;  // overflow: global
  return lds_keys + kSegBytes + 64 * (16 + 4 + 8) + (size_t)max_det * (16 + 4 + 4) + 64 * 4;
}

// LDS layout of nms_kernel: [keys (kSortSmall x 8 B; unused by an image
// whose candidates exceed kSortSmall -- its keys go to the workspace)]
// [segment prefix] [chunk masks / boxes / areas] [kept boxes / areas / slots]
struct NmsLds {
  int* segoff;     // kMaxSeg + 1: exclusive prefix + total
  uint64_t* cmask;  // 64
  float4* cbox;     // chunk boxes (64)
  float* carea;     // 64
  float4* kbox;     // kept offset boxes (max_det)
  float* karea;     // max_det
  int* kslot;       // max_det, then the current chunk's 64 slots
};

// Sort the image's n candidates (keys in LDS or, past kSortSmall, in the
// workspace: KEYS is the pointer's type), greedy NMS, scale_boxes + class
// filter.  Every block thread calls it.
template <class KEYS>
__device__ void nms_body(KEYS* keys, int n, const NmsLds& L, const Cand* __restrict__ cb, int nseg,
                         int b, float max_wh, double iou, int max_det, int max_nms, ScaleArgs sc,
                         const uint32_t* __restrict__ keep4, float* __restrict__ out,
                         int* __restrict__ out_n) {
  const int tid = threadIdx.x;
  int* segoff = L.segoff;
  uint64_t* cmask = L.cmask;
  float4* cbox = L.cbox;
  float* carea = L.carea;
  float4* kbox = L.kbox;
  float* karea = L.karea;
  int* kslot = L.kslot;
  __shared__ int s_nkeep;
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (int i = tid; i < np2; i += blockDim.x) keys[i] = ~0ull;
  __syncthreads();
  for (int sl = tid; sl < nseg * 64; sl += blockDim.x) {
    const int j = sl >> 6, k = sl & 63;
    const int pos = segoff[j] + k;
    const int next = j + 1 == nseg ? segoff[kMaxSeg] : segoff[j + 1];
    if (pos < next && pos < n) {
      const Cand c = cb[sl];
      const uint32_t sb = __float_as_uint(c.score);  // score > conf >= 0: bits are monotonic
      keys[pos] = ((uint64_t)(~sb) << 32) | ((uint64_t)(uint32_t)c.anchor << 16) | (uint64_t)sl;
    }
  }
  __syncthreads();
  if (n <= (int)blockDim.x) {
    // rank sort: thread i's key lands at the number of smaller keys (keys
    // are unique: the slot is in the low bits); every thread reads the
    // same key at the same time (an LDS broadcast), so n keys cost n reads
    // and two barriers instead of log2(np2)^2 / 2 bitonic stages
    const uint64_t mine = tid < n ? keys[tid] : ~0ull;
    int r = 0;
    for (int j = 0; j < n; ++j) r += keys[j] < mine ? 1 : 0;
    __syncthreads();
    if (tid < n) keys[r] = mine;
    __syncthreads();
  } else
  // bitonic sort ascending
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < np2 / 2; i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = keys[lo], c = keys[hi];
        if ((a > c) == up) {
          keys[lo] = c;
          keys[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  // Ultralytics max_nms: only the top max_nms by score enter torchvision nms
  if (n > max_nms) n = max_nms;
  // greedy NMS, chunks of 64 candidates (score order), all 16 waves:
  //  1. wave 0 fetches the chunk's boxes into LDS and clears the chunk masks;
  //  2. wave w tests every chunk candidate (its lane) against the kept boxes
  //     k = w, w + 16, ... (suppressed flags -> one ballot per wave) and
  //     against the later chunk members j = w, w + 16, ... (bits of the
  //     lane's chunk mask, OR-ed into LDS);
  //  3. wave 0 resolves the chunk in order -- q kept iff still alive, then
  //     q's mask kills the later members it overlaps -- with every mask in a
  //     register (read across lanes by readlane, no LDS round trip per q).
  // Same decisions as one wave walking each candidate against every kept
  // box (r04): the IoU test is symmetric, order only matters in step 3.
  // (r04's single-wave form paid a serial LDS read per kept box and per
  // chunk member: 48 us for an image of 129 candidates.)
  __shared__ uint64_t supw[16];
  const int lane = tid & 63, wv = tid >> 6;
  const int nwv = blockDim.x >> 6;
  if (tid == 0) s_nkeep = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 64) {
    const int nkeep = s_nkeep;
    if (nkeep >= max_det) break;  // uniform: read after the last barrier
    if (wv == 0) {
      const int i = base + lane;
      float4 bx = make_float4(0.f, 0.f, 0.f, 0.f);
      float ar = 0.f;
      int slot = -1;
      if (i < n) {
        slot = (int)(keys[i] & 0xFFFF);
        bx = offset_box(cb[slot], max_wh);
        ar = (bx.z - bx.x) * (bx.w - bx.y);
      }
      cbox[lane] = bx;
      carea[lane] = ar;
      cmask[lane] = 0;
      kslot[max_det + lane] = slot;  // staged: the chunk's slots (kslot has max_det + 64 entries)
    }
    __syncthreads();
    {
      const bool valid = base + lane < n;
      const float4 bx = cbox[lane];
      const float ar = carea[lane];
      bool sup = !valid;
      for (int k = wv; k < nkeep && !sup; k += nwv) sup = suppresses(kbox[k], karea[k], bx, ar, iou);
      const uint64_t bal = __ballot(sup);
      if (lane == 0) supw[wv] = bal;
      uint64_t m = 0;
      if (valid)
        for (int j = wv; j < 64 && base + j < n; j += nwv)
          if (j > lane && suppresses(bx, ar, cbox[j], carea[j], iou)) m |= 1ull << j;
      if (m) atomicOr((unsigned long long*)&cmask[lane], (unsigned long long)m);
    }
    __syncthreads();
    if (wv == 0) {
      uint64_t supall = 0;
      for (int w = 0; w < nwv; ++w) supall |= supw[w];
      uint64_t alive = ~supall;
      const uint64_t mine = cmask[lane];
      const uint32_t mlo = (uint32_t)mine, mhi = (uint32_t)(mine >> 32);
      uint64_t kept = 0;
      int room = max_det - nkeep;
      while (alive && room > 0) {  // uniform
        const int q = __builtin_ctzll(alive);
        kept |= 1ull << q;
        const uint64_t mq = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(mhi, q) << 32) |
                            (uint64_t)(uint32_t)__builtin_amdgcn_readlane(mlo, q);
        alive &= ~(mq | (1ull << q));
        --room;
      }
      if ((kept >> lane) & 1ull) {
        const int pos = nkeep + __popcll(kept & ((1ull << lane) - 1ull));
        kbox[pos] = cbox[lane];
        karea[pos] = carea[lane];
        kslot[pos] = kslot[max_det + lane];
      }
      if (lane == 0) s_nkeep = nkeep + __popcll(kept);
    }
    __syncthreads();
  }
  // scale_boxes + clip + post-NMS class filter, order preserved
  if (tid < 64) {
    const int nkeep = s_nkeep;
    int w = 0;
    for (int base = 0; base < nkeep; base += 64) {
      const int k = base + tid;
      bool ok = false;
      Cand c;
      if (k < nkeep) {
        c = cb[kslot[k]];
        ok = keep4 == nullptr || ((keep4[(c.cls >> 5) & 3] >> (c.cls & 31)) & 1u);
      }
      const uint64_t bal = __ballot(ok);
      if (ok) {
        const int pos = w + __popcll(bal & ((1ull << tid) - 1ull));
        float x1 = (c.x1 - sc.pad_x) / sc.gain, y1 = (c.y1 - sc.pad_y) / sc.gain;
        float x2 = (c.x2 - sc.pad_x) / sc.gain, y2 = (c.y2 - sc.pad_y) / sc.gain;
        x1 = fminf(fmaxf(x1, 0.f), sc.clip_w);
        y1 = fminf(fmaxf(y1, 0.f), sc.clip_h);
        x2 = fminf(fmaxf(x2, 0.f), sc.clip_w);
        y2 = fminf(fmaxf(y2, 0.f), sc.clip_h);
        float* o = out + ((size_t)b * max_det + pos) * 6;
        o[0] = x1;
        o[1] = y1;
        o[2] = x2;
        o[3] = y2;
        o[4] = c.score;
        o[5] = (float)c.cls;
      }
      w += __popcll(bal);
    }
    if (tid == 0) out_n[b] = w;
  }
}

// One workgroup per image: segment prefix, then nms_body with the keys in
// LDS (n <= kSortSmall: ~41 KB of LDS, so conv blocks still fit beside it
// when the track stage overlaps the next forward) or in the workspace
// (kSortCap = 65536 covers every slot of the candidate layout, so no
// candidate is ever dropped before the sort) -- one launch either way.
__global__ __launch_bounds__(1024) void nms_kernel(const Cand* __restrict__ cand,
                                                   const int* __restrict__ seg_n, int nseg, int cap,
                                                   float max_wh, double iou, int max_det,
                                                   int max_nms, ScaleArgs sc, const uint32_t* __restrict__ keep4,
                                                   float* __restrict__ out, int* __restrict__ out_n,
                                                   int* __restrict__ cand_total,
                                                   uint64_t* __restrict__ gkeys) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  constexpr size_t kLdsKeys = (size_t)kSortSmall * 8;
  NmsLds L;
  L.segoff = (int*)(smem + kLdsKeys);
  L.cmask = (uint64_t*)(smem + kLdsKeys + kSegBytes);
  L.cbox = (float4*)(L.cmask + 64);
  L.carea = (float*)(L.cbox + 64);
  L.kbox = (float4*)(L.carea + 64);
  L.karea = (float*)(L.kbox + max_det);
  L.kslot = (int*)(L.karea + max_det);
  int* segoff = L.segoff;
  __shared__ int wsum[16];
  const Cand* cb = cand + (size_t)b * cap;
  // segment counts -> exclusive prefix (one segment per thread, nseg <= 1024)
  int cnt = 0;
  if (tid < nseg) cnt = min(max(seg_n[(size_t)b * nseg + tid], 0), 64);
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off);
    if ((tid & 63) >= off) incl += v;
  }
  if ((tid & 63) == 63) wsum[tid >> 6] = incl;
  __syncthreads();
  int wpre = 0;
  for (int w = 0; w < (tid >> 6); ++w) wpre += wsum[w];
  if (tid < nseg) segoff[tid] = wpre + incl - cnt;
  if (tid == 0) {
    int tot = 0;
    for (int w = 0; w < 16; ++w) tot += wsum[w];
    segoff[kMaxSeg] = tot;
  }
  __syncthreads();
  const int n = segoff[kMaxSeg];
  if (cand_total && tid == 0) cand_total[b] = n;
  // n <= nseg * 64 <= cap <= kSortCap (checked by the host entry)
  if (n <= kSortSmall)
    nms_body((uint64_t*)smem, n, L, cb, nseg, b, max_wh, iou, max_det, max_nms, sc, keep4, out, out_n);
  else
    nms_body(gkeys + (size_t)b * kSortCap, n, L, cb, nseg, b, max_wh, iou, max_det, max_nms, sc, keep4,
             out, out_n);
}

// Reference-layout candidates: raw (B, 4+nc, A) -> Cand rows (xc filter,
// xywh2xyxy, best class), i.e. the first half of non_max_suppression.  One
// wave per 64-anchor segment, written in the segmented layout of
// rv_nms_postprocess (slot = 64 * segment + rank in anchor order).
__global__ __launch_bounds__(64) void raw_candidates_kernel(const float* __restrict__ raw, int nc,
                                                            int A, float conf,
                                                            Cand* __restrict__ cand, int cap,
                                                            int* __restrict__ seg_n) {
  const int j = blockIdx.x, lane = threadIdx.x;
  const int a = j * 64 + lane;
  const int b = blockIdx.y;
  const float* r = raw + (size_t)b * (4 + nc) * A;
  float best = -INFINITY;
  int bc = 0;
  if (a < A)
    for (int c = 0; c < nc; ++c) {
      const float s = r[(size_t)(4 + c) * A + a];
      if (s > best) {
        best = s;
        bc = c;
      }
    }
  const bool pass = a < A && best > conf;
  const unsigned long long m = __ballot(pass);
  if (lane == 0) seg_n[(size_t)b * gridDim.x + j] = __popcll(m);
  if (!pass) return;
  const int i = j * 64 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  const float cx = r[a], cy = r[(size_t)A + a], w = r[(size_t)2 * A + a], h = r[(size_t)3 * A + a];
  const float hw = w / 2.0f, hh = h / 2.0f;
  if (i < cap) {
    Cand c;
    c.x1 = cx - hw;
    c.y1 = cy - hh;
    c.x2 = cx + hw;
    c.y2 = cy + hh;
    c.score = best;
    c.cls = bc;
    c.anchor = a;
    c.pad = 0;
    cand[(size_t)b * cap + i] = c;
  }
}

}  // namespace rv

using namespace rv;

// LDS of the first pass at the largest max_det (the overflow pass needs less)
extern "C" size_t rv_nms_smem_bytes(void) { return nms_smem(kSortSmall, kMaxDet); }

// Workspace of rv_nms_postprocess: the overflow pass's sort keys.
extern "C" size_t rv_nms_ws_bytes(int B) { return (size_t)(B > 0 ? B : 0) * kSortCap * 8; }

extern "C" int rv_nms_postprocess(const void* cand, const int* seg_n, int B, int cap, int nseg,
                                  float iou, int max_det, int max_nms, float max_wh,
                                  const float* scale5,
                                  const uint32_t* keep_mask4, float* out, int* out_n,
                                  int* cand_total, void* ws, size_t ws_bytes, void* stream) {
  RV_CHECK_ARG(cand && seg_n && out && out_n && scale5, "null pointer");
  RV_CHECK_ARG(B >= 0 && cap > 0 && cap <= 65536, "cap %d outside (0, 65536]", cap);
  RV_CHECK_ARG(nseg > 0 && nseg <= kMaxSeg && nseg * 64 <= cap,
               "nseg %d: need 0 < nseg <= %d and nseg * 64 <= cap %d", nseg, kMaxSeg, cap);
  RV_CHECK_ARG(max_det > 0 && max_det <= kMaxDet, "max_det %d outside (0, %d]", max_det, kMaxDet);
  RV_CHECK_ARG(max_nms > 0, "max_nms %d must be positive", max_nms);
  static_assert(kSortCap >= 65536, "the overflow pass must hold every slot of cap <= 65536");
  RV_CHECK_ARG(ws && ws_bytes >= rv_nms_ws_bytes(B), "workspace %zu B < rv_nms_ws_bytes(%d) = %zu",
               ws_bytes, B, rv_nms_ws_bytes(B));
  if (B == 0) return RV_OK;
  ScaleArgs sc;
  sc.gain = scale5[0];
  sc.pad_x = scale5[1];
  sc.pad_y = scale5[2];
  sc.clip_w = scale5[3];
  sc.clip_h = scale5[4];
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)nms_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)rv_nms_smem_bytes());
    if (e != hipSuccess) {
      set_error("hipFuncSetAttribute(NMS LDS): %s", hipGetErrorString(e));
      (void)hipGetLastError();
      return -(int)e;
    }
    attr = true;
  }
  nms_kernel<<<B, 1024, nms_smem(kSortSmall, max_det), as_stream(stream)>>>(
      (const Cand*)cand, seg_n, nseg, cap, max_wh, (double)iou, max_det, max_nms, sc, keep_mask4,
      out, out_n, cand_total, (uint64_t*)ws);
  return launch_status("rv_nms_postprocess");
}

extern "C" int rv_cand_segments(int A) { return A > 0 ? ceil_div(A, 64) : 0; }

extern "C" int rv_candidates_from_raw(const float* raw, int B, int nc, int A, float conf,
                                      void* cand, int cap, int* seg_n, void* stream) {
  RV_CHECK_ARG(raw && cand && seg_n, "null pointer");
  RV_CHECK_ARG(B >= 0 && nc > 0 && A > 0 && A < 65536 && cap >= ceil_div(A, 64) * 64,
               "bad raw shape / cap < 64 * ceil(A / 64)");
  if (B == 0) return RV_OK;
  raw_candidates_kernel<<<dim3(ceil_div(A, 64), B), 64, 0, as_stream(stream)>>>(
      raw, nc, A, conf, (Cand*)cand, cap, seg_n);
  return launch_status("rv_candidates_from_raw");
}
