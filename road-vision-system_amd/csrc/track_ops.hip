// Standalone tracker / geometry entries (SURVEY §8(b) Tracker and Geometry
// rows): the pieces of SortTracker.update a maintainer can swap in one at a
// time, batched over S independent camera streams.  The fused per-stream
// kernel (sort.hip, rv_sort_update) runs the same math inside one launch.
//
//   rv_iou_matrix_batched     _iou_matrix   sort_tracker.py:74-80 (+ _iou :55-71)
//   rv_greedy_assign_batched  _associate    sort_tracker.py:182-210 (the loop)
//   rv_homography_project_f64 project_bbox + distance, projector.py:30-47,74-84
//   rv_untracked_metrics      the tracker-off branch of main_preview.py:101-109:
//                             no track ids or speeds, distance_for_bbox per det
//
// All latency-bound small work: one workgroup per stream for the IoU and
// the assignment, one thread per box for the projection.
#include <math.h>
#include "common.h"
#include "track_math.h"

namespace rv {

namespace {

__global__ __launch_bounds__(256) void iou_matrix_kernel(const float* __restrict__ trk,
                                                         const int* __restrict__ T,
                                                         const float* __restrict__ det,
                                                         const int* __restrict__ D,
                                                         float* __restrict__ out, int Tmax,
                                                         int Dmax) {
  const int s = blockIdx.y;
  const int nt = min(max(T[s], 0), Tmax), nd = min(max(D[s], 0), Dmax);
  const float4* tb = (const float4*)(trk + (size_t)s * Tmax * 4);
  const float4* db = (const float4*)(det + (size_t)s * Dmax * 4);
  float* o = out + (size_t)s * Tmax * Dmax;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < Tmax * Dmax;
       i += gridDim.x * blockDim.x) {
    const int t = i / Dmax, d = i - t * Dmax;
    o[i] = (t < nt && d < nd) ? iou_f32(tb[t], db[d]) : 0.0f;
  }
}

// The reference loop literally: idx = argmax(M) (first max in row-major
// order) -> stop if M[idx] < thr -> record (t, d) if both are free -> mask
// row t and column d with -1.  M (the stream's T x D block, row stride Dmax)
// is modified in place as in the reference.
__global__ __launch_bounds__(256) void greedy_assign_kernel(
    float* __restrict__ M, const int* __restrict__ T, const int* __restrict__ D, int Tmax,
    int Dmax, double thr, int* __restrict__ match_t, int* __restrict__ match_d,
    int* __restrict__ n_match, int* __restrict__ trk_match, int* __restrict__ det_match) {
  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const int nt = min(max(T[s], 0), Tmax), nd = min(max(D[s], 0), Dmax);
  const int mcap = min(Tmax, Dmax);
  float* m = M + (size_t)s * Tmax * Dmax;
  int* tm = trk_match + (size_t)s * Tmax;
  int* dm = det_match + (size_t)s * Dmax;
  int* mt = match_t + (size_t)s * mcap;
  int* md = match_d + (size_t)s * mcap;
  for (int i = tid; i < Tmax; i += 256) tm[i] = -1;
  for (int i = tid; i < Dmax; i += 256) dm[i] = -1;
  __shared__ float s_v[4];
  __shared__ int s_i[4];
  __shared__ int s_n;
  if (tid == 0) s_n = 0;
  __syncthreads();
  const int n = nt * nd;
  // each accepted pair masks a row, so at most min(nt, nd) rounds accept;
  // a round that picks an already-masked pair (only when thr <= -1, where
  // the reference would loop forever) ends the loop
  for (int round = 0; n > 0 && round <= min(nt, nd); ++round) {
    float bv = -INFINITY;
    int bi = 0x7FFFFFFF;
    for (int i = tid; i < n; i += 256) {
      const int t = i / nd, d = i - t * nd;
      const float v = m[t * Dmax + d];
      if (v > bv || (v == bv && i < bi)) {
        bv = v;
        bi = i;
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const float ov = __shfl_xor(bv, off);
      const int oi = __shfl_xor(bi, off);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if ((tid & 63) == 0) {
      s_v[tid >> 6] = bv;
      s_i[tid >> 6] = bi;
    }
    __syncthreads();
    bv = s_v[0];
    bi = s_i[0];
    for (int w = 1; w < 4; ++w)
      if (s_v[w] > bv || (s_v[w] == bv && s_i[w] < bi)) {
        bv = s_v[w];
        bi = s_i[w];
      }
    __syncthreads();  // everyone has read s_v / s_i
    if (!((double)bv >= thr)) break;  // max_iou < iou_threshold (f64 compare, NaN-safe)
    const int t = bi / nd, d = bi - (bi / nd) * nd;
    const bool fresh = tm[t] < 0 && dm[d] < 0;
    if (!fresh) break;
    if (tid == 0) {
      tm[t] = d;
      dm[d] = t;
      mt[s_n] = t;
      md[s_n] = d;
      s_n = s_n + 1;
    }
    for (int j = tid; j < nd; j += 256) m[t * Dmax + j] = -1.0f;
    for (int i = tid; i < nt; i += 256) m[i * Dmax + d] = -1.0f;
    __syncthreads();
  }
  if (tid == 0) n_match[s] = s_n;
}

__global__ void project_kernel(const double* __restrict__ H, const float* __restrict__ boxes,
                               int n, const float* __restrict__ origin, double max_distance,
                               double* __restrict__ out_xy, double* __restrict__ out_dist) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* b = boxes + 4 * (size_t)i;
  // project_bbox: foot point (0.5 * (x1 + x2), y2) in float64
  const double cx = 0.5 * ((double)b[0] + (double)b[2]);
  const double cy = (double)b[3];
  double X, Y;
  if (project_h(H, cx, cy, X, Y)) {
    out_xy[2 * i] = X;
    out_xy[2 * i + 1] = Y;
    if (out_dist) out_dist[i] = origin ? distance_o(origin, max_distance, X, Y) : NAN;
  } else {
    out_xy[2 * i] = NAN;
    out_xy[2 * i + 1] = NAN;
    if (out_dist) out_dist[i] = NAN;
  }
}

// The tracker-off branch of the reference loop (main_preview.py:101-109):
// every detection keeps track_id / speed_kmh None and, with a projector,
// gets distance_m = projector.distance_for_bbox(bbox) (None stays None).
// One thread per (stream, detection) slot; slots past det_n[s] are written
// as None too, so the hand-back record is well defined.
struct UntrackedParams {
  double H[9];
  float origin[2];
  double max_distance;
  int has_proj;
};

__global__ void untracked_metrics_kernel(const float* __restrict__ dets,
                                         const int* __restrict__ det_n, int S, int dmax,
                                         UntrackedParams p, int* __restrict__ out_id,
                                         double* __restrict__ out_dist,
                                         double* __restrict__ out_speed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S * dmax) return;
  const int s = i / dmax, d = i - s * dmax;
  double dist = NAN;
  if (p.has_proj && d < min(max(det_n[s], 0), dmax)) {
    const float* b = dets + 6 * (size_t)i;
    const double cx = 0.5 * ((double)b[0] + (double)b[2]);
    const double cy = (double)b[3];
    double X, Y;
    if (project_h(p.H, cx, cy, X, Y)) dist = distance_o(p.origin, p.max_distance, X, Y);
  }
  out_id[i] = -1;
  out_dist[i] = dist;
  out_speed[i] = NAN;
}

}  // namespace

extern "C" int rv_iou_matrix_batched(const float* trk, const int* T, const float* det,
                                     const int* D, float* out, int S, int Tmax, int Dmax,
                                     void* stream) {
  RV_CHECK_ARG(trk != nullptr && T != nullptr && det != nullptr && D != nullptr &&
                   out != nullptr,
               "null pointer");
  RV_CHECK_ARG(S >= 0 && Tmax >= 1 && Dmax >= 1, "bad shape S=%d Tmax=%d Dmax=%d", S, Tmax,
               Dmax);
  RV_CHECK_ARG((size_t)Tmax * Dmax < (1u << 30), "Tmax*Dmax too large");
  if (S == 0) return RV_OK;
  const int blocks = min(64, ceil_div(Tmax * Dmax, 256));
  iou_matrix_kernel<<<dim3(blocks, S), 256, 0, as_stream(stream)>>>(trk, T, det, D, out, Tmax,
                                                                    Dmax);
  return launch_status("rv_iou_matrix_batched");
}

extern "C" int rv_greedy_assign_batched(float* M, const int* T, const int* D, int S, int Tmax,
                                        int Dmax, double thr, int* match_t, int* match_d,
                                        int* n_match, int* trk_match, int* det_match,
                                        void* stream) {
  RV_CHECK_ARG(M != nullptr && T != nullptr && D != nullptr && match_t != nullptr &&
                   match_d != nullptr && n_match != nullptr && trk_match != nullptr &&
                   det_match != nullptr,
               "null pointer");
  RV_CHECK_ARG(S >= 0 && Tmax >= 1 && Dmax >= 1, "bad shape S=%d Tmax=%d Dmax=%d", S, Tmax,
               Dmax);
  RV_CHECK_ARG((size_t)Tmax * Dmax < (1u << 30), "Tmax*Dmax too large");
  if (S == 0) return RV_OK;
  greedy_assign_kernel<<<S, 256, 0, as_stream(stream)>>>(M, T, D, Tmax, Dmax, thr, match_t,
                                                         match_d, n_match, trk_match, det_match);
  return launch_status("rv_greedy_assign_batched");
}

extern "C" int rv_homography_project_f64(const double* H9, const float* boxes, int n,
                                         const float* origin2, double max_distance,
                                         double* out_xy, double* out_dist, void* stream) {
  RV_CHECK_ARG(H9 != nullptr && out_xy != nullptr && (n == 0 || boxes != nullptr),
               "null pointer");
  RV_CHECK_ARG(n >= 0, "n %d < 0", n);
  if (n == 0) return RV_OK;
  project_kernel<<<ceil_div(n, 256), 256, 0, as_stream(stream)>>>(H9, boxes, n, origin2,
                                                                  max_distance, out_xy, out_dist);
  return launch_status("rv_homography_project_f64");
}

extern "C" int rv_untracked_metrics(const float* dets, const int* det_n, int S, int dmax,
                                    const double* H9, const float* origin2, double max_distance,
                                    int* out_id, double* out_dist, double* out_speed,
                                    void* stream) {
  RV_CHECK_ARG(dets != nullptr && det_n != nullptr && out_id != nullptr && out_dist != nullptr &&
                   out_speed != nullptr,
               "null pointer");
  RV_CHECK_ARG(S >= 0 && dmax >= 1, "bad shape S=%d dmax=%d", S, dmax);
  RV_CHECK_ARG(H9 == nullptr || origin2 != nullptr, "a projector needs its origin");
  if (S == 0) return RV_OK;
  UntrackedParams p{};
  p.has_proj = H9 != nullptr;
  if (H9)
    for (int i = 0; i < 9; ++i) p.H[i] = H9[i];
  if (origin2) {
    p.origin[0] = origin2[0];
    p.origin[1] = origin2[1];
  }
  p.max_distance = max_distance;
  const int n = S * dmax;
  untracked_metrics_kernel<<<ceil_div(n, 256), 256, 0, as_stream(stream)>>>(
      dets, det_n, S, dmax, p, out_id, out_dist, out_speed);
  return launch_status("rv_untracked_metrics");
}

}  // namespace rv
