// Batched SORT tracker + ground-plane homography on gfx950.
//
// Reference: SortTracker.update (src/track/sort_tracker.py:212-278) with
// _associate (:182-210), _iou/_iou_matrix (:55-80), _Track (:83-168),
// _bbox_to_z/_x_to_bbox (:22-41) and the filterpy KalmanFilter equations it
// delegates to (predict: x=Fx, P=FPF'+Q; update: y=z-Hx, S=HPH'+R, K=PH'S^-1,
// x+=Ky, P=(I-KH)P(I-KH)'+KRK'); GroundProjector / HomographyProjector
// (src/geometry/projector.py:13-84).
//
// One workgroup per camera stream (streams are independent; frames of one
// stream must be processed in time order, so a batch is stream-major: S
// streams x 1 frame).  Track state lives in HBM in two ping-pong buffers per
// call (in -> out, surviving tracks compacted in list order, new tracks
// appended in detection order, exactly the reference's list semantics).
//
// Association: the reference's greedy loop (repeat argmax -> accept if
// >= thr -> mask row and column) is equal to scanning all pairs with
// IoU >= thr in (IoU desc, flat index asc) order and accepting a pair whose
// row and column are still free.  Candidates are bitonic-sorted in LDS; a
// single lane scans.  If more than kKeyCap pairs qualify (e.g. thr <= 0) the
// kernel falls back to the literal argmax loop over the IoU matrix in HBM.
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "common.h"
#include "track_math.h"

namespace rv {

constexpr int kHist = 33;     // speed history (32 kept after each append)
constexpr int kKeyCap = 1024;  // sorted IoU pairs in LDS (8 KB); more -> the argmax loop over M

struct Track {
  double x[7];
  double P[49];
  double t_pred, t_upd;
  double cur_dist, cur_speed;  // NaN = None
  double hist[kHist][3];       // (t, X, Y): a ring, oldest at hist_h
  int id, hits, streak, cls;
  float conf;
  int hist_n, hist_h;
  int pad[3];
};
static_assert(sizeof(Track) % 16 == 0, "Track alignment");

struct StreamHdr {
  int T, next_id, overflow, pad;
};

struct SortParams {
  double max_staleness, iou_thr, speed_window;
  int min_hits;
  int tmax, dmax;
  int has_proj;
  double H[9];
  float origin[2];
  double max_distance;  // < 0: None
};

__device__ __forceinline__ bool isnone(double v) { return v != v; }

// _bbox_to_z (f64 math, f32 result)
__device__ __forceinline__ void bbox_to_z(double x1, double y1, double x2, double y2, double z[4]) {
  const double w = fmax(1e-3, x2 - x1);
  const double h = fmax(1e-3, y2 - y1);
  const double cx = x1 + 0.5 * w;
  const double cy = y1 + 0.5 * h;
  z[0] = (double)(float)cx;
  z[1] = (double)(float)cy;
  z[2] = (double)(float)(w * h);
  z[3] = (double)(float)(w / h);
}

// _x_to_bbox -> f32 box
__device__ __forceinline__ float4 x_to_bbox(const double* x) {
  const double cx = x[0], cy = x[1], s = x[2], r = x[3];
  const double w = sqrt(fmax(1e-6, s * r));
  const double h = s / fmax(1e-6, w);
  return make_float4((float)(cx - 0.5 * w), (float)(cy - 0.5 * h), (float)(cx + 0.5 * w),
                     (float)(cy + 0.5 * h));
}

// _update_motion_matrix(dt) + kf.predict(), in place row by row (few live
// registers): row i of F P F^T needs P rows i and i + 4 (i < 3) or row i
// alone, and rows 4..6 are read (for rows 0..2) before they are rewritten.
// Same expressions, same rounding as the whole-matrix form.
__device__ void kf_predict(Track& t, double dt_raw) {
  const double dt = fmax(1e-3, dt_raw);
  // x = F x
  t.x[0] = t.x[0] + dt * t.x[4];
  t.x[1] = t.x[1] + dt * t.x[5];
  t.x[2] = t.x[2] + dt * t.x[6];
  // P = F P F^T + Q, F = I + dt E (E: (0,4),(1,5),(2,6))
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    double f[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) f[j] = t.P[i * 7 + j] + (i < 3 ? dt * t.P[(i + 4) * 7 + j] : 0.0);
#pragma unroll
    for (int j = 0; j < 7; ++j) t.P[i * 7 + j] = f[j] + (j < 3 ? dt * f[j + 4] : 0.0);
  }
  const double q0 = 0.04 * dt * dt;
  t.P[0] += q0;
  t.P[8] += q0;
  t.P[16] += q0;
  t.P[32] += dt;
  t.P[40] += dt;
  t.P[48] += dt;
}

// 4x4 inverse, Gauss-Jordan with partial pivoting (first maximum |a[r][c]|).
// Fully unrolled with compile-time row indices only (a pivot-indexed row
// access would put the matrix in scratch memory).
__device__ void inv4(const double* S, double* Si) {
  double a[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[i][j] = j < 4 ? S[i * 4 + j] : (j - 4 == i ? 1.0 : 0.0);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int p = c;
    double best = fabs(a[c][c]);
#pragma unroll
    for (int r = c + 1; r < 4; ++r)
      if (fabs(a[r][c]) > best) {
        best = fabs(a[r][c]);
        p = r;
      }
#pragma unroll
    for (int r = c + 1; r < 4; ++r)
      if (p == r)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const double tmp = a[c][j];
          a[c][j] = a[r][j];
          a[r][j] = tmp;
        }
    const double d = a[c][c];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[c][j] /= d;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r == c) continue;
      const double f = a[r][c];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[r][j] -= f * a[c][j];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) Si[i * 4 + j] = a[i][j + 4];
}

// kf.update(z) with R = diag(1, 1, 10, 10), H = [I4 0] (Joseph form), on a
// per-lane LDS scratch `sc` (kKfScratch doubles, element e at
// sc[e * stride]): a copy of P, K = P H^T S^-1, then AP = A P and finally
// P = AP A^T + K R K^T written over the track's P.  A = I - K H is formed
// entry by entry from K (never stored).  The outer loops stay rolled over
// LDS-resident operands, so the live set is one row (the whole-matrix
// form held A, AP, K and P at once: 330 VGPRs, one wave per SIMD, and it
// could not share a workgroup with the association).  Every sum keeps its
// k order: bit-identical to the whole-matrix form.
constexpr int kKfP = 0, kKfAP = 49, kKfK = 98, kKfScratch = 126;
// row-parallel form (kf_update_rows): per detection P | Si | K | AP | y
constexpr int kKrP = 0, kKrSi = 49, kKrK = 65, kKrAP = 93, kKrY = 142, kKfRows = 147;
__device__ void kf_update(Track& t, const double z[4], double* sc, int stride) {
  const double R[4] = {1.0, 1.0, 10.0, 10.0};
#define KF_P(i, j) sc[(kKfP + (i) * 7 + (j)) * stride]
#define KF_AP(i, j) sc[(kKfAP + (i) * 7 + (j)) * stride]
#define KF_K(i, j) sc[(kKfK + (i) * 4 + (j)) * stride]
#define KF_A(i, k) (((i) == (k) ? 1.0 : 0.0) - ((k) < 4 ? KF_K(i, k) : 0.0))
  for (int e = 0; e < 49; ++e) sc[(kKfP + e) * stride] = t.P[e];
  double y[4];
  {
    double S[16], Si[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = z[i] - t.x[i];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) S[i * 4 + j] = KF_P(i, j) + (i == j ? R[i] : 0.0);
    inv4(S, Si);
#pragma unroll 1
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += KF_P(i, k) * Si[k * 4 + j];
        KF_K(i, j) = acc;
      }
  }
#pragma unroll 1
  for (int i = 0; i < 7; ++i) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += KF_K(i, k) * y[k];
    t.x[i] += acc;
  }
#pragma unroll 1
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 7; ++k) acc += KF_A(i, k) * KF_P(k, j);
      KF_AP(i, j) = acc;
    }
#pragma unroll 1
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 7; ++k) acc += KF_AP(i, k) * KF_A(j, k);
      double krk = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) krk += KF_K(i, k) * R[k] * KF_K(j, k);
      t.P[i * 7 + j] = acc + krk;
    }
#undef KF_P
#undef KF_AP
#undef KF_K
#undef KF_A
}

// kf.update(z) for one matched track by the 8 lanes of one group (lane r
// of the group owns row r of K, AP and the new P; r = 7 idles in the row
// phases), on the group's LDS block `sc` (kKfRows doubles).  Every element
// is the same expression with the same k order as kf_update (bit-identical);
// only the rows run side by side instead of one after another on one lane.
// The group's 8 lanes are one 8-lane slice of a wave, so LDS order within
// the wave plus a wavefront fence between phases is the only sync needed.
__device__ void kf_update_rows(Track& t, const double z[4], double* sc, int r) {
  const double R[4] = {1.0, 1.0, 10.0, 10.0};
#define KR_P(i, j) sc[kKrP + (i) * 7 + (j)]
#define KR_K(i, j) sc[kKrK + (i) * 4 + (j)]
#define KR_AP(i, j) sc[kKrAP + (i) * 7 + (j)]
#define KR_A(i, k) (((i) == (k) ? 1.0 : 0.0) - ((k) < 4 ? KR_K(i, k) : 0.0))
  auto sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  for (int e = r; e < 49; e += 8) sc[kKrP + e] = t.P[e];
  sync();
  if (r == 0) {
    double S[16], Si[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) sc[kKrY + i] = z[i] - t.x[i];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) S[i * 4 + j] = KR_P(i, j) + (i == j ? R[i] : 0.0);
    inv4(S, Si);
#pragma unroll
    for (int e = 0; e < 16; ++e) sc[kKrSi + e] = Si[e];
  }
  sync();
  if (r < 7) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += KR_P(r, k) * sc[kKrSi + k * 4 + j];
      KR_K(r, j) = acc;
    }
  }
  sync();
  if (r < 7) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += KR_K(r, k) * sc[kKrY + k];
    t.x[r] += acc;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      double a2 = 0.0;
#pragma unroll
      for (int k = 0; k < 7; ++k) a2 += KR_A(r, k) * KR_P(k, j);
      KR_AP(r, j) = a2;
    }
  }
  sync();
  if (r < 7) {
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 7; ++k) acc += KR_AP(r, k) * KR_A(j, k);
      double krk = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) krk += KR_K(r, k) * R[k] * KR_K(j, k);
      t.P[r * 7 + j] = acc + krk;
    }
  }
#undef KR_P
#undef KR_K
#undef KR_AP
#undef KR_A
}

// HomographyProjector.project_point / GroundProjector.distance (track_math.h)
__device__ __forceinline__ bool project(const SortParams& p, double x, double y, double& X,
                                        double& Y) {
  return project_h(p.H, x, y, X, Y);
}
__device__ __forceinline__ double distance(const SortParams& p, double X, double Y) {
  return distance_o(p.origin, p.max_distance, X, Y);
}

// _Track.update_metrics
__device__ void update_metrics(const SortParams& p, Track& t, double x1, double y1, double x2,
                               double y2, double ts) {
  double X, Y;
  const double cx = 0.5 * (x1 + x2), cy = y2;
  if (!project(p, cx, cy, X, Y)) {
    t.cur_dist = NAN;
    t.cur_speed = NAN;
    return;
  }
  t.cur_dist = distance(p, X, Y);
  // the history deque as a ring of kHist entries (at most 32 kept, so the
  // appended slot never overwrites a live one): appending and dropping move
  // the two ends only -- shifting the kept entries down after every drop
  // was a chain of dependent global loads and stores per frame (most of
  // the fused SORT kernel's update phase)
  int n = t.hist_n, h = t.hist_h;
  const int w = h + n < kHist ? h + n : h + n - kHist;
  t.hist[w][0] = ts;
  t.hist[w][1] = X;
  t.hist[w][2] = Y;
  ++n;
  int drop = 0;
  const double win = fmax(0.05, p.speed_window);
  auto at = [&](int i) -> const double* {  // i-th oldest kept entry
    const int k = h + i;
    return t.hist[k < kHist ? k : k - kHist];
  };
  while (drop < n && (ts - at(drop)[0]) > win) ++drop;
  if (n - drop > 32) drop = n - 32;
  h += drop;
  if (h >= kHist) h -= kHist;
  n -= drop;
  t.hist_n = n;
  t.hist_h = h;
  if (n >= 2) {
    const double* f = at(0);
    const double* l = at(n - 1);
    const double dt = fmax(1e-3, l[0] - f[0]);
    const double dist = hypot(l[1] - f[1], l[2] - f[2]);
    t.cur_speed = dist / dt;
  } else {
    t.cur_speed = NAN;
  }
}

__device__ void track_init(Track& t, int id, const float* det, double ts) {
  double z[4];
  bbox_to_z(det[0], det[1], det[2], det[3], z);
  for (int i = 0; i < 7; ++i) t.x[i] = i < 4 ? z[i] : 0.0;
  for (int i = 0; i < 49; ++i) t.P[i] = 0.0;
  for (int i = 0; i < 7; ++i) t.P[i * 8] = i < 4 ? 10.0 : 10000.0;
  t.t_pred = t.t_upd = ts;
  t.cur_dist = t.cur_speed = NAN;
  t.id = id;
  t.hits = 1;
  t.streak = 1;
  t.cls = (int)det[5];
  t.conf = det[4];
  t.hist_n = 0;
  t.hist_h = 0;
}

// ---------------------------------------------------------------------------
// One frame of every stream in three launches (rv_sort_update):
//
//   sort_predict_kernel    one thread per live track of every stream: KF
//                          predict (sort_tracker.py:228-229), the predicted
//                          box and last_update_ts to the workspace;
//   sort_associate_kernel  one workgroup per stream: _iou_matrix pairs >= thr,
//                          sorted (IoU desc, flat index asc), the greedy walk
//                          resolved 64 pairs at a time by wave ballots; the
//                          bookkeeping of :234-276 -- unmatched tracks'
//                          hit_streak = 0, new-track ranks / ids in det
//                          order, pruning by staleness, the new list order
//                          and a pool slot for every new track -- all by
//                          block prefix scans;
//   sort_update_kernel     one thread per detection of every stream: KF
//                          update + metrics of its matched track, or the
//                          new track's init + metrics; the per-detection
//                          outputs.
//
// Tracks live in a fixed per-stream pool of tmax slots; the reference's
// list order is an index array (order[i] = slot of the i-th track), so a
// frame never copies a track.  Survivors keep their order, new tracks are
// appended in detection order and take free slots (pruned tracks' slots are
// reused in the same frame).  Capacity: survivors + new tracks > tmax drops
// the new tracks that do not fit (their ids are still handed out) and sets
// the stream's sticky overflow flag (rv_sort_stats).
// ---------------------------------------------------------------------------
#ifndef RV_ASSOC_THREADS
#define RV_ASSOC_THREADS 1024
#endif
constexpr int kAssocThreads = RV_ASSOC_THREADS;
#ifndef RV_SORT_FUSED_THREADS
#define RV_SORT_FUSED_THREADS 512
#endif

// Association workgroup LDS: tbox (tmax float4), dbox (dmax float4), keys
// (kKeyCap u64), tupd (tmax f64), det_match (dmax), trk_match / ord / rank_t
// / frank (tmax int each), rank_d / newslot (dmax int each), used (tmax u8);
// the fused form adds the KF update scratch (kUpd x 126 f64, from offset 0)
// and the detection jobs (dmax int2) at sort_ljob_off.
constexpr int kUpdLanes = 64;
__host__ __device__ inline size_t sort_assoc_bytes(int tmax, int dmax) {
  return (size_t)(tmax + dmax) * 16 + (size_t)kKeyCap * 8 + (size_t)tmax * 8 + (size_t)dmax * 4 * 3 +
         (size_t)tmax * 4 * 4 + (size_t)tmax;
}
__host__ __device__ inline size_t sort_ljob_off(int tmax, int dmax, int kupd) {
  const size_t a = (sort_assoc_bytes(tmax, dmax) + 15) & ~(size_t)15;
  // kKfScratch doubles per update lane, or (the row-parallel update, at
  // most kupd detections) kKfRows doubles per detection
  const size_t b = (size_t)kupd * (kKfRows > 126 ? kKfRows : 126) * 8;
  return a > b ? a : b;
}

struct SortWs {  // per-frame workspace views (rv_sort_ws_bytes)
  float* M;         // S x tmax x dmax IoU matrix (argmax fallback only)
  float4* tbox;     // S x tmax predicted boxes (list order)
  double* tupd;     // S x tmax last_update_ts (list order)
  int2* det_job;    // S x dmax: {slot, id} per detection (see sort_update_kernel)
};

__global__ __launch_bounds__(256) void sort_predict_kernel(const StreamHdr* __restrict__ hdr,
                                                           const int* __restrict__ order,
                                                           Track* __restrict__ pool,
                                                           const double* __restrict__ ts_arr,
                                                           int tmax, SortWs ws) {
  const int s = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= hdr[s].T) return;
  const double ts = ts_arr[s];
  Track& tr = pool[(size_t)s * tmax + order[(size_t)s * tmax + i]];
  kf_predict(tr, ts - tr.t_pred);
  tr.t_pred = ts;
  ws.tbox[(size_t)s * tmax + i] = x_to_bbox(tr.x);
  ws.tupd[(size_t)s * tmax + i] = tr.t_upd;
}

// Exclusive prefix of flag(i) over [0, n) for a kAssocThreads block,
// chunked: out[i] = rank of i among the flagged, -1 if not flagged; returns
// the total.  `wtot`: kAssocThreads / 64 ints of LDS scratch.
template <int NT, class F>
__device__ int block_rank(F flag, int n, int* out, int* wtot) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int base = 0;
  for (int c0 = 0; c0 < n; c0 += NT) {
    const int i = c0 + tid;
    const bool f = i < n && flag(i);
    const unsigned long long m = __ballot(f);
    if (lane == 0) wtot[w] = __popcll(m);
    __syncthreads();
    int pre = base, tot = 0;
    for (int k = 0; k < NT / 64; ++k) {
      pre += k < w ? wtot[k] : 0;
      tot += wtot[k];
    }
    if (i < n) out[i] = f ? pre + __popcll(m & ((1ull << lane) - 1ull)) : -1;
    base += tot;
    __syncthreads();
  }
  return base;
}

// The per-detection update of sort_update_kernel for detection row d (job j).
__device__ __forceinline__ void sort_update_row(Track* __restrict__ pool, const float* __restrict__ dets,
                                                double ts, int s, int d, int2 j, const SortParams& p,
                                                int* __restrict__ out_id, double* __restrict__ out_dist,
                                                double* __restrict__ out_speed, double* ap,
                                                int ap_stride, bool kf_done = false) {
  const size_t o = (size_t)s * p.dmax + d;
  out_id[o] = -1;
  out_dist[o] = NAN;
  out_speed[o] = NAN;
  if (j.x == -2) return;  // no detection
  if (j.x < 0) {          // a new track that did not fit: the id is still consumed
    out_id[o] = j.y;
    return;
  }
  const float* de = dets + o * 6;
  Track& tr = pool[(size_t)s * p.tmax + j.x];
  if (j.y < 0) {  // matched: _Track.update + update_metrics
    if (!kf_done) {  // (else kf_update_rows ran it)
      double z[4];
      bbox_to_z(de[0], de[1], de[2], de[3], z);
      kf_update(tr, z, ap, ap_stride);
    }
    tr.t_pred = ts;
    tr.t_upd = ts;
    tr.hits += 1;
    tr.streak += 1;
    tr.cls = (int)de[5];
    tr.conf = de[4];
  } else {  // new track
    track_init(tr, j.y, de, ts);
  }
  if (p.has_proj) update_metrics(p, tr, de[0], de[1], de[2], de[3], ts);
  out_id[o] = tr.id;
  if (p.has_proj) {
    if (!isnone(tr.cur_dist)) out_dist[o] = tr.cur_dist;
    if (!isnone(tr.cur_speed)) out_speed[o] = tr.cur_speed * 3.6;
  }
}

#ifdef RV_SORT_PHASE
// timing build (tools/sort_phase.py): per-phase wall-clock ticks (100 MHz)
// of the fused kernel summed over blocks, read back by rv_sort_phase_read
__device__ unsigned long long g_sort_phase[8];
#define RV_PH(i)                                                                       \
  do {                                                                                 \
    __syncthreads();                                                                   \
    if (threadIdx.x == 0) {                                                            \
      const unsigned long long now = wall_clock64();                                   \
      atomicAdd(&g_sort_phase[i], now - ph_t);                                         \
      ph_t = now;                                                                      \
    }                                                                                  \
  } while (0)
#else
#define RV_PH(i) \
  do {           \
  } while (0)
#endif

// FUSED (rv_sort_update's default, one launch per frame): the block also
// runs the KF predict of its stream's tracks (sort_predict_kernel's work,
// boxes and last_update_ts straight into LDS) and, after the bookkeeping,
// the per-detection updates (sort_update_kernel's work, jobs from LDS), so
// a frame is one launch of S workgroups instead of three dependent ones --
// fewer queue waits beside the persistent conv grids and no HBM round trip
// of the predicted boxes and jobs.  A workgroup of NT = 256 threads gives
// the update's f64 Kalman algebra the whole register file (one wave per
// SIMD) without spills.
template <int NT, bool FUSED>
__global__ __launch_bounds__(NT) void sort_associate_kernel(
    StreamHdr* __restrict__ hdr, int* __restrict__ order, Track* __restrict__ pool,
    const float* __restrict__ dets, const int* __restrict__ dcount,
    const double* __restrict__ ts_arr, SortParams p, SortWs ws, int* __restrict__ out_id,
    double* __restrict__ out_dist, double* __restrict__ out_speed) {
  constexpr int kAssocThreads = NT;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int kUpd = NT < kUpdLanes ? NT : kUpdLanes;  // FUSED: threads running the KF updates
  float4* tbox = (float4*)smem;                     // tmax
  float4* dbox = tbox + p.tmax;                     // dmax
  uint64_t* keys = (uint64_t*)(dbox + p.dmax);      // kKeyCap
  double* tupd = (double*)(keys + kKeyCap);         // tmax
  int* det_match = (int*)(tupd + p.tmax);           // dmax: matched track (list index) or -1
  int* trk_match = det_match + p.dmax;              // tmax: matched det or -1
  int* ord = trk_match + p.tmax;                    // tmax: the old list order (slots)
  int* rank_t = ord + p.tmax;                       // tmax: survivor rank
  int* frank = rank_t + p.tmax;                     // tmax: free-slot rank
  int* rank_d = frank + p.tmax;                     // dmax: new-track rank
  int* newslot = rank_d + p.dmax;                   // dmax: slot of the r-th new track
  uint8_t* used = (uint8_t*)(newslot + p.dmax);     // tmax
  // FUSED: the detection jobs, after `used` and after the KF update
  // scratch (kUpd x 126 doubles, which reuses the dead association arrays
  // from offset 0 once the bookkeeping is done)
  int2* ljob = (int2*)(smem + sort_ljob_off(p.tmax, p.dmax, kUpd));
  __shared__ int s_cnt, s_red_v[16], s_red_i[16], wtot[16];

  const int s = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
#ifdef RV_SORT_PHASE
  unsigned long long ph_t = wall_clock64();
  if (threadIdx.x == 0) atomicAdd(&g_sort_phase[7], 1ull);  // blocks timed
#endif
  const StreamHdr h = hdr[s];
  const int T = h.T;
  int D = dcount[s];
  D = D < 0 ? 0 : (D > p.dmax ? p.dmax : D);
  const float* dd = dets + (size_t)s * p.dmax * 6;
  const double ts = ts_arr[s];
  int2* job = ws.det_job + (size_t)s * p.dmax;
  int* ord_g = order + (size_t)s * p.tmax;
  Track* pl = pool + (size_t)s * p.tmax;

  for (int t = tid; t < T; t += kAssocThreads) {
    const int slot = ord_g[t];
    if constexpr (FUSED) {  // sort_predict_kernel's work for list index t
      Track& tr = pl[slot];
      kf_predict(tr, ts - tr.t_pred);
      tr.t_pred = ts;
      tbox[t] = x_to_bbox(tr.x);
      tupd[t] = tr.t_upd;
    } else {
      tbox[t] = ws.tbox[(size_t)s * p.tmax + t];
      tupd[t] = ws.tupd[(size_t)s * p.tmax + t];
    }
    ord[t] = slot;
    trk_match[t] = -1;
  }
  for (int d = tid; d < D; d += kAssocThreads) {
    dbox[d] = make_float4(dd[d * 6], dd[d * 6 + 1], dd[d * 6 + 2], dd[d * 6 + 3]);
    det_match[d] = -1;
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  RV_PH(0);  // predict + loads

  // ---- association (_associate, sort_tracker.py:182-210)
  if (T > 0 && D > 0) {
    // qualifying pairs appended with one LDS atomic per wave (a ballot's
    // popcount), not one per pair; the append order does not matter (the
    // keys are sorted next and unique)
    // pair i = tid + kAssocThreads k is (i / D, i % D), stepped
    // incrementally (an integer division by the runtime D per pair was ~20
    // VALU, as much as the IoU itself)
    const int dt = kAssocThreads / D, dd = kAssocThreads - (kAssocThreads / D) * D;
    int pt = tid / D, pd = tid - (tid / D) * D;
    for (int i0 = 0; i0 < T * D; i0 += kAssocThreads) {
      const int i = i0 + tid;
      bool q = false;
      float v = 0.f;
      if (i < T * D) {
        v = iou_f32(tbox[pt], dbox[pd]);
        q = (double)v >= p.iou_thr;
      }
      pt += dt;
      pd += dd;
      if (pd >= D) {
        pd -= D;
        ++pt;
      }
      const unsigned long long m = __ballot(q);
      if (m) {  // wave-uniform
        int base = 0;
        if (lane == 0) base = atomicAdd(&s_cnt, __popcll(m));
        base = __shfl(base, 0);
        if (q) {
          const int k = base + __popcll(m & ((1ull << lane) - 1ull));
          if (k < kKeyCap) keys[k] = ((uint64_t)(~__float_as_uint(v)) << 32) | (uint64_t)(uint32_t)i;
        }
      }
    }
    __syncthreads();
    RV_PH(1);  // IoU pairs
    const int cnt = s_cnt;
    if (cnt <= kKeyCap) {
      int np2 = 1;
      while (np2 < cnt) np2 <<= 1;
      if (cnt <= kAssocThreads) {
        // rank sort: key i lands at the number of smaller keys (unique:
        // the flat index is in the low bits); every thread reads the same
        // key at once (an LDS broadcast) -- cnt reads and two barriers
        // instead of log2(np2)^2 / 2 bitonic stages
        const uint64_t mine = tid < cnt ? keys[tid] : ~0ull;
        int r = 0;
        for (int j = 0; j < cnt; ++j) r += keys[j] < mine ? 1 : 0;
        __syncthreads();
        if (tid < cnt) keys[r] = mine;
        __syncthreads();
        np2 = 0;  // sorted
      }
      for (int i = cnt + tid; i < np2; i += kAssocThreads) keys[i] = ~0ull;
      __syncthreads();
      for (int size = 2; size <= np2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int i = tid; i < np2 / 2; i += kAssocThreads) {
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
      RV_PH(2);  // sort
      // greedy walk in (IoU desc, flat index asc) order, 64 pairs at a time:
      // a pair is accepted iff its row and column are still free; inside a
      // chunk the lowest remaining lane is accepted and the lanes sharing its
      // row or column are dropped (wave-uniform ballot loop)
      if (tid < 64) {
        for (int base = 0; base < cnt; base += 64) {
          const int i = base + lane;
          int t = -1, d = -2;
          bool ok = false;
          if (i < cnt) {
            const int f = (int)(keys[i] & 0xFFFFFFFFu);
            t = f / D;
            d = f - t * D;
            ok = trk_match[t] < 0 && det_match[d] < 0;
          }
          unsigned long long m = __ballot(ok);
          while (m) {
            const int q = __ffsll((long long)m) - 1;
            const int tq = __shfl(t, q), dq = __shfl(d, q);
            if (lane == q) {
              trk_match[t] = d;
              det_match[d] = t;
            }
            m &= ~__ballot(t == tq || d == dq);
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
      }
    } else {
      // more qualifying pairs than keys: the literal reference loop (argmax
      // with the first maximum, accept, mask row and column) over M in HBM
      float* M = ws.M + (size_t)s * p.tmax * p.dmax;
      for (int i = tid; i < T * D; i += kAssocThreads) {
        const int t = i / D, d = i - (i / D) * D;
        M[i] = iou_f32(tbox[t], dbox[d]);
      }
      __syncthreads();
      for (;;) {
        float bv = -INFINITY;
        int bi = 0x7FFFFFFF;
        for (int i = tid; i < T * D; i += kAssocThreads) {
          const float v = M[i];
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
        if (lane == 0) {
          s_red_v[tid >> 6] = __float_as_int(bv);
          s_red_i[tid >> 6] = bi;
        }
        __syncthreads();
        bv = __int_as_float(s_red_v[0]);
        bi = s_red_i[0];
        for (int w = 1; w < kAssocThreads / 64; ++w) {
          const float ov = __int_as_float(s_red_v[w]);
          if (ov > bv || (ov == bv && s_red_i[w] < bi)) {
            bv = ov;
            bi = s_red_i[w];
          }
        }
        __syncthreads();
        if ((double)bv < p.iou_thr) break;
        const int t = bi / D, d = bi - (bi / D) * D;
        if (tid == 0) {
          trk_match[t] = d;
          det_match[d] = t;
        }
        for (int j = tid; j < D; j += kAssocThreads) M[t * D + j] = -1.0f;
        for (int i = tid; i < T; i += kAssocThreads) M[i * D + d] = -1.0f;
        __syncthreads();
      }
    }
  }
  __syncthreads();
  RV_PH(3);  // greedy walk (or the fallback loop)

  // ---- bookkeeping (sort_tracker.py:234-276)
  const int n_new = block_rank<NT>([&](int d) { return det_match[d] < 0; }, D, rank_d, wtot);
  const int n_surv = block_rank<NT>(
      [&](int t) {
        const double upd = trk_match[t] >= 0 ? ts : tupd[t];
        return (ts - upd) <= p.max_staleness;
      },
      T, rank_t, wtot);
  // survivors keep their slots and their list order; unmatched tracks lose
  // their hit streak
  for (int q = tid; q < p.tmax; q += kAssocThreads) used[q] = 0;
  __syncthreads();
  for (int t = tid; t < T; t += kAssocThreads) {
    if (rank_t[t] >= 0) {
      used[ord[t]] = 1;
      ord_g[rank_t[t]] = ord[t];
    }
    if (trk_match[t] < 0) pl[ord[t]].streak = 0;
  }
  __syncthreads();
  // new tracks (alive unless max_staleness < 0: last_update_ts = ts) take the
  // free slots in ascending slot order, appended in detection order
  const bool new_alive = 0.0 <= p.max_staleness;
  const int room = p.tmax - n_surv;
  const int n_fit = !new_alive ? 0 : (n_new < room ? n_new : room);
  block_rank<NT>([&](int q) { return !used[q]; }, p.tmax, frank, wtot);
  for (int q = tid; q < p.tmax; q += kAssocThreads) {
    const int r = frank[q];
    if (r >= 0 && r < n_fit) newslot[r] = q;
  }
  __syncthreads();
  for (int r = tid; r < n_fit; r += kAssocThreads) ord_g[n_surv + r] = newslot[r];
  // detection jobs for sort_update_kernel, {slot, id}: matched -> (its
  // track's slot, -1); new -> (its slot, new id); new without room or pruned
  // at once -> (-1, new id); no detection in the row -> (-2, -1)
  for (int d = tid; d < p.dmax; d += kAssocThreads) {
    int2 j = make_int2(-2, -1);
    if (d < D) {
      const int t = det_match[d];
      if (t >= 0) {
        j = make_int2(ord[t], -1);
      } else {
        const int r = rank_d[d];
        j = make_int2(r < n_fit ? newslot[r] : -1, h.next_id + r);
      }
    }
    if constexpr (FUSED)
      ljob[d] = j;
    else
      job[d] = j;
  }
  if (tid == 0) {
    StreamHdr o;
    o.T = n_surv + n_fit;
    o.next_id = h.next_id + n_new;
    o.overflow = h.overflow | (new_alive && n_new > room ? 1 : 0);
    o.pad = 0;
    hdr[s] = o;
  }
  if constexpr (FUSED) {
    // sort_update_kernel's work: the streak resets above and the predicted
    // states are this block's own global writes, visible after the barrier
    __syncthreads();
    RV_PH(4);  // bookkeeping
    if (D <= NT / 8 && D <= kUpd) {
      // one 8-lane group per detection: the matched tracks' KF updates row
      // by row (kf_update_rows), then lane 0 of the group does the rest of
      // the row (fields, metrics, outputs) as sort_update_row; rows
      // [D, dmax) get their empty outputs from the lanes beyond
      const int d = tid >> 3, r = tid & 7;
      const int2 j = d < D ? ljob[d] : make_int2(-2, -1);
      const bool matched = d < D && j.x >= 0 && j.y < 0;
      if (matched) {
        double z[4];
        const float* de = dets + ((size_t)s * p.dmax + d) * 6;
        bbox_to_z(de[0], de[1], de[2], de[3], z);
        kf_update_rows(pl[j.x], z, (double*)smem + (size_t)d * kKfRows, r);
      }
      if (r == 0 && d < D)
        sort_update_row(pool, dets, ts, s, d, j, p, out_id, out_dist, out_speed, nullptr, 0,
                        matched);
      for (int e = D + tid; e < p.dmax; e += NT)
        sort_update_row(pool, dets, ts, s, e, ljob[e], p, out_id, out_dist, out_speed, nullptr, 0);
    } else {
      double* ap = (double*)smem + tid;
      if (tid < kUpd)
        for (int d = tid; d < p.dmax; d += kUpd)
          sort_update_row(pool, dets, ts, s, d, ljob[d], p, out_id, out_dist, out_speed, ap, kUpd);
    }
    RV_PH(5);  // KF updates + metrics
  }
}

#ifdef RV_SORT_PHASE
extern "C" int rv_sort_phase_read(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sort_phase), sizeof(unsigned long long) * 8) != hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_sort_phase), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// One thread per detection row of every stream (sort_tracker.py:234-269).
__global__ __launch_bounds__(kUpdLanes) void sort_update_kernel(
    Track* __restrict__ pool, const float* __restrict__ dets, const double* __restrict__ ts_arr,
    SortParams p, SortWs ws, int* __restrict__ out_id, double* __restrict__ out_dist,
    double* __restrict__ out_speed) {
  __shared__ double ap[126 * kUpdLanes];  // KF update scratch (kKfScratch), element-major
  const int s = blockIdx.y;
  const int d = blockIdx.x * kUpdLanes + threadIdx.x;
  if (d >= p.dmax) return;
  sort_update_row(pool, dets, ts_arr[s], s, d, ws.det_job[(size_t)s * p.dmax + d], p, out_id,
                  out_dist, out_speed, ap + threadIdx.x, kUpdLanes);
}

// Per-stream state layout: headers (S x 16 B, padded to 256 B), the list
// orders (S x tmax int32, padded), the track pools (S x tmax x Track).
struct StateView {
  StreamHdr* hdr;
  int* order;
  Track* pool;
};

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static StateView state_view(const void* state, int S, int tmax) {
  uint8_t* b = (uint8_t*)state;
  StateView v;
  v.hdr = (StreamHdr*)b;
  b += align256((size_t)S * sizeof(StreamHdr));
  v.order = (int*)b;
  b += align256((size_t)S * tmax * sizeof(int));
  v.pool = (Track*)b;
  return v;
}

__global__ void sort_export_kernel(const StreamHdr* __restrict__ hdr, const int* __restrict__ order,
                                   const Track* __restrict__ pool, int tmax,
                                   double* __restrict__ x_out, int* __restrict__ meta,
                                   int* __restrict__ T_out) {
  const int s = blockIdx.x;
  const int T = hdr[s].T;
  if (threadIdx.x == 0) T_out[s] = T;
  for (int t = threadIdx.x; t < tmax; t += blockDim.x) {
    const bool v = t < T;
    const Track& k = pool[(size_t)s * tmax + (v ? order[(size_t)s * tmax + t] : 0)];
    for (int i = 0; i < 7; ++i) x_out[((size_t)s * tmax + t) * 7 + i] = v ? k.x[i] : 0.0;
    int* m = meta + ((size_t)s * tmax + t) * 4;
    m[0] = v ? k.id : -1;
    m[1] = v ? k.hits : 0;
    m[2] = v ? k.streak : 0;
    m[3] = v ? k.cls : -1;
  }
}

__global__ void sort_stats_kernel(const StreamHdr* __restrict__ hdr, int S, int* __restrict__ T_out,
                                  int* __restrict__ next_id, int* __restrict__ overflow) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const StreamHdr h = hdr[s];
  T_out[s] = h.T;
  if (next_id) next_id[s] = h.next_id;
  if (overflow) overflow[s] = h.overflow;
}

}  // namespace rv

using namespace rv;

extern "C" size_t rv_sort_state_bytes(int S, int tmax) {
  if (S <= 0 || tmax <= 0) return 0;
  return align256((size_t)S * sizeof(StreamHdr)) + align256((size_t)S * tmax * sizeof(int)) +
         (size_t)S * tmax * sizeof(Track);
}

// M (argmax fallback) + predicted boxes + last_update_ts + detection jobs
static size_t ws_parts(int S, int tmax, int dmax, size_t* off) {
  size_t o = 0;
  off[0] = o;
  o = align256(o + (size_t)S * tmax * dmax * sizeof(float));
  off[1] = o;
  o = align256(o + (size_t)S * tmax * sizeof(float4));
  off[2] = o;
  o = align256(o + (size_t)S * tmax * sizeof(double));
  off[3] = o;
  o = align256(o + (size_t)S * dmax * sizeof(int2));
  return o;
}

extern "C" size_t rv_sort_ws_bytes(int S, int tmax, int dmax) {
  if (S <= 0 || tmax <= 0 || dmax <= 0) return 0;
  size_t off[4];
  return ws_parts(S, tmax, dmax, off);
}

constexpr int kFusedThreads = RV_SORT_FUSED_THREADS;
static size_t sort_smem(int tmax, int dmax, bool fused) {
  const int kupd = kFusedThreads < kUpdLanes ? kFusedThreads : kUpdLanes;
  return fused ? sort_ljob_off(tmax, dmax, kupd) + (size_t)dmax * 8 : sort_assoc_bytes(tmax, dmax);
}

// RV_SORT_FUSED=0: the three-launch form (A/B)
static bool sort_fused() {
  static const int v = getenv("RV_SORT_FUSED") ? atoi(getenv("RV_SORT_FUSED")) : 1;
  return v != 0;
}

extern "C" int rv_sort_init(void* state, int S, int tmax, void* stream) {
  RV_CHECK_ARG(state && S > 0 && tmax > 0, "bad sort state");
  hipError_t e = hipMemsetAsync(state, 0, rv_sort_state_bytes(S, tmax), as_stream(stream));
  if (e != hipSuccess) {
    set_error("memset: %s", hipGetErrorString(e));
    return -(int)e;
  }
  // next_id starts at 1 (sort_tracker.py:180)
  static thread_local std::vector<StreamHdr> tmp;
  tmp.assign(S, StreamHdr{0, 1, 0, 0});
  e = hipMemcpyAsync(state, tmp.data(), sizeof(StreamHdr) * S, hipMemcpyHostToDevice,
                     as_stream(stream));
  if (e != hipSuccess) {
    set_error("memcpy: %s", hipGetErrorString(e));
    return -(int)e;
  }
  return hipStreamSynchronize(as_stream(stream)) == hipSuccess ? RV_OK : RV_EINVAL;
}

extern "C" int rv_sort_update(void* state_in, void* state_out, int S, int tmax,
                              const float* dets, const int* dcount, int dmax, const double* ts,
                              const double* params6, const double* H9, const float* origin2,
                              void* ws, size_t ws_bytes, int* out_id, double* out_dist,
                              double* out_speed, void* stream) {
  RV_CHECK_ARG(state_in && state_out, "null state");
  RV_CHECK_ARG(dets && dcount && ts && params6 && out_id && out_dist && out_speed && ws,
               "null pointer");
  RV_CHECK_ARG(S > 0 && tmax > 0 && tmax <= 8192 && dmax > 0 && dmax <= 4096, "bad sizes");
  RV_CHECK_ARG(ws_bytes >= rv_sort_ws_bytes(S, tmax, dmax), "workspace too small");
  RV_CHECK_ARG((size_t)tmax * dmax < 0xFFFFFFFFull, "tmax*dmax too large");
  SortParams p;
  memset(&p, 0, sizeof(p));
  p.max_staleness = params6[0];
  p.min_hits = (int)params6[1];
  p.iou_thr = params6[2];
  p.speed_window = params6[3];
  p.max_distance = params6[4];
  p.tmax = tmax;
  p.dmax = dmax;
  p.has_proj = H9 != nullptr;
  if (H9)
    for (int i = 0; i < 9; ++i) p.H[i] = H9[i];
  if (origin2) {
    p.origin[0] = origin2[0];
    p.origin[1] = origin2[1];
  }
  const bool fused = sort_fused();
  const size_t smem = sort_smem(tmax, dmax, fused);
  RV_CHECK_ARG(smem <= 160 * 1024, "tmax/dmax need %zu B of LDS", smem);
  hipStream_t st = as_stream(stream);
  int r = RV_OK;
  if (state_out != state_in)  // the update runs in place on state_out
    r = hip_check(hipMemcpyAsync(state_out, state_in, rv_sort_state_bytes(S, tmax),
                                 hipMemcpyDeviceToDevice, st),
                  "rv_sort_update state copy");
  if (r) return r;
  static int attr_set[2] = {0, 0};
  const void* assoc_fn = fused ? (const void*)sort_associate_kernel<kFusedThreads, true>
                               : (const void*)sort_associate_kernel<kAssocThreads, false>;
  if ((int)smem > attr_set[fused]) {  // once per growth, outside steady-state launches
    hipError_t e = hipFuncSetAttribute(assoc_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) {
      set_error("hipFuncSetAttribute(%zu B LDS): %s", smem, hipGetErrorString(e));
      (void)hipGetLastError();
      return -(int)e;
    }
    attr_set[fused] = (int)smem;
  }
  const StateView v = state_view(state_out, S, tmax);
  size_t off[4];
  ws_parts(S, tmax, dmax, off);
  SortWs w;
  w.M = (float*)((uint8_t*)ws + off[0]);
  w.tbox = (float4*)((uint8_t*)ws + off[1]);
  w.tupd = (double*)((uint8_t*)ws + off[2]);
  w.det_job = (int2*)((uint8_t*)ws + off[3]);
  if (fused) {
    sort_associate_kernel<kFusedThreads, true><<<S, kFusedThreads, smem, st>>>(
        v.hdr, v.order, v.pool, dets, dcount, ts, p, w, out_id, out_dist, out_speed);
    return launch_status("rv_sort_update (fused)");
  }
  sort_predict_kernel<<<dim3(ceil_div(tmax, 256), S), 256, 0, st>>>(v.hdr, v.order, v.pool, ts,
                                                                     tmax, w);
  r = launch_status("rv_sort_update (predict)");
  if (r) return r;
  sort_associate_kernel<kAssocThreads, false><<<S, kAssocThreads, smem, st>>>(
      v.hdr, v.order, v.pool, dets, dcount, ts, p, w, out_id, out_dist, out_speed);
  r = launch_status("rv_sort_update (associate)");
  if (r) return r;
  sort_update_kernel<<<dim3(ceil_div(dmax, kUpdLanes), S), kUpdLanes, 0, st>>>(
      v.pool, dets, ts, p, w, out_id, out_dist, out_speed);
  return launch_status("rv_sort_update (update)");
}

extern "C" int rv_sort_export(const void* state, int S, int tmax, double* x_out, int* meta,
                              int* T_out, void* stream) {
  RV_CHECK_ARG(state && x_out && meta && T_out && S > 0 && tmax > 0, "bad args");
  const StateView v = state_view(state, S, tmax);
  sort_export_kernel<<<S, 256, 0, as_stream(stream)>>>(v.hdr, v.order, v.pool, tmax, x_out, meta,
                                                       T_out);
  return launch_status("rv_sort_export");
}

extern "C" int rv_sort_stats(const void* state, int S, int* T_out, int* next_id_out,
                             int* overflow_out, void* stream) {
  RV_CHECK_ARG(state && T_out && S > 0, "bad args");
  sort_stats_kernel<<<ceil_div(S, 256), 256, 0, as_stream(stream)>>>(
      (const StreamHdr*)state, S, T_out, next_id_out, overflow_out);
  return launch_status("rv_sort_stats");
}
