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
#include <string.h>
#include <vector>
#include "common.h"
#include "track_math.h"

namespace rv {

constexpr int kHist = 33;     // speed history (32 kept after each append)
constexpr int kKeyCap = 4096;

struct Track {
  double x[7];
  double P[49];
  double t_pred, t_upd;
  double cur_dist, cur_speed;  // NaN = None
  double hist[kHist][3];       // (t, X, Y)
  int id, hits, streak, cls;
  float conf;
  int hist_n;
  int pad[4];
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

// _update_motion_matrix(dt) + kf.predict()
__device__ void kf_predict(Track& t, double dt_raw) {
  const double dt = fmax(1e-3, dt_raw);
  double x[7];
  for (int i = 0; i < 7; ++i) x[i] = t.x[i];
  // x = F x
  t.x[0] = x[0] + dt * x[4];
  t.x[1] = x[1] + dt * x[5];
  t.x[2] = x[2] + dt * x[6];
  // P = F P F^T + Q, F = I + dt E (E: (0,4),(1,5),(2,6))
  double FP[49];
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 7; ++j) FP[i * 7 + j] = t.P[i * 7 + j] + (i < 3 ? dt * t.P[(i + 4) * 7 + j] : 0.0);
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 7; ++j) t.P[i * 7 + j] = FP[i * 7 + j] + (j < 3 ? dt * FP[i * 7 + j + 4] : 0.0);
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

// kf.update(z) with R = diag(1, 1, 10, 10), H = [I4 0] (Joseph form)
__device__ void kf_update(Track& t, const double z[4]) {
  const double R[4] = {1.0, 1.0, 10.0, 10.0};
  double y[4], S[16], Si[16], K[28];
  for (int i = 0; i < 4; ++i) y[i] = z[i] - t.x[i];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) S[i * 4 + j] = t.P[i * 7 + j] + (i == j ? R[i] : 0.0);
  inv4(S, Si);
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 4; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 4; ++k) acc += t.P[i * 7 + k] * Si[k * 4 + j];
      K[i * 4 + j] = acc;
    }
  for (int i = 0; i < 7; ++i) {
    double acc = 0.0;
    for (int k = 0; k < 4; ++k) acc += K[i * 4 + k] * y[k];
    t.x[i] += acc;
  }
  // A = I - K H (7x7; only the first 4 columns of KH are non-zero)
  double A[49], AP[49];
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 7; ++j) A[i * 7 + j] = (i == j ? 1.0 : 0.0) - (j < 4 ? K[i * 4 + j] : 0.0);
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 7; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 7; ++k) acc += A[i * 7 + k] * t.P[k * 7 + j];
      AP[i * 7 + j] = acc;
    }
  for (int i = 0; i < 7; ++i)
    for (int j = 0; j < 7; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 7; ++k) acc += AP[i * 7 + k] * A[j * 7 + k];
      double krk = 0.0;
      for (int k = 0; k < 4; ++k) krk += K[i * 4 + k] * R[k] * K[j * 4 + k];
      t.P[i * 7 + j] = acc + krk;
    }
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
  int n = t.hist_n;
  t.hist[n][0] = ts;
  t.hist[n][1] = X;
  t.hist[n][2] = Y;
  ++n;
  int drop = 0;
  const double win = fmax(0.05, p.speed_window);
  while (drop < n && (ts - t.hist[drop][0]) > win) ++drop;
  if (n - drop > 32) drop = n - 32;
  if (drop > 0) {
    for (int i = 0; i < n - drop; ++i)
      for (int c = 0; c < 3; ++c) t.hist[i][c] = t.hist[i + drop][c];
    n -= drop;
  }
  t.hist_n = n;
  if (n >= 2) {
    const double dt = fmax(1e-3, t.hist[n - 1][0] - t.hist[0][0]);
    const double dist = hypot(t.hist[n - 1][1] - t.hist[0][1], t.hist[n - 1][2] - t.hist[0][2]);
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
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sort_update_kernel(
    const StreamHdr* __restrict__ hin, Track* __restrict__ tin, StreamHdr* __restrict__ hout,
    Track* __restrict__ tout, const float* __restrict__ dets, const int* __restrict__ dcount,
    const double* __restrict__ ts_arr, SortParams p, float* __restrict__ iou_ws,
    int* __restrict__ out_id, double* __restrict__ out_dist, double* __restrict__ out_speed) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float4* tbox = (float4*)smem;                       // tmax
  float4* dbox = tbox + p.tmax;                       // dmax
  uint64_t* keys = (uint64_t*)(dbox + p.dmax);        // kKeyCap
  int* det_match = (int*)(keys + kKeyCap);            // dmax: matched track or -1
  int* trk_match = det_match + p.dmax;                // tmax: matched det or -1
  int* keep_pos = trk_match + p.tmax;                 // tmax + dmax: output slot or -1
  __shared__ int s_cnt, s_red_v[4], s_red_i[4];

  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const StreamHdr h = hin[s];
  Track* Wk = tin + (size_t)s * p.tmax;  // work copy (the consumed input state)
  Track* T_out = tout + (size_t)s * p.tmax;
  const int T = h.T;
  int D = dcount[s];
  if (D > p.dmax) D = p.dmax;
  const float* dd = dets + (size_t)s * p.dmax * 6;
  const double ts = ts_arr[s];
  int* oid = out_id + (size_t)s * p.dmax;
  double* odist = out_dist + (size_t)s * p.dmax;
  double* ospd = out_speed + (size_t)s * p.dmax;

  for (int d = tid; d < p.dmax; d += 256) {
    oid[d] = -1;
    odist[d] = NAN;
    ospd[d] = NAN;
  }
  if (T == 0 && D == 0) {
    if (tid == 0) hout[s] = h;
    return;
  }
  // predict every track in place in the work copy
  for (int t = tid; t < T; t += 256) {
    Track& tr = Wk[t];
    kf_predict(tr, ts - tr.t_pred);
    tr.t_pred = ts;
    tbox[t] = x_to_bbox(tr.x);
    trk_match[t] = -1;
  }
  for (int d = tid; d < D; d += 256) {
    dbox[d] = make_float4(dd[d * 6], dd[d * 6 + 1], dd[d * 6 + 2], dd[d * 6 + 3]);
    det_match[d] = -1;
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();

  // ---- association
  if (T > 0 && D > 0) {
    float* M = iou_ws + (size_t)s * p.tmax * p.dmax;
    for (int i = tid; i < T * D; i += 256) {
      const int t = i / D, d = i - (i / D) * D;
      const float v = iou_f32(tbox[t], dbox[d]);
      M[i] = v;
      if ((double)v >= p.iou_thr) {
        const int k = atomicAdd(&s_cnt, 1);
        if (k < kKeyCap)
          keys[k] = ((uint64_t)(~__float_as_uint(v)) << 32) | (uint64_t)(uint32_t)i;
      }
    }
    __syncthreads();
    const int cnt = s_cnt;
    if (cnt <= kKeyCap) {
      int np2 = 1;
      while (np2 < cnt) np2 <<= 1;
      for (int i = cnt + tid; i < np2; i += 256) keys[i] = ~0ull;
      __syncthreads();
      for (int size = 2; size <= np2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int i = tid; i < np2 / 2; i += 256) {
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
      if (tid == 0) {
        for (int k = 0; k < cnt; ++k) {
          const int i = (int)(keys[k] & 0xFFFFFFFFu);
          const int t = i / D, d = i - (i / D) * D;
          if (trk_match[t] < 0 && det_match[d] < 0) {
            trk_match[t] = d;
            det_match[d] = t;
          }
        }
      }
    } else {
      // literal reference loop: argmax (first max) -> accept -> mask
      for (;;) {
        float bv = -INFINITY;
        int bi = 0x7FFFFFFF;
        for (int i = tid; i < T * D; i += 256) {
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
        if ((tid & 63) == 0) {
          s_red_v[tid >> 6] = __float_as_int(bv);
          s_red_i[tid >> 6] = bi;
        }
        __syncthreads();
        bv = __int_as_float(s_red_v[0]);
        bi = s_red_i[0];
        for (int w = 1; w < 4; ++w) {
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
        for (int j = tid; j < D; j += 256) M[t * D + j] = -1.0f;
        for (int i = tid; i < T; i += 256) M[i * D + d] = -1.0f;
        __syncthreads();
      }
    }
  }
  __syncthreads();

  // ---- update matched tracks, mark missed
  for (int t = tid; t < T; t += 256) {
    Track& tr = Wk[t];
    const int d = trk_match[t];
    if (d >= 0) {
      const float* de = dd + d * 6;
      double z[4];
      bbox_to_z(de[0], de[1], de[2], de[3], z);
      kf_update(tr, z);
      tr.t_pred = ts;
      tr.t_upd = ts;
      tr.hits += 1;
      tr.streak += 1;
      tr.cls = (int)de[5];
      tr.conf = de[4];
      if (p.has_proj) update_metrics(p, tr, de[0], de[1], de[2], de[3], ts);
      oid[d] = tr.id;
      if (!isnone(tr.cur_dist)) odist[d] = tr.cur_dist;
      if (!isnone(tr.cur_speed)) ospd[d] = tr.cur_speed * 3.6;
    } else {
      tr.streak = 0;
    }
  }
  // ---- new tracks for unmatched detections, ids in ascending det order
  // (rank among unmatched dets by a block prefix count)
  __syncthreads();
  if (tid == 0) {
    int r = 0;
    for (int d = 0; d < D; ++d) {
      if (det_match[d] < 0) {
        keep_pos[p.tmax + d] = r;
        ++r;
      } else {
        keep_pos[p.tmax + d] = -1;
      }
    }
    s_cnt = r;
  }
  __syncthreads();
  const int n_new = s_cnt;
  bool overflow = T + n_new > p.tmax;
  for (int d = tid; d < D; d += 256) {
    const int r = keep_pos[p.tmax + d];
    if (r < 0) continue;
    const int slot = T + r;
    if (slot >= p.tmax) {
      oid[d] = h.next_id + r;  // id is consumed even though the track cannot be stored
      continue;
    }
    Track& tr = Wk[slot];
    track_init(tr, h.next_id + r, dd + d * 6, ts);
    if (p.has_proj) {
      const float* de = dd + d * 6;
      update_metrics(p, tr, de[0], de[1], de[2], de[3], ts);
      if (!isnone(tr.cur_dist)) odist[d] = tr.cur_dist;
      if (!isnone(tr.cur_speed)) ospd[d] = tr.cur_speed * 3.6;
    }
    oid[d] = tr.id;
  }
  __syncthreads();
  // ---- prune stale tracks: stable compaction work -> out, one lane per track
  const int total = min(T + n_new, p.tmax);
  if (tid == 0) {
    int w = 0;
    for (int t = 0; t < total; ++t) {
      const bool alive = (ts - Wk[t].t_upd) <= p.max_staleness;
      keep_pos[t] = alive ? w++ : -1;
    }
    s_cnt = w;
  }
  __syncthreads();
  const int n_alive = s_cnt;
  for (int t = tid; t < total; t += 256) {
    const int dst = keep_pos[t];
    if (dst < 0) continue;
    const uint4* src4 = (const uint4*)&Wk[t];
    uint4* dst4 = (uint4*)&T_out[dst];
    for (int i = 0; i < (int)(sizeof(Track) / 16); ++i) dst4[i] = src4[i];
  }
  if (tid == 0) {
    StreamHdr o;
    o.T = n_alive;
    o.next_id = h.next_id + n_new;
    o.overflow = h.overflow | (overflow ? 1 : 0);
    o.pad = 0;
    hout[s] = o;
  }
}

__global__ void sort_export_kernel(const StreamHdr* __restrict__ hdr, const Track* __restrict__ tr,
                                   int tmax, double* __restrict__ x_out, int* __restrict__ meta,
                                   int* __restrict__ T_out) {
  const int s = blockIdx.x;
  const int T = hdr[s].T;
  if (threadIdx.x == 0) T_out[s] = T;
  for (int t = threadIdx.x; t < tmax; t += blockDim.x) {
    const Track& k = tr[(size_t)s * tmax + t];
    const bool v = t < T;
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
  return (((size_t)S * sizeof(StreamHdr) + 255) & ~(size_t)255) + (size_t)S * tmax * sizeof(Track);
}

extern "C" size_t rv_sort_ws_bytes(int S, int tmax, int dmax) {
  if (S <= 0 || tmax <= 0 || dmax <= 0) return 0;
  return (size_t)S * tmax * dmax * sizeof(float);
}

static size_t sort_smem(int tmax, int dmax) {
  return (size_t)(tmax + dmax) * 16 + (size_t)kKeyCap * 8 + (size_t)(dmax + tmax) * 4 +
         (size_t)(tmax + dmax) * 4;
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
  RV_CHECK_ARG(state_in && state_out && state_in != state_out, "state buffers must differ");
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
  const size_t hb = ((size_t)S * sizeof(StreamHdr) + 255) & ~(size_t)255;
  const StreamHdr* hin = (const StreamHdr*)state_in;
  Track* tin = (Track*)((uint8_t*)state_in + hb);
  StreamHdr* hout = (StreamHdr*)state_out;
  Track* tout = (Track*)((uint8_t*)state_out + hb);
  const size_t smem = sort_smem(tmax, dmax);
  RV_CHECK_ARG(smem <= 160 * 1024, "tmax/dmax need %zu B of LDS", smem);
  static int attr_set = 0;
  if ((int)smem > attr_set) {  // once per growth, outside steady-state launches
    hipError_t e = hipFuncSetAttribute((const void*)sort_update_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) {
      set_error("hipFuncSetAttribute(%zu B LDS): %s", smem, hipGetErrorString(e));
      (void)hipGetLastError();
      return -(int)e;
    }
    attr_set = (int)smem;
  }
  sort_update_kernel<<<S, 256, smem, as_stream(stream)>>>(hin, tin, hout, tout, dets, dcount, ts, p,
                                                          (float*)ws, out_id, out_dist, out_speed);
  return launch_status("rv_sort_update");
}

extern "C" int rv_sort_export(const void* state, int S, int tmax, double* x_out, int* meta,
                              int* T_out, void* stream) {
  RV_CHECK_ARG(state && x_out && meta && T_out && S > 0 && tmax > 0, "bad args");
  const size_t hb = ((size_t)S * sizeof(StreamHdr) + 255) & ~(size_t)255;
  sort_export_kernel<<<S, 256, 0, as_stream(stream)>>>(
      (const StreamHdr*)state, (const Track*)((const uint8_t*)state + hb), tmax, x_out, meta, T_out);
  return launch_status("rv_sort_export");
}

extern "C" int rv_sort_stats(const void* state, int S, int* T_out, int* next_id_out,
                             int* overflow_out, void* stream) {
  RV_CHECK_ARG(state && T_out && S > 0, "bad args");
  sort_stats_kernel<<<ceil_div(S, 256), 256, 0, as_stream(stream)>>>(
      (const StreamHdr*)state, S, T_out, next_id_out, overflow_out);
  return launch_status("rv_sort_stats");
}
