// Hand-back of one step's results to the host.
//
// Reference: the per-frame path ends on the host -- YOLOUltralytics.infer
// copies boxes.xyxy / conf / cls with .cpu().numpy() and builds Detection
// objects (src/detect/yolo_ultralytics.py:44-52); SortTracker.update then
// fills track_id / distance_m / speed_kmh in place (sort_tracker.py:234-247).
// Here the device outputs of a step (NMS rows + counts, SORT ids / metrics)
// are packed into one contiguous record and copied device -> host with a
// single stream-ordered hipMemcpyAsync, so a captured step graph ends with
// its results already in pinned host memory (no per-field copies, no host
// synchronisation inside the step).
//
// Record layout (rv_results_bytes): int32 n[S] (padded to 16 B), then
// S x dmax rows of 48 B {f32 x1, y1, x2, y2, conf; i32 cls, track_id (-1 =
// None), pad; f64 distance_m, speed_kmh (NaN = None)}; rows >= n[s] are
// zero-filled.
#include "common.h"

namespace rv {

struct DetRecord {
  float x1, y1, x2, y2, conf;
  int cls, track_id, pad;
  double dist, speed;
};
static_assert(sizeof(DetRecord) == 48, "record row is 48 bytes");

__host__ __device__ static inline size_t header_bytes(int S) { return ((size_t)S * 4 + 15) & ~(size_t)15; }

// One thread per (stream, row); rows past the stream's count are zeroed so
// the record is fully defined.
__global__ void results_pack_kernel(const float* __restrict__ dets, const int* __restrict__ det_n,
                                    const int* __restrict__ tid, const double* __restrict__ dist,
                                    const double* __restrict__ spd, int S, int dmax,
                                    uint8_t* __restrict__ rec) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S * dmax) return;
  const int s = i / dmax, r = i - s * dmax;
  int n = det_n[s];
  n = n < 0 ? 0 : (n > dmax ? dmax : n);
  if (r == 0) ((int*)rec)[s] = n;
  DetRecord d;
  if (r < n) {
    const float* p = dets + (size_t)i * 6;
    d.x1 = p[0];
    d.y1 = p[1];
    d.x2 = p[2];
    d.y2 = p[3];
    d.conf = p[4];
    d.cls = (int)p[5];
    d.track_id = tid ? tid[i] : -1;
    d.pad = 0;
    d.dist = dist ? dist[i] : __longlong_as_double(0x7FF8000000000000ll);
    d.speed = spd ? spd[i] : __longlong_as_double(0x7FF8000000000000ll);
  } else {
    d.x1 = d.y1 = d.x2 = d.y2 = d.conf = 0.f;
    d.cls = 0;
    d.track_id = -1;
    d.pad = 0;
    d.dist = d.speed = 0.0;
  }
  ((DetRecord*)(rec + header_bytes(S)))[i] = d;
}

}  // namespace rv

using namespace rv;

extern "C" size_t rv_results_bytes(int S, int dmax) {
  if (S <= 0 || dmax <= 0) return 0;
  return header_bytes(S) + (size_t)S * dmax * sizeof(DetRecord);
}

extern "C" int rv_results_handback(const float* dets, const int* det_n, const int* track_id,
                                   const double* distance_m, const double* speed_kmh, int S,
                                   int dmax, void* dev_stage, size_t stage_bytes, void* host_dst,
                                   void* stream) {
  RV_CHECK_ARG(dets && det_n && dev_stage, "null pointer");
  RV_CHECK_ARG(S > 0 && dmax > 0, "bad sizes S=%d dmax=%d", S, dmax);
  const size_t nb = rv_results_bytes(S, dmax);
  RV_CHECK_ARG(stage_bytes >= nb, "stage %zu B < rv_results_bytes = %zu", stage_bytes, nb);
  const int n = S * dmax;
  // A pinned host record the device can address is written by the pack
  // kernel itself (one launch; the kernel's completion, which the caller's
  // event waits for, publishes the writes): no staging copy and no
  // dependent copy launch per step -- at the end of a pipelined run those
  // two gaps separated every SORT launch of the drain.  RV_HANDBACK_DIRECT=0
  // keeps the stage + hipMemcpyAsync form (A/B).
  static const bool direct = !getenv("RV_HANDBACK_DIRECT") || atoi(getenv("RV_HANDBACK_DIRECT")) != 0;
  if (host_dst && direct) {
    void* dptr = nullptr;
    if (hipHostGetDevicePointer(&dptr, host_dst, 0) == hipSuccess && dptr) {
      results_pack_kernel<<<ceil_div(n, 256), 256, 0, as_stream(stream)>>>(
          dets, det_n, track_id, distance_m, speed_kmh, S, dmax, (uint8_t*)dptr);
      return launch_status("rv_results_handback");
    }
    (void)hipGetLastError();  // not a registered host allocation: stage + copy
  }
  results_pack_kernel<<<ceil_div(n, 256), 256, 0, as_stream(stream)>>>(
      dets, det_n, track_id, distance_m, speed_kmh, S, dmax, (uint8_t*)dev_stage);
  int st = launch_status("rv_results_handback");
  if (st || !host_dst) return st;
  return hip_check(hipMemcpyAsync(host_dst, dev_stage, nb, hipMemcpyDeviceToHost, as_stream(stream)),
                   "rv_results_handback hipMemcpyAsync");
}
