// Scalar math shared by the fused SORT kernel (sort.hip) and the standalone
// tracker / geometry entries (track_ops.hip).  Compiled with
// -ffp-contract=off, so every expression rounds like the numpy scalar code
// it restates.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace rv {

// _iou in numpy float32 scalar arithmetic (sort_tracker.py:55-71)
__device__ __forceinline__ float iou_f32(float4 a, float4 b) {
  const float ix1 = fmaxf(a.x, b.x), iy1 = fmaxf(a.y, b.y);
  const float ix2 = fminf(a.z, b.z), iy2 = fminf(a.w, b.w);
  const float iw = fmaxf(0.0f, ix2 - ix1), ih = fmaxf(0.0f, iy2 - iy1);
  const float inter = iw * ih;
  const float area_a = fmaxf(0.0f, a.z - a.x) * fmaxf(0.0f, a.w - a.y);
  const float area_b = fmaxf(0.0f, b.z - b.x) * fmaxf(0.0f, b.w - b.y);
  const float denom = area_a + area_b - inter;
  if (denom <= 0.0f) return 0.0f;
  return inter / denom;
}

// HomographyProjector.project_point (projector.py:74-84): f64 H x [x, y, 1]
__device__ __forceinline__ bool project_h(const double* H, double x, double y, double& X,
                                          double& Y) {
  const double mx = H[0] * x + H[1] * y + H[2];
  const double my = H[3] * x + H[4] * y + H[5];
  const double w = H[6] * x + H[7] * y + H[8];
  if (fabs(w) < 1e-6) return false;
  X = mx / w;
  Y = my / w;
  return isfinite(X) && isfinite(Y);
}

// GroundProjector.distance (projector.py:37-47): f32 norm, optional cap;
// NaN = None.  max_distance < 0 means no cap.
__device__ __forceinline__ double distance_o(const float* origin, double max_distance, double X,
                                             double Y) {
  const float vx = (float)X - origin[0], vy = (float)Y - origin[1];
  const float d = sqrtf(vx * vx + vy * vy);
  if (!isfinite(d)) return NAN;
  double dd = (double)d;
  if (max_distance >= 0.0) dd = fmin(dd, max_distance);
  return dd;
}

}  // namespace rv
