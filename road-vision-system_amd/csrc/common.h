// Shared helpers for the gfx950 kernels behind include/rvhip.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include "../../include/rvhip.h"

namespace rv {

// Thread-local last error text, read back through rv_last_error().
void set_error(const char* fmt, ...);

// Convert a launch status into the ABI's return code.
inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return -(int)e;
  }
  return RV_OK;
}

// A HIP runtime call's status as an ABI code (RV_OK or -(hipError_t)), with
// the call named in rv_last_error() when it failed.
inline int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return RV_OK;
  set_error("%s: %s", what, hipGetErrorString(e));
  return -(int)e;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

#define RV_CHECK_ARG(cond, ...)      \
  do {                               \
    if (!(cond)) {                   \
      ::rv::set_error(__VA_ARGS__);  \
      return RV_EINVAL;              \
    }                                \
  } while (0)

// OpenCV saturate_cast<uchar>(int)
__device__ __forceinline__ int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// OpenCV BGR -> YCrCb, 8U, 14-bit fixed point (RGB2YCrCb_i<uchar>, blueIdx 0).
// Y = (B*1868 + G*9617 + R*4899 + 2^13) >> 14, Cr/Cb around 128.
__device__ __forceinline__ void bgr_to_ycrcb(int b, int g, int r, int& y, int& cr, int& cb) {
  int Y = (b * 1868 + g * 9617 + r * 4899 + 8192) >> 14;
  int Cr = ((r - Y) * 11682 + (128 << 14) + 8192) >> 14;
  int Cb = ((b - Y) * 9241 + (128 << 14) + 8192) >> 14;
  y = sat_u8(Y);
  cr = sat_u8(Cr);
  cb = sat_u8(Cb);
}

// OpenCV YCrCb -> BGR, 8U (YCrCb2RGB_i<uchar>): arithmetic shifts.
__device__ __forceinline__ void ycrcb_to_bgr(int y, int cr, int cb, int& b, int& g, int& r) {
  int dcb = cb - 128, dcr = cr - 128;
  b = sat_u8(y + ((dcb * 29049 + 8192) >> 14));
  g = sat_u8(y + ((dcb * -5636 + dcr * -11698 + 8192) >> 14));
  r = sat_u8(y + ((dcr * 22987 + 8192) >> 14));
}

// Only the Y of BGR -> YCrCb (also the BGR2GRAY value, 14-bit form).
__device__ __forceinline__ int bgr_to_y(int b, int g, int r) {
  return (b * 1868 + g * 9617 + r * 4899 + 8192) >> 14;
}

// OpenCV borderInterpolate(BORDER_REFLECT_101) for p outside [0, n).
__host__ __device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
  }
  return p;
}

}  // namespace rv
