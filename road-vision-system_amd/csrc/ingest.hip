// Frame ingest: NV12 -> interleaved BGR on device (cv2.COLOR_YUV2BGR_NV12,
// 8U; OpenCV color_yuv YUV420sp2RGB8: BT.601 video range, 20-bit fixed
// point).  The reference's capture (src/io_video/capture.py:10-24) hands BGR
// frames to the per-frame path; uploading NV12 instead (1.5 B/pixel) halves
// the PCIe bytes of host-fed frames, and NV12 is what a hardware decoder
// produces, so this pass is the device half of a decode front end.
//
// HBM-bound: 1.5 B read + 3 B written per pixel.  One thread converts a
// 4 x 2 pixel block (one dword of U,V pairs, two dwords of Y, three dwords
// out per row) when rows are dword aligned; a 2 x 2 scalar path otherwise.
#include "common.h"

namespace rv {

namespace {

constexpr int kCY = 1220542, kCUB = 2116026, kCUG = -409993, kCVG = -852492, kCVR = 1673527;
constexpr int kSh = 20;

struct UvTerms {
  int r, g, b;
};

__device__ __forceinline__ UvTerms uv_terms(int u, int v) {
  u -= 128;
  v -= 128;
  return {(1 << (kSh - 1)) + kCVR * v, (1 << (kSh - 1)) + kCVG * v + kCUG * u,
          (1 << (kSh - 1)) + kCUB * u};
}

// An empty asm value barrier.  Without it the gfx950 backend (ROCm 7.2
// LLVM) fuses `sat_u8(a >> 20) | sat_u8(b >> 20) << 8` into
// v_ashr_pk_u8_i32 and then ORs that result into a dword as if its upper 16
// bits were zero; they are not, and bytes 2-3 of every packed dword came out
// wrong (caught by tests/test_preprocess_gpu.py::test_nv12_to_bgr_bit_exact).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// returns b | g << 8 | r << 16
__device__ __forceinline__ uint32_t yuv_px(int y, const UvTerms& t) {
  const int yy = max(y - 16, 0) * kCY;
  const int b = opaque(sat_u8((yy + t.b) >> kSh));
  const int g = opaque(sat_u8((yy + t.g) >> kSh));
  const int r = opaque(sat_u8((yy + t.r) >> kSh));
  return (uint32_t)b | ((uint32_t)g << 8) | ((uint32_t)r << 16);
}

__global__ __launch_bounds__(256) void nv12_vec_kernel(const uint8_t* __restrict__ y,
                                                       const uint8_t* __restrict__ uv,
                                                       int y_pitch, int uv_pitch, size_t y_fstride,
                                                       size_t uv_fstride,
                                                       uint8_t* __restrict__ out, int H, int W,
                                                       int pitch) {
  const int b = blockIdx.y;
  const int gpr = W / 4, n = (H / 2) * gpr;
  const uint8_t* fy = y + b * y_fstride;
  const uint8_t* fuv = uv + b * uv_fstride;
  uint8_t* fo = out + (size_t)b * H * pitch;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r2 = i / gpr, x0 = (i - r2 * gpr) * 4;
    const uint32_t q = *(const uint32_t*)(fuv + (size_t)r2 * uv_pitch + x0);
    const UvTerms t0 = uv_terms(q & 255, (q >> 8) & 255);
    const UvTerms t1 = uv_terms((q >> 16) & 255, q >> 24);
#pragma unroll
    for (int dr = 0; dr < 2; ++dr) {
      const int r = 2 * r2 + dr;
      const uint32_t yw = *(const uint32_t*)(fy + (size_t)r * y_pitch + x0);
      const uint32_t p0 = yuv_px(yw & 255, t0), p1 = yuv_px((yw >> 8) & 255, t0);
      const uint32_t p2 = yuv_px((yw >> 16) & 255, t1), p3 = yuv_px(yw >> 24, t1);
      // 4 BGR pixels = 12 bytes = 3 dwords, little-endian
      uint32_t* d = (uint32_t*)(fo + (size_t)r * pitch + (size_t)x0 * 3);
      d[0] = p0 | (p1 << 24);
      d[1] = (p1 >> 8) | (p2 << 16);
      d[2] = (p2 >> 16) | (p3 << 8);
    }
  }
}

__global__ __launch_bounds__(256) void nv12_scalar_kernel(const uint8_t* __restrict__ y,
                                                          const uint8_t* __restrict__ uv,
                                                          int y_pitch, int uv_pitch,
                                                          size_t y_fstride, size_t uv_fstride,
                                                          uint8_t* __restrict__ out, int H,
                                                          int W, int pitch) {
  const int b = blockIdx.y;
  const int cpr = W / 2, n = (H / 2) * cpr;
  const uint8_t* fy = y + b * y_fstride;
  const uint8_t* fuv = uv + b * uv_fstride;
  uint8_t* fo = out + (size_t)b * H * pitch;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r2 = i / cpr, c2 = i - r2 * cpr;
    const uint8_t* q = fuv + (size_t)r2 * uv_pitch + 2 * c2;
    const UvTerms t = uv_terms(q[0], q[1]);
#pragma unroll
    for (int dr = 0; dr < 2; ++dr)
#pragma unroll
      for (int dc = 0; dc < 2; ++dc) {
        const int r = 2 * r2 + dr, c = 2 * c2 + dc;
        const uint32_t p = yuv_px(fy[(size_t)r * y_pitch + c], t);
        uint8_t* d = fo + (size_t)r * pitch + (size_t)c * 3;
        d[0] = p & 255;
        d[1] = (p >> 8) & 255;
        d[2] = (p >> 16) & 255;
      }
  }
}

}  // namespace

extern "C" int rv_nv12_to_bgr_u8(const uint8_t* y, const uint8_t* uv, int y_pitch, int uv_pitch,
                                 size_t y_frame_stride, size_t uv_frame_stride, uint8_t* out,
                                 int B, int H, int W, int pitch, void* stream) {
  RV_CHECK_ARG(y != nullptr && uv != nullptr && out != nullptr, "null pointer");
  RV_CHECK_ARG(B >= 0 && H > 0 && W > 0 && H % 2 == 0 && W % 2 == 0,
               "bad NV12 shape B=%d H=%d W=%d (H, W even)", B, H, W);
  RV_CHECK_ARG(y_pitch >= W && uv_pitch >= W && pitch >= 3 * W, "pitch too small");
  RV_CHECK_ARG(y_frame_stride >= (size_t)H * y_pitch &&
                   uv_frame_stride >= (size_t)(H / 2) * uv_pitch,
               "frame stride too small");
  if (B == 0) return RV_OK;
  hipStream_t s = as_stream(stream);
  const bool vec = W % 4 == 0 && y_pitch % 4 == 0 && uv_pitch % 4 == 0 && pitch % 4 == 0 &&
                   y_frame_stride % 4 == 0 && uv_frame_stride % 4 == 0 &&
                   (((uintptr_t)y | (uintptr_t)uv | (uintptr_t)out) % 4 == 0);
  if (vec) {
    const int blocks = min(2048, ceil_div((H / 2) * (W / 4), 256));
    nv12_vec_kernel<<<dim3(blocks, B), 256, 0, s>>>(y, uv, y_pitch, uv_pitch, y_frame_stride,
                                                    uv_frame_stride, out, H, W, pitch);
  } else {
    const int blocks = min(2048, ceil_div((H / 2) * (W / 2), 256));
    nv12_scalar_kernel<<<dim3(blocks, B), 256, 0, s>>>(y, uv, y_pitch, uv_pitch, y_frame_stride,
                                                       uv_frame_stride, out, H, W, pitch);
  }
  return launch_status("rv_nv12_to_bgr_u8");
}

}  // namespace rv
