// Ultralytics LetterBox on gfx950 (the pre-transform inside model.predict,
// reached from src/detect/yolo_ultralytics.py:28-35).
//
// Restated semantics:
//   r = min(imgsz/H, imgsz/W); new = (round(W r), round(H r));
//   dw, dh = (imgsz - new) % stride / 2;
//   top, bottom = round(dh -/+ 0.1); left, right = round(dw -/+ 0.1)
//   cv2.resize(INTER_LINEAR) 8U fixed point (11-bit coefficients,
//   VResizeLinear<uchar> rounding), cv2.copyMakeBorder(BORDER_CONSTANT, 114).
// At 1920x1080 the scale is exactly 1/3, every source coordinate is integral
// (3x+1, 3y+1) and the resize is an exact decimation; at 640x640 and 640x480
// it is the identity.
#include "lbgeo.h"

namespace rv {

// One thread per output pixel.
__global__ __launch_bounds__(256) void letterbox_kernel(const uint8_t* __restrict__ in,
                                                        uint8_t* __restrict__ out, int H, int W,
                                                        int pitch, LbGeo g) {
  const int b = blockIdx.z;
  const int oy = blockIdx.y;
  const int ox = blockIdx.x * 256 + threadIdx.x;
  if (ox >= g.out_w) return;
  uint8_t* dst = out + (((size_t)b * g.out_h + oy) * g.out_w + ox) * 3;
  const int dy = oy - g.top, dx = ox - g.left;
  if (dy < 0 || dy >= g.new_h || dx < 0 || dx >= g.new_w) {
    dst[0] = 114;
    dst[1] = 114;
    dst[2] = 114;
    return;
  }
  const uint8_t* frame = in + (size_t)b * H * pitch;
  if (g.new_h == H && g.new_w == W) {  // no resize
    const uint8_t* s = frame + (size_t)dy * pitch + (size_t)dx * 3;
    dst[0] = s[0];
    dst[1] = s[1];
    dst[2] = s[2];
    return;
  }
  const LbTap tx = lb_tap_x(dx, g.scale_x, W), ty = lb_tap_y(dy, g.scale_y, H);
  const uint8_t* r0 = frame + (size_t)ty.s0 * pitch;
  const uint8_t* r1 = frame + (size_t)ty.s1 * pitch;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int d0 = r0[tx.s0 * 3 + c] * tx.w0 + r0[tx.s1 * 3 + c] * tx.w1;
    const int d1 = r1[tx.s0 * 3 + c] * tx.w0 + r1[tx.s1 * 3 + c] * tx.w1;
    dst[c] = (uint8_t)lb_vmix(d0, d1, ty.w0, ty.w1);
  }
}

// The constant-114 border of a letterbox whose interior another kernel
// writes (the fused preprocess pass): only the pad pixels are touched.
__global__ __launch_bounds__(256) void letterbox_pad_kernel(uint8_t* __restrict__ out, LbGeo g) {
  const int b = blockIdx.y;
  const int right = g.out_w - g.left - g.new_w;
  const int band = g.top * g.out_w;                             // top rows
  const int bottom = (g.out_h - g.top - g.new_h) * g.out_w;     // bottom rows
  const int side = g.new_h * (g.left + right);                  // left/right columns
  const int n = band + bottom + side;
  uint8_t* img = out + (size_t)b * g.out_h * g.out_w * 3;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int oy, ox;
    if (i < band) {
      oy = i / g.out_w;
      ox = i - oy * g.out_w;
    } else if (i < band + bottom) {
      const int j = i - band;
      oy = g.top + g.new_h + j / g.out_w;
      ox = j - (j / g.out_w) * g.out_w;
    } else {
      const int j = i - band - bottom;
      const int w = g.left + right;
      oy = g.top + j / w;
      const int c = j - (j / w) * w;
      ox = c < g.left ? c : g.left + g.new_w + (c - g.left);
    }
    uint8_t* d = img + ((size_t)oy * g.out_w + ox) * 3;
    d[0] = 114;
    d[1] = 114;
    d[2] = 114;
  }
}

int launch_letterbox_pad(uint8_t* out, int B, const LbGeo& g, hipStream_t s) {
  const int n = g.out_h * g.out_w - g.new_h * g.new_w;
  if (n <= 0 || B == 0) return RV_OK;
  letterbox_pad_kernel<<<dim3(ceil_div(n, 256), B), 256, 0, s>>>(out, g);
  return launch_status("letterbox_pad");
}

}  // namespace rv

using namespace rv;

extern "C" int rv_letterbox_geometry(int H, int W, int imgsz, int stride, int* geo) {
  RV_CHECK_ARG(geo != nullptr && H > 0 && W > 0 && imgsz > 0 && stride > 0, "bad letterbox args");
  const double r = fmin((double)imgsz / H, (double)imgsz / W);
  const int new_w = (int)nearbyint(W * r), new_h = (int)nearbyint(H * r);
  double dw = (double)((imgsz - new_w) % stride), dh = (double)((imgsz - new_h) % stride);
  if (dw < 0) dw += stride;  // np.mod semantics
  if (dh < 0) dh += stride;
  dw /= 2.0;
  dh /= 2.0;
  const int top = (int)nearbyint(dh - 0.1), bottom = (int)nearbyint(dh + 0.1);
  const int left = (int)nearbyint(dw - 0.1), right = (int)nearbyint(dw + 0.1);
  geo[0] = new_h + top + bottom;
  geo[1] = new_w + left + right;
  geo[2] = new_h;
  geo[3] = new_w;
  geo[4] = top;
  geo[5] = left;
  return RV_OK;
}

extern "C" int rv_letterbox_u8(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                               const int* geo, void* stream) {
  RV_CHECK_ARG(in != nullptr && out != nullptr && geo != nullptr, "null pointer");
  RV_CHECK_ARG(B >= 0 && H > 0 && W > 0 && pitch >= 3 * W, "bad frame shape");
  LbGeo g;
  RV_CHECK_ARG(lbgeo_from(geo, H, W, g), "inconsistent letterbox geometry");
  if (B == 0) return RV_OK;
  dim3 grid(ceil_div(g.out_w, 256), g.out_h, B);
  letterbox_kernel<<<grid, 256, 0, as_stream(stream)>>>(in, out, H, W, pitch, g);
  return launch_status("rv_letterbox_u8");
}
