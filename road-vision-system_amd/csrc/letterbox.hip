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
#include <math.h>
#include "common.h"

namespace rv {

struct LbGeo {
  int out_h, out_w, new_h, new_w, top, left;
  double scale_x, scale_y;  // source / destination
};

__device__ __forceinline__ int round_short(float v) {
  int r = __float2int_rn(v);
  return r < -32768 ? -32768 : (r > 32767 ? 32767 : r);
}

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
  // horizontal coefficients (resizeGeneric_ xofs/ialpha)
  float fx = (float)((dx + 0.5) * g.scale_x - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) {
    fx = 0.f;
    sx = 0;
  }
  bool single = false;
  if (sx >= W - 1) {
    fx = 0.f;
    sx = W - 1;
    single = true;
  }
  const int a0 = round_short((1.f - fx) * 2048.f), a1 = round_short(fx * 2048.f);
  // vertical coefficients (yofs/ibeta); rows clamped, weights kept
  float fy = (float)((dy + 0.5) * g.scale_y - 0.5);
  int sy = (int)floorf(fy);
  fy -= (float)sy;
  const int b0 = round_short((1.f - fy) * 2048.f), b1 = round_short(fy * 2048.f);
  const int r0 = min(max(sy, 0), H - 1), r1 = min(max(sy + 1, 0), H - 1);
  const uint8_t* s0 = frame + (size_t)r0 * pitch + (size_t)sx * 3;
  const uint8_t* s1 = frame + (size_t)r1 * pitch + (size_t)sx * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int d0, d1;
    if (single) {
      d0 = s0[c] * 2048;
      d1 = s1[c] * 2048;
    } else {
      d0 = s0[c] * a0 + s0[c + 3] * a1;
      d1 = s1[c] * a0 + s1[c + 3] * a1;
    }
    // VResizeLinear<uchar, int, short, FixedPtCast<int,uchar,22>>
    dst[c] = (uint8_t)((((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2);
  }
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
  g.out_h = geo[0];
  g.out_w = geo[1];
  g.new_h = geo[2];
  g.new_w = geo[3];
  g.top = geo[4];
  g.left = geo[5];
  RV_CHECK_ARG(g.new_h > 0 && g.new_w > 0 && g.top >= 0 && g.left >= 0 &&
                   g.top + g.new_h <= g.out_h && g.left + g.new_w <= g.out_w,
               "inconsistent letterbox geometry");
  if (B == 0) return RV_OK;
  // cv::resize: inv_scale = dsize/ssize, scale = 1/inv_scale
  g.scale_x = 1.0 / ((double)g.new_w / W);
  g.scale_y = 1.0 / ((double)g.new_h / H);
  dim3 grid(ceil_div(g.out_w, 256), g.out_h, B);
  letterbox_kernel<<<grid, 256, 0, as_stream(stream)>>>(in, out, H, W, pitch, g);
  return launch_status("rv_letterbox_u8");
}
