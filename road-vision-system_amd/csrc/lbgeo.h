// Ultralytics LetterBox geometry and the cv2.resize(INTER_LINEAR) 8U
// per-axis coefficients, shared by the standalone letterbox kernel
// (letterbox.hip) and the fused CLAHE+median+letterbox pass (preprocess.hip)
// so both produce the same bytes.
#pragma once
#include <math.h>
#include "common.h"

namespace rv {

struct LbGeo {
  int out_h, out_w, new_h, new_w, top, left;
  double scale_x, scale_y;  // source / destination (cv::resize scale)
};

// One axis of the resize: destination d reads source s0 (weight w0) and s1
// (weight w1), 11-bit weights; s0/s1 already clamped to [0, n).  A zero
// weight's index is redirected to the other tap, so it never leaves the
// support of the nonzero taps (the arithmetic is unchanged: 0 * v = 0).
struct LbTap {
  int s0, s1, w0, w1;
};

__host__ __device__ inline int lb_round_short(float v) {
  int r = (int)nearbyintf(v);  // cvRound/saturate_cast<short>, half-even
  return r < -32768 ? -32768 : (r > 32767 ? 32767 : r);
}

// horizontal taps: resizeGeneric_ xofs / ialpha (sx clamped on both sides,
// the right edge collapses to a single tap of weight 2048)
__host__ __device__ inline LbTap lb_tap_x(int dx, double scale, int n) {
  float fx = (float)((dx + 0.5) * scale - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) {
    fx = 0.f;
    sx = 0;
  }
  LbTap t;
  if (sx >= n - 1) {
    t.s0 = t.s1 = n - 1;
    t.w0 = 2048;
    t.w1 = 0;
    return t;
  }
  t.s0 = sx;
  t.s1 = sx + 1;
  t.w0 = lb_round_short((1.f - fx) * 2048.f);
  t.w1 = lb_round_short(fx * 2048.f);
  if (t.w1 == 0) t.s1 = t.s0;
  if (t.w0 == 0) t.s0 = t.s1;
  return t;
}

// vertical taps: yofs / ibeta; rows clamped, weights kept
__host__ __device__ inline LbTap lb_tap_y(int dy, double scale, int n) {
  float fy = (float)((dy + 0.5) * scale - 0.5);
  int sy = (int)floorf(fy);
  fy -= (float)sy;
  LbTap t;
  t.w0 = lb_round_short((1.f - fy) * 2048.f);
  t.w1 = lb_round_short(fy * 2048.f);
  t.s0 = sy < 0 ? 0 : (sy > n - 1 ? n - 1 : sy);
  t.s1 = sy + 1 < 0 ? 0 : (sy + 1 > n - 1 ? n - 1 : sy + 1);
  if (t.w1 == 0) t.s1 = t.s0;
  if (t.w0 == 0) t.s0 = t.s1;
  return t;
}

// VResizeLinear<uchar, int, short, FixedPtCast<int, uchar, 22>> on the two
// horizontally resized rows d0 = p00*wx0 + p01*wx1, d1 = p10*wx0 + p11*wx1.
__host__ __device__ inline int lb_vmix(int d0, int d1, int wy0, int wy1) {
  return (((wy0 * (d0 >> 4)) >> 16) + ((wy1 * (d1 >> 4)) >> 16) + 2) >> 2;
}

// geo6 = {out_h, out_w, new_h, new_w, top, left} (rv_letterbox_geometry)
// -> LbGeo with cv::resize's scale = 1 / (dsize / ssize).  0 if inconsistent.
inline bool lbgeo_from(const int* geo, int H, int W, LbGeo& g) {
  g.out_h = geo[0];
  g.out_w = geo[1];
  g.new_h = geo[2];
  g.new_w = geo[3];
  g.top = geo[4];
  g.left = geo[5];
  g.scale_x = 1.0 / ((double)g.new_w / W);
  g.scale_y = 1.0 / ((double)g.new_h / H);
  return g.new_h > 0 && g.new_w > 0 && g.top >= 0 && g.left >= 0 &&
         g.top + g.new_h <= g.out_h && g.left + g.new_w <= g.out_w;
}

// Fill only the 114 border of B letterboxed images (letterbox.hip).
int launch_letterbox_pad(uint8_t* out, int B, const LbGeo& g, hipStream_t s);

}  // namespace rv
