// 8U sRGB/D65 BGR <-> Lab for CLAHEDehaze's LAB path
// (src/preprocess/ops/clahe_dehaze.py:21-25: cv2.COLOR_BGR2LAB, CLAHE on L,
// cv2.COLOR_LAB2BGR).  Restates OpenCV 4.x color_lab.cpp's 8-bit integer
// paths: RGB2Lab_b (gamma table x 2^3, 12-bit XYZ coefficients, 15-bit cube
// root table, L = (296 fY - 1336934) >> 15 rounded) and Lab2RGBinteger
// (14-bit y / f(y) per L, fixed-point a/500 and b/200 dividers, piecewise
// f^-1, 4096-entry inverse gamma).  The tables are built once on the host in
// double with round-half-even and copied into device memory on first use.
#pragma once
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

namespace rv {

struct LabTables {
  uint16_t gamma[256];  // sRGB u8 -> linear x 255*8
  uint16_t cbrt[3072];  // f(t) x 2^15, t = i / (255*8)
  uint16_t yf[512];     // per L: {y x 2^14, f(y) x 2^14}
  uint16_t invg[4096];  // linear i/4096 -> sRGB u8
  int32_t cf[9];        // rows X,Y,Z over (B,G,R): M_rgb2xyz / white x 2^12
  int32_t ci[9];        // rows B,G,R over (X,Y,Z): M_xyz2rgb * white x 2^12
};
static_assert(sizeof(LabTables) == 2 * (256 + 3072 + 512 + 4096) + 4 * 18, "packed layout");

inline void build_lab_tables(LabTables& t) {
  static const double m[9] = {0.412453, 0.357580, 0.180423, 0.212671, 0.715160,
                              0.072169, 0.019334, 0.119193, 0.950227};  // sRGB -> XYZ (D65)
  static const double mi[9] = {3.240479, -1.53715, -0.498535, -0.969256, 1.875991,
                               0.041556, 0.055648, -0.204043, 1.057311};  // XYZ -> sRGB
  static const double wp[3] = {0.950456, 1.0, 1.088754};
  for (int i = 0; i < 256; ++i) {
    const double x = i / 255.0;
    const double lin = x <= 0.04045 ? x / 12.92 : std::pow((x + 0.055) / 1.055, 2.4);
    t.gamma[i] = (uint16_t)std::nearbyint(2040.0 * lin);
  }
  for (int i = 0; i < 3072; ++i) {
    const double x = i / 2040.0;
    const double f = x < 216.0 / 24389.0 ? x * (841.0 / 108.0) + 16.0 / 116.0 : std::cbrt(x);
    t.cbrt[i] = (uint16_t)std::nearbyint(32768.0 * f);
  }
  const double base = 16384.0;
  for (int i = 0; i < 256; ++i) {
    double y, fy;
    if (i <= 20) {  // linear segment of f^-1 below L = 8
      y = std::nearbyint(i * base * 180.0 / 414613.0);
      fy = std::nearbyint(base * (16.0 / 116.0 + i * 5.0 / 1479.0));
    } else {
      const double f = i * 100.0 * base / (255.0 * 116.0) + 16.0 * base / 116.0;
      fy = std::nearbyint(f);
      y = std::nearbyint(f * f * f / (base * base));
    }
    t.yf[2 * i] = (uint16_t)y;
    t.yf[2 * i + 1] = (uint16_t)fy;
  }
  for (int i = 0; i < 4096; ++i) {
    const double x = i / 4096.0;
    const double v = x <= 0.0031308 ? 12.92 * x : 1.055 * std::pow(x, 1.0 / 2.4) - 0.055;
    t.invg[i] = (uint16_t)std::nearbyint(255.0 * v);
  }
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      t.cf[r * 3 + c] = (int32_t)std::nearbyint(4096.0 * m[r * 3 + (2 - c)] / wp[r]);
      t.ci[r * 3 + c] = (int32_t)std::nearbyint(4096.0 * mi[(2 - r) * 3 + c] * wp[c]);
    }
}

__device__ __forceinline__ int lab_sat(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// L only (the CLAHE histogram pass needs nothing else).
__device__ __forceinline__ int lab_l(const LabTables& t, int b, int g, int r) {
  const int B = t.gamma[b], G = t.gamma[g], R = t.gamma[r];
  const int Y = (t.cf[3] * B + t.cf[4] * G + t.cf[5] * R + 2048) >> 12;
  return lab_sat((296 * (int)t.cbrt[Y] - 1336934 + (1 << 14)) >> 15);
}

__device__ __forceinline__ void bgr_to_lab(const LabTables& t, int b, int g, int r, int& L,
                                           int& A, int& Bo) {
  const int B = t.gamma[b], G = t.gamma[g], R = t.gamma[r];
  const int X = (t.cf[0] * B + t.cf[1] * G + t.cf[2] * R + 2048) >> 12;
  const int Y = (t.cf[3] * B + t.cf[4] * G + t.cf[5] * R + 2048) >> 12;
  const int Z = (t.cf[6] * B + t.cf[7] * G + t.cf[8] * R + 2048) >> 12;
  const int fX = t.cbrt[X], fY = t.cbrt[Y], fZ = t.cbrt[Z];
  L = lab_sat((296 * fY - 1336934 + (1 << 14)) >> 15);
  A = lab_sat((500 * (fX - fY) + (128 << 15) + (1 << 14)) >> 15);
  Bo = lab_sat((200 * (fY - fZ) + (128 << 15) + (1 << 14)) >> 15);
}

// f^-1 on the 14-bit scale: linear below 6/29 (x 2^14 = 3390), cube above.
__device__ __forceinline__ int lab_finv(int v) {
  return v <= 3390 ? v * 108 / 841 - 290 : v * v / 16384 * v / 16384;
}

__device__ __forceinline__ void lab_to_bgr(const LabTables& t, int L, int a, int b, int& ob,
                                           int& og, int& orr) {
  const int y = t.yf[2 * L], fy = t.yf[2 * L + 1];
  const int adiv = ((5 * a * 53687 + (1 << 7)) >> 13) - 4194;   // a/500 x 2^14 - 128/500
  const int bdiv = ((b * 41943 + (1 << 4)) >> 9) - 10485 + 1;   // b/200 x 2^14 - 128/200
  const int x = lab_finv(fy + adiv), z = lab_finv(fy - bdiv);
  int o[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    int v = (t.ci[r * 3] * x + t.ci[r * 3 + 1] * y + t.ci[r * 3 + 2] * z + (1 << 13)) >> 14;
    v = v < 0 ? 0 : (v > 4095 ? 4095 : v);
    o[r] = t.invg[v];
  }
  ob = o[0];
  og = o[1];
  orr = o[2];
}

}  // namespace rv
