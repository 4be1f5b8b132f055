// Preprocess kernels for gfx950: CLAHE (YCrCb luma), k x k median, and the
// fused CLAHE+median pass used by the default chain.
//
// Reference interface: src/preprocess/ops/clahe_dehaze.py:13-32 (CLAHEDehaze)
// and src/preprocess/ops/median_derain.py:10-14 (MedianDerain).  The
// arithmetic those ops delegate to OpenCV is restated here:
//   * BGR<->YCrCb 8U: 14-bit fixed point (common.h)
//   * cv::CLAHE 8UC1: per-tile 256-bin histogram, integer clip +
//     redistribution, float CDF LUT, float bilinear blend of 4 tile LUTs
//     (cvRound = round-half-even).  Compiled with -ffp-contract=off so the
//     blend rounds exactly like the scalar C++.
//   * cv::medianBlur 8UC3: exact per-channel median, BORDER_REPLICATE.
//
// HBM layout: frames are B x H x pitch bytes (interleaved BGR).  The LUT
// workspace is B x tiles^2 x 256 u8 (16 KB per frame at 8x8).
#include <cstring>
#include <mutex>
#include "lab.h"
#include "lbgeo.h"

// Cache policy of the preprocess's streaming traffic: the frames are read
// twice (LUT pass, then the median pass) and proc is written once and never
// read back on the device.  Non-temporal loads / stores (global_* nt) keep
// those ~600 MB per 32-frame step from evicting the detector's activations
// out of L2 / the Infinity Cache while the passes overlap the forward:
// +1.5 % frames/s in the bench (5 interleaved runs each, profiles/r06/).
// The letterbox output (read by the stem) stays temporal.  Build with
// -DRV_PRE_TEMPORAL for plain loads / stores (A/B).
#ifndef RV_PRE_TEMPORAL
#define RV_LUT_LD(p) __builtin_nontemporal_load(p)
#define RV_MED_LD(p) __builtin_nontemporal_load(p)
#define RV_MED_ST(p, v) __builtin_nontemporal_store((v), (p))
#else
#define RV_LUT_LD(p) (*(p))
#define RV_MED_LD(p) (*(p))
#define RV_MED_ST(p, v) (*(p) = (v))
#endif

namespace rv {

struct ClaheGeo {
  int tiles;       // tiles per axis
  int tw, th;      // tile size in the (possibly reflect-101 extended) image
  int clip_limit;  // integer clip (0 = no clipping)
  float lut_scale; // 255.f / (tw*th)
  float inv_tw, inv_th;
};

// cv::CLAHE_Impl::apply geometry (imgproc/src/clahe.cpp): when either axis
// is not divisible by the grid, BOTH axes are extended by
// tiles - (n % tiles) (a full extra tile-row of padding on a divisible axis).
static ClaheGeo make_geo(int H, int W, int tiles, double clip) {
  ClaheGeo g;
  g.tiles = tiles;
  if (W % tiles == 0 && H % tiles == 0) {
    g.tw = W / tiles;
    g.th = H / tiles;
  } else {
    g.tw = (W + tiles - (W % tiles)) / tiles;
    g.th = (H + tiles - (H % tiles)) / tiles;
  }
  int area = g.tw * g.th;
  g.lut_scale = 255.0f / (float)area;
  g.clip_limit = 0;
  if (clip > 0.0) {
    g.clip_limit = (int)(clip * area / 256);
    if (g.clip_limit < 1) g.clip_limit = 1;
  }
  g.inv_tw = 1.0f / (float)g.tw;
  g.inv_th = 1.0f / (float)g.th;
  return g;
}

// Lab tables (lab.h) in device memory, filled once on first LAB use.
__device__ LabTables g_lab;

enum ClaheSpace { kYCrCb = 0, kLab = 1 };

template <int SPACE>
__device__ __forceinline__ int clahe_luma(int b, int g, int r) {
  if (SPACE == kLab) return lab_l(g_lab, b, g, r);
  return bgr_to_y(b, g, r);
}

// ---------------------------------------------------------------------------
// Kernel A: per (tile, frame) histogram of Y -> clip -> redistribute -> LUT.
// One 256-thread workgroup per tile.
// PACKED (every tile whose counts fit 16 bits; the default at 1080p): 32
// LDS histogram copies, copy = lane & 31, two bins per word as u16 counts:
// bin y of copy c is half y & 1 of word 32 (y >> 1) + c.  An atomic add's
// bank is then (word mod 32/64) = c + 32 ((y >> 1) & 1): the 32 lanes of a
// lane group always hit 32 different banks and never one address, whatever
// the image -- conflict-free.  The reduction reads a row's 32 words as 8
// rotated 16-B quads (conflict-free) and, for tiles below 2^16 pixels, adds
// whole words before extracting the bin's half.  16 KB of LDS, as before.
// Otherwise (tiles of > 2M pixels): 16 u32 copies, copy = lane & 15, word
// 257 c + y.
// (r02/r03: copy = wave x lane & 3, bin-major -- a wave reached only 16 banks
// and up to 16 lanes hit one address, SQ_LDS_BANK_CONFLICT /
// SQ_LDS_IDX_ACTIVE 0.78; the 257-word form alone: 0.68.  r02's one copy
// per lane with u16 counters in 33 KB halved the resident blocks: slower.)
// ---------------------------------------------------------------------------
template <int SPACE, bool PACKED>
__device__ __forceinline__ void clahe_lut_body(const uint8_t* __restrict__ in,
                                               uint8_t* __restrict__ lut, int H, int W, int pitch,
                                               const ClaheGeo& g, int tile, int b, int t) {
  constexpr int kCopies = PACKED ? 32 : 16;
  constexpr int kStride = PACKED ? 0 : 257;  // u32 form: words per copy
  constexpr int kWords = PACKED ? 128 * 32 : kStride * kCopies;
  __shared__ __attribute__((aligned(16))) int hist[kWords];
  __shared__ int wsum[4], wtot[4];
  const int wave = t >> 6;
  const int r_lo = 0, r_hi = g.th;
  const int ty = tile / g.tiles, tx = tile - (tile / g.tiles) * g.tiles;
  const int x0 = tx * g.tw, y0 = ty * g.th;
  const uint8_t* frame = in + (size_t)b * H * pitch;

  for (int i = t; i < kWords; i += 256) hist[i] = 0;
  __syncthreads();

  const bool inside = (x0 + g.tw <= W) && (y0 + g.th <= H);
  const bool vec = inside && (g.tw % 4 == 0) && (pitch % 4 == 0) &&
                   ((((uintptr_t)frame) + (uintptr_t)x0 * 3) % 4 == 0);
  int* h = hist + (t & (kCopies - 1)) * (PACKED ? 1 : kStride);
  auto bump = [&](int y) {
    if constexpr (PACKED)
      atomicAdd(&h[(y >> 1) * 32], 1 << ((y & 1) << 4));
    else
      atomicAdd(&h[y], 1);
  };
  if (vec) {
    // thread t takes the 4-pixel groups i = t + 256 k of the tile (row i /
    // groups, column i % groups), two batches of 4 in flight: batch k + 1's
    // loads are issued before batch k's pixels are binned, and a group's
    // byte offset is stepped incrementally (a division per group was ~20 VALU
    // of the ~70 a group costs)
    const int groups = g.tw >> 2, rows = r_hi - r_lo;
    const int dr = 256 / groups, dg = 256 - dr * groups;  // block-uniform steps
    const int step_b = dr * pitch + dg * 12, wrap_b = pitch - groups * 12;
    const uint8_t* base = frame + (size_t)(y0 + r_lo) * pitch + (size_t)x0 * 3;
    int r = t / groups, gi = t - (t / groups) * groups;
    int off = r * pitch + gi * 12;
    auto advance = [&]() {
      off += step_b;
      r += dr;
      gi += dg;
      if (gi >= groups) {
        gi -= groups;
        ++r;
        off += wrap_b;
      }
    };
    auto load4 = [&](uint32_t (&w)[4][3], bool (&ok)[4]) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ok[u] = r < rows;
        w[u][0] = w[u][1] = w[u][2] = 0;
        if (ok[u]) {
          const uint32_t* q = (const uint32_t*)(base + off);
          w[u][0] = RV_LUT_LD(q);
          w[u][1] = RV_LUT_LD(q + 1);
          w[u][2] = RV_LUT_LD(q + 2);
        }
        advance();
      }
    };
    auto bin4 = [&](const uint32_t (&w)[4][3], const bool (&ok)[4]) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (!ok[u]) break;
        const uint32_t w0 = w[u][0], w1 = w[u][1], w2 = w[u][2];
        // bytes little-endian: w0 = b0 g0 r0 b1 | w1 = g1 r1 b2 g2 | w2 = r2 b3 g3 r3
        bump(clahe_luma<SPACE>(w0 & 255, (w0 >> 8) & 255, (w0 >> 16) & 255));
        bump(clahe_luma<SPACE>(w0 >> 24, w1 & 255, (w1 >> 8) & 255));
        bump(clahe_luma<SPACE>((w1 >> 16) & 255, w1 >> 24, w2 & 255));
        bump(clahe_luma<SPACE>((w2 >> 8) & 255, (w2 >> 16) & 255, w2 >> 24));
      }
    };
    uint32_t wa[4][3], wb[4][3];
    bool oka[4], okb[4];
    load4(wa, oka);
    while (oka[0]) {  // groups are in row order: once one is past the tile, so are the rest
      load4(wb, okb);
      bin4(wa, oka);
      if (!okb[0]) break;
      load4(wa, oka);
      bin4(wb, okb);
    }
  } else {
    const int total = g.tw * (r_hi - r_lo);
    for (int i = t; i < total; i += 256) {
      const int r = r_lo + i / g.tw;
      const int c = i - r * g.tw;
      int sy = y0 + r;
      if (sy >= H) sy = reflect101(sy, H);
      int sx = x0 + c;
      if (sx >= W) sx = reflect101(sx, W);
      const uint8_t* p = frame + (size_t)sy * pitch + (size_t)sx * 3;
      bump(clahe_luma<SPACE>(p[0], p[1], p[2]));
    }
  }
  __syncthreads();

  int v = 0;
  if constexpr (PACKED) {
    // bin t = half t & 1 of the 32 copies' words of row t >> 1, read as 8
    // 16-B quads (quad j rotated by the row: lanes of one ds_read_b128 group
    // cover 8 rows x 2 bin halves on 16 distinct bank slots)
    const int rw = t >> 1, sh = (t & 1) << 4;
    const uint4* row = (const uint4*)(hist + rw * 32);
    if ((long)g.tw * g.th <= 65535) {
      // the low halves' sum is the bin's count (<= tile pixels < 2^16): add
      // whole words, extract once
      uint32_t sum = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint4 q = row[(j + rw) & 7];
        sum += q.x + q.y + q.z + q.w;
      }
      v = (int)((sum >> sh) & 0xFFFF);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint4 q = row[(j + rw) & 7];
        v += (int)(((q.x >> sh) & 0xFFFF) + ((q.y >> sh) & 0xFFFF) + ((q.z >> sh) & 0xFFFF) +
                   ((q.w >> sh) & 0xFFFF));
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < kCopies; ++c) v += hist[c * kStride + t];
  }
  if (g.clip_limit > 0) {
    int ex = v > g.clip_limit ? v - g.clip_limit : 0;
    v = v > g.clip_limit ? g.clip_limit : v;
    // block sum of the clipped excess
    for (int off = 32; off > 0; off >>= 1) ex += __shfl_xor(ex, off);
    if ((t & 63) == 0) wsum[wave] = ex;
    __syncthreads();
    const int clipped = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    const int batch = clipped / 256;
    const int residual = clipped - batch * 256;
    v += batch;
    if (residual != 0) {
      int step = 256 / residual;
      if (step < 1) step = 1;
      if (t % step == 0 && t / step < residual) v += 1;
    }
  }
  // inclusive prefix sum over the 256 bins: wave scans, then the totals of
  // the lower waves
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(v, off);
    if ((t & 63) >= off) v += y;
  }
  if ((t & 63) == 63) wtot[wave] = v;
  __syncthreads();
  for (int w = 0; w < wave; ++w) v += wtot[w];
  const float f = (float)v * g.lut_scale;
  uint8_t* dst = lut + ((size_t)b * g.tiles * g.tiles + tile) * 256;
  dst[t] = (uint8_t)sat_u8(__float2int_rn(f));
}

template <int SPACE, bool PACKED>
__global__ __launch_bounds__(256) void clahe_lut_kernel(const uint8_t* __restrict__ in,
                                                        uint8_t* __restrict__ lut, int H, int W,
                                                        int pitch, ClaheGeo g) {
  clahe_lut_body<SPACE, PACKED>(in, lut, H, W, pitch, g, blockIdx.x, blockIdx.y, threadIdx.x);
}

// u16 counts per (copy, bin) fit: a copy is shared by 8 threads (lanes c,
// c + 32 of 4 waves), each bumping at most 4 ceil(tw/4 th / 256) (vector
// path) or ceil(tw th / 256) pixels
static bool clahe_packed_ok(const ClaheGeo& g) {
  const long per_thread = 4L * (((long)(g.tw / 4) * g.th + 255) / 256) + ((long)g.tw * g.th + 255) / 256;
  return 8 * per_thread <= 65535;
}

template <int SPACE>
static void launch_clahe_lut(const uint8_t* in, uint8_t* lut, int B, int H, int W, int pitch,
                             const ClaheGeo& g, hipStream_t s) {
  if (clahe_packed_ok(g))
    clahe_lut_kernel<SPACE, true><<<dim3(g.tiles * g.tiles, B), 256, 0, s>>>(in, lut, H, W, pitch, g);
  else
    clahe_lut_kernel<SPACE, false><<<dim3(g.tiles * g.tiles, B), 256, 0, s>>>(in, lut, H, W, pitch, g);
}

// CLAHE_Interpolation_Body per-axis coefficients.
struct Interp {
  int i1, i2;   // clamped tile indices
  float a, a1;  // weight of i2 / of i1
};
__device__ __forceinline__ Interp interp_axis(int p, float inv, int tiles) {
  Interp r;
  const float f = (float)p * inv - 0.5f;
  const int i1 = (int)floorf(f);
  r.a = f - (float)i1;
  r.a1 = 1.0f - r.a;
  r.i1 = i1 < 0 ? 0 : i1;
  r.i2 = (i1 + 1) > tiles - 1 ? tiles - 1 : i1 + 1;
  return r;
}

// res = (L11*xa1 + L12*xa)*ya1 + (L21*xa1 + L22*xa)*ya, then cvRound+saturate.
__device__ __forceinline__ int clahe_blend(int l11, int l12, int l21, int l22, const Interp& ix,
                                           const Interp& iy) {
  const float res = ((float)l11 * ix.a1 + (float)l12 * ix.a) * iy.a1 +
                    ((float)l21 * ix.a1 + (float)l22 * ix.a) * iy.a;
  return sat_u8(__float2int_rn(res));
}

// ---------------------------------------------------------------------------
// Kernel B (standalone CLAHEDehaze): per pixel YCrCb, blend of the 4 tile
// LUTs (read through L2), YCrCb->BGR.  One workgroup per 8-row strip.
// ---------------------------------------------------------------------------
constexpr int kApplyRows = 8;

template <int SPACE>
__global__ __launch_bounds__(256) void clahe_apply_kernel(const uint8_t* __restrict__ in,
                                                          uint8_t* __restrict__ out,
                                                          const uint8_t* __restrict__ lut, int H,
                                                          int W, int pitch, ClaheGeo g) {
  const int b = blockIdx.z;
  const uint8_t* fin = in + (size_t)b * H * pitch;
  uint8_t* fout = out + (size_t)b * H * pitch;
  const uint8_t* flut = lut + (size_t)b * g.tiles * g.tiles * 256;
  const int yb = blockIdx.y * kApplyRows;
  const int ye = min(H, yb + kApplyRows);
  for (int y = yb; y < ye; ++y) {
    const Interp iy = interp_axis(y, g.inv_th, g.tiles);
    const uint8_t* r1 = flut + (size_t)iy.i1 * g.tiles * 256;
    const uint8_t* r2 = flut + (size_t)iy.i2 * g.tiles * 256;
    const uint8_t* src = fin + (size_t)y * pitch;
    uint8_t* dst = fout + (size_t)y * pitch;
    for (int x = threadIdx.x; x < W; x += 256) {
      const Interp ix = interp_axis(x, g.inv_tw, g.tiles);
      int Y, Cr, Cb;  // (L, a, b) for SPACE == kLab
      if (SPACE == kLab)
        bgr_to_lab(g_lab, src[3 * x], src[3 * x + 1], src[3 * x + 2], Y, Cr, Cb);
      else
        bgr_to_ycrcb(src[3 * x], src[3 * x + 1], src[3 * x + 2], Y, Cr, Cb);
      const int y2 = clahe_blend(r1[ix.i1 * 256 + Y], r1[ix.i2 * 256 + Y], r2[ix.i1 * 256 + Y],
                                 r2[ix.i2 * 256 + Y], ix, iy);
      int bb, gg, rr;
      if (SPACE == kLab)
        lab_to_bgr(g_lab, y2, Cr, Cb, bb, gg, rr);
      else
        ycrcb_to_bgr(y2, Cr, Cb, bb, gg, rr);
      dst[3 * x] = (uint8_t)bb;
      dst[3 * x + 1] = (uint8_t)gg;
      dst[3 * x + 2] = (uint8_t)rr;
    }
  }
}

// ---------------------------------------------------------------------------
// Median (+ optional fused CLAHE) on an LDS tile with halo.
// Block = 256 threads -> BW x BH = 128 x 16 output pixels; each thread owns
// two horizontal runs of 4 pixels (12 contiguous output bytes each).
// Stage 1: raw rows (+halo, clamped) HBM -> LDS with 16-byte loads.
// Stage 2: (optional CLAHE + colour round trip) raw -> processed tile,
//          replicate-clamped columns.
// Stage 3: median from the processed tile -> HBM.
// ---------------------------------------------------------------------------
constexpr int kBW = 128, kBH = 16;
constexpr int kLutWinMax = 48;  // LUT tiles resident in LDS (12 KB)

template <int K>
struct MedTile {
  static constexpr int R = K / 2;
  static constexpr int TW = kBW + 2 * R;  // halo tile width (px)
  static constexpr int TH = kBH + 2 * R;
  static constexpr int RAWP = ((TW * 3 + 15 + 15) / 16) * 16 + 16;  // raw row stride (bytes)
  static constexpr int PROC = TW * 3;                                // processed row stride
};

__device__ __forceinline__ uint8_t med3u(int a, int b, int c) {
  return (uint8_t)max(min(a, b), min(max(a, b), c));
}

// 3x3: sort each column (lo, mid, hi) once, then
// median = med3(max3(lo), med3(mid), min3(hi))  (exact for 9 samples).
__device__ __forceinline__ void median3_run4(const uint8_t* __restrict__ tile, int stride, int hx,
                                             int hy, uint8_t* __restrict__ o) {
  // columns hx-1 .. hx+4 (tile coords already include the +R halo offset)
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int lo[6], mi[6], hi[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int col = (hx - 1 + j) * 3 + c;
      const int a = tile[(hy - 1) * stride + col];
      const int b = tile[hy * stride + col];
      const int d = tile[(hy + 1) * stride + col];
      lo[j] = min(min(a, b), d);
      hi[j] = max(max(a, b), d);
      mi[j] = max(min(a, b), min(max(a, b), d));
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int l = max(max(lo[p], lo[p + 1]), lo[p + 2]);
      const int m = med3u(mi[p], mi[p + 1], mi[p + 2]);
      const int h = min(min(hi[p], hi[p + 1]), hi[p + 2]);
      o[p * 3 + c] = med3u(l, m, h);
    }
  }
}

// Generic odd K: radix select of rank K*K/2 over the window held in VGPRs.
template <int K>
__device__ __forceinline__ uint8_t median_radix(const uint8_t* __restrict__ tile, int stride,
                                                int hx, int hy, int c) {
  constexpr int N = K * K;
  constexpr int RANK = N / 2;
  int w[N];
#pragma unroll
  for (int dy = 0; dy < K; ++dy)
#pragma unroll
    for (int dx = 0; dx < K; ++dx)
      w[dy * K + dx] = tile[(hy - K / 2 + dy) * stride + (hx - K / 2 + dx) * 3 + c];
  int res = 0;
#pragma unroll
  for (int bit = 7; bit >= 0; --bit) {
    const int cand = res | (1 << bit);
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) cnt += w[i] < cand ? 1 : 0;
    if (cnt <= RANK) res = cand;
  }
  return (uint8_t)res;
}

template <int K, bool CLAHE>
__global__ __launch_bounds__(256) void median_tile_kernel(const uint8_t* __restrict__ in,
                                                          uint8_t* __restrict__ out,
                                                          const uint8_t* __restrict__ lut, int H,
                                                          int W, int pitch, ClaheGeo g) {
  using T = MedTile<K>;
  constexpr int R = T::R;
  __shared__ __attribute__((aligned(16))) uint8_t raw[T::TH * T::RAWP];
  __shared__ __attribute__((aligned(16))) uint8_t proc[T::TH * T::PROC + 16];
  __shared__ __attribute__((aligned(16))) uint8_t lwin[CLAHE ? kLutWinMax * 256 : 16];

  const int tid = threadIdx.x;
  const int b = blockIdx.z;
  const int x0 = blockIdx.x * kBW, y0 = blockIdx.y * kBH;
  const uint8_t* frame = in + (size_t)b * H * pitch;
  const int rowbytes = W * 3;

  // global byte window of the clamped halo columns
  const int gx_lo = max(x0 - R, 0), gx_hi = min(x0 + kBW + R, W);  // [lo, hi)
  const int bx0 = gx_lo * 3, bx1 = gx_hi * 3;
  const int base = bx0 & ~15;
  const int nch = ((bx1 + 15) & ~15) / 16 - base / 16;

  // Stage 1: raw rows -> LDS
  for (int i = tid; i < T::TH * nch; i += 256) {
    const int hr = i / nch;
    const int ch = i - hr * nch;
    const int gy = min(max(y0 - R + hr, 0), H - 1);
    const uint8_t* row = frame + (size_t)gy * pitch;
    const int o = base + ch * 16;
    uint8_t* dst = raw + hr * T::RAWP + ch * 16;
    const uint8_t* src = row + o;
    if (o + 16 <= rowbytes && (((uintptr_t)src) & 15) == 0) {
      *(uint4*)dst = *(const uint4*)src;
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (o + j < rowbytes) dst[j] = src[j];
    }
  }

  // LUT window for the halo region (CLAHE only)
  int wtx0 = 0, wty0 = 0, wtw = 0;
  Interp iy_rows[1];
  (void)iy_rows;
  if constexpr (CLAHE) {
    const uint8_t* flut = lut + (size_t)b * g.tiles * g.tiles * 256;
    const int gy_lo = max(y0 - R, 0), gy_hi = min(y0 + kBH + R, H) - 1;
    wtx0 = interp_axis(gx_lo, g.inv_tw, g.tiles).i1;
    const int wtx1 = interp_axis(gx_hi - 1, g.inv_tw, g.tiles).i2;
    wty0 = interp_axis(gy_lo, g.inv_th, g.tiles).i1;
    const int wty1 = interp_axis(gy_hi, g.inv_th, g.tiles).i2;
    wtw = wtx1 - wtx0 + 1;
    const int wth = wty1 - wty0 + 1;
    // host guarantees wtw*wth <= kLutWinMax
    for (int i = tid; i < wtw * wth * 16; i += 256) {
      const int tt = i >> 4, q = i & 15;
      const int r = tt / wtw, c = tt - r * wtw;
      const uint4* s = (const uint4*)(flut + ((size_t)(wty0 + r) * g.tiles + (wtx0 + c)) * 256);
      ((uint4*)lwin)[i] = s[q];
    }
  }
  __syncthreads();

  // Stage 2: processed tile (clamped columns), optional CLAHE
  for (int i = tid; i < T::TH * T::TW; i += 256) {
    const int hr = i / T::TW;
    const int hc = i - hr * T::TW;
    const int gx = min(max(x0 - R + hc, 0), W - 1);
    const uint8_t* p = raw + hr * T::RAWP + (gx * 3 - base);
    int bb = p[0], gg = p[1], rr = p[2];
    if constexpr (CLAHE) {
      const int gy = min(max(y0 - R + hr, 0), H - 1);
      const Interp ix = interp_axis(gx, g.inv_tw, g.tiles);
      const Interp iy = interp_axis(gy, g.inv_th, g.tiles);
      int Y, Cr, Cb;
      bgr_to_ycrcb(bb, gg, rr, Y, Cr, Cb);
      const uint8_t* l1 = lwin + (iy.i1 - wty0) * wtw * 256;
      const uint8_t* l2 = lwin + (iy.i2 - wty0) * wtw * 256;
      const int c1 = (ix.i1 - wtx0) * 256 + Y, c2 = (ix.i2 - wtx0) * 256 + Y;
      const int y2 = clahe_blend(l1[c1], l1[c2], l2[c1], l2[c2], ix, iy);
      ycrcb_to_bgr(y2, Cr, Cb, bb, gg, rr);
    }
    uint8_t* q = proc + hr * T::PROC + hc * 3;
    q[0] = (uint8_t)bb;
    q[1] = (uint8_t)gg;
    q[2] = (uint8_t)rr;
  }
  __syncthreads();

  // Stage 3: medians, 2 runs of 4 px per thread
  uint8_t* fout = out + (size_t)b * H * pitch;
#pragma unroll
  for (int run = 0; run < 2; ++run) {
    const int idx = tid + run * 256;     // 0..511
    const int ry = idx >> 5;             // 0..15
    const int rx = (idx & 31) * 4;       // 0..124
    const int y = y0 + ry, x = x0 + rx;
    if (y >= H || x >= W) continue;
    uint8_t o[12];
    if constexpr (K == 3) {
      median3_run4(proc, T::PROC, rx + R, ry + R, o);
    } else {
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int c = 0; c < 3; ++c) o[p * 3 + c] = median_radix<K>(proc, T::PROC, rx + p + R, ry + R, c);
    }
    uint8_t* dst = fout + (size_t)y * pitch + (size_t)x * 3;
    const int n = min(4, W - x) * 3;
    if (n == 12 && (((uintptr_t)dst) & 3) == 0) {
      uint32_t w0 = o[0] | (o[1] << 8) | (o[2] << 16) | ((uint32_t)o[3] << 24);
      uint32_t w1 = o[4] | (o[5] << 8) | (o[6] << 16) | ((uint32_t)o[7] << 24);
      uint32_t w2 = o[8] | (o[9] << 8) | (o[10] << 16) | ((uint32_t)o[11] << 24);
      ((uint32_t*)dst)[0] = w0;
      ((uint32_t*)dst)[1] = w1;
      ((uint32_t*)dst)[2] = w2;
    } else {
      for (int j = 0; j < n; ++j) dst[j] = o[j];
    }
  }
}

// ---------------------------------------------------------------------------
// 3x3 fast path: med3_kernel<CLAHE, LB>.
// Block = 256 threads -> 128 x 32 output pixels of one frame.
//  1. the (32+2) x (128+2) halo tile is loaded as 32 four-pixel groups per
//     row (12 bytes, three dword loads) plus the two side pixels, all issued
//     first so their latency overlaps step 2.
//  2. (CLAHE) the block's interpolation cells go to LDS as packed u32
//     entries: cell (cy, cx) = the 4 tile LUTs one pixel blends, so a pixel
//     costs ONE ds_read_b32 for its l11|l12|l21|l22.  The cell area is
//     dynamic LDS sized by the host for the geometry (4 KB at 1080p/8x8).
//  3. the groups are CLAHE'd in registers and stored to LDS as 3 dwords.
//  4. each thread produces a 4 x 4 block of medians (4 px wide, 4 rows):
//     it reads 6 tile rows x 20 bytes with dword loads, sorts every 3-row
//     column once (min3/med3/max3) and combines 3 columns per output:
//     med = med3(max3(lo), med3(mid), min3(hi))  -- exact for 9 samples.
//  5. (LB) the medians overwrite the halo tile in LDS (after a barrier:
//     every thread holds its 6 rows in registers) and the letterbox pixels
//     whose bilinear support lies in this block are produced from them
//     (cv2.resize INTER_LINEAR fixed point, lbgeo.h).  The host only picks
//     LB when every letterbox pixel's support falls inside one block.
// LDS: 14.1 KB tile + cells + 1.3 KB taps, so 5-6 blocks fit a CU.
// ---------------------------------------------------------------------------
constexpr int kM3W = 128, kM3H = 32;
constexpr int kM3TW = kM3W + 8;         // tile bytes cover px x0-4 .. x0+131 (x0-1 .. x0+128 used)
constexpr int kM3TH = kM3H + 2;         // tile rows y0-1 .. y0+32
constexpr int kM3Stride = 416;          // tile row bytes (408 used; median tile 384)
constexpr int kCellMax = 16;            // packed LUT cells per block (<= 16 KB)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Two output channels of ycrcb_to_bgr at once.  lo4/hi4 are the channel
// terms scaled by 4 ((4x) >> 16 == x >> 14, so each term is the high half);
// one v_perm_b32 gathers both, v_pk_add_u16 adds the luma of each half
// (ylo / yhi: only their low 16 bits count)
// (|y + term| < 2^15, so the i16 view is exact) and v_sat_pk_u8_i16
// saturates and packs: bytes {sat(ylo + lo), sat(yhi + hi)} in the low half.
__device__ __forceinline__ uint32_t ycc_pair(int lo4, int hi4, uint32_t ylo, uint32_t yhi) {
  const uint32_t t = __builtin_amdgcn_perm((uint32_t)hi4, (uint32_t)lo4, 0x07060302u);
  const uint32_t y = __builtin_amdgcn_perm(yhi, ylo, 0x05040100u);  // low halves
  const u16x2 s = __builtin_bit_cast(u16x2, t) + __builtin_bit_cast(u16x2, y);
  uint32_t r;
  asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(__builtin_bit_cast(uint32_t, s)));
  return r;
}

// four values < 256 -> one dword (a in byte 0): three v_perm_b32
// (selector byte 0x0c yields zero)
__device__ __forceinline__ uint32_t pack_u8x4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t ab = __builtin_amdgcn_perm(b, a, 0x0c0c0400u);
  const uint32_t cd = __builtin_amdgcn_perm(d, c, 0x0c0c0400u);
  return __builtin_amdgcn_perm(cd, ab, 0x05040100u);
}

// low 16 bits of a, then low 16 bits of b
__device__ __forceinline__ uint32_t pack_lo16(uint32_t a, uint32_t b) {
  return __builtin_amdgcn_perm(b, a, 0x05040100u);
}

// v_med3_u32 (written out: the min/max form gets CSE'd with the column
// min3/max3 and loses the 3-input instructions)
__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

struct LbFuse {
  LbGeo g;
  uint8_t* out;  // B x out_h x out_w x 3
  // every tap of both axes has weight (2048, 0): an exact integer
  // decimation (1080p -> 640 wide: source pixel 3d + 1), where
  // cv2.resize(INTER_LINEAR) returns the source byte itself
  // (lb_vmix(2048 p, ., 2048, 0) = p), so the blend is a copy
  int copy;
};

static bool lb_is_copy(const LbGeo& G, int H, int W) {
  for (int dx = 0; dx < G.new_w; ++dx)
    if (lb_tap_x(dx, G.scale_x, W).w1 != 0) return false;
  for (int dy = 0; dy < G.new_h; ++dy)
    if (lb_tap_y(dy, G.scale_y, H).w1 != 0) return false;
  return true;
}

__device__ __forceinline__ int clahe_cell_index(int p, float inv) {
  return (int)floorf((float)p * inv - 0.5f);
}

// CLAHE_Interpolation_Body, x part: weights {xa1, xa} and the byte offset
// of image column gx's cell column (cells are 256 x u32).
__device__ __forceinline__ void clahe_x(int gx, float inv_tw, int cx0, f32x2& xw, int& xoffb) {
  const float fx = (float)gx * inv_tw - 0.5f;
  const int ix = (int)floorf(fx);
  const float xa = fx - (float)ix;
  xw = f32x2{1.0f - xa, xa};
  xoffb = (ix - cx0) * 1024;
}

// y part for image row y (clamped): weights {ya1, ya} and the cell row.
__device__ __forceinline__ const uint32_t* clahe_row(int y, int H, float inv_th, int cy0, int ncx,
                                                     const uint32_t* cells, f32x2& yw) {
  const int gy = min(max(y, 0), H - 1);
  const float fy = (float)gy * inv_th - 0.5f;
  const int iy = (int)floorf(fy);
  const float ya = fy - (float)iy;
  yw = f32x2{1.0f - ya, ya};
  return cells + (iy - cy0) * ncx * 256;
}

// One pixel: bgr_to_ycrcb, the blended LUT luma y2 (in the low 16 bits of
// y2, see below), and the ycrcb_to_bgr terms x4 for ycc_pair.  `cellx` is
// the cell row plus the pixel's cell column, in bytes.  Cr/Cb are kept as Cr-128 / Cb-128: for arithmetic
// shifts (v + (128 << 14)) >> 14 == (v >> 14) + 128, so the u8 saturation
// becomes one clamp to [-128, 127] (Y itself is always <= 255).
__device__ __forceinline__ void clahe_ycc(int bb, int gg, int rr, const uint8_t* cellx, f32x2 xw,
                                          f32x2 yw, uint32_t& y2, int& tb, int& tg, int& tr) {
  const int Y = bgr_to_y(bb, gg, rr);
  const int dcr = min(max(((rr - Y) * 11682 + 8192) >> 14, -128), 127);
  const int dcb = min(max(((bb - Y) * 9241 + 8192) >> 14, -128), 127);
  const uint32_t q = *(const uint32_t*)(cellx + Y * 4);
  // (l11*xa1 + l12*xa, l21*xa1 + l22*xa) as one packed-f32 pair, then
  // top*ya1 + bottom*ya: the scalar expression's exact op order
  const f32x2 l1 = {(float)(q & 255), (float)((q >> 16) & 255)};
  const f32x2 l2 = {(float)((q >> 8) & 255), (float)(q >> 24)};
  const f32x2 tt = l1 * xw.x + l2 * xw.y;
  const f32x2 tw = tt * yw;
  // a convex blend of u8 LUT entries: cvRound lands in [0, 255], so the
  // saturate_cast is the identity.  cvRound (half-even) by the 1.5 * 2^23
  // addend: the f32 add rounds to an integer, which then sits in the low
  // mantissa bits; only the low 16 bits of y2 are used (ycc_pair).
  y2 = __float_as_uint((tw.x + tw.y) + 12582912.0f);
  tb = dcb * (29049 * 4) + 8192 * 4;
  tg = dcb * (-5636 * 4) + dcr * (-11698 * 4) + 8192 * 4;
  tr = dcr * (22987 * 4) + 8192 * 4;
}

// One 128 x 32 block (b, x0, y0).
template <bool CLAHE, bool LB>
__device__ __forceinline__ void med3_body(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                          const uint8_t* __restrict__ lut, int H, int W, int pitch,
                                          int vec, const ClaheGeo& g, const LbFuse& lb, int b,
                                          int x0, int y0, int tid) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kM3TH * kM3Stride];  // halo, then medians
  extern __shared__ __attribute__((aligned(16))) uint32_t cells[];  // CLAHE cells (host-sized)

  const uint8_t* frame = in + (size_t)b * H * pitch;

  // ---- 1. halo loads.  Thread -> 4-pixel group gc = tid & 31 (px x0+4gc ..
  //      x0+4gc+3) of rows rs, rs+8, rs+16, rs+24 and, in wave 0 only, 32+rs;
  //      the side columns x0-1 and x0+128 are 68 single pixels for threads
  //      64..131.  Every load is issued before any use.  In the tile, group
  //      gc sits at byte 12*(gc+1) and the side pixels at bytes 9 and 396.
  constexpr int kIt = 5;
  const int gc = tid & 31, rs = tid >> 5;
  const int px0 = x0 + gc * 4;
  const bool vrow = vec && px0 + 3 < W;
  uint32_t d[kIt][3];
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int hr = rs + 8 * it;  // < 32 for it < 4; it == 4: wave 0 only
    d[it][0] = d[it][1] = d[it][2] = 0;
    if (hr < kM3TH) {
      const int gy = min(max(y0 - 1 + hr, 0), H - 1);
      const uint8_t* row = frame + (size_t)gy * pitch;
      if (vrow) {
        const uint32_t* p = (const uint32_t*)(row + px0 * 3);
        d[it][0] = RV_MED_LD(p);
        d[it][1] = RV_MED_LD(p + 1);
        d[it][2] = RV_MED_LD(p + 2);
      } else {
        uint8_t v[12];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int gx = min(px0 + j, W - 1);
          v[3 * j] = row[gx * 3];
          v[3 * j + 1] = row[gx * 3 + 1];
          v[3 * j + 2] = row[gx * 3 + 2];
        }
#pragma unroll
        for (int w = 0; w < 3; ++w)
          d[it][w] = v[4 * w] | (v[4 * w + 1] << 8) | (v[4 * w + 2] << 16) |
                     ((uint32_t)v[4 * w + 3] << 24);
      }
    }
  }
  const int sk = tid - 64;  // side pixel: row sk >> 1, right column if sk & 1
  const bool side = sk >= 0 && sk < 2 * kM3TH;
  const int s_hr = sk >> 1, s_px = (sk & 1) ? min(x0 + kM3W, W - 1) : max(x0 - 1, 0);
  int sb = 0, sg = 0, sr = 0;
  if (side) {
    const uint8_t* sp = frame + (size_t)min(max(y0 - 1 + s_hr, 0), H - 1) * pitch + s_px * 3;
    sb = sp[0];
    sg = sp[1];
    sr = sp[2];
  }

  // ---- 2. packed LUT cells of this block: wave w builds cells w, w+4, ..;
  //      lane l gathers Y = 4l..4l+3 of the 4 tile LUTs with one dword load
  //      each and transposes the 4x4 bytes with v_perm_b32.
  int cx0 = 0, cy0 = 0, ncx = 1;
  if constexpr (CLAHE) {
    const int gx_lo = max(x0 - 1, 0), gx_hi = min(x0 + kM3W, W - 1);
    const int gy_lo = max(y0 - 1, 0), gy_hi = min(y0 + kM3H, H - 1);
    cx0 = clahe_cell_index(gx_lo, g.inv_tw);
    cy0 = clahe_cell_index(gy_lo, g.inv_th);
    ncx = clahe_cell_index(gx_hi, g.inv_tw) - cx0 + 1;
    const int ncy = clahe_cell_index(gy_hi, g.inv_th) - cy0 + 1;
    const uint32_t* flut = (const uint32_t*)(lut + (size_t)b * g.tiles * g.tiles * 256);
    const int lane = tid & 63;
    for (int c = tid >> 6; c < ncx * ncy; c += 4) {
      const int cy = c / ncx, cx = c - (c / ncx) * ncx;
      const int iy = cy0 + cy, ix = cx0 + cx;
      const int r1 = max(iy, 0), r2 = min(iy + 1, g.tiles - 1);
      const int c1 = max(ix, 0), c2 = min(ix + 1, g.tiles - 1);
      const uint32_t l11 = flut[(r1 * g.tiles + c1) * 64 + lane];
      const uint32_t l12 = flut[(r1 * g.tiles + c2) * 64 + lane];
      const uint32_t l21 = flut[(r2 * g.tiles + c1) * 64 + lane];
      const uint32_t l22 = flut[(r2 * g.tiles + c2) * 64 + lane];
      const uint32_t p_lo = __builtin_amdgcn_perm(l12, l11, 0x05010400u);  // a0 b0 a1 b1
      const uint32_t p_hi = __builtin_amdgcn_perm(l12, l11, 0x07030602u);  // a2 b2 a3 b3
      const uint32_t q_lo = __builtin_amdgcn_perm(l22, l21, 0x05010400u);
      const uint32_t q_hi = __builtin_amdgcn_perm(l22, l21, 0x07030602u);
      uint4 v;
      v.x = __builtin_amdgcn_perm(q_lo, p_lo, 0x05040100u);
      v.y = __builtin_amdgcn_perm(q_lo, p_lo, 0x07060302u);
      v.z = __builtin_amdgcn_perm(q_hi, p_hi, 0x05040100u);
      v.w = __builtin_amdgcn_perm(q_hi, p_hi, 0x07060302u);
      *(uint4*)(cells + c * 256 + 4 * lane) = v;
    }
  }

  // ---- 3. CLAHE in registers -> LDS
  // per-pixel x interpolation (CLAHE_Interpolation_Body xa/xa1/ind)
  f32x2 xw[4];   // {xa1, xa}
  int xoff[4];   // cell column byte offset
  if constexpr (CLAHE) {
#pragma unroll
    for (int j = 0; j < 4; ++j) clahe_x(min(px0 + j, W - 1), g.inv_tw, cx0, xw[j], xoff[j]);
    __syncthreads();  // cells visible
  }
#pragma unroll
  for (int it = 0; it < kIt; ++it) {
    const int hr = rs + 8 * it;
    if (hr >= kM3TH) break;
    uint32_t* dst = (uint32_t*)(tile + hr * kM3Stride + (gc + 1) * 12);
    if constexpr (CLAHE) {
      f32x2 yw;
      const uint32_t* crow = clahe_row(y0 - 1 + hr, H, g.inv_th, cy0, ncx, cells, yw);
      uint32_t y2[4];
      int tb[4], tg[4], tr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int bb = (d[it][(3 * j) >> 2] >> (8 * ((3 * j) & 3))) & 255;
        const int gg = (d[it][(3 * j + 1) >> 2] >> (8 * ((3 * j + 1) & 3))) & 255;
        const int rr = (d[it][(3 * j + 2) >> 2] >> (8 * ((3 * j + 2) & 3))) & 255;
        clahe_ycc(bb, gg, rr, (const uint8_t*)crow + xoff[j], xw[j], yw, y2[j], tb[j], tg[j], tr[j]);
      }
      // bytes b0 g0 r0 b1 | g1 r1 b2 g2 | r2 b3 g3 r3 as six channel pairs
      dst[0] = pack_lo16(ycc_pair(tb[0], tg[0], y2[0], y2[0]), ycc_pair(tr[0], tb[1], y2[0], y2[1]));
      dst[1] = pack_lo16(ycc_pair(tg[1], tr[1], y2[1], y2[1]), ycc_pair(tb[2], tg[2], y2[2], y2[2]));
      dst[2] = pack_lo16(ycc_pair(tr[2], tb[3], y2[2], y2[3]), ycc_pair(tg[3], tr[3], y2[3], y2[3]));
    } else {
      dst[0] = d[it][0];
      dst[1] = d[it][1];
      dst[2] = d[it][2];
    }
  }
  if (side) {
    uint8_t* dst = tile + s_hr * kM3Stride + ((sk & 1) ? 12 * (kM3W / 4 + 1) : 9);
    if constexpr (CLAHE) {
      f32x2 sxw, yw;
      int sxoff;
      clahe_x(s_px, g.inv_tw, cx0, sxw, sxoff);
      const uint32_t* crow = clahe_row(y0 - 1 + s_hr, H, g.inv_th, cy0, ncx, cells, yw);
      uint32_t y2;
      int tb, tg, tr;
      clahe_ycc(sb, sg, sr, (const uint8_t*)crow + sxoff, sxw, yw, y2, tb, tg, tr);
      const uint32_t bg = ycc_pair(tb, tg, y2, y2), rr = ycc_pair(tr, tr, y2, y2);
      sb = bg & 255;
      sg = (bg >> 8) & 255;
      sr = rr & 255;
    }
    dst[0] = (uint8_t)sb;
    dst[1] = (uint8_t)sg;
    dst[2] = (uint8_t)sr;
  }
  __syncthreads();

  // ---- 4. medians: thread -> 4 px (rx..rx+3) x 4 rows (ry..ry+3)
  const int rx = (tid & 31) * 4, ry = (tid >> 5) * 4;
  uint32_t rw[6][5];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const uint32_t* p = (const uint32_t*)(tile + (ry + r) * kM3Stride + rx * 3 + 8);
#pragma unroll
    for (int j = 0; j < 5; ++j) rw[r][j] = p[j];
  }
  if constexpr (LB) __syncthreads();  // the halo tile is in registers: reuse it for medians
  // byte (column jj in 0..5 = px rx-1+jj, channel c) of row r sits at window
  // byte 1 + 3*jj + c
#define RV_B(r, k) ((rw[r][(k) >> 2] >> (8 * ((k) & 3))) & 255u)
  const int x = x0 + rx;
  // row pointer stepped by pitch (no per-row 64-bit multiply)
  uint8_t* orow = out + ((size_t)b * H + y0 + ry) * pitch + (size_t)x * 3;
#pragma unroll
  for (int o = 0; o < 4; ++o, orow += pitch) {
    const int y = y0 + ry + o;
    uint32_t v12[12];  // medians, byte order b0 g0 r0 b1 ...
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      uint32_t lo[6], mi[6], hi[6];
#pragma unroll
      for (int jj = 0; jj < 6; ++jj) {
        const uint32_t a = RV_B(o, 1 + 3 * jj + c), bq = RV_B(o + 1, 1 + 3 * jj + c),
                       e = RV_B(o + 2, 1 + 3 * jj + c);
        lo[jj] = min(min(a, bq), e);
        hi[jj] = max(max(a, bq), e);
        mi[jj] = med3_u32(a, bq, e);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint32_t l = max(max(lo[p], lo[p + 1]), lo[p + 2]);
        const uint32_t m = med3_u32(mi[p], mi[p + 1], mi[p + 2]);
        const uint32_t h = min(min(hi[p], hi[p + 1]), hi[p + 2]);
        v12[3 * p + c] = med3_u32(l, m, h);
      }
    }
    uint32_t res[3];
#pragma unroll
    for (int w = 0; w < 3; ++w) res[w] = pack_u8x4(v12[4 * w], v12[4 * w + 1], v12[4 * w + 2], v12[4 * w + 3]);
    if constexpr (LB) {
      uint32_t* od = (uint32_t*)(tile + (ry + o) * kM3Stride + rx * 3);
      od[0] = res[0];
      od[1] = res[1];
      od[2] = res[2];
    }
    if (y < H && x < W) {
      uint8_t* dst = orow;
      if (vec && x + 3 < W) {
        RV_MED_ST((uint32_t*)dst, res[0]);
        RV_MED_ST((uint32_t*)dst + 1, res[1]);
        RV_MED_ST((uint32_t*)dst + 2, res[2]);
      } else {
        const int n = min(4, W - x) * 3;
        for (int j = 0; j < n; ++j) dst[j] = (uint8_t)(res[j >> 2] >> (8 * (j & 3)));
      }
    }
  }
#undef RV_B

  // ---- 5. letterbox pixels owned by this block: per-axis taps once into
  //      LDS, then 2-D from the median tile
  if constexpr (LB) {
    __shared__ LbTap tapx[kM3W + 8], tapy[kM3H + 8];
    __shared__ int ntap[2], dlo[2];
    const LbGeo& G = lb.g;
    if (tid < 2) {
      const double inv = tid == 0 ? 1.0 / G.scale_x : 1.0 / G.scale_y;
      const int o0 = tid == 0 ? x0 : y0, span = tid == 0 ? kM3W : kM3H;
      const int nmax = tid == 0 ? G.new_w : G.new_h;
      const int lo = max(0, (int)floor((o0 + 0.5) * inv - 0.5) - 2);
      const int hi = min(nmax - 1, (int)ceil((o0 + span - 0.5) * inv - 0.5) + 2);
      dlo[tid] = lo;
      ntap[tid] = max(0, min(hi - lo + 1, span + 8));
    }
    __syncthreads();  // also: the median tile is complete
    const int nx = ntap[0], ny = ntap[1];
    if (tid < nx) tapx[tid] = lb_tap_x(dlo[0] + tid, G.scale_x, W);
    else if (tid >= 192 && tid - 192 < ny) tapy[tid - 192] = lb_tap_y(dlo[1] + tid - 192, G.scale_y, H);
    __syncthreads();
    // lane -> letterbox column jx, wave -> rows jy = w, w+4, ..: the row's
    // ownership test is wave-uniform, the tap tables are read once per lane
    const size_t orow = (size_t)G.out_w * 3;
    uint8_t* lbo = lb.out + ((size_t)b * G.out_h + G.top + dlo[1]) * orow +
                   (size_t)(G.left + dlo[0]) * 3;
    for (int jx = tid & 63; jx < nx; jx += 64) {
      const LbTap tx = tapx[jx];
      // owner: the block holding the first tap (host checked: all taps)
      const bool own_x = tx.s0 >= x0 && tx.s0 < x0 + kM3W;
      const int c0 = (tx.s0 - x0) * 3, c1 = (tx.s1 - x0) * 3;
      for (int jy = tid >> 6; jy < ny; jy += 4) {
        const LbTap ty = tapy[jy];
        if (ty.s0 < y0 || ty.s0 >= y0 + kM3H || !own_x) continue;
        const uint8_t* r0 = tile + (ty.s0 - y0) * kM3Stride;
        const uint8_t* r1 = tile + (ty.s1 - y0) * kM3Stride;
        uint8_t* dst = lbo + jy * orow + jx * 3;
        if (lb.copy) {
          dst[0] = r0[c0];
          dst[1] = r0[c0 + 1];
          dst[2] = r0[c0 + 2];
          continue;
        }
        // lb_vmix with 24-bit multiplies (u8 x 11-bit weights, (d >> 4) <
        // 2^15): the full-rate v_mul_u32_u24 instead of v_mul_lo_u32
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const uint32_t d0 = __umul24(r0[c0 + c], tx.w0) + __umul24(r0[c1 + c], tx.w1);
          const uint32_t d1 = __umul24(r1[c0 + c], tx.w0) + __umul24(r1[c1 + c], tx.w1);
          dst[c] = (uint8_t)(((__umul24(ty.w0, d0 >> 4) >> 16) + (__umul24(ty.w1, d1 >> 4) >> 16) + 2) >> 2);
        }
      }
    }
  }
}

template <bool CLAHE, bool LB>
__global__ __launch_bounds__(256) void med3_kernel(const uint8_t* __restrict__ in,
                                                   uint8_t* __restrict__ out,
                                                   const uint8_t* __restrict__ lut, int H, int W,
                                                   int pitch, int vec, ClaheGeo g, LbFuse lb) {
  // XCD-aware tile order: workgroups go round-robin to the 8 XCDs, so
  // dispatch slot L runs on XCD L % 8; give each XCD one contiguous run of
  // tiles (row-major within a frame) so the halo rows and the 12-byte side
  // halos shared by neighbouring tiles hit that XCD's L2.
  const int ntx = (W + kM3W - 1) / kM3W, nty = (H + kM3H - 1) / kM3H;
  const int n = gridDim.x, L = blockIdx.x;
  const int q = n >> 3, r = n & 7, xcd = L & 7, slot = L >> 3;
  const int t = xcd < r ? xcd * (q + 1) + slot : r * (q + 1) + (xcd - r) * q + slot;
  const int b = t / (ntx * nty);
  const int f = t - b * (ntx * nty);
  med3_body<CLAHE, LB>(in, out, lut, H, W, pitch, vec, g, lb, b,
                              (f - (f / ntx) * ntx) * kM3W, (f / ntx) * kM3H, threadIdx.x);
}

static size_t lut_bytes(int B, int tiles) { return (size_t)B * tiles * tiles * 256; }

// Host checks for med3_kernel.
// Upper bound of ncx * ncy in the kernel: distinct floor(p/t - 0.5) over a
// span of n consecutive p <= ceil(n/t) + 1 (+1 more for float rounding of
// p * inv), and at most tiles + 1 values (-1 .. tiles-1).
static int med3_cells(const ClaheGeo& g) {
  const int ncx = min((kM3TW + g.tw - 1) / g.tw + 2, g.tiles + 1);
  const int ncy = min((kM3TH + g.th - 1) / g.th + 2, g.tiles + 1);
  return ncx * ncy;
}

static bool med3_cells_fit(const ClaheGeo& g, int H, int W) {
  (void)H;
  (void)W;
  return med3_cells(g) <= kCellMax;
}

// every letterbox pixel's nonzero taps must lie in the block of its first tap
static bool med3_lb_fits(const LbGeo& G, int H, int W) {
  // downscale / identity only: a block then owns <= 128 + 5 columns and
  // <= 32 + 5 rows of letterbox pixels (the LDS tap tables)
  if (G.new_w > W || G.new_h > H) return false;
  for (int dx = 0; dx < G.new_w; ++dx) {
    const LbTap t = lb_tap_x(dx, G.scale_x, W);
    if (t.s0 / kM3W != t.s1 / kM3W) return false;
  }
  for (int dy = 0; dy < G.new_h; ++dy) {
    const LbTap t = lb_tap_y(dy, G.scale_y, H);
    if (t.s0 / kM3H != t.s1 / kM3H) return false;
  }
  return true;
}

template <bool CLAHE, bool LB>
static void launch_med3(const uint8_t* in, uint8_t* out, const uint8_t* lut, int B, int H, int W,
                        int pitch, const ClaheGeo& g, const LbFuse& lb, hipStream_t s) {
  const int vec = (pitch % 4 == 0) && (((uintptr_t)in) % 4 == 0) && (((uintptr_t)out) % 4 == 0);
  const dim3 grid(ceil_div(W, kM3W) * ceil_div(H, kM3H) * B);  // tiles, mapped in the kernel
  const size_t cell_bytes = CLAHE ? (size_t)med3_cells(g) * 1024 : 0;
  med3_kernel<CLAHE, LB><<<grid, 256, cell_bytes, s>>>(in, out, lut, H, W, pitch, vec, g, lb);
}

// Gray span for the low-contrast gate (pipeline.py:24-30).
__global__ __launch_bounds__(256) void gray_span_kernel(const uint8_t* __restrict__ in, int H,
                                                        int W, int pitch, int* __restrict__ mn_mx) {
  const int b = blockIdx.y;
  const uint8_t* frame = in + (size_t)b * H * pitch;
  int mn = 255, mx = 0;
  const int total = H * W;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int y = i / W, x = i - (i / W) * W;
    const uint8_t* p = frame + (size_t)y * pitch + (size_t)x * 3;
    const int v = bgr_to_y(p[0], p[1], p[2]);
    mn = min(mn, v);
    mx = max(mx, v);
  }
  for (int off = 32; off > 0; off >>= 1) {
    mn = min(mn, __shfl_xor(mn, off));
    mx = max(mx, __shfl_xor(mx, off));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mn_mx[2 * b], mn);
    atomicMax(&mn_mx[2 * b + 1], mx);
  }
}
__global__ void gray_span_init(int* mn_mx, int B) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) {
    mn_mx[2 * i] = 255;
    mn_mx[2 * i + 1] = 0;
  }
}
__global__ void gray_span_finish(const int* mn_mx, int* span, int B) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) span[i] = mn_mx[2 * i + 1] - mn_mx[2 * i];
}

static bool lut_window_fits(const ClaheGeo& g, int K) {
  const int R = K / 2;
  // worst-case tile columns/rows touched by one (kBW+2R) x (kBH+2R) halo tile
  const int cols = (kBW + 2 * R - 1) / g.tw + 3;
  const int rows = (kBH + 2 * R - 1) / g.th + 3;
  return min(cols, g.tiles) * min(rows, g.tiles) <= kLutWinMax;
}

template <int K, bool CLAHE>
static void launch_median(const uint8_t* in, uint8_t* out, const uint8_t* lut, int B, int H,
                          int W, int pitch, const ClaheGeo& g, hipStream_t s) {
  dim3 grid(ceil_div(W, kBW), ceil_div(H, kBH), B);
  median_tile_kernel<K, CLAHE><<<grid, 256, 0, s>>>(in, out, lut, H, W, pitch, g);
}

template <bool CLAHE>
static void dispatch_median(int k, const uint8_t* in, uint8_t* out, const uint8_t* lut, int B,
                            int H, int W, int pitch, const ClaheGeo& g, hipStream_t s) {
  switch (k) {
    case 3: launch_median<3, CLAHE>(in, out, lut, B, H, W, pitch, g, s); break;
    case 5: launch_median<5, CLAHE>(in, out, lut, B, H, W, pitch, g, s); break;
    case 7: launch_median<7, CLAHE>(in, out, lut, B, H, W, pitch, g, s); break;
    default: launch_median<9, CLAHE>(in, out, lut, B, H, W, pitch, g, s); break;
  }
}

}  // namespace rv

using namespace rv;

static int check_frames(const uint8_t* in, const void* out, int B, int H, int W, int pitch) {
  RV_CHECK_ARG(in != nullptr && out != nullptr, "null frame pointer");
  RV_CHECK_ARG(B >= 0 && H > 0 && W > 0, "bad frame shape B=%d H=%d W=%d", B, H, W);
  RV_CHECK_ARG(pitch >= 3 * W, "pitch %d < 3*W", pitch);
  RV_CHECK_ARG((const void*)in != out, "in and out must not alias");
  return RV_OK;
}

// B x tiles^2 LUTs of 256 bytes
extern "C" size_t rv_clahe_ws_bytes(int B, int tiles) {
  if (B <= 0 || tiles <= 0) return 0;
  return lut_bytes(B, tiles);
}

extern "C" int rv_clahe_ycrcb_u8(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                                 int tiles, double clip, void* ws, size_t ws_bytes, void* stream) {
  int st = check_frames(in, out, B, H, W, pitch);
  if (st) return st;
  RV_CHECK_ARG(tiles >= 1 && tiles <= 64, "tiles %d out of range", tiles);
  RV_CHECK_ARG(ws != nullptr && ws_bytes >= rv_clahe_ws_bytes(B, tiles), "workspace too small");
  if (B == 0) return RV_OK;
  ClaheGeo g = make_geo(H, W, tiles, clip);
  hipStream_t s = as_stream(stream);
  uint8_t* lut = (uint8_t*)ws;
  launch_clahe_lut<kYCrCb>(in, lut, B, H, W, pitch, g, s);
  clahe_apply_kernel<kYCrCb><<<dim3(1, ceil_div(H, kApplyRows), B), 256, 0, s>>>(in, out, lut, H, W,
                                                                          pitch, g);
  return launch_status("rv_clahe_ycrcb_u8");
}

extern "C" int rv_median_u8c3(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                              int k, void* stream) {
  int st = check_frames(in, out, B, H, W, pitch);
  if (st) return st;
  RV_CHECK_ARG(k == 3 || k == 5 || k == 7 || k == 9, "median k=%d must be 3,5,7,9", k);
  if (B == 0) return RV_OK;
  ClaheGeo g{};
  if (k == 3)
    launch_med3<false, false>(in, out, nullptr, B, H, W, pitch, g, LbFuse{}, as_stream(stream));
  else
    dispatch_median<false>(k, in, out, nullptr, B, H, W, pitch, g, as_stream(stream));
  return launch_status("rv_median_u8c3");
}

static LabTables g_lab_host;
static std::once_flag g_lab_built;
static std::mutex g_lab_mu;
static uint64_t g_lab_devices = 0;  // bit d: tables uploaded to device d

// Upload the Lab tables to the current device once (per device: a process
// may drive several GPUs).  Synchronous; call rv_lab_init() before capture.
static int ensure_lab_tables() {
  std::call_once(g_lab_built, [] { build_lab_tables(g_lab_host); });
  int dev = 0;
  int st = hip_check(hipGetDevice(&dev), "hipGetDevice");
  if (st) return st;
  RV_CHECK_ARG(dev >= 0 && dev < 64, "device %d out of range", dev);
  std::lock_guard<std::mutex> lock(g_lab_mu);
  if (g_lab_devices >> dev & 1) return RV_OK;
  st = hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_lab), &g_lab_host, sizeof(LabTables)),
                 "Lab table upload");
  if (!st) g_lab_devices |= 1ull << dev;
  return st;
}

extern "C" int rv_lab_init(void) { return ensure_lab_tables(); }

extern "C" int rv_lab_tables_host(void* out, size_t bytes) {
  RV_CHECK_ARG(out != nullptr && bytes == sizeof(LabTables), "need %zu bytes",
               sizeof(LabTables));
  LabTables t;
  build_lab_tables(t);
  memcpy(out, &t, sizeof(t));
  return RV_OK;
}

extern "C" int rv_clahe_lab_u8(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                               int tiles, double clip, void* ws, size_t ws_bytes, void* stream) {
  int st = check_frames(in, out, B, H, W, pitch);
  if (st) return st;
  RV_CHECK_ARG(tiles >= 1 && tiles <= 64, "tiles %d out of range", tiles);
  RV_CHECK_ARG(ws != nullptr && ws_bytes >= rv_clahe_ws_bytes(B, tiles), "workspace too small");
  st = ensure_lab_tables();
  if (st) return st;
  if (B == 0) return RV_OK;
  ClaheGeo g = make_geo(H, W, tiles, clip);
  hipStream_t s = as_stream(stream);
  uint8_t* lut = (uint8_t*)ws;
  launch_clahe_lut<kLab>(in, lut, B, H, W, pitch, g, s);
  clahe_apply_kernel<kLab><<<dim3(1, ceil_div(H, kApplyRows), B), 256, 0, s>>>(in, out, lut, H,
                                                                              W, pitch, g);
  return launch_status("rv_clahe_lab_u8");
}

extern "C" int rv_clahe_median_u8(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                                  int tiles, double clip, int k, void* ws, size_t ws_bytes,
                                  void* stream) {
  int st = check_frames(in, out, B, H, W, pitch);
  if (st) return st;
  RV_CHECK_ARG(tiles >= 1 && tiles <= 64, "tiles %d out of range", tiles);
  RV_CHECK_ARG(k == 3 || k == 5 || k == 7 || k == 9, "median k=%d must be 3,5,7,9", k);
  RV_CHECK_ARG(ws != nullptr && ws_bytes >= rv_clahe_ws_bytes(B, tiles), "workspace too small");
  if (B == 0) return RV_OK;
  ClaheGeo g = make_geo(H, W, tiles, clip);
  hipStream_t s = as_stream(stream);
  uint8_t* lut = (uint8_t*)ws;
  if (k == 3 && med3_cells_fit(g, H, W)) {
    launch_clahe_lut<kYCrCb>(in, lut, B, H, W, pitch, g, s);
    launch_med3<true, false>(in, out, lut, B, H, W, pitch, g, LbFuse{}, s);
    return launch_status("rv_clahe_median_u8");
  }
  RV_CHECK_ARG(lut_window_fits(g, k),
               "LUT window too large for the fused pass (tiles=%d, tile %dx%d); "
               "use rv_clahe_ycrcb_u8 + rv_median_u8c3",
               tiles, g.tw, g.th);
  launch_clahe_lut<kYCrCb>(in, lut, B, H, W, pitch, g, s);
  dispatch_median<true>(k, in, out, lut, B, H, W, pitch, g, s);
  return launch_status("rv_clahe_median_u8");
}

extern "C" int rv_clahe_median_fits(int H, int W, int tiles, int k) {
  if (H <= 0 || W <= 0 || tiles < 1 || tiles > 64) return 0;
  const ClaheGeo g = make_geo(H, W, tiles, 0.0);
  if (k == 3 && med3_cells_fit(g, H, W)) return 1;
  return lut_window_fits(g, k) ? 1 : 0;
}

extern "C" int rv_clahe_median_letterbox_fits(int H, int W, int tiles, int k, const int* geo) {
  if (H <= 0 || W <= 0 || tiles < 1 || tiles > 64 || k != 3 || geo == nullptr) return 0;
  LbGeo G;
  if (!lbgeo_from(geo, H, W, G)) return 0;
  return med3_cells_fit(make_geo(H, W, tiles, 0.0), H, W) && med3_lb_fits(G, H, W) ? 1 : 0;
}

extern "C" int rv_clahe_median_letterbox_u8(const uint8_t* in, uint8_t* out, int B, int H, int W,
                                            int pitch, int tiles, double clip, int k, void* ws,
                                            size_t ws_bytes, uint8_t* lb_out, const int* geo,
                                            void* stream) {
  int st = check_frames(in, out, B, H, W, pitch);
  if (st) return st;
  RV_CHECK_ARG(tiles >= 1 && tiles <= 64, "tiles %d out of range", tiles);
  RV_CHECK_ARG(ws != nullptr && ws_bytes >= rv_clahe_ws_bytes(B, tiles), "workspace too small");
  RV_CHECK_ARG(lb_out != nullptr && geo != nullptr, "null letterbox pointer");
  RV_CHECK_ARG(rv_clahe_median_letterbox_fits(H, W, tiles, k, geo),
               "geometry not supported by the fused pass (k=%d, %dx%d, tiles=%d); use "
               "rv_clahe_median_u8 + rv_letterbox_u8", k, W, H, tiles);
  if (B == 0) return RV_OK;
  ClaheGeo g = make_geo(H, W, tiles, clip);
  LbFuse lb;
  lbgeo_from(geo, H, W, lb.g);
  lb.out = lb_out;
  lb.copy = lb_is_copy(lb.g, H, W) ? 1 : 0;
  hipStream_t s = as_stream(stream);
  uint8_t* lut = (uint8_t*)ws;
  st = launch_letterbox_pad(lb_out, B, lb.g, s);
  if (st) return st;
  launch_clahe_lut<kYCrCb>(in, lut, B, H, W, pitch, g, s);
  launch_med3<true, true>(in, out, lut, B, H, W, pitch, g, lb, s);
  return launch_status("rv_clahe_median_letterbox_u8");
}

extern "C" int rv_gray_span_u8(const uint8_t* in, int B, int H, int W, int pitch, int* ws,
                               int* span_out, void* stream) {
  RV_CHECK_ARG(in != nullptr && ws != nullptr && span_out != nullptr, "null pointer");
  RV_CHECK_ARG(B >= 0 && H > 0 && W > 0 && pitch >= 3 * W, "bad frame shape");
  if (B == 0) return RV_OK;
  hipStream_t s = as_stream(stream);
  gray_span_init<<<ceil_div(B, 256), 256, 0, s>>>(ws, B);
  const int blocks = min(256, ceil_div(H * W, 256));
  gray_span_kernel<<<dim3(blocks, B), 256, 0, s>>>(in, H, W, pitch, ws);
  gray_span_finish<<<ceil_div(B, 256), 256, 0, s>>>(ws, span_out, B);
  return launch_status("rv_gray_span_u8");
}
