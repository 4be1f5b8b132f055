/*
 * rv_oracle.c — CPU restatement of the reference hot path, used ONLY as the
 * parity checker (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * It is never linked into, loaded by, or called from the product path.
 *
 * Provenance.  The reference (YJxyzxyz/road-vision-system) delegates this
 * arithmetic to third-party libraries that are absent from this container
 * and unpinned by the reference (requirements.txt:1-9):
 *   - OpenCV (opencv-python, ~4.10-4.12 by snapshot date): cvtColor
 *     BGR<->YCrCb 8U (color_yuv: RGB2YCrCb_i / YCrCb2RGB_i, yuv_shift 14),
 *     CLAHE 8UC1 (imgproc/src/clahe.cpp: CLAHE_CalcLut_Body,
 *     CLAHE_Interpolation_Body), medianBlur 8UC3 (BORDER_REPLICATE),
 *     resize INTER_LINEAR 8U (resizeGeneric_ + VResizeLinear<uchar>).
 *     Call sites: src/preprocess/ops/clahe_dehaze.py:19-30,
 *     src/preprocess/ops/median_derain.py:14.
 *   - Ultralytics (~8.3.x) LetterBox / non_max_suppression / scale_boxes and
 *     torchvision.ops.nms (CPU kernel: stable descending sort, greedy
 *     suppression with `ovr > iou_threshold` in double).  Call site:
 *     src/detect/yolo_ultralytics.py:28-35.
 * These functions restate the published scalar algorithms; parity against
 * the real libraries is UNPINNED in this container (none is installed).
 * The SORT association helpers restate src/track/sort_tracker.py:55-80 and
 * :182-210 and are pinned against vectors produced by the reference code
 * itself (tests/golden/make_golden.py).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp; SSE2 scalar
 * floats, no excess precision, no FMA contraction).  The per-pixel loops are
 * OpenMP-parallel over independent rows / tiles (OMP_NUM_THREADS), as
 * OpenCV's parallel_for_ is, so the CPU baseline uses the host's cores; the
 * results do not depend on the thread count.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int sat_u8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

static int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
  }
  return p;
}

/* cvtColor COLOR_BGR2YCrCb, 8U */
void oracle_bgr2ycrcb(const uint8_t* in, uint8_t* out, int n) {
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    int b = in[3 * i], g = in[3 * i + 1], r = in[3 * i + 2];
    int Y = (b * 1868 + g * 9617 + r * 4899 + 8192) >> 14;
    int Cr = ((r - Y) * 11682 + (128 << 14) + 8192) >> 14;
    int Cb = ((b - Y) * 9241 + (128 << 14) + 8192) >> 14;
    out[3 * i] = (uint8_t)sat_u8(Y);
    out[3 * i + 1] = (uint8_t)sat_u8(Cr);
    out[3 * i + 2] = (uint8_t)sat_u8(Cb);
  }
}

/* cvtColor COLOR_YCrCb2BGR, 8U */
void oracle_ycrcb2bgr(const uint8_t* in, uint8_t* out, int n) {
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    int Y = in[3 * i], Cr = in[3 * i + 1], Cb = in[3 * i + 2];
    int b = Y + (((Cb - 128) * 29049 + 8192) >> 14);
    int g = Y + (((Cb - 128) * -5636 + (Cr - 128) * -11698 + 8192) >> 14);
    int r = Y + (((Cr - 128) * 22987 + 8192) >> 14);
    out[3 * i] = (uint8_t)sat_u8(b);
    out[3 * i + 1] = (uint8_t)sat_u8(g);
    out[3 * i + 2] = (uint8_t)sat_u8(r);
  }
}

/* cv::CLAHE::apply on one 8UC1 plane (src pitch = W). */
void oracle_clahe_u8c1(const uint8_t* src, uint8_t* dst, int H, int W, int tiles, double clip) {
  int tw, th;
  if (W % tiles == 0 && H % tiles == 0) {
    tw = W / tiles;
    th = H / tiles;
  } else {
    tw = (W + tiles - (W % tiles)) / tiles;
    th = (H + tiles - (H % tiles)) / tiles;
  }
  const int area = tw * th;
  const float lut_scale = (float)255 / area;
  int clip_limit = 0;
  if (clip > 0.0) {
    clip_limit = (int)(clip * area / 256);
    if (clip_limit < 1) clip_limit = 1;
  }
  uint8_t* lut = (uint8_t*)malloc((size_t)tiles * tiles * 256);
#pragma omp parallel for collapse(2) schedule(static)
  for (int ty = 0; ty < tiles; ++ty)
    for (int tx = 0; tx < tiles; ++tx) {
      int hist[256];
      memset(hist, 0, sizeof(hist));
      for (int r = 0; r < th; ++r) {
        int sy = ty * th + r;
        if (sy >= H) sy = reflect101(sy, H);
        for (int c = 0; c < tw; ++c) {
          int sx = tx * tw + c;
          if (sx >= W) sx = reflect101(sx, W);
          hist[src[(size_t)sy * W + sx]]++;
        }
      }
      if (clip_limit > 0) {
        int clipped = 0;
        for (int i = 0; i < 256; ++i)
          if (hist[i] > clip_limit) {
            clipped += hist[i] - clip_limit;
            hist[i] = clip_limit;
          }
        int batch = clipped / 256;
        int residual = clipped - batch * 256;
        for (int i = 0; i < 256; ++i) hist[i] += batch;
        if (residual != 0) {
          int step = 256 / residual;
          if (step < 1) step = 1;
          for (int i = 0; i < 256 && residual > 0; i += step, residual--) hist[i]++;
        }
      }
      int sum = 0;
      uint8_t* l = lut + ((size_t)ty * tiles + tx) * 256;
      for (int i = 0; i < 256; ++i) {
        sum += hist[i];
        l[i] = (uint8_t)sat_u8((int)lrintf((float)sum * lut_scale));
      }
    }
  const float inv_tw = 1.0f / tw, inv_th = 1.0f / th;
#pragma omp parallel for schedule(static)
  for (int y = 0; y < H; ++y) {
    float tyf = y * inv_th - 0.5f;
    int ty1 = (int)floorf(tyf);
    int ty2 = ty1 + 1;
    float ya = tyf - ty1, ya1 = 1.0f - ya;
    ty1 = ty1 < 0 ? 0 : ty1;
    ty2 = ty2 > tiles - 1 ? tiles - 1 : ty2;
    const uint8_t* p1 = lut + (size_t)ty1 * tiles * 256;
    const uint8_t* p2 = lut + (size_t)ty2 * tiles * 256;
    for (int x = 0; x < W; ++x) {
      float txf = x * inv_tw - 0.5f;
      int tx1 = (int)floorf(txf);
      int tx2 = tx1 + 1;
      float xa = txf - tx1, xa1 = 1.0f - xa;
      tx1 = tx1 < 0 ? 0 : tx1;
      tx2 = tx2 > tiles - 1 ? tiles - 1 : tx2;
      int v = src[(size_t)y * W + x];
      int i1 = tx1 * 256 + v, i2 = tx2 * 256 + v;
      float res = (p1[i1] * xa1 + p1[i2] * xa) * ya1 + (p2[i1] * xa1 + p2[i2] * xa) * ya;
      dst[(size_t)y * W + x] = (uint8_t)sat_u8((int)lrintf(res));
    }
  }
  free(lut);
}

/* CLAHEDehaze YCrCb path on one BGR frame (pitch = 3W). */
void oracle_clahe_ycrcb(const uint8_t* in, uint8_t* out, int H, int W, int tiles, double clip) {
  size_t n = (size_t)H * W;
  uint8_t* ycc = (uint8_t*)malloc(n * 3);
  uint8_t* y = (uint8_t*)malloc(n);
  uint8_t* y2 = (uint8_t*)malloc(n);
  oracle_bgr2ycrcb(in, ycc, (int)n);
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)n; ++i) y[i] = ycc[3 * i];
  oracle_clahe_u8c1(y, y2, H, W, tiles, clip);
#pragma omp parallel for schedule(static)
  for (long i = 0; i < (long)n; ++i) ycc[3 * i] = y2[i];
  oracle_ycrcb2bgr(ycc, out, (int)n);
  free(ycc);
  free(y);
  free(y2);
}

/* cv::medianBlur 8UC3, odd k, BORDER_REPLICATE (exact median: partial
 * insertion sort of the k*k window). */
static int min2(int a, int b) { return a < b ? a : b; }
static int max2(int a, int b) { return a > b ? a : b; }
static int med3(int a, int b, int c) { return max2(min2(a, b), min2(max2(a, b), c)); }

/* k = 3 fast path: sort each column of 3, median = med3(max(lo), med(mid), min(hi)). */
static void median3(const uint8_t* in, uint8_t* out, int H, int W) {
#pragma omp parallel for schedule(static)
  for (int y = 0; y < H; ++y) {
    const uint8_t* r0 = in + (size_t)clampi(y - 1, 0, H - 1) * W * 3;
    const uint8_t* r1 = in + (size_t)y * W * 3;
    const uint8_t* r2 = in + (size_t)clampi(y + 1, 0, H - 1) * W * 3;
    for (int x = 0; x < W; ++x)
      for (int c = 0; c < 3; ++c) {
        int lo[3], mi[3], hi[3];
        for (int j = 0; j < 3; ++j) {
          const int xx = clampi(x - 1 + j, 0, W - 1) * 3 + c;
          const int a = r0[xx], b = r1[xx], d = r2[xx];
          lo[j] = min2(min2(a, b), d);
          hi[j] = max2(max2(a, b), d);
          mi[j] = med3(a, b, d);
        }
        out[((size_t)y * W + x) * 3 + c] = (uint8_t)med3(max2(max2(lo[0], lo[1]), lo[2]),
                                                         med3(mi[0], mi[1], mi[2]),
                                                         min2(min2(hi[0], hi[1]), hi[2]));
      }
  }
}

void oracle_median_u8c3(const uint8_t* in, uint8_t* out, int H, int W, int k) {
  if (k == 3) {
    median3(in, out, H, W);
    return;
  }
  const int r = k / 2, n = k * k, rank = n / 2;
#pragma omp parallel for schedule(static)
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x)
      for (int c = 0; c < 3; ++c) {
        int w[81];
        int m = 0;
        for (int dy = -r; dy <= r; ++dy) {
          int sy = clampi(y + dy, 0, H - 1);
          for (int dx = -r; dx <= r; ++dx) {
            int sx = clampi(x + dx, 0, W - 1);
            int v = in[((size_t)sy * W + sx) * 3 + c];
            int j = m++;
            while (j > 0 && w[j - 1] > v) {
              w[j] = w[j - 1];
              --j;
            }
            w[j] = v;
          }
        }
        out[((size_t)y * W + x) * 3 + c] = (uint8_t)w[rank];
      }
}

/* Ultralytics LetterBox(imgsz, auto=True, stride) geometry. */
void oracle_letterbox_geometry(int H, int W, int imgsz, int stride, int* geo) {
  double r = fmin((double)imgsz / H, (double)imgsz / W);
  int new_w = (int)nearbyint(W * r), new_h = (int)nearbyint(H * r);
  double dw = (double)(((imgsz - new_w) % stride + stride) % stride);
  double dh = (double)(((imgsz - new_h) % stride + stride) % stride);
  dw /= 2.0;
  dh /= 2.0;
  int top = (int)nearbyint(dh - 0.1), bottom = (int)nearbyint(dh + 0.1);
  int left = (int)nearbyint(dw - 0.1), right = (int)nearbyint(dw + 0.1);
  geo[0] = new_h + top + bottom;
  geo[1] = new_w + left + right;
  geo[2] = new_h;
  geo[3] = new_w;
  geo[4] = top;
  geo[5] = left;
}

static int round_short(float v) {
  int r = (int)lrintf(v);
  return r < -32768 ? -32768 : (r > 32767 ? 32767 : r);
}

/* cv2.resize(INTER_LINEAR) 8UC3 + copyMakeBorder(114), one frame. */
void oracle_letterbox(const uint8_t* in, uint8_t* out, int H, int W, const int* geo) {
  int out_h = geo[0], out_w = geo[1], new_h = geo[2], new_w = geo[3], top = geo[4], left = geo[5];
  double scale_x = 1.0 / ((double)new_w / W), scale_y = 1.0 / ((double)new_h / H);
#pragma omp parallel for schedule(static)
  for (int oy = 0; oy < out_h; ++oy)
    for (int ox = 0; ox < out_w; ++ox) {
      uint8_t* d = out + ((size_t)oy * out_w + ox) * 3;
      int dy = oy - top, dx = ox - left;
      if (dy < 0 || dy >= new_h || dx < 0 || dx >= new_w) {
        d[0] = d[1] = d[2] = 114;
        continue;
      }
      if (new_h == H && new_w == W) {
        memcpy(d, in + ((size_t)dy * W + dx) * 3, 3);
        continue;
      }
      float fx = (float)((dx + 0.5) * scale_x - 0.5);
      int sx = (int)floorf(fx);
      fx -= sx;
      int single = 0;
      if (sx < 0) {
        fx = 0;
        sx = 0;
      }
      if (sx >= W - 1) {
        fx = 0;
        sx = W - 1;
        single = 1;
      }
      int a0 = round_short((1.f - fx) * 2048.f), a1 = round_short(fx * 2048.f);
      float fy = (float)((dy + 0.5) * scale_y - 0.5);
      int sy = (int)floorf(fy);
      fy -= sy;
      int b0 = round_short((1.f - fy) * 2048.f), b1 = round_short(fy * 2048.f);
      int r0 = clampi(sy, 0, H - 1), r1 = clampi(sy + 1, 0, H - 1);
      const uint8_t* s0 = in + ((size_t)r0 * W + sx) * 3;
      const uint8_t* s1 = in + ((size_t)r1 * W + sx) * 3;
      for (int c = 0; c < 3; ++c) {
        int d0 = single ? s0[c] * 2048 : s0[c] * a0 + s0[c + 3] * a1;
        int d1 = single ? s1[c] * 2048 : s1[c] * a0 + s1[c + 3] * a1;
        d[c] = (uint8_t)((((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2);
      }
    }
}

/* ---- SORT association (src/track/sort_tracker.py:55-80, 182-210) ---- */

/* _iou in numpy float32 scalar arithmetic. */
float oracle_iou(const float* a, const float* b) {
  float ix1 = a[0] > b[0] ? a[0] : b[0];
  float iy1 = a[1] > b[1] ? a[1] : b[1];
  float ix2 = a[2] < b[2] ? a[2] : b[2];
  float iy2 = a[3] < b[3] ? a[3] : b[3];
  float iw = ix2 - ix1;
  iw = iw > 0.0f ? iw : 0.0f;
  float ih = iy2 - iy1;
  ih = ih > 0.0f ? ih : 0.0f;
  float inter = iw * ih;
  float aw = a[2] - a[0], ah = a[3] - a[1], bw = b[2] - b[0], bh = b[3] - b[1];
  float area_a = (aw > 0.0f ? aw : 0.0f) * (ah > 0.0f ? ah : 0.0f);
  float area_b = (bw > 0.0f ? bw : 0.0f) * (bh > 0.0f ? bh : 0.0f);
  float denom = area_a + area_b - inter;
  if (denom <= 0.0f) return 0.0f;
  return inter / denom;
}

void oracle_iou_matrix(const float* trk, int T, const float* det, int D, float* out) {
  for (int i = 0; i < T; ++i)
    for (int j = 0; j < D; ++j) out[(size_t)i * D + j] = oracle_iou(trk + 4 * i, det + 4 * j);
}

/* Greedy argmax association; returns the number of matches. match_t/d get
 * the matches in acceptance order; m is destroyed. */
int oracle_greedy(float* m, int T, int D, float thr, int* match_t, int* match_d) {
  int n = 0;
  if (T == 0 || D == 0) return 0;
  for (;;) {
    size_t best = 0;
    float bv = m[0];
    for (size_t i = 1; i < (size_t)T * D; ++i)
      if (m[i] > bv) {
        bv = m[i];
        best = i;
      }
    if (bv < thr) break;
    int t = (int)(best / D), d = (int)(best % D);
    match_t[n] = t;
    match_d[n] = d;
    ++n;
    for (int j = 0; j < D; ++j) m[(size_t)t * D + j] = -1.0f;
    for (int i = 0; i < T; ++i) m[(size_t)i * D + d] = -1.0f;
  }
  return n;
}

/* ---- torchvision.ops.nms (CPU kernel) on class-offset boxes ---- */

typedef struct {
  float s;
  int i;
} ScoreIdx;
static int cmp_desc_stable(const void* a, const void* b) {
  const ScoreIdx* x = (const ScoreIdx*)a;
  const ScoreIdx* y = (const ScoreIdx*)b;
  if (x->s > y->s) return -1;
  if (x->s < y->s) return 1;
  return x->i - y->i;
}

/* boxes: n x 4 (already offset by class), scores: n.  Writes kept indices
 * (into the input) in keep order; returns count (<= max_keep). */
int oracle_nms(const float* boxes, const float* scores, int n, double iou_thr, int max_keep,
               int* keep) {
  ScoreIdx* order = (ScoreIdx*)malloc(sizeof(ScoreIdx) * (n > 0 ? n : 1));
  uint8_t* sup = (uint8_t*)calloc(n > 0 ? n : 1, 1);
  float* area = (float*)malloc(sizeof(float) * (n > 0 ? n : 1));
  for (int i = 0; i < n; ++i) {
    order[i].s = scores[i];
    order[i].i = i;
    area[i] = (boxes[4 * i + 2] - boxes[4 * i]) * (boxes[4 * i + 3] - boxes[4 * i + 1]);
  }
  qsort(order, n, sizeof(ScoreIdx), cmp_desc_stable);
  int nk = 0;
  for (int a = 0; a < n; ++a) {
    int i = order[a].i;
    if (sup[i]) continue;
    if (nk < max_keep) keep[nk] = i;
    nk++;
    const float* bi = boxes + 4 * i;
    for (int c = a + 1; c < n; ++c) {
      int j = order[c].i;
      if (sup[j]) continue;
      const float* bj = boxes + 4 * j;
      float xx1 = bi[0] > bj[0] ? bi[0] : bj[0];
      float yy1 = bi[1] > bj[1] ? bi[1] : bj[1];
      float xx2 = bi[2] < bj[2] ? bi[2] : bj[2];
      float yy2 = bi[3] < bj[3] ? bi[3] : bj[3];
      float w = xx2 - xx1;
      w = w > 0.f ? w : 0.f;
      float h = yy2 - yy1;
      h = h > 0.f ? h : 0.f;
      float inter = w * h;
      float ovr = inter / (area[i] + area[j] - inter);
      if ((double)ovr > iou_thr) sup[j] = 1;
    }
  }
  free(order);
  free(sup);
  free(area);
  return nk < max_keep ? nk : max_keep;
}

/* ------------------------------------------------------------------------
 * CLAHEDehaze LAB path (src/preprocess/ops/clahe_dehaze.py:21-25):
 * cv2.COLOR_BGR2LAB -> CLAHE on L -> cv2.COLOR_LAB2BGR, 8U, sRGB, D65.
 * Restates OpenCV 4.x imgproc/src/color_lab.cpp's 8-bit integer paths
 * (RGB2Lab_b: gamma_shift 3, lab_shift 12, 15-bit cube-root table;
 * Lab2RGBinteger: 14-bit base, L -> (y, f(y)) table, a/b dividers, 4096-entry
 * inverse-gamma table).  Tables are computed here in double with
 * round-half-even (OpenCV builds them with softfloat/softdouble).  UNPINNED
 * against real OpenCV (absent); pinned by CIE known-answer values in
 * tests/test_oracle_preprocess.py.
 * ---------------------------------------------------------------------- */
typedef struct {
  uint16_t gamma[256];  /* sRGB -> linear, x 255*8 */
  uint16_t cbrt[3072];  /* f(t) x 2^15 for t = i / (255*8) */
  uint16_t yf[512];     /* per L: y x 2^14, f(y) x 2^14 */
  uint16_t invg[4096];  /* linear (i/4096) -> sRGB u8 */
  int32_t cf[9];        /* BGR-ordered rows X, Y, Z: M_rgb2xyz / white x 2^12 */
  int32_t ci[9];        /* rows B, G, R over (X, Y, Z): M_xyz2rgb * white x 2^12 */
} OracleLab;

static const double kRgb2Xyz[9] = {0.412453, 0.357580, 0.180423, 0.212671, 0.715160,
                                   0.072169, 0.019334, 0.119193, 0.950227};
static const double kXyz2Rgb[9] = {3.240479, -1.53715, -0.498535, -0.969256, 1.875991,
                                   0.041556, 0.055648, -0.204043, 1.057311};
static const double kD65[3] = {0.950456, 1.0, 1.088754};

void oracle_lab_tables(OracleLab* t) {
  for (int i = 0; i < 256; ++i) {
    double x = i / 255.0;
    double g = x <= 0.04045 ? x / 12.92 : pow((x + 0.055) / 1.055, 2.4);
    t->gamma[i] = (uint16_t)nearbyint(255.0 * 8.0 * g);
  }
  for (int i = 0; i < 3072; ++i) {
    double x = i / (255.0 * 8.0);
    double f = x < 216.0 / 24389.0 ? x * (841.0 / 108.0) + 16.0 / 116.0 : cbrt(x);
    t->cbrt[i] = (uint16_t)nearbyint(32768.0 * f);
  }
  const double base = 16384.0;
  for (int i = 0; i < 256; ++i) {
    double y, ify;
    if (i <= 20) {
      y = nearbyint(i * base * 20.0 * 9.0 / (17.0 * 29.0 * 29.0 * 29.0));
      ify = nearbyint(base * (16.0 / 116.0 + i * 5.0 / (3.0 * 17.0 * 29.0)));
    } else {
      double fy = i * 100.0 * base / (255.0 * 116.0) + 16.0 * base / 116.0;
      ify = nearbyint(fy);
      y = nearbyint(fy * fy * fy / (base * base));
    }
    t->yf[2 * i] = (uint16_t)y;
    t->yf[2 * i + 1] = (uint16_t)ify;
  }
  for (int i = 0; i < 4096; ++i) {
    double x = i / 4096.0;
    double v = x <= 0.0031308 ? 12.92 * x : 1.055 * pow(x, 1.0 / 2.4) - 0.055;
    t->invg[i] = (uint16_t)nearbyint(255.0 * v);
  }
  /* forward rows X, Y, Z; columns in BGR order (src[0] = B) */
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      t->cf[r * 3 + c] = (int32_t)nearbyint(4096.0 * kRgb2Xyz[r * 3 + (2 - c)] / kD65[r]);
  /* inverse rows B, G, R; columns X, Y, Z */
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      t->ci[r * 3 + c] = (int32_t)nearbyint(4096.0 * kXyz2Rgb[(2 - r) * 3 + c] * kD65[c]);
}

static OracleLab g_olab;
static int g_olab_ready = 0;
static const OracleLab* olab(void) {
  if (!g_olab_ready) {
    oracle_lab_tables(&g_olab);
    g_olab_ready = 1;
  }
  return &g_olab;
}

/* RGB2Lab_b: CV_DESCALE(x, n) = (x + 2^(n-1)) >> n (arithmetic shift). */
static void bgr2lab_px(const OracleLab* t, int b, int g, int r, int* L, int* A, int* B) {
  int B_ = t->gamma[b], G_ = t->gamma[g], R_ = t->gamma[r];
  int X = (t->cf[0] * B_ + t->cf[1] * G_ + t->cf[2] * R_ + 2048) >> 12;
  int Y = (t->cf[3] * B_ + t->cf[4] * G_ + t->cf[5] * R_ + 2048) >> 12;
  int Z = (t->cf[6] * B_ + t->cf[7] * G_ + t->cf[8] * R_ + 2048) >> 12;
  int fX = t->cbrt[X], fY = t->cbrt[Y], fZ = t->cbrt[Z];
  *L = sat_u8((296 * fY - 1336934 + (1 << 14)) >> 15);
  *A = sat_u8((500 * (fX - fY) + 128 * (1 << 15) + (1 << 14)) >> 15);
  *B = sat_u8((200 * (fY - fZ) + 128 * (1 << 15) + (1 << 14)) >> 15);
}

static int ab_to_xz(int v) {
  return v <= 3390 ? v * 108 / 841 - 16384 * 16 / 116 * 108 / 841 : v * v / 16384 * v / 16384;
}

/* Lab2RGBinteger::process, BGR output. */
static void lab2bgr_px(const OracleLab* t, int L, int a, int b, int* ob, int* og, int* orr) {
  int y = t->yf[2 * L], ify = t->yf[2 * L + 1];
  int adiv = ((5 * a * 53687 + (1 << 7)) >> 13) - 128 * 16384 / 500;
  int bdiv = ((b * 41943 + (1 << 4)) >> 9) - 128 * 16384 / 200 + 1;
  int x = ab_to_xz(ify + adiv), z = ab_to_xz(ify - bdiv);
  int o[3];
  for (int r = 0; r < 3; ++r) {
    int v = (t->ci[r * 3] * x + t->ci[r * 3 + 1] * y + t->ci[r * 3 + 2] * z + (1 << 13)) >> 14;
    v = clampi(v, 0, 4095);
    o[r] = t->invg[v];
  }
  *ob = o[0];
  *og = o[1];
  *orr = o[2];
}

void oracle_bgr2lab(const uint8_t* in, uint8_t* out, int n) {
  const OracleLab* t = olab();
  for (int i = 0; i < n; ++i) {
    int L, A, B;
    bgr2lab_px(t, in[3 * i], in[3 * i + 1], in[3 * i + 2], &L, &A, &B);
    out[3 * i] = (uint8_t)L;
    out[3 * i + 1] = (uint8_t)A;
    out[3 * i + 2] = (uint8_t)B;
  }
}

void oracle_lab2bgr(const uint8_t* in, uint8_t* out, int n) {
  const OracleLab* t = olab();
  for (int i = 0; i < n; ++i) {
    int b, g, r;
    lab2bgr_px(t, in[3 * i], in[3 * i + 1], in[3 * i + 2], &b, &g, &r);
    out[3 * i] = (uint8_t)b;
    out[3 * i + 1] = (uint8_t)g;
    out[3 * i + 2] = (uint8_t)r;
  }
}

/* CLAHEDehaze LAB path on one BGR frame (pitch = 3W). */
void oracle_clahe_lab(const uint8_t* in, uint8_t* out, int H, int W, int tiles, double clip) {
  size_t n = (size_t)H * W;
  uint8_t* lab = (uint8_t*)malloc(n * 3);
  uint8_t* l = (uint8_t*)malloc(n);
  uint8_t* l2 = (uint8_t*)malloc(n);
  oracle_bgr2lab(in, lab, (int)n);
  for (size_t i = 0; i < n; ++i) l[i] = lab[3 * i];
  oracle_clahe_u8c1(l, l2, H, W, tiles, clip);
  for (size_t i = 0; i < n; ++i) lab[3 * i] = l2[i];
  oracle_lab2bgr(lab, out, (int)n);
  free(lab);
  free(l);
  free(l2);
}

/* ------------------------------------------------------------------------
 * cv2.cvtColor(COLOR_YUV2BGR_NV12), 8U (OpenCV color_yuv: YUV420sp2RGB8,
 * ITU-R BT.601 video range, 20-bit fixed point).  The device half of a
 * decode front end (src/io_video/capture.py:10-24 hands BGR frames to the
 * pipeline; a hardware decoder hands NV12).  Y plane H x W (y_pitch), then
 * the interleaved U,V plane H/2 x W (uv_pitch); H and W even.
 * ---------------------------------------------------------------------- */
void oracle_nv12_to_bgr(const uint8_t* y, const uint8_t* uv, int y_pitch, int uv_pitch,
                        uint8_t* out, int H, int W) {
  const int CY = 1220542, CUB = 2116026, CUG = -409993, CVG = -852492, CVR = 1673527;
  const int SH = 20;
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c) {
      const int u = uv[(r / 2) * uv_pitch + (c & ~1)] - 128;
      const int v = uv[(r / 2) * uv_pitch + (c & ~1) + 1] - 128;
      const int ruv = (1 << (SH - 1)) + CVR * v;
      const int guv = (1 << (SH - 1)) + CVG * v + CUG * u;
      const int buv = (1 << (SH - 1)) + CUB * u;
      int yy = y[r * y_pitch + c] - 16;
      if (yy < 0) yy = 0;
      yy *= CY;
      uint8_t* o = out + ((size_t)r * W + c) * 3;
      o[0] = (uint8_t)sat_u8((yy + buv) >> SH);
      o[1] = (uint8_t)sat_u8((yy + guv) >> SH);
      o[2] = (uint8_t)sat_u8((yy + ruv) >> SH);
    }
}
