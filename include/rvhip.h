/*
 * rvhip.h — C ABI of the MI355X-native (gfx950) road-vision hot path.
 *
 * One shared library (librvhip.so, built by road-vision-system_amd/csrc/Makefile)
 * exports every function declared here.  Conventions, identical for every entry:
 *
 *   - plain pointers and sizes only; no torch / STL types cross the boundary;
 *   - device buffers are owned by the caller (torch tensors on the host side),
 *     the library never allocates or frees device memory inside a launch
 *     function, so every launch function is hipGraph-capturable;
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream);
 *     all work is stream-ordered, nothing synchronises the host;
 *   - return value: 0 = ok, RV_EINVAL (-1000) = bad argument (shape / pointer /
 *     capacity), RV_ECAP (-1001) = a capacity limit was exceeded, and
 *     -(hipError_t) for a HIP launch error.  Nothing throws across the ABI.
 *     rv_last_error() returns a static, thread-local description of the last
 *     non-zero status.
 *
 * Frames are interleaved BGR uint8, H x W x 3, `pitch` bytes between rows and
 * H*pitch bytes between frames of a batch (B frames = B independent camera
 * streams, stream-major).  Each entry cites the reference interface it
 * replaces (paths relative to YJxyzxyz/road-vision-system).
 */
#ifndef RVHIP_H
#define RVHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RV_OK 0
#define RV_EINVAL (-1000)
#define RV_ECAP (-1001)

/* ABI version (bumped on any signature change) and last-error text. */
int rv_abi_version(void);
const char* rv_last_error(void);

/* ------------------------------------------------------------------------ */
/* Preprocess: CLAHEDehaze (src/preprocess/ops/clahe_dehaze.py:13-32,       */
/* cv2.createCLAHE(...).apply on the Y plane of cv2.COLOR_BGR2YCrCb, then    */
/* cv2.COLOR_YCrCb2BGR) and MedianDerain (src/preprocess/ops/                */
/* median_derain.py:10-14, cv2.medianBlur).                                  */
/* ------------------------------------------------------------------------ */

/* Workspace bytes rv_clahe_ycrcb_u8 needs for B frames with a tiles x tiles
 * grid (one 256-entry u8 LUT per tile per frame). */
size_t rv_clahe_ws_bytes(int B, int tiles);

/* CLAHE on the luma of BGR frames, returned as BGR (YCrCb path of
 * clahe_dehaze.py:27-30).  `tiles` is the already-clamped grid
 * (clahe_dehaze.py:17: max(2, tile_grid)); `clip` the clipLimit.
 * in and out may not alias. */
int rv_clahe_ycrcb_u8(const uint8_t* in, uint8_t* out, int B, int H, int W,
                      int pitch, int tiles, double clip, void* ws,
                      size_t ws_bytes, void* stream);

/* Exact per-channel k x k median with replicated borders (cv2.medianBlur on
 * 8UC3).  k is the already-normalised kernel size (median_derain.py:11-13:
 * odd, clamped to [3, 9]). in and out may not alias. */
int rv_median_u8c3(const uint8_t* in, uint8_t* out, int B, int H, int W,
                   int pitch, int k, void* stream);

/* The default chain [CLAHEDehaze(YCrCb), MedianDerain(k)] of
 * configs/default.yaml:21-31 in one pass over HBM after the LUT pass: CLAHE
 * apply + colour round trip + k x k median, writing `out` (the observable
 * `proc` frame of main_preview.py:94).  Bit-identical to calling
 * rv_clahe_ycrcb_u8 then rv_median_u8c3.  ws as for rv_clahe_ws_bytes. */
int rv_clahe_median_u8(const uint8_t* in, uint8_t* out, int B, int H, int W,
                       int pitch, int tiles, double clip, int k, void* ws,
                       size_t ws_bytes, void* stream);

/* 1 if rv_clahe_median_u8 can run this geometry (the LUT window of one
 * output tile fits in LDS), 0 if the caller must use the unfused pair. */
int rv_clahe_median_fits(int H, int W, int tiles, int k);

/* Low-contrast auto gate (src/preprocess/pipeline.py:24-30): per frame,
 * span_out[b] = max(gray) - min(gray), gray = cv2.COLOR_BGR2GRAY (14-bit
 * fixed point).  ws: 2*B ints of device scratch. */
int rv_gray_span_u8(const uint8_t* in, int B, int H, int W, int pitch,
                    int* ws, int* span_out, void* stream);

/* ------------------------------------------------------------------------ */
/* Detect: YOLOUltralytics (src/detect/yolo_ultralytics.py:26-53).           */
/* ------------------------------------------------------------------------ */

/* Ultralytics LetterBox(640, auto=True, stride=32) geometry for an H x W
 * frame: writes {out_h, out_w, new_h, new_w, top, left} into geo[6]. */
int rv_letterbox_geometry(int H, int W, int imgsz, int stride, int* geo);

/* LetterBox pixels: cv2.resize(INTER_LINEAR, 8U fixed point) to new_h x
 * new_w, then cv2.copyMakeBorder(top, ., left, ., BORDER_CONSTANT, 114).
 * Output is BGR u8, B x out_h x out_w x 3, tightly packed. */
int rv_letterbox_u8(const uint8_t* in, uint8_t* out, int B, int H, int W,
                    int pitch, const int* geo, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RVHIP_H */
