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
#define RV_EOF 1 /* rv_capture_*: the source has no more frames */

/* ABI version (bumped on any signature change) and last-error text. */
int rv_abi_version(void);
const char* rv_last_error(void);
/* Measurement plumbing (no reference counterpart): an empty kernel whose
 * dispatch marks a point in a rocprofv3 kernel trace (bench.py brackets its
 * timed region with tags 1 and 2). */
int rv_trace_marker(int tag, void* stream);
/* Diagnostics (no reference counterpart): on a fatal signal write the native
 * stack to stderr, then chain to the previously installed handler (e.g.
 * Python's faulthandler).  Idempotent. */
int rv_install_crash_handler(void);

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

/* CLAHEDehaze space="LAB" (clahe_dehaze.py:21-25): cv2.COLOR_BGR2LAB, CLAHE
 * on L, cv2.COLOR_LAB2BGR, 8U sRGB / D65 integer paths (OpenCV color_lab.cpp
 * RGB2Lab_b / Lab2RGBinteger, restated; csrc/lab.h).  Same arguments and
 * workspace as rv_clahe_ycrcb_u8.  The first LAB call on a device uploads
 * the Lab tables to it synchronously; call rv_lab_init() (current device)
 * once before capturing the op in a graph. */
int rv_clahe_lab_u8(const uint8_t* in, uint8_t* out, int B, int H, int W,
                    int pitch, int tiles, double clip, void* ws,
                    size_t ws_bytes, void* stream);
int rv_lab_init(void);
/* Host copy of the Lab tables (parity tests): {u16 gamma[256], cbrt[3072],
 * yf[512], invg[4096]; i32 cf[9], ci[9]}, exactly 15944 bytes. */
int rv_lab_tables_host(void* out, size_t bytes);

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

/* The default chain plus the detector's LetterBox in one pass:
 * rv_clahe_median_u8 (k = 3) writing `out`, and the Ultralytics letterbox of
 * `out` (geo from rv_letterbox_geometry) into lb_out (B x geo[0] x geo[1] x 3),
 * byte-identical to rv_clahe_median_u8 followed by rv_letterbox_u8.  Replaces
 * the pipeline -> detector hand-over of main_preview.py:99-101
 * (PreprocessPipeline.__call__ then YOLOUltralytics.infer's LetterBox,
 * src/detect/yolo_ultralytics.py:28-35).  RV_EINVAL unless
 * rv_clahe_median_letterbox_fits() says 1. */
int rv_clahe_median_letterbox_u8(const uint8_t* in, uint8_t* out, int B, int H, int W,
                                 int pitch, int tiles, double clip, int k, void* ws,
                                 size_t ws_bytes, uint8_t* lb_out, const int* geo,
                                 void* stream);

/* 1 if rv_clahe_median_letterbox_u8 supports this geometry: k = 3, the LUT
 * cells of a 128 x 32 tile fit in LDS and every letterbox pixel's bilinear
 * taps fall in one tile. */
int rv_clahe_median_letterbox_fits(int H, int W, int tiles, int k, const int* geo);

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


/* --- YOLOv8 model (the Ultralytics graph run by model.predict,
 * yolo_ultralytics.py:16-35).  variant: 0=n 1=s 2=m 3=l 4=x (yolov8.yaml
 * scales).  Weights are BN-fused conv weights + biases in Ultralytics
 * state_dict order (rv_yolo_conv_info), flattened as, per conv,
 * weight[cout][cin][k][k] then bias[cout] (f32). */
int rv_yolo_num_convs(int variant);
/* info[5] = {cin, cout, k, stride, silu}; name = "model.2.m.0.cv1" etc. */
int rv_yolo_conv_info(int variant, int idx, int* info, char* name, int name_cap);
size_t rv_yolo_flat_floats(int variant);
size_t rv_yolo_packed_bytes(int variant);
/* Host-side packer: flat f32 -> device layout (bf16 [Cout16][ky][kx][Cin32],
 * f32 biases); the caller copies host_out to device memory it owns. */
int rv_yolo_pack(int variant, const float* flat, size_t n, void* host_out, size_t out_bytes);
/* Plan a model for in_h x in_w letterboxed inputs (multiples of 32) and up
 * to max_B images; dev_packed must stay valid for the handle's lifetime. */
int rv_yolo_create(int variant, const void* dev_packed, int max_B, int in_h, int in_w,
                   void** handle);
int rv_yolo_destroy(void* handle);
/* Handle options.  RV_YOLO_OPT_RAW_UNFUSED (default 1): a forward asked for
 * raw_out runs the unfused stem, so the P1 map (X0) lands in the workspace
 * for layer-wise inspection (and the C2f blocks unfused); 0: raw forwards
 * run the production kernel sequence, so raw_out is what the candidate
 * path computed. */
#define RV_YOLO_OPT_RAW_UNFUSED 1
/* RV_YOLO_OPT_FUSE_C2F: the narrow C2f blocks run as cv1 + one fused launch
 * for the bottlenecks and cv2 (bit-identical to the unfused convs): 1
 * (default) the hidden-width-16 blocks (YOLOv8n model.2), 2 also the
 * width-32 ones (model.4 / model.15; measured slower than unfused), 0 none:
 * one launch per conv. */
#define RV_YOLO_OPT_FUSE_C2F 2
/* RV_YOLO_OPT_STEM_X1 (default 0): the fused stem (conv0 + model.1, and
 * model.2.cv1 from its registers) also writes the X1 map; by default X1
 * never reaches HBM when model.2.cv1 is fused. */
#define RV_YOLO_OPT_STEM_X1 3
/* RV_YOLO_OPT_HEAD_STREAMS (default 1): the P3 / P4 Detect heads run on two
 * side streams of the handle (forked / joined with events) so they overlap
 * the rest of the neck; 0 keeps them on the caller's stream (a pipelined
 * caller whose stages already overlap).  The environment variable
 * RV_HEAD_STREAMS=0/1 overrides it. */
#define RV_YOLO_OPT_HEAD_STREAMS 4
/* RV_YOLO_OPT_FUSE_CV1 (default 1): model.3 and model.4.cv1 (the C2f's
 * first 1x1) run as one launch -- the 1x1 works on model.3's output tile in
 * LDS, so that map never reaches HBM; bit-identical to the two launches.
 * Raw parity forwards with RV_YOLO_OPT_RAW_UNFUSED keep them separate. */
#define RV_YOLO_OPT_FUSE_CV1 5
/* RV_YOLO_OPT_HEAD_CHAIN (default 0): candidate forwards of the YOLOv8n-
 * shaped bf16 head run each branch's last 1x1 conv inside its 3x3 conv's
 * launch (box: + DFL, class: + sigmoid / first maximum) and form the
 * candidates in one small kernel; the same candidates as the decode
 * kernel, whose head features and logits then never reach HBM.  Raw
 * forwards (raw_out) keep the decode kernel.  Off by default: on MI355X the
 * chained 3x3 launches cost what the decode saves. */
#define RV_YOLO_OPT_HEAD_CHAIN 6
/* RV_YOLO_OPT_C2F_TAP_PAIRS (default 1): the fused hidden-width-16 C2f chain
 * (model.2 of YOLOv8n) runs its 3x3 convs on tap pairs -- two taps' 16
 * channels per 32-deep MFMA k-step, 5 k-steps instead of 9 half-zero ones;
 * the sums round differently (within 1 bf16 ulp of the per-tap order).
 * 0: the per-tap k order, bit-identical to the unfused launches. */
#define RV_YOLO_OPT_C2F_TAP_PAIRS 7

/* One bf16 NHWC conv through the detector's conv launcher (layer tests;
 * the building block behind rv_yolo_forward, which the reference's
 * model.predict call replaces, src/detect/yolo_ultralytics.py:28-35):
 * k in {1, 3} (pad k / 2), stride 1 or 2, bias, SiLU when act != 0, plus an
 * optional bf16 residual view of the output's shape.  w: packed
 * [Cout_pad16][k*k][Cin_pad32] bf16, bias: f32 [Cout_pad16].  cfg6
 * (nullable): {MR, NR, G, resw, persist, kind} as rv_yolo_tuned_config
 * reports; RV_EINVAL when it is not valid for the layer. */
int rv_conv_bf16(const void* in, int B, int Hin, int Win, int Cin, int in_cs, const void* w,
                 const float* bias, int Cout, int k, int stride, void* out, int out_cs,
                 const void* res, int res_cs, int act, const int* cfg6, void* stream);
int rv_yolo_set_option(void* handle, int opt, int value);

/* fp8 plans (BASELINE configs[4]: "YOLOv8m 1280x1280 fp8 MFMA conv path").
 * dtype RV_YOLO_DTYPE_FP8: every conv except conv 0 (f32 weights, u8 input)
 * and the Detect head's last 1x1 stage (bf16, inside the decode) runs on
 * v_mfma_f32_16x16x32_fp8_fp8 with OCP e4m3fn weights (per output channel
 * power-of-two scale, round to nearest even, saturated at 448) and e4m3
 * activations (one power-of-two scale per activation buffer, value = code *
 * scale, set with rv_yolo_set_act_scales before the first forward; the
 * head's .1 stage writes bf16 features for the decode).  Packed layout per
 * fp8 conv: e4m3 [Cout16][ky][kx][Cin64], f32 bias [Cout16], f32 weight
 * scales [Cout16].  dtype RV_YOLO_DTYPE_BF16 = rv_yolo_pack / rv_yolo_create. */
#define RV_YOLO_DTYPE_BF16 0
#define RV_YOLO_DTYPE_FP8 1
size_t rv_yolo_packed_bytes2(int variant, int dtype);
int rv_yolo_pack2(int variant, int dtype, const float* flat, size_t n, void* host_out,
                  size_t out_bytes);
int rv_yolo_create2(int variant, int dtype, const void* dev_packed, int max_B, int in_h, int in_w,
                    void** handle);
/* scales[n]: one per activation buffer (n = rv_yolo_num_buffers; entries of
 * bf16 / f32 buffers are ignored), each a positive power of two. */
int rv_yolo_set_act_scales(void* handle, const float* scales, int n);
/* Per activation buffer: element bytes (1 fp8, 2 bf16, 4 f32), and its name
 * in the plan ("X0", "C2", "CAT14", "SP", "DA0", "model.2.m.0", ...: the
 * tensor or concat it holds; the fp8 oracle keys its scales by these). */
int rv_yolo_buffer_esize(void* handle, int buf);
int rv_yolo_buffer_name(void* handle, int buf, char* name, int cap);
/* The power-of-two scale for a tensor of absolute maximum amax (the rule the
 * packer and calibration use). */
float rv_fp8_scale(double amax);
size_t rv_yolo_ws_bytes(void* handle, int B);
int rv_yolo_num_anchors(void* handle);
/* Forward on B letterboxed u8 BGR images (B x in_h x in_w x 3).  raw_out
 * (nullable): the reference's raw prediction (B, 4+nc, A) f32 = cat(xywh *
 * stride, sigmoid(cls)).  cand (nullable): NMS candidate rows
 * {x1,y1,x2,y2,score,cls,anchor,pad} (32 B) of every anchor whose best class
 * score > conf, in the SEGMENTED layout: per image cand_cap rows, segment j
 * (64 consecutive anchors of one head level, nseg = rv_yolo_cand_segments)
 * owns rows [64 j, 64 j + cand_n[b * nseg + j]) in anchor order; cand_cap
 * >= 64 * nseg.  No atomics, no pre-zeroing. */
int rv_yolo_cand_segments(void* handle);
int rv_yolo_forward(void* handle, const uint8_t* lb, int B, void* ws, size_t ws_bytes,
                    float* raw_out, float conf, void* cand, int cand_cap, int* cand_n,
                    void* stream);
/* The forward in two parts: part 1 = stem .. model.15 (lb used), part 2 =
 * the bottom-up neck, the Detect heads and the decode (lb unused; reads part
 * 1's activations from the same workspace; cand / raw as above; raw_out
 * only with part 0 = the whole forward).  Part 2 needs a part 0 or part 1
 * forward of the same handle before it (launch numbering of the autotuned
 * configurations).  With two handles + workspaces a pipelined caller runs
 * part 2 of step j-1 beside part 1 of step j.  Part 1 itself may run as
 * part 3 (the stem and model.2, lb used) then part 4 (model.3 .. model.15,
 * lb unused; it must continue the handle's last part 3 with the same B and
 * workspace), so a caller can order other work after the stem. */
int rv_yolo_forward_part(void* handle, const uint8_t* lb, int B, void* ws, size_t ws_bytes,
                         float* raw_out, float conf, void* cand, int cand_cap, int* cand_n,
                         void* stream, int part);

/* Introspection for layer-wise parity tests: activation buffers (NHWC,
 * info = {H, W, C, is_f32}, byte offset inside the workspace for batch B)
 * and the conv launches of the last forward (24 ints each: conv index,
 * input view {buf, cs, co, Hin, Win}, Ho, Wo, two output views {buf, cs, co,
 * upsample}, residual view {buf, cs, co}, then a 1x1 conv's virtual concat
 * input {in_up, in2 buf, in2 cs, in2 co, split}: channels [0, split) are the
 * input view's (read upsampled 2x when in_up), the rest in2's; in2 buf -1:
 * none).  Returns the record count. */
int rv_yolo_num_buffers(void* handle);
int rv_yolo_buffer_info(void* handle, int B, int buf, int* info, size_t* off_bytes);
int rv_yolo_trace(void* handle, int* recs, int max_recs);

/* Live device timing of the conv launches (HIP events recorded on the launch
 * stream around every conv_mfma launch of the next max_forwards forwards;
 * 0 disables).  rv_yolo_profile_read synchronises on the events and returns,
 * per conv launch index, the summed ms over the recorded forwards, the
 * algorithmic FLOPs of one launch (2*M*N*K) and the conv index. */
int rv_yolo_profile(void* handle, int max_forwards);
/* The same with every profiled conv launched `reps` times back to back
 * between its event pair (same inputs and output); profile_read then
 * reports the time of ONE launch, free of the per-event dispatch gap. */
int rv_yolo_profile_reps(void* handle, int max_forwards, int reps);
int rv_yolo_profile_read(void* handle, double* ms, double* flops, int* conv, int n);
/* Algorithmic HBM bytes of one launch per conv launch index (inputs read
 * once, outputs written, residual, weights); returns the entries written. */
int rv_yolo_profile_bytes(void* handle, double* bytes, int n);
/* [start, end) in ms of every recorded conv launch of `handle`, after the
 * first recorded event of handle `ref` (same device clock), so the launches
 * of several forward contexts merge into the conv family's chip-wide busy
 * time.  Writes at most n pairs; returns the interval count. */
int rv_yolo_profile_times(void* handle, void* ref, double* t0, double* t1, int n);

/* Per-layer autotuning of the conv kernels (no reference counterpart: it
 * picks, per conv launch of this handle's forward, the fastest of the valid
 * LDS-staged kernel configurations on the given letterboxed batch; later
 * forwards use the choices).  Synchronous, not graph-capturable; call once
 * after rv_yolo_create.  verify != 0: every configuration's output is also
 * compared with the default's (they are bit-identical by construction) and
 * *n_bad counts the ones that were not.  reps: timed launches per config. */
int rv_yolo_autotune(void* handle, const uint8_t* lb, int B, void* ws, size_t ws_bytes,
                     int reps, int verify, int* n_bad, void* stream);
/* cfg6 = {MR, NR, G, resw, persist, kind} of conv launch idx (kind 0: LDS-staged
 * patch kernel, 1: direct-B 1x1 kernel; MR 0 = default
 * heuristic); returns the number of tuned launches (0 before autotuning). */
int rv_yolo_tuned_config(void* handle, int idx, int* cfg6);
/* Install a saved configuration (cfg6 as above) for conv launch idx of a
 * plan with n launches (e.g. reloaded from a file written after an earlier
 * autotune), so a run can skip the autotuner; an invalid entry falls back to
 * the default heuristic at launch. */
int rv_yolo_set_tuned(void* handle, int n, int idx, const int* cfg6);
/* The valid configurations of conv launch idx of the last whole forward
 * (cfg6 entries as above, at most cap written); returns the count (0 for a
 * fused C2f launch). */
int rv_yolo_conv_candidates(void* handle, int idx, int* cfg6, int cap);

/* --- Ultralytics non_max_suppression + scale_boxes + class filter
 * (yolo_ultralytics.py:28-53), one workgroup per image. */
size_t rv_nms_smem_bytes(void);
/* cand / seg_n: the segmented candidate layout of rv_yolo_forward (nseg
 * segments of 64 rows, cap <= 65536 rows per image).  Every candidate is
 * sorted (score desc, anchor asc); only the first max_nms of them enter the
 * greedy pass (Ultralytics non_max_suppression's max_nms = 30000: top
 * max_nms by score).  scale5 = {gain (f32 of the python gain), pad_x, pad_y,
 * clip_w, clip_h}; keep_mask4 (nullable = keep all): 128-bit class mask
 * (classes_keep); out: B x max_det x 6 {x1,y1,x2,y2,conf,cls} in score
 * order, out_n[B]; cand_total (nullable): candidates per image before
 * max_nms; ws: rv_nms_ws_bytes(B) bytes of device workspace. */
int rv_nms_postprocess(const void* cand, const int* seg_n, int B, int cap, int nseg,
                       float iou, int max_det, int max_nms, float max_wh, const float* scale5,
                       const uint32_t* keep_mask4, float* out, int* out_n, int* cand_total,
                       void* ws, size_t ws_bytes, void* stream);
/* Device workspace rv_nms_postprocess needs for B images (sort keys of
 * images with more than 4096 candidates: 65536 x 8 B per image). */
size_t rv_nms_ws_bytes(int B);
/* Segments of 64 anchors for a raw prediction with A anchors. */
int rv_cand_segments(int A);
/* Candidate rows from a reference-layout raw prediction (B, 4+nc, A), in the
 * segmented layout (segment j = anchors [64 j, 64 j + 64)); cap >= 64 *
 * rv_cand_segments(A). */
int rv_candidates_from_raw(const float* raw, int B, int nc, int A, float conf, void* cand,
                           int cap, int* seg_n, void* stream);

/* ------------------------------------------------------------------------ */
/* Track: SortTracker.update (src/track/sort_tracker.py:212-278) batched over */
/* S independent streams, with GroundProjector metrics (projector.py:13-84). */
/* ------------------------------------------------------------------------ */
size_t rv_sort_state_bytes(int S, int tmax);
size_t rv_sort_ws_bytes(int S, int tmax, int dmax);
/* Zero the state (no tracks, next_id = 1); synchronises `stream`.  Layout:
 * per-stream headers, list orders (tmax int32 each) and track pools (tmax
 * slots each); a track keeps its slot for life, the reference's list order
 * is the order array. */
int rv_sort_init(void* state, int S, int tmax, void* stream);
/* One frame per stream, three stream-ordered launches (KF predict over every
 * track; one workgroup per stream for _associate + bookkeeping; KF update /
 * new tracks over every detection).  The update runs in place on state_out;
 * pass state_in == state_out (if they differ, state_in is first copied to
 * state_out).  dets: S x dmax x 6 {x1,y1,x2,y2,conf,cls} f32 (post
 * class-filter), dcount[S]; ts[S] seconds.  params6 = {max_staleness,
 * min_hits, iou_threshold, speed_window, max_distance (<0 = None), 0}.  H9
 * (nullable = no projector): row-major f64 homography; origin2: projector
 * origin (f32).  Outputs per detection (S x dmax): track id (-1 = None),
 * distance_m and speed_kmh (NaN = None).  tmax <= 8192 and the association
 * workgroup's LDS (about 41 B x tmax + 28 B x dmax + 32 KB) <= 160 KB. */
int rv_sort_update(void* state_in, void* state_out, int S, int tmax, const float* dets,
                   const int* dcount, int dmax, const double* ts, const double* params6,
                   const double* H9, const float* origin2, void* ws, size_t ws_bytes,
                   int* out_id, double* out_dist, double* out_speed, void* stream);
/* Per-stream capacity report (device outputs, S ints each): live tracks T,
 * next track id, and the sticky overflow flag -- 1 once a frame had more
 * surviving + new tracks than tmax; the new tracks that did not fit were dropped
 * (their ids were still handed out), so that stream's ids diverge from the
 * reference's unbounded track list from then on.  next_id_out / overflow_out
 * are nullable. */
int rv_sort_stats(const void* state, int S, int* T_out, int* next_id_out, int* overflow_out,
                  void* stream);
/* Debug/parity export: per track x[7] (f64) and {id, hits, hit_streak, cls}. */
int rv_sort_export(const void* state, int S, int tmax, double* x_out, int* meta, int* T_out,
                   void* stream);

/* ------------------------------------------------------------------------ */
/* Result hand-back (yolo_ultralytics.py:44-52 `.cpu().numpy()` + Detection  */
/* construction; sort_tracker.py:234-247 fills track_id / distance_m /       */
/* speed_kmh).  One record per step: int32 n[S] (padded to 16 B), then       */
/* S x dmax rows of 48 B {f32 x1,y1,x2,y2,conf; i32 cls, track_id (-1 =      */
/* None), pad; f64 distance_m, speed_kmh (NaN = None)}, rows >= n[s] zeroed. */
/* ------------------------------------------------------------------------ */
size_t rv_results_bytes(int S, int dmax);
/* Packs the NMS rows (S x dmax x 6 f32) + counts and the SORT outputs
 * (track_id / distance_m / speed_kmh, S x dmax; each nullable = None) into
 * dev_stage (>= rv_results_bytes) and, when host_dst is non-null (pinned
 * host memory), copies the record there with one stream-ordered
 * hipMemcpyAsync.  Graph-capturable. */
int rv_results_handback(const float* dets, const int* det_n, const int* track_id,
                        const double* distance_m, const double* speed_kmh, int S, int dmax,
                        void* dev_stage, size_t stage_bytes, void* host_dst, void* stream);

/* --- Standalone pieces of SortTracker.update / GroundProjector, batched over
 * S streams (csrc/track_ops.hip; rv_sort_update fuses the same math). */
/* _iou_matrix (sort_tracker.py:74-80, _iou :55-71) in f32 scalar order.
 * trk: S x Tmax x 4, det: S x Dmax x 4 (x1,y1,x2,y2) f32; T[S], D[S] valid
 * counts (device).  out: S x Tmax x Dmax, zero outside T[s] x D[s]. */
int rv_iou_matrix_batched(const float* trk, const int* T, const float* det, const int* D,
                          float* out, int S, int Tmax, int Dmax, void* stream);
/* _associate's greedy loop (sort_tracker.py:196-208): argmax (first max in
 * row-major order), stop below thr (f64 compare), accept if row and column
 * are free, mask both with -1.  M (S x Tmax x Dmax, e.g. from
 * rv_iou_matrix_batched) is modified in place like the reference's matrix.
 * Outputs (device): match_t / match_d (S x min(Tmax, Dmax)) in acceptance
 * order, n_match[S], trk_match (S x Tmax: det index or -1), det_match
 * (S x Dmax: track index or -1); the reference's unmatched lists are the
 * -1 entries in ascending order.  thr <= -1 (an endless loop in the
 * reference) stops once every row is masked. */
int rv_greedy_assign_batched(float* M, const int* T, const int* D, int S, int Tmax, int Dmax,
                             double thr, int* match_t, int* match_d, int* n_match,
                             int* trk_match, int* det_match, void* stream);
/* GroundProjector.project_bbox + distance (projector.py:30-47, 74-84): foot
 * point (0.5*(x1+x2), y2) through the f64 homography H9 (device, row-major);
 * out_xy (n x 2 f64, NaN = None); out_dist (nullable, n f64, NaN = None):
 * f32 norm to origin2 (device, nullable = no distance), capped at
 * max_distance when >= 0. */
int rv_homography_project_f64(const double* H9, const float* boxes, int n,
                              const float* origin2, double max_distance,
                              double* out_xy, double* out_dist, void* stream);

/* The tracker-off branch of the per-frame loop (main_preview.py:101-109:
 * `tracker is None`): for dets (S x dmax x 6 f32, device) with det_n (S,
 * device) valid rows per stream, out_id = -1 (track_id None), out_speed NaN
 * (speed_kmh None) and out_dist = projector.distance_for_bbox(bbox)
 * (projector.py:49-51; NaN = None) when H9 (host, 3x3 f64 row-major) is
 * given, else NaN.  origin2 (host, 2 f32) is required with H9;
 * max_distance < 0 = no cap.  Every out array is S x dmax, device. */
int rv_untracked_metrics(const float* dets, const int* det_n, int S, int dmax,
                         const double* H9, const float* origin2, double max_distance,
                         int* out_id, double* out_dist, double* out_speed, void* stream);

/* ------------------------------------------------------------------------ */
/* Ingest: NV12 -> BGR (cv2.COLOR_YUV2BGR_NV12, 8U, BT.601 video range,      */
/* 20-bit fixed point).  The device half of a decode front end for           */
/* src/io_video/capture.py:10-24: host-fed NV12 is 1.5 B/pixel over PCIe     */
/* instead of 3.  y: B frames of H x W (y_pitch, y_frame_stride bytes apart); */
/* uv: interleaved U,V, H/2 x W (uv_pitch, uv_frame_stride); H, W even.      */
/* A packed NV12 batch is y = base, uv = base + H*W, both strides H*W*3/2.   */
/* ------------------------------------------------------------------------ */
int rv_nv12_to_bgr_u8(const uint8_t* y, const uint8_t* uv, int y_pitch, int uv_pitch,
                      size_t y_frame_stride, size_t uv_frame_stride, uint8_t* out,
                      int B, int H, int W, int pitch, void* stream);

/* ------------------------------------------------------------------------ */
/* Augment: fog + rain synthetic inputs (EnhancedFogSynthesizer.synthesize,  */
/* src/augment/fog.py:239-299; tools/fog_batch.py:7-34 drives it offline).   */
/* Restated subset: depth proxy, value-noise beta map, transmission, airlight */
/* gradient map, scattering I = J t + A (1 - t), global veil, tint, gamma,    */
/* plus rain streaks.  Parameters are drawn on the host                       */
/* (rvs_amd/augment/fog.py); the OpenCV filters are not restated. */
/* ------------------------------------------------------------------------ */
#define RV_FOG_NCONST 26
#define RV_FOG_NPARAM 16
/* consts (host, RV_FOG_NCONST f32): {vx, vy, dv_max, d_min, d_range, 0,
 *   rain_p, rain_len, n_oct, [gh, gw, amp, 0] x 4 octaves, norm}.
 * scene (device f32, 4*H + W + 3*n_oct*(H + W)): per-row 0.7*dp/dp_max,
 *   depth factor (sky boost x road damp), global-veil weight, airlight
 *   vertical gradient; the per-column airlight horizontal gradient; then per
 *   octave the noise sample taps: rows {y0[H], y1[H], wy[H]}, columns
 *   {x0[W], x1[W], wx[W]} (ys = (y*gh)/H in f32, y0 = floor, y1 = min(y0+1,
 *   gh), wy = ys - y0; the same along x).
 * frame_params (device, B x RV_FOG_NPARAM f32): {beta, A_b, A_g, A_r,
 *   A_scale, tint_b, tint_g, tint_r, gamma, rain_seed (< 2^24), 0...}.
 * grids (device, B x grid_stride f32): per frame, the octaves' value-noise
 *   grids, (gh+1) x (gw+1) each, concatenated.
 * ws: rv_fog_ws_bytes(B) bytes of device scratch (noise min / max). */
size_t rv_fog_ws_bytes(int B);
int rv_fog_rain_u8(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                   const float* consts, int n_consts, const float* scene,
                   const float* frame_params, const float* grids, int grid_stride,
                   void* ws, size_t ws_bytes, void* stream);

/* The whole EnhancedFogSynthesizer.synthesize (fog.py:227-299) with every
 * filter, as opencv-python runs it: the image airlight (band luminance
 * 0.9-quantile, masked mean, tint, filtered gradient map; fog.py:120-139),
 * the edge-guided transmission (_guided_filter's bilateralFilter fallback,
 * d 17, sigma 12 / 12; fog.py:55-67,172-179), scattering + global veil,
 * _glow (fog.py:182-191), _depth_blur (fog.py:194-214),
 * _local_contrast_fade (fog.py:217-224), tint, gamma, sensor noise, rain.
 * consts / scene / grids / rain as rv_fog_rain_u8.
 * full (host, RV_FOG_NFULL f32): {band_h, k, t, edge_guided, 0...}: the
 *   airlight band rows (max(10, int(0.12 H))) and np.quantile's f32 'linear'
 *   constants for n = band_h * W (k = floor((n-1)*0.9f), t = remainder).
 * depth (device f32 H x W): _depth_proxy's clipped depth.
 * amap_unit (device f32 H x W): the airlight filter applied to vgrad x xgrad
 *   (the per-channel map is a_c times it; rvs_amd.augment.airlight_unit_map).
 * bands (device u8 H x W): the _depth_blur band of each pixel (0..2, 3 none).
 * frame_params (device, B x RV_FOG_NPARAM_FULL f32): {beta, airlight tint
 *   b/g/r, airlight target mean, tint b/g/r, gamma, rain_seed, glow strength,
 *   contrast drop, has_noise, band kernel sizes x 3 (0 = skip), glow mask
 *   kernel k, glow image kernel k2, fade diameter d, 0...}; k, k2, band sizes
 *   <= 63, d <= 15.
 * noise (device f32 B x H x W x 3 or NULL): the sensor-noise normals of the
 *   frames whose has_noise is set.
 * ws: rv_fog_full_ws_bytes(B, H, W) bytes (56 B per pixel + partials).
 * H, W >= 64. */
#define RV_FOG_NPARAM_FULL 24
#define RV_FOG_NFULL 8
size_t rv_fog_full_ws_bytes(int B, int H, int W);
int rv_fog_full_u8(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                   const float* consts, int n_consts, const float* full, int n_full,
                   const float* scene, const float* depth, const float* amap_unit,
                   const uint8_t* bands, const float* frame_params, const float* grids,
                   int grid_stride, const float* noise, void* ws, size_t ws_bytes,
                   void* stream);

/* ------------------------------------------------------------------------ */
/* Capture front end (VideoSource, src/io_video/capture.py:10-24; README    */
/* module 8's async pipeline).  One reader thread per source fills a ring of */
/* pinned host slots from a file; frames are stamped with the wall-clock    */
/* time they were read (capture.py:20).  Formats: YUV4MPEG2 4:2:0 (handed   */
/* out as NV12), raw NV12, raw BGR.  No bitstream decoder / camera here.    */
/* ------------------------------------------------------------------------ */
#define RV_CAP_Y4M 0
#define RV_CAP_NV12 1
#define RV_CAP_BGR 2
/* W, H are read from the header for Y4M; nbuf in [2, 64] slots; loop != 0
 * rewinds at end of file.  *handle owns a reader thread. */
int rv_capture_open(const char* path, int fmt, int W, int H, int nbuf, int loop, void** handle);
/* info[6] = {W, H, fmt, frame bytes (NV12: 3WH/2, BGR: 3WH), pinned, nbuf} */
int rv_capture_info(void* handle, int* info);
/* Next frame in order (blocks until read): RV_OK with the slot's host pointer,
 * read time (s since the epoch) and frame index, or RV_EOF.  The slot stays
 * held until rv_capture_release. */
int rv_capture_next(void* handle, uint8_t** frame, double* ts, int64_t* index, int* slot);
int rv_capture_release(void* handle, int slot);
/* One frame of each of S sources -> dev + s * dev_stride (H2D on `stream`);
 * each slot returns to its reader once an event recorded behind its copy has
 * completed, so the rings refill while the device works.  ts / index (host, S) may be
 * NULL.  RV_EOF when a source ended (frames already queued are still
 * copied); rv_capture_close waits for copies still in flight. */
int rv_capture_upload_batch(void* const* handles, int S, uint8_t* dev, size_t dev_stride,
                            double* ts, int64_t* index, void* stream);
int rv_capture_close(void* handle);

/* --- Native launch schedule (csrc/sched.hip; no reference counterpart: the
 * reference runs its chain synchronously, main_preview.py:94-109).  A run of
 * K pipelined steps recorded once as a list of stream-ordered calls of this
 * library plus event record / wait nodes, issued by rv_sched_run with one
 * call.  rvs_amd/schedule.py records it.  Op argument arrays follow the C
 * signature of the op with float-class arguments moved, in order, to fargs
 * and the stream removed (it is the node's `stream`); a host-array argument
 * is passed as its byte offset into `host` (copied at record time) or -1. */
#define RV_SCHED_CLAHE_MEDIAN_LETTERBOX 0 /* rv_clahe_median_letterbox_u8 */
#define RV_SCHED_CLAHE_MEDIAN 1           /* rv_clahe_median_u8 */
#define RV_SCHED_LETTERBOX 2              /* rv_letterbox_u8 */
#define RV_SCHED_YOLO_FORWARD_PART 3      /* rv_yolo_forward_part */
#define RV_SCHED_NMS 4                    /* rv_nms_postprocess */
#define RV_SCHED_SORT_UPDATE 5            /* rv_sort_update */
#define RV_SCHED_HANDBACK 6               /* rv_results_handback */
#define RV_SCHED_UNTRACKED 7              /* rv_untracked_metrics */
#define RV_SCHED_NUM_OPS 8
int rv_sched_create(void** handle);
int rv_sched_destroy(void* handle);
int rv_sched_add_op(void* handle, int op, const int64_t* iargs, int ni, const double* fargs,
                    int nf, const void* host, size_t host_bytes, void* stream);
/* An event recorded on `stream` at this point of the run; its id -> *event.
 * timing != 0: a timing event (rv_sched_event_elapsed). */
int rv_sched_add_record(void* handle, void* stream, int timing, int* event);
/* `stream` waits for event `event` (an earlier record node). */
int rv_sched_add_wait(void* handle, void* stream, int event);
int rv_sched_num_nodes(void* handle);
/* Host wait (this thread only) for record node `event` of the last run.
 * Valid only after rv_sched_run returned RV_OK for that run: RV_EINVAL
 * before the first run, while a run is issuing, after a run that failed
 * part-way, or for an event the latest run did not issue.  Single issuer:
 * waits must not overlap an rv_sched_run of the same handle from another
 * thread (issue a run, wait on its events, then issue the next run); the
 * RV_EINVAL check covers a wait that starts while a run is issuing, not a
 * run that starts while a wait polls. */
int rv_sched_event_sync(void* handle, int event);
/* Non-blocking form: 1 = completed, 0 = not yet, < 0 = error (same
 * validity rule as rv_sched_event_sync). */
int rv_sched_event_query(void* handle, int event);
/* Milliseconds between two timing record nodes of the last run (same
 * validity rule as rv_sched_event_sync). */
int rv_sched_event_elapsed(void* handle, int a, int b, float* ms);
/* Issue the whole schedule: every stream it uses waits for `origin`'s work
 * so far, the nodes are issued in record order, and `origin` waits for every
 * stream at the end.  Asynchronous (no host synchronisation). */
int rv_sched_run(void* handle, void* origin);

#ifdef __cplusplus
}
#endif
#endif /* RVHIP_H */
