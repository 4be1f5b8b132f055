// Internal interface of the YOLOv8 conv / head kernels (conv.hip) used by the
// model plan (yolo.hip).  Activations are NHWC bf16 (raw uint16 bits);
// a "view" is (base pointer, channel stride of the buffer, channel offset),
// so concatenation is free: producers write into a slice of a wider buffer
// and consumers read a slice.
#pragma once
#include "common.h"

namespace rv {

typedef uint16_t bf16_t;

struct ConvArgs {
  // input view
  const bf16_t* in;
  int in_cs, in_co;
  int Hin, Win, Cin;
  // packed weights [Cout_pad16][k*k][Cin_pad32] bf16, bias [Cout_pad16] f32
  const bf16_t* w;
  const float* bias;
  int Cout, k, stride, pad;
  int Ho, Wo, B;
  // up to two output views; up = 1 writes a nearest-2x upsampled copy
  void* out0;
  int out0_cs, out0_co, out0_up;
  void* out1;
  int out1_cs, out1_co, out1_up;
  int out_f32;  // 1: outputs are f32 (detect logits), else bf16
  // optional residual view (same spatial size as the output): v += res
  const bf16_t* res;
  int res_cs, res_co;
  int act;  // 1: SiLU
  // optional second group (a block-diagonal conv: the Detect head's
  // parallel cv2 / cv3 branches in one launch).  Output channels
  // [g2_cout0, Cout) read input channels [g2_in_co, g2_in_co + g2_Cin) of
  // the same input buffer with their own packed weights and bias; output
  // channel g2_cout0 + j is that group's channel j.  g2_cout0 = 0: one group.
  int g2_cout0, g2_in_co, g2_Cin;
  const bf16_t* g2_w;
  const float* g2_bias;
  // > 0: this launch record stands for a fused C2f chain (yolo.hip's
  // Model::fused[fused - 1]); the autotuner leaves it alone
  int fused;
  // fp8 (OCP e4m3fn) path: in8 = 1 -> the input (and residual) views hold
  // fp8 codes with per-tensor scales s_in / s_res (value = code * s), the
  // weights are fp8 [Cout_pad16][ky][kx][Cin_pad64] with per-cout scales
  // `wscale` (g2: g2_wscale); out*_8 = 1 -> that output view stores fp8
  // codes of value / s_out*, else bf16 (f32 when out_f32).
  int in8, out0_8, out1_8;
  float s_in, s_res, s_out0, s_out1;
  const float* wscale;
  const float* g2_wscale;
  // virtual concat input of a 1x1 conv (conv1x1_direct_kernel only): input
  // channels [0, split) come from the `in` view -- read at (y/2, x/2) of a
  // half-resolution map when in_up, i.e. the nearest-2x upsample the
  // reference materialises (torch.cat([Upsample(x), y])) is never written --
  // and [split, Cin) from the in2 view (channel stride in2_cs, offset in2_co,
  // full resolution).  split = 0 and in_up = 0: `in` only.
  const bf16_t* in2;
  int in2_cs, in2_co, split, in_up;
  // chained 1x1 conv (conv_patch_kernel CH form): a C2f cv1 (Cout -> Cout,
  // SiLU) fused into the conv producing its input.  ch_w: its packed
  // weights [Cout][Cout] bf16, ch_b: its bias.  The launch's output view
  // (out0) is then the 1x1's; the producer's own output stays in LDS.
  const bf16_t* ch_w;
  const float* ch_b;
  // 1: SiLU, the 1x1's bf16 output stored to out0; 2: a Detect box
  // branch's last conv, DFL to four f32 distances per pixel (out0: 4 f32
  // per pixel); 3: a Detect class branch's last conv, sigmoid and first
  // maximum (out0: {f32 score, i32 class} per pixel)
  int ch_mode;
};

// One configuration of the LDS-staged conv kernel: MR x NR 16x16 fragments
// per wave, G input-channel chunks (32 ch) per pipeline stage, resident
// weights, persistent grid.
struct ConvCfg {
  int mr, nr, G, resw, persist;
  int kind = 0;  // 0: LDS-staged patch kernel (4 waves); 1: 1x1 direct-B kernel (G, resw
                 // unused); 2: the patch kernel with 8 waves per workgroup (bf16 3x3)
};

// Implicit-GEMM conv on MFMA (v_mfma_f32_16x16x32_bf16), default config.
int launch_conv(const ConvArgs& a, hipStream_t s);
// The same with an explicit configuration; whether a configuration is valid
// for a layer; the valid configurations of a layer (the autotuner's search
// space: returns the count, fills at most cap).
int launch_conv_cfg(const ConvArgs& a, const ConvCfg& c, hipStream_t s);
bool conv_cfg_ok(const ConvArgs& a, const ConvCfg& c);
int conv_candidates(const ConvArgs& a, ConvCfg* out, int cap);

// First conv (3 -> C0, k3 s2, p1) straight from the u8 BGR letterboxed
// frame (the reference's predictor preprocess im[..., ::-1] / 255 folded into
// the weights), on i8 MFMAs over the window bytes with exact i32 sums; the
// weights in the integer form yolo.hip's packer writes (pack_conv0q).
struct Conv0Q {
  const int8_t* d;   // [3][C0][64] balanced base-256 digits of Q (k = 16 ky + 3 kx + ch, BGR)
  const float* s;    // [C0] value scale
  const float* b;    // [C0] bias
  const int32_t* c;  // [3][C0] 128 sum_k D_i[k]: digit i's accumulator start
};
int launch_conv0(const uint8_t* img, int B, int H, int W, const Conv0Q& q, int C0, bf16_t* out,
                 int out_cs, hipStream_t s);
// The same with an fp8 output (codes of value / s_out, channel stride out_cs
// bytes).
int launch_conv0_fp8(const uint8_t* img, int B, int H, int W, const Conv0Q& q, int C0,
                     uint8_t* out, int out_cs, float s_out, hipStream_t s);

// conv0 and model.1 (C0 = 16 -> C1 = 32, k3 s2) fused: the P1 map never
// leaves LDS.  w1/b1: model.1's packed weights / bias; out (nullable): X1
// (NHWC, channel stride out_cs).  w2/b2/out2 (nullable): the following 1x1
// conv 32 -> 32 (model.2.cv1) run from the registers into out2 (channel
// stride out2_cs), bit-identical to the unfused 1x1 kernels.
int launch_stem(const uint8_t* img, int B, int H, int W, const Conv0Q& q0, int C0,
                const bf16_t* w1, const float* b1, int C1, bf16_t* out, int out_cs,
                hipStream_t s, const bf16_t* w2 = nullptr, const float* b2 = nullptr,
                bf16_t* out2 = nullptr, int out2_cs = 0);

// SPPF pooling: buf holds x in channels [0, c); writes maxpool5, maxpool5^2
// and maxpool5^3 (= clipped 5/9/13 windows) into [c,2c), [2c,3c), [3c,4c).
int launch_sppf_pool(bf16_t* buf, int B, int H, int W, int c, hipStream_t s);
// fp8 buffer (one scale for the whole buffer: max pooling is scale-free).
int launch_sppf_pool_fp8(uint8_t* buf, int B, int H, int W, int c, hipStream_t s);

// Fused C2f bottleneck chain + cv2 (c2f.hip) for C2f blocks with hidden
// width C in {16, 32} and N in {1, 2} bottlenecks (C = 16: N = 1): reads
// y0 / y1 (cv1's output, channels [cat_co, cat_co + 2C) of the block's
// concat buffer), writes cv2's 2C channels to the output view.  Every
// intermediate stays in LDS.  Bit-identical to the unfused launches (C = 16
// with tap_pairs: within 1 bf16 ulp).
struct C2fArgs {
  const bf16_t* cat;
  int cat_cs, cat_co;
  int H, W, B;
  const bf16_t* wa[2];
  const float* ba[2];
  const bf16_t* wb[2];
  const float* bb[2];
  const bf16_t* w2;
  const float* b2;
  bf16_t* out;
  int out_cs, out_co;
  // C = 16: the 3x3 convs on tap pairs (two taps' 16 channels per 32-deep
  // k-step; within 1 bf16 ulp of the per-tap k order) instead of one
  // half-zero k-step per tap (bit-identical to the unfused launches)
  int tap_pairs;
};
bool c2f_fusable(int C, int N, int cat_cs, int cat_co, int out_cs, int out_co);
int launch_c2f_chain(const C2fArgs& a, int C, int N, bool shortcut, hipStream_t s);

struct HeadLevel {
  const float* logits;  // [B][H][W][cs] f32: [0,4*reg) box bins, [4*reg, 4*reg+nc) classes
  int H, W, cs;
  float stride;
  // fused form (feat != nullptr): the last 1x1 convs of the level run inside
  // the decode from the bf16 features [box feats (cin_b) | class feats
  // (cin_c)] (channel stride feat_cs) with packed weights [cout][cin_pad32]
  // and f32 biases; logits_out (nullable) receives the f32 logits.
  const bf16_t* feat;
  int feat_cs, cin_b, cin_c;
  const bf16_t* w_box;
  const bf16_t* w_cls;
  const float* b_box;
  const float* b_cls;
  float* logits_out;
};

// The chained Detect head's outputs per level (conv_patch_kernel ch_mode 2 /
// 3): bx = 4 f32 DFL distances per pixel, sc = {f32 score, i32 class} per
// pixel, B x H x W each; start / blk: first anchor / first 64-anchor
// segment of each level (+ totals at [nlv]).
struct HeadCombine {
  const float* bx[4];
  const float* sc[4];
  int H[4], W[4];
  float stride[4];
  int start[5], blk[5];
  int nlv;
};

struct Cand {  // one detection candidate (Ultralytics NMS row before NMS)
  float x1, y1, x2, y2, score;
  int cls, anchor, pad;
};

// DFL + dist2bbox + sigmoid for all anchors.  Optionally writes the
// reference's raw output (B, 4+nc, A) and every anchor whose best class
// score > conf as a candidate row: segment j (64 consecutive anchors of one
// level) fills cand[b][64 j ...] in anchor order, its count in
// seg_n[b][j] (nseg = decode_segments()).
int decode_segments(const HeadLevel* lv, int nlv);
int launch_detect_decode(const HeadLevel* lv, int nlv, int B, int nc, int reg_max, float conf,
                         float* raw, Cand* cand, int cand_cap, int* seg_n, hipStream_t s);

// Candidates of the chained head (HeadCombine): the fixed decode's output
// for the same logits, in the segmented layout of rv_yolo_forward.
int launch_head_combine(const HeadCombine& h, int B, float conf, Cand* cand, int cand_cap,
                        int* cand_n, hipStream_t s);

}  // namespace rv
