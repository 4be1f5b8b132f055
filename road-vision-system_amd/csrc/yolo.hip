// YOLOv8 model plan + C ABI (the detector backend behind
// src/detect/yolo_ultralytics.py:7-53, restating the Ultralytics yolov8.yaml
// graph: Conv / C2f / SPPF / Detect(DFL)).
//
// The plan is built natively here: the canonical conv list (Ultralytics
// state_dict order, BN already fused into conv weight + bias), the weight
// packer, the activation-buffer layout in one caller-owned HBM workspace, and
// the launch sequence of a forward.  Concats are free (producers write into
// channel slices of the concat buffers); nearest-2x upsamples are extra
// epilogue writes of the producing conv.
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>
#include <cstring>
#include <cmath>
#include "conv.h"

namespace rv {

struct ConvSpec {
  std::string name;
  int cin, cout, k, s, act;
  size_t w_off = 0, b_off = 0;  // byte offsets in the packed blob
  size_t ws_off = 0;            // fp8 convs: per-cout weight scales (f32)
  bool f8 = false;              // fp8 weights / inputs (RV_YOLO_DTYPE_FP8 plans)
};

struct Variant {
  int c1, c2, c3, c4, c5;   // backbone widths (P1..P5)
  int h12, h15, h18, h21;   // head widths
  int nb, nm;               // C2f repeats for "3" and "6"
  int c2d, c3d;             // Detect branch widths
  int nc = 80, reg = 16;
};

static int make_div8(double x) { return (int)(std::ceil(x / 8.0) * 8); }

static bool variant_widths(int variant, Variant& v) {
  // yolov8.yaml scales: n [0.33, 0.25, 1024], s [0.33, 0.50, 1024],
  // m [0.67, 0.75, 768], l [1.00, 1.00, 512], x [1.00, 1.25, 512]
  static const double S[5][3] = {{0.33, 0.25, 1024}, {0.33, 0.50, 1024}, {0.67, 0.75, 768},
                                 {1.00, 1.00, 512},  {1.00, 1.25, 512}};
  if (variant < 0 || variant > 4) return false;
  const double d = S[variant][0], w = S[variant][1], mc = S[variant][2];
  auto ch = [&](int c) { return make_div8(std::min((double)c, mc) * w); };
  auto rep = [&](int n) { return std::max((int)std::lround(n * d), 1); };
  v.c1 = ch(64);
  v.c2 = ch(128);
  v.c3 = ch(256);
  v.c4 = ch(512);
  v.c5 = ch(1024);
  v.h12 = ch(512);
  v.h15 = ch(256);
  v.h18 = ch(512);
  v.h21 = ch(1024);
  v.nb = rep(3);
  v.nm = rep(6);
  v.c2d = std::max(std::max(16, v.h15 / 4), v.reg * 4);
  v.c3d = std::max(v.h15, std::min(v.nc, 100));
  return true;
}

struct ModelDef {
  Variant v;
  int dtype = 0;  // RV_YOLO_DTYPE_BF16 / RV_YOLO_DTYPE_FP8
  std::vector<ConvSpec> convs;
  // conv 0's integer form (the i8 MFMA conv0, conv.h Conv0Q), after every
  // conv's block: digits [3][C0][64] i8, scales [C0] f32, biases [C0] f32,
  // accumulator starts [3][C0] i32
  size_t q_off = 0, q_bytes = 0;
  int add(const std::string& n, int ci, int co, int k, int s, int act = 1) {
    ConvSpec c;
    c.name = n;
    c.cin = ci;
    c.cout = co;
    c.k = k;
    c.s = s;
    c.act = act;
    convs.push_back(c);
    return (int)convs.size() - 1;
  }
  void c2f(const std::string& p, int c1, int c2, int n) {
    const int c = c2 / 2;
    add(p + ".cv1", c1, 2 * c, 1, 1);
    add(p + ".cv2", (2 + n) * c, c2, 1, 1);
    for (int i = 0; i < n; ++i) {
      add(p + ".m." + std::to_string(i) + ".cv1", c, c, 3, 1);
      add(p + ".m." + std::to_string(i) + ".cv2", c, c, 3, 1);
    }
  }
  int find(const std::string& n) const {
    for (size_t i = 0; i < convs.size(); ++i)
      if (convs[i].name == n) return (int)i;
    return -1;
  }
};

static size_t conv0q_bytes(int C0) { return 3 * (size_t)C0 * 64 + 20 * (size_t)C0; }

static bool build_def(int variant, ModelDef& m, int dtype = RV_YOLO_DTYPE_BF16) {
  if (!variant_widths(variant, m.v)) return false;
  if (dtype != RV_YOLO_DTYPE_BF16 && dtype != RV_YOLO_DTYPE_FP8) return false;
  m.dtype = dtype;
  const Variant& v = m.v;
  m.add("model.0", 3, v.c1, 3, 2);
  m.add("model.1", v.c1, v.c2, 3, 2);
  m.c2f("model.2", v.c2, v.c2, v.nb);
  m.add("model.3", v.c2, v.c3, 3, 2);
  m.c2f("model.4", v.c3, v.c3, v.nm);
  m.add("model.5", v.c3, v.c4, 3, 2);
  m.c2f("model.6", v.c4, v.c4, v.nm);
  m.add("model.7", v.c4, v.c5, 3, 2);
  m.c2f("model.8", v.c5, v.c5, v.nb);
  m.add("model.9.cv1", v.c5, v.c5 / 2, 1, 1);
  m.add("model.9.cv2", v.c5 / 2 * 4, v.c5, 1, 1);
  m.c2f("model.12", v.c5 + v.c4, v.h12, v.nb);
  m.c2f("model.15", v.h12 + v.c3, v.h15, v.nb);
  m.add("model.16", v.h15, v.h15, 3, 2);
  m.c2f("model.18", v.h15 + v.h12, v.h18, v.nb);
  m.add("model.19", v.h18, v.h18, 3, 2);
  m.c2f("model.21", v.h18 + v.c5, v.h21, v.nb);
  const int chs[3] = {v.h15, v.h18, v.h21};
  for (int i = 0; i < 3; ++i) {
    const std::string p = "model.22.cv2." + std::to_string(i);
    m.add(p + ".0", chs[i], v.c2d, 3, 1);
    m.add(p + ".1", v.c2d, v.c2d, 3, 1);
    m.add(p + ".2", v.c2d, 4 * v.reg, 1, 1, 0);
  }
  for (int i = 0; i < 3; ++i) {
    const std::string p = "model.22.cv3." + std::to_string(i);
    m.add(p + ".0", chs[i], v.c3d, 3, 1);
    m.add(p + ".1", v.c3d, v.c3d, 3, 1);
    m.add(p + ".2", v.c3d, v.nc, 1, 1, 0);
  }
  // packed layout: conv 0 keeps f32 OIHW (VALU conv), the rest bf16
  // [Cout_pad16][ky][kx][Cin_pad32]; biases f32 [Cout_pad16]; 256-B aligned.
  // fp8 plans: every conv but conv 0 and the Detect head's last 1x1 stage
  // (run inside the decode kernel on bf16 features) is fp8 e4m3
  // [Cout_pad16][ky][kx][Cin_pad64] + f32 per-cout scales [Cout_pad16].
  size_t off = 0;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  for (size_t i = 0; i < m.convs.size(); ++i) {
    ConvSpec& c = m.convs[i];
    c.f8 = dtype == RV_YOLO_DTYPE_FP8 && i > 0 &&
           !(c.name.compare(0, 9, "model.22.") == 0 && c.name.size() > 2 &&
             c.name.compare(c.name.size() - 2, 2, ".2") == 0);
    const int cop = (c.cout + 15) & ~15;
    const int cip = c.f8 ? (c.cin + 63) & ~63 : (c.cin + 31) & ~31;
    c.w_off = off;
    off = al(off + (i == 0 ? (size_t)c.cout * c.cin * c.k * c.k * 4
                           : (size_t)cop * c.k * c.k * cip * (c.f8 ? 1 : 2)));
    c.b_off = off;
    off = al(off + (size_t)cop * 4);
    if (c.f8) {
      c.ws_off = off;
      off = al(off + (size_t)cop * 4);
    }
  }
  m.q_off = off;
  m.q_bytes = conv0q_bytes(m.convs[0].cout);
  return true;
}

static size_t packed_bytes(const ModelDef& m) {
  return (m.q_off + m.q_bytes + 255) & ~(size_t)255;
}

// Integer form of conv 0 (conv.h Conv0Q): per output channel o, the f64
// weights V[k] = w[o][2-ch][ky][kx] / 255 (RGB order and 1/255 folded in;
// k = 16 ky + 3 kx + ch over the window's BGR bytes, k % 16 >= 9 zero) as
// integers Q[k] = round(V[k] / s), s = max|V| / (127 * 2^16), split into
// balanced base-256 digits Q = 65536 D0 + 256 D1 + D2 (each in [-128, 127]).
// The kernel feeds x - 128 (the byte XOR 0x80) to one i8 MFMA per digit,
// starting each accumulator at 128 sum_k D_i[k], so it holds T_i = sum_k
// D_i[k] x[k] exactly (|T_i| <= 27 * 128 * 255 < 2^24: exact in f32 too);
// the value is s (65536 T0 + 256 T1 + T2) + b, f32 to 2^-23 of the weight
// scale with no offset cancellation.
static void pack_conv0q(const float* w, const float* b, int C0, uint8_t* dst) {
  int8_t* D = (int8_t*)dst;
  float* S = (float*)(dst + 3 * (size_t)C0 * 64);
  float* Bv = S + C0;
  int32_t* Cq = (int32_t*)(Bv + C0);
  for (int o = 0; o < C0; ++o) {
    double V[64] = {0.0}, M = 0.0;
    for (int ky = 0; ky < 3; ++ky)
      for (int kx = 0; kx < 3; ++kx)
        for (int ch = 0; ch < 3; ++ch) {
          const double v = (double)w[((o * 3 + (2 - ch)) * 3 + ky) * 3 + kx] / 255.0;
          V[16 * ky + 3 * kx + ch] = v;
          M = std::max(M, std::fabs(v));
        }
    const float s = M > 0.0 ? (float)(M / (127.0 * 65536.0)) : 1.0f;
    long long sd[3] = {0, 0, 0};
    for (int k = 0; k < 64; ++k) {
      const long long q = std::llround(V[k] / (double)s);
      const long long d2 = ((q + 128) & 255) - 128;
      const long long q1 = (q - d2) / 256;
      const long long d1 = ((q1 + 128) & 255) - 128;
      const long long d0 = (q1 - d1) / 256;
      const long long d[3] = {d0, d1, d2};
      for (int t = 0; t < 3; ++t) {
        D[((size_t)t * C0 + o) * 64 + k] = (int8_t)d[t];
        sd[t] += d[t];
      }
    }
    S[o] = s;
    Bv[o] = b[o];
    for (int t = 0; t < 3; ++t) Cq[t * C0 + o] = (int32_t)(128 * sd[t]);
  }
}

static size_t flat_floats(const ModelDef& m) {
  size_t n = 0;
  for (const ConvSpec& c : m.convs) n += (size_t)c.cout * c.cin * c.k * c.k + c.cout;
  return n;
}

// OCP e4m3fn code of x (|x| saturated to 448, round to nearest even,
// subnormals in 2^-9 steps) -- the rounding of v_cvt_pk_fp8_f32
static uint8_t host_f2e4m3(float x) {
  const uint8_t sgn = std::signbit(x) ? 0x80 : 0;
  double a = std::fabs((double)x);
  if (a > 448.0) a = 448.0;
  if (a < std::ldexp(1.0, -6)) return sgn | (uint8_t)std::nearbyint(a * 512.0);  // 8 -> 2^-6
  int e;
  const double m = std::frexp(a, &e);  // a = m 2^e, m in [0.5, 1)
  int q = (int)std::nearbyint((m * 2.0 - 1.0) * 8.0);
  int E = e - 1 + 7;
  if (q == 8) {
    q = 0;
    ++E;
  }
  return sgn | (uint8_t)((E << 3) | q);
}

// smallest power of two s with amax / s <= 448 (1 for amax == 0)
static float pow2_scale(double amax) {
  if (!(amax > 0.0)) return 1.0f;
  return (float)std::ldexp(1.0, (int)std::ceil(std::log2(amax / 448.0)));
}

static uint16_t host_f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)(u >> 16);  // inf/nan
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// ---------------------------------------------------------------------------
// Plan: activation buffers (element offsets into the bf16 workspace, per B)
// ---------------------------------------------------------------------------
struct View {
  int buf;  // buffer id
  int cs, co;
};

struct Buf {
  size_t elems_per_img;
  bool f32;
  size_t off_bytes;  // filled per B
  int esize = 2;     // bytes per element: 4 (f32 logits), 2 (bf16), 1 (fp8 codes)
};

struct TraceRec {
  int conv, in_buf, in_cs, in_co, Hin, Win, Ho, Wo;
  int out0_buf, out0_cs, out0_co, up0, out1_buf, out1_cs, out1_co, up1;
  int res_buf, res_cs, res_co;
  int in_up, in2_buf, in2_cs, in2_co, split;  // virtual concat input (ConvArgs::split)
};

// A 1x1 conv's virtual concat input (ConvArgs::in2 / split / in_up):
// channels [0, split) from view a (read upsampled 2x when up), the rest
// from view b.
struct VIn {
  View a;
  int up;
  View b;
  int split;
};

// Live per-launch timing of conv_mfma (bench roofline): one hipEvent pair
// per conv launch per forward, recorded on the launch stream.
struct Profile {
  bool on = false;
  int cap_fwd = 0, n_fwd = 0, per_fwd = 0;
  int reps = 1;  // launches of each conv between its event pair (rv_yolo_profile_reps)
  std::vector<hipEvent_t> ev;     // [cap_fwd][per_fwd][2]
  std::vector<double> flops;      // per conv launch index (algorithmic, 2*M*N*K)
  std::vector<double> bytes;      // per conv launch index (algorithmic HBM bytes, launch_bytes)
  std::vector<int> conv_of;       // conv spec index per launch index
};

struct Model {
  ModelDef def;
  Profile prof;
  std::vector<TraceRec> trace;  // conv specs run by the last forward (one record each)
  std::vector<ConvArgs> launches;  // conv kernel launches of the last forward
  std::vector<ConvCfg> tuned;      // per launch index: autotuned config (mr 0 = default)
  struct FusedC2f {
    C2fArgs a;
    int C, N;
    bool shortcut;
  };
  std::vector<FusedC2f> fused;     // fused C2f chains of the last forward (ConvArgs::fused)
  std::vector<std::pair<std::string, int>> tmps;  // bottleneck temp buffer per "prefix.m.i"
  int tmp_of(const std::string& k) const {
    for (auto& t : tmps)
      if (t.first == k) return t.second;
    return -1;
  }
  const uint8_t* dev = nullptr;  // packed weights (caller-owned device memory)
  // side streams + events for the forked P3 / P4 Detect heads
  hipStream_t side[2] = {nullptr, nullptr};
  hipEvent_t ev_fork[2] = {nullptr, nullptr}, ev_join[2] = {nullptr, nullptr};
  ~Model() {
    for (int i = 0; i < 2; ++i) {
      // teardown: a failure here leaves nothing to report or undo
      if (side[i]) (void)hipStreamDestroy(side[i]);
      if (ev_fork[i]) (void)hipEventDestroy(ev_fork[i]);
      if (ev_join[i]) (void)hipEventDestroy(ev_join[i]);
    }
  }
  int max_B = 0, H = 0, W = 0;
  // forward parts (rv_yolo_forward_part): launch index base of this call
  // (part 2 continues part 1's launch numbering) and part 1's launch count
  int li_base = 0, n_part1 = -1;
  int n_part1a = -1;               // launches of the last part 3 (stem .. model.2)
  int part1a_B = 0;
  void* part1a_ws = nullptr;
  int part1_B = 0;                // batch and workspace of the last part 0 / part 1 forward:
  const void* part1_ws = nullptr;  // part 2 must continue exactly that forward
  // fp8 plans: per-buffer activation scales (value = code * scale), powers
  // of two; set by rv_yolo_set_act_scales before the first forward
  std::vector<float> act_scale;
  bool scales_set = false;
  // RV_YOLO_OPT_RAW_UNFUSED: forwards that return the raw prediction run the
  // unfused stem, so every activation (X0 included) is in the workspace
  int raw_unfused = 1;
  // RV_YOLO_OPT_FUSE_C2F: narrow C2f blocks as cv1 + one fused chain launch
  // (1: the hidden-width-16 chains only, 2: width 16 and 32, 0: none)
  int fuse_c2f = 1;
  // RV_YOLO_OPT_STEM_X1: the fused stem also writes X1 (parity tests)
  int stem_x1 = 0;
  int head_streams = 1;            // RV_YOLO_OPT_HEAD_STREAMS
  int fuse_cv1 = 1;                // RV_YOLO_OPT_FUSE_CV1
  int head_chain = 0;              // RV_YOLO_OPT_HEAD_CHAIN (measured neutral: DESIGN.md)
  int c2f_tap_pairs = 1;           // RV_YOLO_OPT_C2F_TAP_PAIRS
  std::vector<Buf> bufs;
  int nA = 0;
  int map_h[6], map_w[6];  // stride 2^i maps

  std::vector<int> buf_h, buf_w, buf_c;
  std::vector<std::string> buf_name;
  int newbuf(const std::string& name, int s, int c, bool f32 = false, bool bf16 = false) {
    Buf b;
    b.elems_per_img = (size_t)map_h[s] * map_w[s] * c;
    b.f32 = f32;
    b.off_bytes = 0;
    b.esize = f32 ? 4 : (def.dtype == RV_YOLO_DTYPE_FP8 && !bf16 ? 1 : 2);
    bufs.push_back(b);
    buf_h.push_back(map_h[s]);
    buf_w.push_back(map_w[s]);
    buf_c.push_back(c);
    buf_name.push_back(name);
    return (int)bufs.size() - 1;
  }
  // buffer ids
  int X0, X1, C2, X2, X3, C4, CAT14, X5, C6, CAT11, X7, C8, X8, SP, CAT20, C12, CAT17, C15,
      X15, C18, X18, C21, X21;
  int DA[3], DB[3], HD[3];
  int BX[3], SC[3];  // chained head: DFL distances / (score, class) per pixel

  size_t ws_bytes(int B) const {
    size_t off = 0;
    for (const Buf& b : bufs)
      off = (off + b.elems_per_img * B * b.esize + 255) & ~(size_t)255;
    return off;
  }
};

static void plan(Model& M) {
  const Variant& v = M.def.v;
  for (int i = 0; i < 6; ++i) {
    M.map_h[i] = M.H >> i;
    M.map_w[i] = M.W >> i;
  }
  M.X0 = M.newbuf("X0", 1, v.c1);
  M.X1 = M.newbuf("X1", 2, v.c2);
  M.C2 = M.newbuf("C2", 2, (2 + v.nb) * (v.c2 / 2));
  M.X2 = M.newbuf("X2", 2, v.c2);
  M.X3 = M.newbuf("X3", 3, v.c3);
  M.C4 = M.newbuf("C4", 3, (2 + v.nm) * (v.c3 / 2));
  M.CAT14 = M.newbuf("CAT14", 3, v.h12 + v.c3);
  M.X5 = M.newbuf("X5", 4, v.c4);
  M.C6 = M.newbuf("C6", 4, (2 + v.nm) * (v.c4 / 2));
  M.CAT11 = M.newbuf("CAT11", 4, v.c5 + v.c4);
  M.X7 = M.newbuf("X7", 5, v.c5);
  M.C8 = M.newbuf("C8", 5, (2 + v.nb) * (v.c5 / 2));
  M.X8 = M.newbuf("X8", 5, v.c5);
  M.SP = M.newbuf("SP", 5, 4 * (v.c5 / 2));
  M.CAT20 = M.newbuf("CAT20", 5, v.h18 + v.c5);
  M.C12 = M.newbuf("C12", 4, (2 + v.nb) * (v.h12 / 2));
  M.CAT17 = M.newbuf("CAT17", 4, v.h15 + v.h12);
  M.C15 = M.newbuf("C15", 3, (2 + v.nb) * (v.h15 / 2));
  M.X15 = M.newbuf("X15", 3, v.h15);
  M.C18 = M.newbuf("C18", 4, (2 + v.nb) * (v.h18 / 2));
  M.X18 = M.newbuf("X18", 4, v.h18);
  M.C21 = M.newbuf("C21", 5, (2 + v.nb) * (v.h21 / 2));
  M.X21 = M.newbuf("X21", 5, v.h21);
  for (int i = 0; i < 3; ++i) {
    const std::string l = std::to_string(i);
    M.DA[i] = M.newbuf("DA" + l, 3 + i, v.c2d + v.c3d);
    M.DB[i] = M.newbuf("DB" + l, 3 + i, v.c2d + v.c3d, false, true);  // bf16: the decode's features
    M.HD[i] = M.newbuf("HD" + l, 3 + i, 4 * v.reg + v.nc, true);
    M.BX[i] = M.newbuf("BX" + l, 3 + i, 4, true);
    M.SC[i] = M.newbuf("SC" + l, 3 + i, 2, true);
  }
  // one temp per bottleneck (its first conv's output): no buffer is ever
  // overwritten inside a forward, so every layer stays inspectable
  struct C2fDef {
    const char* p;
    int level, c2, n;
  };
  const C2fDef cs[] = {{"model.2", 2, v.c2, v.nb},  {"model.4", 3, v.c3, v.nm},
                       {"model.6", 4, v.c4, v.nm},  {"model.8", 5, v.c5, v.nb},
                       {"model.12", 4, v.h12, v.nb}, {"model.15", 3, v.h15, v.nb},
                       {"model.18", 4, v.h18, v.nb}, {"model.21", 5, v.h21, v.nb}};
  for (const C2fDef& c : cs)
    for (int i = 0; i < c.n; ++i) {
      const std::string q = std::string(c.p) + ".m." + std::to_string(i);
      M.tmps.push_back({q, M.newbuf(q, c.level, c.c2 / 2)});
    }
  M.nA = M.map_h[3] * M.map_w[3] + M.map_h[4] * M.map_w[4] + M.map_h[5] * M.map_w[5];
}

struct Exec {
  Model* M;
  uint8_t* ws;
  int B;
  hipStream_t s;
  std::vector<size_t> off;
  int status = 0;

  void* ptr(int buf) const { return ws + off[buf]; }
  const bf16_t* wptr(const ConvSpec& c) const { return (const bf16_t*)(M->dev + c.w_off); }
  const float* bptr(const ConvSpec& c) const { return (const float*)(M->dev + c.b_off); }
  const float* wsptr(const ConvSpec& c) const {
    return c.f8 ? (const float*)(M->dev + c.ws_off) : nullptr;
  }
  float scale(int buf) const { return buf >= 0 ? M->act_scale[buf] : 1.0f; }

  int spec(const std::string& name) {
    const int idx = M->def.find(name);
    if (idx < 0 && !status) {
      set_error("plan: unknown conv %s", name.c_str());
      status = RV_EINVAL;
    }
    return idx;
  }

  ConvArgs args(const ConvSpec& c, View in, int li, View o0, int up0, View o1, int up1,
                View res) const {
    ConvArgs a;
    memset(&a, 0, sizeof(a));
    a.in = (const bf16_t*)ptr(in.buf);
    a.in_cs = in.cs;
    a.in_co = in.co;
    a.Hin = M->map_h[li];
    a.Win = M->map_w[li];
    a.Cin = c.cin;
    a.w = wptr(c);
    a.bias = bptr(c);
    a.Cout = c.cout;
    a.k = c.k;
    a.stride = c.s;
    a.pad = c.k / 2;
    a.Ho = (a.Hin + 2 * a.pad - c.k) / c.s + 1;
    a.Wo = (a.Win + 2 * a.pad - c.k) / c.s + 1;
    a.B = B;
    a.out0 = ptr(o0.buf);
    a.out0_cs = o0.cs;
    a.out0_co = o0.co;
    a.out0_up = up0;
    if (o1.buf >= 0) {
      a.out1 = ptr(o1.buf);
      a.out1_cs = o1.cs;
      a.out1_co = o1.co;
      a.out1_up = up1;
    }
    a.out_f32 = M->bufs[o0.buf].f32 ? 1 : 0;
    if (res.buf >= 0) {
      a.res = (const bf16_t*)ptr(res.buf);
      a.res_cs = res.cs;
      a.res_co = res.co;
    }
    a.act = c.act;
    if (c.f8) {
      a.in8 = 1;
      a.s_in = scale(in.buf);
      a.wscale = wsptr(c);
      a.out0_8 = M->bufs[o0.buf].esize == 1;
      a.s_out0 = scale(o0.buf);
      if (o1.buf >= 0) {
        a.out1_8 = M->bufs[o1.buf].esize == 1;
        a.s_out1 = scale(o1.buf);
      }
      if (res.buf >= 0) a.s_res = scale(res.buf);
    }
    return a;
  }

  // one record per conv spec (layer-wise parity tests read these back)
  void trace(int idx, const ConvArgs& a, View in, View o0, int up0, View o1, int up1, View res,
             const VIn* vin = nullptr) {
    TraceRec r;
    memset(&r, 0, sizeof(r));
    r.in2_buf = -1;
    if (vin) {
      in = vin->a;
      r.in_up = vin->up;
      r.in2_buf = vin->b.buf;
      r.in2_cs = vin->b.cs;
      r.in2_co = vin->b.co;
      r.split = vin->split;
    }
    r.conv = idx;
    r.in_buf = in.buf;
    r.in_cs = in.cs;
    r.in_co = in.co;
    r.Hin = a.Hin;
    r.Win = a.Win;
    r.Ho = a.Ho;
    r.Wo = a.Wo;
    r.out0_buf = o0.buf;
    r.out0_cs = o0.cs;
    r.out0_co = o0.co;
    r.up0 = up0;
    r.out1_buf = o1.buf;
    r.out1_cs = o1.cs;
    r.out1_co = o1.co;
    r.up1 = up1;
    r.res_buf = res.buf;
    r.res_cs = res.cs;
    r.res_co = res.co;
    M->trace.push_back(r);
  }

  // Algorithmic HBM bytes of one conv launch: every input channel slice it
  // reads (once), every output / upsampled copy it writes, the residual it
  // adds and its packed weights -- each byte once, however the kernel tiles.
  static double launch_bytes(const ConvArgs& a) {
    const double px_in = (double)a.B * a.Hin * a.Win, px_out = (double)a.B * a.Ho * a.Wo;
    if (a.split > 0 || a.in_up) {  // virtual concat: each source read once
      const double cin1 = a.split > 0 ? a.split : a.Cin;
      const double src = (a.in_up ? px_in / 4 : px_in) * cin1 + px_in * (a.Cin - cin1);
      const double outs = (a.out0 ? (a.out0_up ? 4 : 1) : 0) + (a.out1 ? (a.out1_up ? 4 : 1) : 0);
      return 2.0 * src + 2.0 * px_out * a.Cout * outs + 2.0 * a.Cout * a.Cin;
    }
    const bool g2 = a.g2_cout0 > 0;
    const int cout1 = g2 ? a.g2_cout0 : a.Cout, cout2 = g2 ? a.Cout - a.g2_cout0 : 0;
    double in_ch = a.Cin;
    if (g2 && (a.g2_in_co != a.in_co || a.g2_Cin != a.Cin)) in_ch += a.g2_Cin;
    const double eb = a.in8 ? 1.0 : 2.0;  // input / residual / weight element bytes
    auto ob = [&](int o8) { return a.out_f32 ? 4.0 : (o8 ? 1.0 : 2.0); };
    const double outs = (a.out0 ? (a.out0_up ? 4 : 1) * ob(a.out0_8) : 0) +
                        (a.out1 ? (a.out1_up ? 4 : 1) * ob(a.out1_8) : 0);
    const double w = eb * a.k * a.k * ((double)cout1 * a.Cin + (double)cout2 * (g2 ? a.g2_Cin : 0)) +
                     (a.ch_w ? 2.0 * a.Cout * a.Cout : 0.0);  // a chained 1x1's weights
    return px_in * in_ch * eb + px_out * a.Cout * outs + (a.res ? px_out * a.Cout * eb : 0.0) + w;
  }

  static double flops_of(const ConvSpec& c, const ConvArgs& a) {
    return 2.0 * a.B * a.Ho * a.Wo * (double)c.cout * c.cin * c.k * c.k;
  }

  // One kernel launch: the autotuned configuration of this launch index if
  // there is a valid one, else the default; live HIP-event timing when
  // profiling is on.
  void launch(const ConvArgs& a, int idx, double flops) {
    const int li_ = M->li_base + (int)M->launches.size();
    M->launches.push_back(a);
    Profile& P = M->prof;
    const bool rec = P.on && P.n_fwd < P.cap_fwd && li_ < P.per_fwd;
    const int ev0 =
        rec ? hip_check(hipEventRecord(P.ev[((size_t)P.n_fwd * P.per_fwd + li_) * 2], s),
                        "profile hipEventRecord")
            : RV_OK;
    // profiled forwards may launch each conv `reps` times back to back
    // between its events (the same inputs, the same output): the event pair
    // then times reps kernels, not reps dispatch latencies
    const int nrep = rec ? P.reps : 1;
    for (int r = 0; r < nrep && !status; ++r) {
      if (a.fused > 0) {
        const Model::FusedC2f& f = M->fused[a.fused - 1];
        status = launch_c2f_chain(f.a, f.C, f.N, f.shortcut, s);
      } else if (li_ < (int)M->tuned.size() && M->tuned[li_].mr > 0 &&
                 conv_cfg_ok(a, M->tuned[li_])) {
        status = launch_conv_cfg(a, M->tuned[li_], s);
      } else {
        status = launch_conv(a, s);
      }
    }
    if (!status) status = ev0;
    if (rec && !status)
      status = hip_check(hipEventRecord(P.ev[((size_t)P.n_fwd * P.per_fwd + li_) * 2 + 1], s),
                         "profile hipEventRecord");
    if (P.on && P.n_fwd == 0 && li_ < P.per_fwd) {
      P.flops[li_] = flops;
      P.bytes[li_] = a.fused > 0 ? fused_bytes : launch_bytes(a);
      P.conv_of[li_] = idx;
    }
  }
  double fused_bytes = 0.0;  // algorithmic bytes of the next fused launch

  // conv `name`: input view at map level li -> up to two output views
  // (vin: a 1x1 conv's virtual concat input instead of `in`)
  void conv(const std::string& name, View in, int li, View o0, int up0 = 0, View o1 = {-1, 0, 0},
            int up1 = 0, View res = {-1, 0, 0}, const VIn* vin = nullptr) {
    if (status) return;
    const int idx = spec(name);
    if (idx < 0) return;
    const ConvSpec& c = M->def.convs[idx];
    ConvArgs a = args(c, vin ? vin->a : in, li, o0, up0, o1, up1, res);
    if (vin) {
      a.in_up = vin->up;
      a.in2 = (const bf16_t*)ptr(vin->b.buf);
      a.in2_cs = vin->b.cs;
      a.in2_co = vin->b.co;
      a.split = vin->split;
    }
    trace(idx, a, in, o0, up0, o1, up1, res, vin);
    launch(a, idx, flops_of(c, a));
  }

  // Two convs that share their input buffer, kernel size, stride and
  // activation and write adjacent channel slices of one output view -- the
  // Detect head's cv2 / cv3 branches -- as one grouped launch
  // (ConvArgs::g2_*).  Default: grouped in fp8 plans only.  bf16 plans launch
  // the branches separately: with the 8-wave patch kernel each branch runs
  // as ONE cout tile of its own width (box 64, class 80) reading the input
  // once, where the grouped launch's 64-wide tiles padded the class branch
  // to 128 (r04: P3 head 306 -> 260 us per 128-frame unit,
  // profiles/r04/conv_table_eager_*).  RV_HEAD_PAIR=1 / 0 forces either.
  void conv_pair(const std::string& n1, View in1, const std::string& n2, View in2, int li,
                 View o0) {
    if (status) return;
    const int i1 = spec(n1), i2 = spec(n2);
    if (i1 < 0 || i2 < 0) return;
    const ConvSpec& c1 = M->def.convs[i1];
    const ConvSpec& c2 = M->def.convs[i2];
    const View o2{o0.buf, o0.cs, o0.co + c1.cout};
    static const int env = getenv("RV_HEAD_PAIR") ? atoi(getenv("RV_HEAD_PAIR")) : -1;
    const bool pair = env >= 0 ? env != 0 : c1.f8;
    if (!pair || in1.buf != in2.buf || in1.cs != in2.cs || c1.k != c2.k || c1.s != c2.s ||
        c1.act != c2.act || c1.cout % 64 != 0) {
      conv(n1, in1, li, o0);
      conv(n2, in2, li, o2);
      return;
    }
    const View none{-1, 0, 0};
    ConvArgs a = args(c1, in1, li, o0, 0, none, 0, none);
    const ConvArgs a2 = args(c2, in2, li, o2, 0, none, 0, none);
    trace(i1, a, in1, o0, 0, none, 0, none);
    trace(i2, a2, in2, o2, 0, none, 0, none);
    const double fl = flops_of(c1, a) + flops_of(c2, a2);
    a.Cout = c1.cout + c2.cout;
    a.g2_cout0 = c1.cout;
    a.g2_in_co = in2.co;
    a.g2_Cin = c2.cin;
    a.g2_w = wptr(c2);
    a.g2_bias = bptr(c2);
    a.g2_wscale = wsptr(c2);
    launch(a, i1, fl);
  }

  // conv n1 (3x3, output view `mid`, never written) with the 1x1 conv n2
  // (Cout -> Cout, SiLU: a C2f cv1) chained inside the same launch
  // (ConvArgs::ch_w, conv_patch_kernel CH form) writing view o0.  false
  // when the pair does not have the chained form's shape (the caller then
  // runs them as two launches).
  bool conv_chain(const std::string& n1, View in, int li, View mid, const std::string& n2,
                  View o0) {
    if (status) return false;
    const int i1 = M->def.find(n1), i2 = M->def.find(n2);
    if (i1 < 0 || i2 < 0) return false;
    const ConvSpec& c1 = M->def.convs[i1];
    const ConvSpec& c2 = M->def.convs[i2];
    if (c1.f8 || c2.f8 || c1.k != 3 || c1.cout != 64 || c2.k != 1 || c2.cin != c1.cout ||
        c2.cout != c1.cout || !c1.act || !c2.act)
      return false;
    const View none{-1, 0, 0};
    ConvArgs a = args(c1, in, li, o0, 0, none, 0, none);
    ConvCfg probe{4, 1, 1, 1, 1, 0};
    a.ch_w = wptr(c2);
    a.ch_b = bptr(c2);
    a.ch_mode = 1;
    if (!conv_cfg_ok(a, probe)) return false;
    // trace records: the two convs as the unfused plan runs them
    trace(i1, args(c1, in, li, mid, 0, none, 0, none), in, mid, 0, none, 0, none);
    const ConvArgs a2 = args(c2, mid, li + 1, o0, 0, none, 0, none);
    trace(i2, a2, mid, o0, 0, none, 0, none);
    launch(a, i1, flops_of(c1, a) + flops_of(c2, a2));
    return true;
  }

  // The Detect head's branch of level li: its 3x3 conv n1 (input view in,
  // nominal output `mid` -- never written) with its last 1x1 conv n2
  // chained in the same launch (ch_mode 2: box, DFL distances to o0; 3:
  // class, best (score, class) to o0).  probe_only: just report whether the
  // shapes have a chained configuration.
  bool head_chain(const std::string& n1, View in, int li, View mid, const std::string& n2,
                  View o0, int mode, bool probe_only) {
    if (status) return false;
    const int i1 = M->def.find(n1), i2 = M->def.find(n2);
    if (i1 < 0 || i2 < 0) return false;
    const ConvSpec& c1 = M->def.convs[i1];
    const ConvSpec& c2 = M->def.convs[i2];
    if (c1.f8 || c2.f8 || c1.k != 3 || c1.s != 1 || c2.k != 1 || c2.cin != c1.cout ||
        c2.cout != c1.cout || !c1.act || c2.act || c1.cout != (mode == 2 ? 64 : 80))
      return false;
    const View none{-1, 0, 0};
    ConvArgs a = args(c1, in, li, o0, 0, none, 0, none);
    a.ch_w = wptr(c2);
    a.ch_b = bptr(c2);
    a.ch_mode = mode;
    if (!conv_cfg_ok(a, ConvCfg{mode == 2 ? 4 : 5, 1, 1, 1, 1, 0}) &&
        !conv_cfg_ok(a, ConvCfg{mode == 2 ? 4 : 5, 1, 1, 0, 1, 0}))
      return false;
    if (probe_only) return true;
    trace(i1, args(c1, in, li, mid, 0, none, 0, none), in, mid, 0, none, 0, none);
    const ConvArgs a2 = args(c2, mid, li, o0, 0, none, 0, none);
    trace(i2, a2, mid, o0, 0, none, 0, none);
    launch(a, i1, flops_of(c1, a) + flops_of(c2, a2));
    return true;
  }

  static bool c2f_will_fuse(int c, int n, bool fuse, int up0, View o1, View o0) {
    return fuse && up0 == 0 && o1.buf < 0 && c2f_fusable(c, n, 2 * c, 0, o0.cs, o0.co);
  }

  // C2f(prefix): in view (map li) -> concat buffer cb -> outputs.  With
  // `fuse`, narrow blocks run cv1 and then one fused launch for the
  // bottlenecks + cv2 (c2f.hip; intermediates stay in LDS).
  void c2f(const std::string& p, View in, int li, int cb, int c2, int n, bool shortcut, View o0,
           int up0 = 0, View o1 = {-1, 0, 0}, int up1 = 0, bool fuse = false,
           bool cv1_done = false, const VIn* vin = nullptr) {
    const int c = c2 / 2;
    // a fused chain keeps z_i in LDS, so its concat buffer holds y0, y1
    // only: pixel stride 2c (denser cv1 stores and chain reads)
    const bool fused = c2f_will_fuse(c, n, fuse, up0, o1, o0);
    const int cs = fused ? 2 * c : (2 + n) * c;
    if (!cv1_done)
      conv(p + ".cv1", in, li, View{cb, cs, 0}, 0, View{-1, 0, 0}, 0, View{-1, 0, 0}, vin);
    if (fused && !status) {
      Model::FusedC2f f;
      memset(&f.a, 0, sizeof(f.a));
      f.C = c;
      f.N = n;
      f.shortcut = shortcut;
      f.a.cat = (const bf16_t*)ptr(cb);
      f.a.cat_cs = cs;
      f.a.cat_co = 0;
      f.a.H = M->map_h[li];
      f.a.W = M->map_w[li];
      f.a.B = B;
      f.a.tap_pairs = M->c2f_tap_pairs;
      double flops = 0.0;
      ConvArgs rec;
      for (int i = 0; i < n; ++i) {
        const std::string q = p + ".m." + std::to_string(i);
        const int ia = spec(q + ".cv1"), ib = spec(q + ".cv2");
        if (ia < 0 || ib < 0) return;
        const ConvSpec& ca = M->def.convs[ia];
        const ConvSpec& cbv = M->def.convs[ib];
        f.a.wa[i] = wptr(ca);
        f.a.ba[i] = bptr(ca);
        f.a.wb[i] = wptr(cbv);
        f.a.bb[i] = bptr(cbv);
        // trace records keep the layer list complete (the buffers are not
        // written: parity forwards run unfused; the records show the unfused
        // concat layout)
        const int tmp = M->tmp_of(q);
        const int cs_u = (2 + n) * c;
        const View bin{cb, cs_u, (1 + i) * c};
        const View none{-1, 0, 0};
        ConvArgs aa = args(ca, bin, li, View{tmp, c, 0}, 0, none, 0, none);
        trace(ia, aa, bin, View{tmp, c, 0}, 0, none, 0, none);
        ConvArgs ab = args(cbv, View{tmp, c, 0}, li, View{cb, cs_u, (2 + i) * c}, 0, none, 0,
                           shortcut ? bin : none);
        trace(ib, ab, View{tmp, c, 0}, View{cb, cs_u, (2 + i) * c}, 0, none, 0, shortcut ? bin : none);
        flops += flops_of(ca, aa) + flops_of(cbv, ab);
      }
      const int i2 = spec(p + ".cv2");
      if (i2 < 0) return;
      const ConvSpec& c2s = M->def.convs[i2];
      f.a.w2 = wptr(c2s);
      f.a.b2 = bptr(c2s);
      f.a.out = (bf16_t*)ptr(o0.buf);
      f.a.out_cs = o0.cs;
      f.a.out_co = o0.co;
      const int cs_u = (2 + n) * c;  // cv2's Cin: the unfused concat width
      rec = args(c2s, View{cb, cs_u, 0}, li, o0, 0, View{-1, 0, 0}, 0, View{-1, 0, 0});
      trace(i2, rec, View{cb, cs_u, 0}, o0, 0, View{-1, 0, 0}, 0, View{-1, 0, 0});
      flops += flops_of(c2s, rec);
      M->fused.push_back(f);
      rec.fused = (int)M->fused.size();
      // algorithmic bytes: y0 + y1 read once, cv2's output written once,
      // every weight of the chain read once
      double wbytes = 0.0;
      for (int i = 0; i < n; ++i) wbytes += 2.0 * 2 * 9 * c * 32;
      wbytes += 2.0 * c2 * ((cs_u + 31) / 32 * 32);
      fused_bytes = (double)B * f.a.H * f.a.W * (2.0 * c * 2 + 2.0 * c2) + wbytes;
      launch(rec, i2, flops);
      return;
    }
    for (int i = 0; i < n; ++i) {
      const View bin{cb, cs, (1 + i) * c};
      const std::string q = p + ".m." + std::to_string(i);
      const int tmp = M->tmp_of(q);
      conv(q + ".cv1", bin, li, View{tmp, c, 0});
      conv(q + ".cv2", View{tmp, c, 0}, li, View{cb, cs, (2 + i) * c}, 0, {-1, 0, 0}, 0,
           shortcut ? bin : View{-1, 0, 0});
    }
    conv(p + ".cv2", View{cb, cs, 0}, li, o0, up0, o1, up1);
  }
};

}  // namespace rv

using namespace rv;

extern "C" int rv_yolo_num_convs(int variant) {
  ModelDef m;
  if (!build_def(variant, m)) return RV_EINVAL;
  return (int)m.convs.size();
}

extern "C" int rv_yolo_conv_info(int variant, int idx, int* info, char* name, int name_cap) {
  ModelDef m;
  RV_CHECK_ARG(build_def(variant, m), "unknown variant %d", variant);
  RV_CHECK_ARG(idx >= 0 && idx < (int)m.convs.size() && info, "bad conv index %d", idx);
  const ConvSpec& c = m.convs[idx];
  info[0] = c.cin;
  info[1] = c.cout;
  info[2] = c.k;
  info[3] = c.s;
  info[4] = c.act;
  if (name && name_cap > 0) {
    strncpy(name, c.name.c_str(), name_cap - 1);
    name[name_cap - 1] = 0;
  }
  return RV_OK;
}

extern "C" size_t rv_yolo_flat_floats(int variant) {
  ModelDef m;
  if (!build_def(variant, m)) return 0;
  return flat_floats(m);
}

extern "C" size_t rv_yolo_packed_bytes2(int variant, int dtype) {
  ModelDef m;
  if (!build_def(variant, m, dtype)) return 0;
  return packed_bytes(m);
}

extern "C" size_t rv_yolo_packed_bytes(int variant) {
  return rv_yolo_packed_bytes2(variant, RV_YOLO_DTYPE_BF16);
}

extern "C" float rv_fp8_scale(double amax) { return pow2_scale(amax); }

extern "C" int rv_yolo_pack(int variant, const float* flat, size_t n, void* host_out,
                            size_t out_bytes) {
  return rv_yolo_pack2(variant, RV_YOLO_DTYPE_BF16, flat, n, host_out, out_bytes);
}

extern "C" int rv_yolo_pack2(int variant, int dtype, const float* flat, size_t n, void* host_out,
                             size_t out_bytes) {
  ModelDef m;
  RV_CHECK_ARG(build_def(variant, m, dtype), "unknown variant %d / dtype %d", variant, dtype);
  RV_CHECK_ARG(flat && host_out, "null pointer");
  RV_CHECK_ARG(n == flat_floats(m), "flat weights: got %zu floats, need %zu", n, flat_floats(m));
  RV_CHECK_ARG(out_bytes >= packed_bytes(m), "packed buffer too small");
  uint8_t* out = (uint8_t*)host_out;
  memset(out, 0, packed_bytes(m));
  const float* p = flat;
  for (size_t i = 0; i < m.convs.size(); ++i) {
    const ConvSpec& c = m.convs[i];
    const size_t nw = (size_t)c.cout * c.cin * c.k * c.k;
    const float* w = p;
    const float* b = p + nw;
    p += nw + c.cout;
    if (i == 0) {
      memcpy(out + c.w_off, w, nw * 4);
      pack_conv0q(w, b, c.cout, out + m.q_off);
    } else if (c.f8) {
      // per output channel: scale = 2^ceil(log2(amax / 448)), codes RNE
      const int cip = (c.cin + 63) & ~63;
      const int kk = c.k * c.k;
      uint8_t* dst = out + c.w_off;
      float* wsc = (float*)(out + c.ws_off);
      for (int o = 0; o < c.cout; ++o) {
        double amax = 0.0;
        for (size_t j = 0; j < (size_t)c.cin * kk; ++j)
          amax = std::max(amax, (double)std::fabs(w[(size_t)o * c.cin * kk + j]));
        const float sc = pow2_scale(amax);
        wsc[o] = sc;
        for (int ky = 0; ky < c.k; ++ky)
          for (int kx = 0; kx < c.k; ++kx)
            for (int ci = 0; ci < c.cin; ++ci)
              dst[((size_t)o * kk + ky * c.k + kx) * cip + ci] =
                  host_f2e4m3(w[(((size_t)o * c.cin + ci) * c.k + ky) * c.k + kx] / sc);
      }
    } else {
      const int cip = (c.cin + 31) & ~31;
      uint16_t* dst = (uint16_t*)(out + c.w_off);
      for (int o = 0; o < c.cout; ++o)
        for (int ky = 0; ky < c.k; ++ky)
          for (int kx = 0; kx < c.k; ++kx)
            for (int ci = 0; ci < c.cin; ++ci)
              dst[((size_t)o * c.k * c.k + ky * c.k + kx) * cip + ci] =
                  host_f2bf(w[(((size_t)o * c.cin + ci) * c.k + ky) * c.k + kx]);
    }
    memcpy(out + c.b_off, b, (size_t)c.cout * 4);
  }
  return RV_OK;
}

extern "C" int rv_yolo_create(int variant, const void* dev_packed, int max_B, int in_h, int in_w,
                              void** handle) {
  return rv_yolo_create2(variant, RV_YOLO_DTYPE_BF16, dev_packed, max_B, in_h, in_w, handle);
}

extern "C" int rv_yolo_create2(int variant, int dtype, const void* dev_packed, int max_B, int in_h,
                               int in_w, void** handle) {
  RV_CHECK_ARG(handle && dev_packed, "null pointer");
  RV_CHECK_ARG(max_B > 0 && in_h > 0 && in_w > 0 && in_h % 32 == 0 && in_w % 32 == 0,
               "input %dx%d must be positive multiples of 32", in_h, in_w);
  Model* M = new Model();
  if (!build_def(variant, M->def, dtype)) {
    delete M;
    set_error("unknown variant %d / dtype %d", variant, dtype);
    return RV_EINVAL;
  }
  M->dev = (const uint8_t*)dev_packed;
  for (int i = 0; i < 2; ++i) {
    if (hipStreamCreateWithFlags(&M->side[i], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&M->ev_fork[i], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&M->ev_join[i], hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      M->side[0] = M->side[1] = nullptr;  // sequential heads
    }
  }
  M->max_B = max_B;
  M->H = in_h;
  M->W = in_w;
  plan(*M);
  M->act_scale.assign(M->bufs.size(), 1.0f);
  M->scales_set = dtype == RV_YOLO_DTYPE_BF16;
  *handle = M;
  return RV_OK;
}

extern "C" int rv_yolo_set_act_scales(void* h, const float* scales, int n) {
  RV_CHECK_ARG(h && scales, "null pointer");
  Model* M = (Model*)h;
  RV_CHECK_ARG(n == (int)M->bufs.size(), "got %d scales, the plan has %d buffers", n,
               (int)M->bufs.size());
  for (int i = 0; i < n; ++i) {
    if (M->bufs[i].esize != 1) continue;
    int e;
    const float f = std::frexp(scales[i], &e);
    RV_CHECK_ARG(scales[i] > 0.f && std::isfinite(scales[i]) && f == 0.5f,
                 "buffer %d: scale %g is not a positive power of two", i, (double)scales[i]);
  }
  for (int i = 0; i < n; ++i) M->act_scale[i] = M->bufs[i].esize == 1 ? scales[i] : 1.0f;
  M->scales_set = true;
  return RV_OK;
}

extern "C" int rv_yolo_buffer_name(void* h, int buf, char* name, int cap) {
  RV_CHECK_ARG(h && name && cap > 0, "bad args");
  Model* M = (Model*)h;
  RV_CHECK_ARG(buf >= 0 && buf < (int)M->bufs.size(), "bad buffer %d", buf);
  strncpy(name, M->buf_name[buf].c_str(), cap - 1);
  name[cap - 1] = 0;
  return RV_OK;
}

extern "C" int rv_yolo_buffer_esize(void* h, int buf) {
  RV_CHECK_ARG(h, "null handle");
  Model* M = (Model*)h;
  RV_CHECK_ARG(buf >= 0 && buf < (int)M->bufs.size(), "bad buffer %d", buf);
  return M->bufs[buf].esize;
}

extern "C" int rv_yolo_destroy(void* h) {
  delete (Model*)h;
  return RV_OK;
}

extern "C" int rv_yolo_set_option(void* h, int opt, int value) {
  RV_CHECK_ARG(h, "null handle");
  Model* M = (Model*)h;
  switch (opt) {
    case RV_YOLO_OPT_RAW_UNFUSED:
      M->raw_unfused = value != 0;
      return RV_OK;
    case RV_YOLO_OPT_FUSE_C2F:
      M->fuse_c2f = value < 0 ? 0 : (value > 2 ? 2 : value);
      return RV_OK;
    case RV_YOLO_OPT_STEM_X1:
      M->stem_x1 = value != 0;
      return RV_OK;
    case RV_YOLO_OPT_HEAD_STREAMS:
      M->head_streams = value != 0;
      return RV_OK;
    case RV_YOLO_OPT_FUSE_CV1:
      M->fuse_cv1 = value != 0;
      return RV_OK;
    case RV_YOLO_OPT_HEAD_CHAIN:
      M->head_chain = value != 0;
      return RV_OK;
    case RV_YOLO_OPT_C2F_TAP_PAIRS:
      M->c2f_tap_pairs = value != 0;
      return RV_OK;
    default:
      set_error("unknown yolo option %d", opt);
      return RV_EINVAL;
  }
}

extern "C" size_t rv_yolo_ws_bytes(void* h, int B) {
  if (!h || B <= 0) return 0;
  return ((Model*)h)->ws_bytes(B);
}

extern "C" int rv_yolo_num_anchors(void* h) { return h ? ((Model*)h)->nA : 0; }

extern "C" int rv_yolo_cand_segments(void* h) {
  if (!h) return 0;
  const Model* M = (const Model*)h;
  HeadLevel hl[3];
  for (int i = 0; i < 3; ++i) {
    hl[i].H = M->map_h[3 + i];
    hl[i].W = M->map_w[3 + i];
  }
  return decode_segments(hl, 3);
}

extern "C" int rv_yolo_forward_part(void* h, const uint8_t* lb, int B, void* ws, size_t ws_bytes,
                                    float* raw_out, float conf, void* cand, int cand_cap,
                                    int* cand_n, void* stream, int part);

extern "C" int rv_yolo_forward(void* h, const uint8_t* lb, int B, void* ws, size_t ws_bytes,
                               float* raw_out, float conf, void* cand, int cand_cap, int* cand_n,
                               void* stream) {
  return rv_yolo_forward_part(h, lb, B, ws, ws_bytes, raw_out, conf, cand, cand_cap, cand_n, stream,
                              0);
}

// part 0: the whole forward.  part 1: stem .. model.15 (the backbone and the
// top-down neck: the bandwidth-heavy P2/P3 layers).  part 2: the rest (the
// bottom-up neck, the Detect heads and the decode: small latency-bound
// launches), reading part 1's activations from the same workspace.  A
// pipelined caller with two workspaces runs part 2 of step j-1 beside
// part 1 of step j.
extern "C" int rv_yolo_forward_part(void* h, const uint8_t* lb, int B, void* ws, size_t ws_bytes,
                                    float* raw_out, float conf, void* cand, int cand_cap,
                                    int* cand_n, void* stream, int part) {
  RV_CHECK_ARG(h && ws && (lb || part == 2 || part == 4), "null pointer");
  RV_CHECK_ARG(part >= 0 && part <= 4, "part %d not in {0, 1, 2, 3, 4}", part);
  Model* M = (Model*)h;
  RV_CHECK_ARG(part != 4 || M->n_part1a >= 0, "forward part 4 before any part 3 of this handle");
  RV_CHECK_ARG(part != 4 || (B == M->part1a_B && ws == M->part1a_ws),
               "forward part 4 (B=%d, ws %p) does not continue the last part 3 of this handle "
               "(B=%d, ws %p)", B, ws, M->part1a_B, M->part1a_ws);
  RV_CHECK_ARG(part != 2 || M->n_part1 >= 0,
               "forward part 2 before any part 0 / part 1 forward of this handle");
  RV_CHECK_ARG(part != 2 || (B == M->part1_B && ws == M->part1_ws),
               "forward part 2 (B=%d, ws %p) does not continue the last part 1 of this handle "
               "(B=%d, ws %p)", B, ws, M->part1_B, M->part1_ws);
  RV_CHECK_ARG((part != 1 && part != 3 && part != 4) || !raw_out,
               "raw_out needs the whole forward (part 0)");
  RV_CHECK_ARG(B > 0 && B <= M->max_B, "B=%d outside (0, %d]", B, M->max_B);
  RV_CHECK_ARG(ws_bytes >= M->ws_bytes(B), "workspace %zu < %zu bytes", ws_bytes, M->ws_bytes(B));
  RV_CHECK_ARG(!cand || (cand_n && cand_cap > 0), "candidate buffers incomplete");
  RV_CHECK_ARG(M->scales_set, "fp8 plan: activation scales not set (rv_yolo_set_act_scales)");
  const Variant& v = M->def.v;
  const bool f8 = M->def.dtype == RV_YOLO_DTYPE_FP8;
  Exec E;
  E.M = M;
  E.ws = (uint8_t*)ws;
  E.B = B;
  E.s = as_stream(stream);
  size_t off = 0;
  for (const Buf& b : M->bufs) {
    E.off.push_back(off);
    off = (off + b.elems_per_img * B * b.esize + 255) & ~(size_t)255;
  }
  M->trace.clear();
  M->launches.clear();
  M->fused.clear();
  M->li_base = part == 2 ? M->n_part1 : (part == 4 ? M->n_part1a : 0);
  // fused C2f chains (c2f.hip) unless a raw parity forward keeps every
  // activation (RV_YOLO_OPT_RAW_UNFUSED) or RV_FUSE_C2F=0
  static const bool c2f_env = !getenv("RV_FUSE_C2F") || atoi(getenv("RV_FUSE_C2F")) != 0;
  const bool fuse_c2f = c2f_env && !f8 && M->fuse_c2f && !(raw_out && M->raw_unfused);
  // the hidden-width-32 chains (model.4, model.15 of YOLOv8n) measured
  // faster unfused since the patch kernel's buffer-DMA / fast-epilogue work
  // (r03: 188 + 86 us per 128-frame unit fused, 142 + 79 unfused): only
  // the C = 16 chain (model.2 at P2, 122 fused vs 191 unfused) stays fused
  // unless RV_FUSE_C2F32=1 or RV_YOLO_OPT_FUSE_C2F = 2
  static const bool c2f32_env = getenv("RV_FUSE_C2F32") && atoi(getenv("RV_FUSE_C2F32")) != 0;
  const bool fuse_c2f32 = fuse_c2f && (c2f32_env || M->fuse_c2f == 2);
  const int cat14 = v.h12 + v.c3, cat11 = v.c5 + v.c4, cat20 = v.h18 + v.c5,
            cat17 = v.h15 + v.h12;
  // The neck's two Upsample + Concat pairs (yolov8.yaml layers 10-11 and
  // 13-14): bf16 plans read the upsampled half of model.12.cv1's and
  // model.15.cv1's input straight from the half-resolution map (a virtual
  // concat, ConvArgs::split / in_up), so the 4x upsampled copies are never
  // written; fp8 plans (patch kernel only) and RV_VCAT=0 materialise them
  // into CAT11[0, c5) / CAT14[0, h12) as before.
  static const bool vcat_env = !getenv("RV_VCAT") || atoi(getenv("RV_VCAT")) != 0;
  const bool vcat = vcat_env && !f8;
  const View none{-1, 0, 0};
  const VIn vin12{View{M->CAT20, cat20, v.h18}, 1, View{M->CAT11, cat11, v.c5}, v.c5};
  const VIn vin15{View{M->CAT17, cat17, v.h15}, 1, View{M->CAT14, cat14, v.h12}, v.h12};
  auto c2f12 = [&]() {
    E.c2f("model.12", View{M->CAT11, cat11, 0}, 4, M->C12, v.h12, v.nb, false,
          View{M->CAT17, cat17, v.h15}, 0, vcat ? none : View{M->CAT14, cat14, 0}, vcat ? 0 : 1,
          false, false, vcat ? &vin12 : nullptr);
  };
  auto c2f15 = [&]() {
    E.c2f("model.15", View{M->CAT14, cat14, 0}, 3, M->C15, v.h15, v.nb, false,
          View{M->X15, v.h15, 0}, 0, View{-1, 0, 0}, 0, v.h15 / 2 == 16 ? fuse_c2f : fuse_c2f32,
          false, vcat ? &vin15 : nullptr);
  };
  // where part 1 ends (parts 1 / 4 vs part 2): after model.15 (15, default),
  // model.12 (12) or SPPF (9) (RV_FWD_SPLIT).  Part 1 is the busier half
  // (its stream 70 % busy against 45 % in the r04 trace), but moving the
  // top-down neck's C2f blocks into part 2 measured slower (three A/B
  // triples, r04: 44.6-45.1k at 15, 43.9-45.2k at 12, 43.6-44.7k at 9)
  static const int split = getenv("RV_FWD_SPLIT") ? atoi(getenv("RV_FWD_SPLIT")) : 15;
  int st;
  if (part != 2) {
  if (part != 4) {  // part 4 continues after model.2
  // backbone
  const ConvSpec& c0 = M->def.convs[0];
  const uint8_t* qb = M->dev + M->def.q_off;
  const float* qs = (const float*)(qb + 3 * (size_t)c0.cout * 64);
  const Conv0Q q0{(const int8_t*)qb, qs, qs + c0.cout, (const int32_t*)(qs + 2 * c0.cout)};
  // conv0 + model.1 fused (the P1 map stays in LDS) unless the caller asked
  // for the raw prediction with RV_YOLO_OPT_RAW_UNFUSED set (layer parity
  // forwards keep every activation in the workspace) or RV_FUSE_STEM=0
  static const bool stem_env = !getenv("RV_FUSE_STEM") || atoi(getenv("RV_FUSE_STEM")) != 0;
  const int i1 = M->def.find("model.1");
  const bool fuse_stem =
      stem_env && !f8 && !(raw_out && M->raw_unfused) && c0.cout == 16 && v.c2 == 32 && i1 >= 0;
  // the fused stem also runs model.2.cv1 (32 -> 32 1x1) from its registers
  // into the model.2 concat buffer when the shapes allow
  const int i2cv1 = M->def.find("model.2.cv1");
  const int c2cs = E.c2f_will_fuse(v.c2 / 2, v.nb, fuse_c2f, 0, View{-1, 0, 0}, View{M->X2, v.c2, 0})
                       ? v.c2
                       : (2 + v.nb) * (v.c2 / 2);
  const bool stem_cv1 = fuse_stem && i2cv1 >= 0 && M->def.convs[i2cv1].cin == 32 &&
                        M->def.convs[i2cv1].cout == 32 && M->def.convs[i2cv1].k == 1;
  if (fuse_stem) {
    const ConvSpec& c1 = M->def.convs[i1];
    const View none{-1, 0, 0};
    E.trace(i1, E.args(c1, View{M->X0, v.c1, 0}, 1, View{M->X1, v.c2, 0}, 0, none, 0, none),
            View{M->X0, v.c1, 0}, View{M->X1, v.c2, 0}, 0, none, 0, none);
    const ConvSpec* cv = stem_cv1 ? &M->def.convs[i2cv1] : nullptr;
    if (cv)
      E.trace(i2cv1, E.args(*cv, View{M->X1, v.c2, 0}, 2, View{M->C2, c2cs, 0}, 0, none, 0, none),
              View{M->X1, v.c2, 0}, View{M->C2, c2cs, 0}, 0, none, 0, none);
    // the stem is timed with the conv launches (profile slot per_fwd - 1,
    // which no conv launch index reaches: a forward has fewer launches than
    // convs)
    Profile& P = M->prof;
    const int slot = P.per_fwd - 1;
    const bool rec = P.on && P.n_fwd < P.cap_fwd && slot >= 0;
    const bool x1_out = !cv || M->stem_x1;
    if (rec) {
      const double px0 = (double)B * M->map_h[1] * M->map_w[1];
      const double px1 = (double)B * M->map_h[2] * M->map_w[2];
      P.flops[slot] = 2.0 * px0 * c0.cout * 27 + 2.0 * px1 * c1.cout * c1.cin * 9 +
                      (cv ? 2.0 * px1 * cv->cout * cv->cin : 0.0);
      // letterbox read once, X1 / the cv1 slice written once, weights once
      P.bytes[slot] = (double)B * M->H * M->W * 3 + px1 * 2.0 * (x1_out ? c1.cout : 0) +
                      (cv ? px1 * 2.0 * cv->cout : 0.0) + M->def.q_bytes + 2.0 * c1.cout * 9 * 32 +
                      (cv ? 2.0 * cv->cout * 32 : 0.0);
      P.conv_of[slot] = 0;
      st = hip_check(hipEventRecord(P.ev[((size_t)P.n_fwd * P.per_fwd + slot) * 2], E.s),
                     "profile hipEventRecord");
      if (st) return st;
    }
    for (int r = 0; r < (rec ? P.reps : 1); ++r) {
      st = launch_stem(lb, B, M->H, M->W, q0, c0.cout, E.wptr(c1), E.bptr(c1), c1.cout,
                       x1_out ? (bf16_t*)E.ptr(M->X1) : nullptr, v.c2, E.s,
                       cv ? E.wptr(*cv) : nullptr, cv ? E.bptr(*cv) : nullptr,
                       cv ? (bf16_t*)E.ptr(M->C2) : nullptr, c2cs);
      if (st) return st;
    }
    if (rec) {
      st = hip_check(hipEventRecord(P.ev[((size_t)P.n_fwd * P.per_fwd + slot) * 2 + 1], E.s),
                     "profile hipEventRecord");
      if (st) return st;
    }
  } else {
    st = f8 ? launch_conv0_fp8(lb, B, M->H, M->W, q0, c0.cout, (uint8_t*)E.ptr(M->X0), v.c1,
                               E.scale(M->X0), E.s)
            : launch_conv0(lb, B, M->H, M->W, q0, c0.cout, (bf16_t*)E.ptr(M->X0), v.c1, E.s);
    if (st) return st;
    E.conv("model.1", View{M->X0, v.c1, 0}, 1, View{M->X1, v.c2, 0});
  }
  E.c2f("model.2", View{M->X1, v.c2, 0}, 2, M->C2, v.c2, v.nb, true, View{M->X2, v.c2, 0}, 0,
        View{-1, 0, 0}, 0, fuse_c2f, stem_cv1);
  if (E.status) return E.status;
  if (part == 3) {  // the stem and model.2: the VALU-heavy start of part 1
    M->n_part1a = M->li_base + (int)M->launches.size();
    M->part1a_B = B;
    M->part1a_ws = ws;
    // part 3 rewrote the start of the workspace: a part 2 now needs the part 4
    // that finishes this forward, not the part 1 of an earlier one
    M->n_part1 = -1;
    M->part1_B = 0;
    M->part1_ws = nullptr;
    return RV_OK;
  }
  }  // part != 4
  // model.3 + model.4.cv1 in one launch (the chained 1x1: model.3's output
  // map is only ever read by model.4.cv1) unless a raw parity forward keeps
  // every activation (RV_YOLO_OPT_RAW_UNFUSED), RV_YOLO_OPT_FUSE_CV1 = 0 or
  // RV_FUSE_CV1=0
  {
    static const bool cv1_env = !getenv("RV_FUSE_CV1") || atoi(getenv("RV_FUSE_CV1")) != 0;
    const bool f4 = v.c3 / 2 == 16 ? fuse_c2f : fuse_c2f32;
    const int c4 = v.c3 / 2;
    const int c4cs = E.c2f_will_fuse(c4, v.nm, f4, 0, View{-1, 0, 0}, View{M->CAT14, cat14, v.h12})
                         ? 2 * c4
                         : (2 + v.nm) * c4;
    const bool chained = cv1_env && M->fuse_cv1 && !f8 && !(raw_out && M->raw_unfused) &&
                         E.conv_chain("model.3", View{M->X2, v.c2, 0}, 2, View{M->X3, v.c3, 0},
                                      "model.4.cv1", View{M->C4, c4cs, 0});
    if (!chained) E.conv("model.3", View{M->X2, v.c2, 0}, 2, View{M->X3, v.c3, 0});
    E.c2f("model.4", View{M->X3, v.c3, 0}, 3, M->C4, v.c3, v.nm, true,
          View{M->CAT14, cat14, v.h12}, 0, View{-1, 0, 0}, 0, f4, chained);
  }
  E.conv("model.5", View{M->CAT14, cat14, v.h12}, 3, View{M->X5, v.c4, 0});
  E.c2f("model.6", View{M->X5, v.c4, 0}, 4, M->C6, v.c4, v.nm, true,
        View{M->CAT11, cat11, v.c5});
  E.conv("model.7", View{M->CAT11, cat11, v.c5}, 4, View{M->X7, v.c5, 0});
  E.c2f("model.8", View{M->X7, v.c5, 0}, 5, M->C8, v.c5, v.nb, true, View{M->X8, v.c5, 0});
  // SPPF
  const int sc = v.c5 / 2;
  E.conv("model.9.cv1", View{M->X8, v.c5, 0}, 5, View{M->SP, 4 * sc, 0});
  if (E.status) return E.status;
  st = f8 ? launch_sppf_pool_fp8((uint8_t*)E.ptr(M->SP), B, M->map_h[5], M->map_w[5], sc, E.s)
          : launch_sppf_pool((bf16_t*)E.ptr(M->SP), B, M->map_h[5], M->map_w[5], sc, E.s);
  if (st) return st;
  E.conv("model.9.cv2", View{M->SP, 4 * sc, 0}, 5, View{M->CAT20, cat20, v.h18}, 0,
         vcat ? none : View{M->CAT11, cat11, 0}, vcat ? 0 : 1);
  // head
  if (split >= 12) c2f12();
  if (split >= 15) c2f15();
  if (E.status) return E.status;
  M->n_part1 = M->li_base + (int)M->launches.size();
  M->part1_B = B;
  M->part1_ws = ws;
  if (part == 1 || part == 4) return RV_OK;
  }  // part != 2
  // the top-down neck's C2f blocks after the split run at the start of part 2
  if (split < 12) c2f12();
  if (split < 15) c2f15();
  if (E.status) return E.status;
  // Detect head of level i: box (cv2) and class (cv3) branches, one grouped
  // launch per stage; the last 1x1 stage runs inside the decode kernel
  // (RV_FUSE_HEAD=0: separate launches and f32 logits in HBM).  The P3 and
  // P4 heads are forked onto side streams as soon as their input map exists,
  // so they overlap the rest of the neck (small, latency-bound launches);
  // RV_YOLO_OPT_HEAD_STREAMS = 0 (a pipelined caller: its stages already
  // overlap, and two more streams per handle share the process's 4 hardware
  // queues -- r04: +3 % in the pipeline with the heads on the caller's
  // stream) or RV_HEAD_STREAMS=0 / 1 (overrides) keeps everything on the
  // caller's stream.
  const View P[3] = {View{M->X15, v.h15, 0}, View{M->X18, v.h18, 0}, View{M->X21, v.h21, 0}};
  const int dcs = v.c2d + v.c3d, hcs = 4 * v.reg + v.nc;
  static const bool fuse_env = !getenv("RV_FUSE_HEAD") || atoi(getenv("RV_FUSE_HEAD")) != 0;
  const bool fuse_head = fuse_env && v.c2d % 8 == 0 && v.c3d % 8 == 0;
  static const int streams_env = getenv("RV_HEAD_STREAMS") ? atoi(getenv("RV_HEAD_STREAMS")) != 0 : -1;
  const bool streams_on = streams_env >= 0 ? streams_env != 0 : M->head_streams != 0;
  // profiled forwards time every launch alone (per-launch roofline), so the
  // heads stay on the caller's stream there; so do batches under 8, whose
  // few-us head launches gain less from the overlap than the fork / join
  // event round trips cost (batch 1, r05: 0.356 -> 0.308 ms device time per
  // forward, launch submission 284 -> 218 us, tools/c2_host.py)
  const bool fork = streams_on && B >= 8 && M->side[0] && M->side[1] &&
                    !(M->prof.on && M->prof.n_fwd < M->prof.cap_fwd);
  const hipStream_t main_s = E.s;
  // The chained head (RV_YOLO_OPT_HEAD_CHAIN; RV_HEAD_CHAIN=0/1 overrides):
  // each branch's .1 conv runs its .2 1x1 on the tile in LDS and keeps only
  // the DFL distances (box) / the best (score, class) (class), and one small
  // kernel (head_combine_kernel) forms the candidates -- the DB features and
  // the f32 logits never reach HBM.  Candidate forwards of the bf16
  // YOLOv8n-shaped head only (raw forwards keep the decode kernel); the same
  // candidates as the fixed decode.
  static const int chain_env = getenv("RV_HEAD_CHAIN") ? atoi(getenv("RV_HEAD_CHAIN")) : -1;
  bool hchain = (chain_env < 0 ? M->head_chain != 0 : chain_env != 0) && !f8 && fuse_head && !raw_out && cand && v.nc == 80 &&
                v.reg == 16 && v.c2d == 64 && v.c3d == 80;
  for (int i = 0; i < 3 && hchain; ++i) {
    const std::string a = "model.22.cv2." + std::to_string(i), c = "model.22.cv3." + std::to_string(i);
    hchain = E.head_chain(a + ".1", View{M->DA[i], dcs, 0}, 3 + i, View{M->DB[i], dcs, 0}, a + ".2",
                          View{M->BX[i], 4, 0}, 2, true) &&
             E.head_chain(c + ".1", View{M->DA[i], dcs, v.c2d}, 3 + i, View{M->DB[i], dcs, v.c2d},
                          c + ".2", View{M->SC[i], 2, 0}, 3, true);
  }
  auto head_level = [&](int i) {
    const std::string a = "model.22.cv2." + std::to_string(i), c = "model.22.cv3." + std::to_string(i);
    E.conv_pair(a + ".0", P[i], c + ".0", P[i], 3 + i, View{M->DA[i], dcs, 0});
    if (hchain) {
      E.head_chain(a + ".1", View{M->DA[i], dcs, 0}, 3 + i, View{M->DB[i], dcs, 0}, a + ".2",
                   View{M->BX[i], 4, 0}, 2, false);
      E.head_chain(c + ".1", View{M->DA[i], dcs, v.c2d}, 3 + i, View{M->DB[i], dcs, v.c2d}, c + ".2",
                   View{M->SC[i], 2, 0}, 3, false);
      return E.status;
    }
    E.conv_pair(a + ".1", View{M->DA[i], dcs, 0}, c + ".1", View{M->DA[i], dcs, v.c2d}, 3 + i,
                View{M->DB[i], dcs, 0});
    if (!fuse_head) {
      E.conv_pair(a + ".2", View{M->DB[i], dcs, 0}, c + ".2", View{M->DB[i], dcs, v.c2d}, 3 + i,
                  View{M->HD[i], hcs, 0});
    } else {  // run inside the decode kernel; trace records keep the layer list complete
      const View none{-1, 0, 0};
      const int ia = E.spec(a + ".2"), ic = E.spec(c + ".2");
      if (ia < 0 || ic < 0) return E.status;
      const ConvSpec& sa = M->def.convs[ia];
      const ConvSpec& sc = M->def.convs[ic];
      E.trace(ia, E.args(sa, View{M->DB[i], dcs, 0}, 3 + i, View{M->HD[i], hcs, 0}, 0, none, 0, none),
              View{M->DB[i], dcs, 0}, View{M->HD[i], hcs, 0}, 0, none, 0, none);
      E.trace(ic, E.args(sc, View{M->DB[i], dcs, v.c2d}, 3 + i, View{M->HD[i], hcs, 4 * v.reg}, 0,
                         none, 0, none),
              View{M->DB[i], dcs, v.c2d}, View{M->HD[i], hcs, 4 * v.reg}, 0, none, 0, none);
    }
    return E.status;
  };
  auto forked_head = [&](int i) {  // level i's head on side stream i (joined before decode)
    if (!fork) return head_level(i);
    int e = hip_check(hipEventRecord(M->ev_fork[i], main_s), "head fork hipEventRecord");
    if (!e) e = hip_check(hipStreamWaitEvent(M->side[i], M->ev_fork[i], 0), "head fork wait");
    if (e) return E.status = e;
    E.s = M->side[i];
    const int r = head_level(i);
    e = hip_check(hipEventRecord(M->ev_join[i], M->side[i]), "head join hipEventRecord");
    E.s = main_s;
    if (!r && e) E.status = e;
    return r ? r : e;
  };
  if (E.status || forked_head(0)) return E.status;
  E.conv("model.16", View{M->X15, v.h15, 0}, 3, View{M->CAT17, cat17, 0});
  E.c2f("model.18", View{M->CAT17, cat17, 0}, 4, M->C18, v.h18, v.nb, false,
        View{M->X18, v.h18, 0});
  if (E.status || forked_head(1)) return E.status;
  E.conv("model.19", View{M->X18, v.h18, 0}, 4, View{M->CAT20, cat20, 0});
  E.c2f("model.21", View{M->CAT20, cat20, 0}, 5, M->C21, v.h21, v.nb, false,
        View{M->X21, v.h21, 0});
  if (E.status || head_level(2)) return E.status;
  if (fork)
    for (int i = 0; i < 2 && !E.status; ++i)
      E.status = hip_check(hipStreamWaitEvent(main_s, M->ev_join[i], 0), "head join wait");
  if (E.status) return E.status;
  if (M->prof.on && M->prof.n_fwd < M->prof.cap_fwd) M->prof.n_fwd++;
  if (hchain) {
    HeadCombine hc;
    memset(&hc, 0, sizeof(hc));
    hc.nlv = 3;
    for (int i = 0; i < 3; ++i) {
      hc.bx[i] = (const float*)E.ptr(M->BX[i]);
      hc.sc[i] = (const float*)E.ptr(M->SC[i]);
      hc.H[i] = M->map_h[3 + i];
      hc.W[i] = M->map_w[3 + i];
      hc.stride[i] = (float)(8 << i);
      hc.start[i + 1] = hc.start[i] + hc.H[i] * hc.W[i];
      hc.blk[i + 1] = hc.blk[i] + ceil_div(hc.H[i] * hc.W[i], 64);
    }
    return launch_head_combine(hc, B, conf, (Cand*)cand, cand_cap, cand_n, E.s);
  }
  HeadLevel hl[3];
  memset(hl, 0, sizeof(hl));
  for (int i = 0; i < 3; ++i) {
    hl[i].logits = (const float*)E.ptr(M->HD[i]);
    hl[i].H = M->map_h[3 + i];
    hl[i].W = M->map_w[3 + i];
    hl[i].cs = hcs;
    hl[i].stride = (float)(8 << i);
    if (fuse_head) {
      const ConvSpec& sa = M->def.convs[M->def.find("model.22.cv2." + std::to_string(i) + ".2")];
      const ConvSpec& sc = M->def.convs[M->def.find("model.22.cv3." + std::to_string(i) + ".2")];
      hl[i].feat = (const bf16_t*)E.ptr(M->DB[i]);
      hl[i].feat_cs = dcs;
      hl[i].cin_b = sa.cin;
      hl[i].cin_c = sc.cin;
      hl[i].w_box = E.wptr(sa);
      hl[i].w_cls = E.wptr(sc);
      hl[i].b_box = E.bptr(sa);
      hl[i].b_cls = E.bptr(sc);
      hl[i].logits_out = raw_out ? (float*)E.ptr(M->HD[i]) : nullptr;
    }
  }
  return launch_detect_decode(hl, 3, B, v.nc, v.reg, conf, raw_out, (Cand*)cand, cand_cap, cand_n,
                              E.s);
}

// ---- introspection (parity tests / debugging) ------------------------------
extern "C" int rv_yolo_num_buffers(void* h) { return h ? (int)((Model*)h)->bufs.size() : 0; }

extern "C" int rv_yolo_buffer_info(void* h, int B, int buf, int* info, size_t* off_bytes) {
  RV_CHECK_ARG(h && info && off_bytes && B > 0, "bad args");
  Model* M = (Model*)h;
  RV_CHECK_ARG(buf >= 0 && buf < (int)M->bufs.size(), "bad buffer %d", buf);
  size_t off = 0;
  for (int i = 0; i < buf; ++i)
    off = (off + M->bufs[i].elems_per_img * B * M->bufs[i].esize + 255) & ~(size_t)255;
  *off_bytes = off;
  info[0] = M->buf_h[buf];
  info[1] = M->buf_w[buf];
  info[2] = M->buf_c[buf];
  info[3] = M->bufs[buf].f32 ? 1 : 0;
  return RV_OK;
}

// 20 ints per conv launch of the last forward; returns the record count
extern "C" int rv_yolo_trace(void* h, int* recs, int max_recs) {
  if (!h) return RV_EINVAL;
  Model* M = (Model*)h;
  const int n = (int)M->trace.size();
  if (recs)
    for (int i = 0; i < n && i < max_recs; ++i) memcpy(recs + 24 * i, &M->trace[i], 24 * sizeof(int));
  return n;
}

// ---- live conv timing ------------------------------------------------------
extern "C" int rv_yolo_profile_reps(void* h, int max_forwards, int reps) {
  RV_CHECK_ARG(h && max_forwards >= 0 && reps >= 1, "bad args");
  Model* M = (Model*)h;
  Profile& P = M->prof;
  P.reps = reps;
  for (hipEvent_t e : P.ev) (void)hipEventDestroy(e);  // teardown
  P.ev.clear();
  P.on = max_forwards > 0;
  P.n_fwd = 0;
  P.cap_fwd = max_forwards;
  P.per_fwd = (int)M->def.convs.size();
  P.flops.assign(P.per_fwd, 0.0);
  P.bytes.assign(P.per_fwd, 0.0);
  P.conv_of.assign(P.per_fwd, -1);
  if (!P.on) return RV_OK;
  P.ev.resize((size_t)P.cap_fwd * P.per_fwd * 2);
  for (auto& e : P.ev)
    if (hipEventCreate(&e) != hipSuccess) {
      set_error("hipEventCreate failed");
      return RV_EINVAL;
    }
  return RV_OK;
}

extern "C" int rv_yolo_profile(void* h, int max_forwards) {
  return rv_yolo_profile_reps(h, max_forwards, 1);
}

// After the profiled forwards (synchronises): per conv launch index i,
// ms[i] = total device time over the recorded forwards, flops[i] =
// algorithmic FLOPs of ONE launch, conv[i] = conv spec index.  Returns the
// number of recorded forwards.
extern "C" int rv_yolo_profile_read(void* h, double* ms, double* flops, int* conv, int n) {
  RV_CHECK_ARG(h && ms && flops && conv, "bad args");
  Model* M = (Model*)h;
  Profile& P = M->prof;
  if (!P.on) return 0;
  for (int i = 0; i < n && i < P.per_fwd; ++i) {
    double tot = 0.0;
    for (int f = 0; f < P.n_fwd; ++f) {
      float t = 0.f;
      hipEvent_t a = P.ev[((size_t)f * P.per_fwd + i) * 2], b = P.ev[((size_t)f * P.per_fwd + i) * 2 + 1];
      if (P.conv_of[i] >= 0 && hipEventSynchronize(b) == hipSuccess &&
          hipEventElapsedTime(&t, a, b) == hipSuccess)
        tot += t;
    }
    ms[i] = tot / P.reps;
    flops[i] = P.flops[i];
    conv[i] = P.conv_of[i];
  }
  return P.n_fwd;
}

// After the profiled forwards (synchronises): the [start, end) interval of
// every recorded conv launch of handle h, in ms after the first recorded
// event of handle `ref` (forward 0; ref may be h).  Handles of one device
// share the clock, so the intervals of several forward contexts (lanes)
// can be merged into the chip-wide busy time of the conv family.  Writes
// at most n pairs; returns the number of intervals.
extern "C" int rv_yolo_profile_times(void* h, void* ref, double* t0, double* t1, int n) {
  RV_CHECK_ARG(h && ref && (n == 0 || (t0 && t1)), "bad args");
  Model* M = (Model*)h;
  const Profile& P = M->prof;
  const Profile& R = ((Model*)ref)->prof;
  if (!P.on || !R.on || R.n_fwd == 0) return 0;
  hipEvent_t e0 = nullptr;
  for (int i = 0; i < R.per_fwd && !e0; ++i)
    if (R.conv_of[i] >= 0) e0 = R.ev[(size_t)i * 2];
  if (!e0) return 0;
  int k = 0;
  for (int f = 0; f < P.n_fwd; ++f)
    for (int i = 0; i < P.per_fwd; ++i) {
      if (P.conv_of[i] < 0) continue;
      hipEvent_t a = P.ev[((size_t)f * P.per_fwd + i) * 2], b = P.ev[((size_t)f * P.per_fwd + i) * 2 + 1];
      float ta = 0.f, tb = 0.f;
      if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ta, e0, a) != hipSuccess ||
          hipEventElapsedTime(&tb, e0, b) != hipSuccess) {
        (void)hipGetLastError();
        set_error("rv_yolo_profile_times: event query failed");
        return RV_EINVAL;
      }
      if (k < n) {
        t0[k] = ta;
        t1[k] = tb;
      }
      ++k;
    }
  return k;
}

// ---- per-layer autotuning ---------------------------------------------------
namespace rv {

// Bytes of the buffer an output view lives in (the view's base pointer is
// the buffer start): B x (2x upsampled) rows x channel stride x element.
static size_t out_bytes(const ConvArgs& a, int d) {
  const void* p = d == 0 ? a.out0 : a.out1;
  if (!p) return 0;
  const int up = d == 0 ? a.out0_up : a.out1_up;
  const int cs = d == 0 ? a.out0_cs : a.out1_cs;
  const int o8 = d == 0 ? a.out0_8 : a.out1_8;
  return (size_t)a.B * a.Ho * a.Wo * (up ? 4 : 1) * cs * (a.out_f32 ? 4 : (o8 ? 1 : 2));
}

__global__ void count_diff_kernel(const uint32_t* __restrict__ x, const uint32_t* __restrict__ y,
                                  size_t n, unsigned* __restrict__ cnt) {
  unsigned c = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    c += x[i] != y[i];
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

}  // namespace rv

// Time every valid kernel configuration of every conv launch of a forward on
// this input (the activations of one default forward, so every launch sees
// its real operands) and keep the fastest per launch index for later
// forwards of this handle.  Synchronous; not capturable.  verify != 0 also
// compares each configuration's output buffers with the default's (all
// configurations accumulate in the same k order, so they must be bit-equal);
// *n_bad = configurations that differed.
extern "C" int rv_yolo_autotune(void* h, const uint8_t* lb, int B, void* ws, size_t ws_bytes,
                                int reps, int verify, int* n_bad, void* stream) {
  RV_CHECK_ARG(h && lb && ws, "null pointer");
  Model* M = (Model*)h;
  hipStream_t s = as_stream(stream);
  reps = reps < 1 ? 1 : reps;
  M->tuned.clear();
  int st = rv_yolo_forward(h, lb, B, ws, ws_bytes, nullptr, 1.0f, nullptr, 0, nullptr, stream);
  if (st) return st;
  const std::vector<ConvArgs> L = M->launches;
  std::vector<ConvCfg> best(L.size(), ConvCfg{0, 0, 0, 0, 0});
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
    set_error("hipEventCreate failed");
    return RV_EINVAL;
  }
  size_t maxb = 0;
  for (const ConvArgs& a : L) maxb = std::max(maxb, std::max(out_bytes(a, 0), out_bytes(a, 1)));
  uint8_t* ref = nullptr;
  unsigned* cnt = nullptr;
  if (verify && (hipMalloc((void**)&ref, 2 * maxb) != hipSuccess ||
                 hipMalloc((void**)&cnt, sizeof(unsigned)) != hipSuccess)) {
    set_error("autotune: hipMalloc of %zu verification bytes failed", 2 * maxb);
    st = RV_EINVAL;
  }
  int bad = 0;
  static const int dbg = getenv("RV_CONV_DEBUG") ? atoi(getenv("RV_CONV_DEBUG")) : 0;
  std::vector<ConvCfg> cands(512);
  for (size_t i = 0; i < L.size() && !st; ++i) {
    const ConvArgs& a = L[i];
    if (a.fused > 0) continue;  // fused C2f chains have one kernel configuration
    if (verify)
      for (int d = 0; d < 2; ++d)
        if (out_bytes(a, d))
          if (!st)
            st = hip_check(hipMemcpyAsync(ref + d * maxb, d == 0 ? a.out0 : a.out1,
                                          out_bytes(a, d), hipMemcpyDeviceToDevice, s),
                           "autotune reference copy");
    auto time_cfg = [&](const ConvCfg* c) -> float {
      int r = c ? launch_conv_cfg(a, *c, s) : launch_conv(a, s);  // warm-up launch
      if (!r) r = hip_check(hipEventRecord(e0, s), "autotune hipEventRecord");
      for (int k = 0; k < reps && !r; ++k) r = c ? launch_conv_cfg(a, *c, s) : launch_conv(a, s);
      if (!r) r = hip_check(hipEventRecord(e1, s), "autotune hipEventRecord");
      if (r || hipEventSynchronize(e1) != hipSuccess) {
        if (!st) st = r ? r : RV_EINVAL;
        return 1e30f;
      }
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 1e30f;  // never chosen
      return ms / reps;
    };
    const float t0 = time_cfg(nullptr);
    float tbest = t0;
    const int n = std::min(conv_candidates(a, cands.data(), (int)cands.size()), (int)cands.size());
    for (int j = 0; j < n && !st; ++j) {
      const float t = time_cfg(&cands[j]);
      if (dbg >= 2)
        fprintf(stderr, "[autotune]   launch %2zu cand MR=%d NR=%d G=%d resw=%d persist=%d kind=%d %7.1f us\n",
                i, cands[j].mr, cands[j].nr, cands[j].G, cands[j].resw, cands[j].persist,
                cands[j].kind, t * 1e3);
      if (verify) {
        unsigned diff = 0;
        for (int d = 0; d < 2; ++d) {
          const size_t nb = out_bytes(a, d);
          if (!nb) continue;
          int vs = hip_check(hipMemsetAsync(cnt, 0, sizeof(unsigned), s), "autotune verify");
          count_diff_kernel<<<1024, 256, 0, s>>>((const uint32_t*)(ref + d * maxb),
                                                 (const uint32_t*)(d == 0 ? a.out0 : a.out1),
                                                 nb / 4, cnt);
          unsigned h_cnt = 0;
          if (!vs)
            vs = hip_check(hipMemcpyAsync(&h_cnt, cnt, sizeof(unsigned), hipMemcpyDeviceToHost, s),
                           "autotune verify");
          if (!vs) vs = hip_check(hipStreamSynchronize(s), "autotune verify");
          if (vs && !st) st = vs;
          diff += h_cnt;
        }
        if (diff) ++bad;
      }
      if (t < tbest) {
        tbest = t;
        best[i] = cands[j];
      }
    }
    if (dbg)
      fprintf(stderr, "[autotune] launch %2zu %3dx%-3d k%d s%d %4d->%-4d default %7.1f us best %7.1f us"
                      " MR=%d NR=%d G=%d resw=%d persist=%d kind=%d (%d cfgs)\n",
              i, a.Ho, a.Wo, a.k, a.stride, a.Cin, a.Cout, t0 * 1e3, tbest * 1e3, best[i].mr,
              best[i].nr, best[i].G, best[i].resw, best[i].persist, best[i].kind, n);
  }
  // teardown of the autotuner's private buffers: nothing to report
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (ref) (void)hipFree(ref);
  if (cnt) (void)hipFree(cnt);
  if (n_bad) *n_bad = bad;
  if (!st) M->tuned = best;
  return st;
}

// The autotuned configuration of conv launch `idx` (cfg6 = {MR, NR, G, resw,
// persist, kind}; MR = 0: the default heuristic).  Returns the number of launches.
extern "C" int rv_yolo_tuned_config(void* h, int idx, int* cfg6) {
  if (!h) return RV_EINVAL;
  Model* M = (Model*)h;
  if (cfg6 && idx >= 0 && idx < (int)M->tuned.size()) {
    const ConvCfg& c = M->tuned[idx];
    cfg6[0] = c.mr;
    cfg6[1] = c.nr;
    cfg6[2] = c.G;
    cfg6[3] = c.resw;
    cfg6[4] = c.persist;
    cfg6[5] = c.kind;
  }
  return (int)M->tuned.size();
}

// Install a configuration for conv launch idx (saved from rv_yolo_tuned_config
// of an earlier autotune of the same plan): n = number of launches of the
// plan (resizes the table; entries not set keep the default heuristic).
// Invalid configurations fall back to the default at launch (conv_cfg_ok).
extern "C" int rv_yolo_set_tuned(void* h, int n, int idx, const int* cfg6) {
  RV_CHECK_ARG(h && cfg6 && n > 0 && idx >= 0 && idx < n, "bad args");
  Model* M = (Model*)h;
  if ((int)M->tuned.size() != n) M->tuned.assign(n, ConvCfg{0, 0, 0, 0, 0});
  M->tuned[idx] = ConvCfg{cfg6[0], cfg6[1], cfg6[2], cfg6[3], cfg6[4], cfg6[5]};
  return RV_OK;
}

// The valid kernel configurations of conv launch idx of the last whole
// forward (the autotuner's search space for it; fused C2f launches have
// none): writes up to cap entries of cfg6 = {MR, NR, G, resw, persist, kind}
// and returns the count.  A caller that times configurations in its own
// schedule (bench.py's in-pipeline tuning) installs them with
// rv_yolo_set_tuned.
extern "C" int rv_yolo_conv_candidates(void* h, int idx, int* cfg6, int cap) {
  RV_CHECK_ARG(h, "null handle");
  Model* M = (Model*)h;
  RV_CHECK_ARG(idx >= 0 && idx < (int)M->launches.size(),
               "launch %d not in the last forward (%d launches)", idx, (int)M->launches.size());
  const ConvArgs& a = M->launches[idx];
  if (a.fused > 0) return 0;
  std::vector<ConvCfg> c(512);
  const int n = std::min(conv_candidates(a, c.data(), (int)c.size()), (int)c.size());
  for (int i = 0; i < n && i < cap && cfg6; ++i) {
    cfg6[6 * i] = c[i].mr;
    cfg6[6 * i + 1] = c[i].nr;
    cfg6[6 * i + 2] = c[i].G;
    cfg6[6 * i + 3] = c[i].resw;
    cfg6[6 * i + 4] = c[i].persist;
    cfg6[6 * i + 5] = c[i].kind;
  }
  return n;
}

// Algorithmic HBM bytes of each conv launch of the profiled forwards (same
// indexing as rv_yolo_profile_read); returns the number of entries written.
extern "C" int rv_yolo_profile_bytes(void* h, double* bytes, int n) {
  RV_CHECK_ARG(h && bytes, "bad args");
  Model* M = (Model*)h;
  const Profile& P = M->prof;
  int k = 0;
  for (; k < n && k < (int)P.bytes.size(); ++k) bytes[k] = P.bytes[k];
  return k;
}
