// YOLOv8 stem kernels for gfx950: conv0 (model.0, 3 -> 16, k3 s2 from the u8
// letterbox on i8 MFMAs) alone, and the fused stem (conv0 + model.1 +
// model.2.cv1) with the P1 map kept in LDS.
//
// Reference: the first layers of the YOLOv8 graph Ultralytics runs inside
// model.predict (src/detect/yolo_ultralytics.py:28-35; Conv = conv + fused
// BN + SiLU).  Own translation unit: built with -mllvm
// -amdgpu-mfma-vgpr-form=1 (Makefile), so the i8 / bf16 MFMA accumulators
// live in VGPRs -- conv0's epilogue reads its three digit sums per output
// without v_accvgpr_read (they are the stem's VALU hot spot).
#include "conv_common.h"

namespace rv {

// ---------------------------------------------------------------------------
// conv0: 3 -> C0, k3 s2 p1, from letterboxed u8 BGR, SiLU, bf16 out.
// ---------------------------------------------------------------------------
// conv0 on integer MFMA (v_mfma_i32_16x16x64_i8).  GEMM view: D[cout][px] =
// sum_k Q[cout][k] x[k][px] over the 3x3 window's 27 BGR bytes,
// k = 16 ky + 3 kx + ch (lane quad q supplies the 9 bytes of window row
// ky = q; quad 3 and k % 16 >= 9 carry zero weights).  The window row is 9
// contiguous bytes of the letterbox row, so a lane's B operand is three
// dword loads, three v_alignbyte_b32 and an XOR 0x80 each (u8 x -> i8
// x - 128): no per-byte conversion.  The weights are the integers Q =
// round(V / s) of V = w[rgb][ky][kx] / 255 at 2^-23 of the channel's largest
// |V| (yolo.hip pack_conv0q) in three balanced base-256 i8 digits, one MFMA
// each, the accumulator started at 128 sum_k D_i[k] so it ends at
// T_i = sum_k D_i[k] x[k] exactly (< 2^24, exact in f32).  The value is
// s (65536 T0 + (256 T1 + T2)) + b in f32, with 256 T1 + T2 summed exactly in
// i32 (|T_i| <= 27 * 128 * 255 < 2^20) and one fma -- the f64 reference within
// 1 bf16 ulp (test_first_conv_sppf_and_decode).
// Out-of-image window bytes read zeros through the buffer range check
// (voffset kOOB), i.e. the zero padding of the normalised image.
// ---------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) int i32x4;

// raw window words of X0 map pixel (Y, X), lane quad q: lb row 2Y - 1 + q,
// bytes 6X - 3 .. 6X + 5 of it inside the three dwords from its aligned base
struct C0Win {
  uint32_t w0, w1, w2;
  int sh;
};

__device__ __forceinline__ C0Win conv0_window(__amdgpu_buffer_rsrc_t r, int Y, int X, int quad, int H,
                                              int rowb, bool valid) {
  const int row = 2 * Y - 1 + quad;
  const int start = 6 * X - 3;
  C0Win w;
  w.sh = start & 3;
  const bool ok = valid && quad < 3 && (unsigned)row < (unsigned)H;
  const uint32_t vb = ok ? (uint32_t)(row * rowb + start - w.sh) : kOOB;
  // X = 0: the dword before the window's first byte is the left padding
  const uint32_t v0 = X > 0 ? vb : kOOB;
  w.w0 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)v0, 0, 0);
  w.w1 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)(vb + 4u), 0, 0);
  w.w2 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)(vb + 8u), 0, 0);
  return w;
}

__device__ __forceinline__ i32x4 conv0_bop(const C0Win& w) {
  const uint32_t b0 = __builtin_amdgcn_alignbyte(w.w1, w.w0, w.sh) ^ 0x80808080u;
  const uint32_t b1 = __builtin_amdgcn_alignbyte(w.w2, w.w1, w.sh) ^ 0x80808080u;
  const uint32_t b2 = __builtin_amdgcn_alignbyte(w.w2, w.w2, w.sh) ^ 0x80808080u;
  return i32x4{(int)b0, (int)b1, (int)b2, 0};
}

// the digits of cout rows 16 m + col (A operands) and the lane's 4 output
// channels' scale / folded bias
template <int MR>
struct C0Wts {
  i32x4 d[MR][3], c[MR][3];
  f32x4 s[MR], b[MR];
  __device__ __forceinline__ void load(const Conv0Q& q, int C0, int col, int quad) {
#pragma unroll
    for (int m = 0; m < MR; ++m) {
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        d[m][t] = *(const i32x4*)(q.d + ((size_t)t * C0 + 16 * m + col) * 64 + 16 * quad);
        c[m][t] = *(const i32x4*)(q.c + (size_t)t * C0 + 16 * m + 4 * quad);
      }
      s[m] = *(const f32x4*)(q.s + 16 * m + 4 * quad);
      b[m] = *(const f32x4*)(q.b + 16 * m + 4 * quad);
    }
  }
};

// one 16-pixel fragment: lane (col, quad) -> SiLU(conv0) of output channels
// 16 m + 4 quad .. +3 of the fragment's pixel col
template <int MR>
__device__ __forceinline__ void conv0_frag(const C0Wts<MR>& W, const i32x4 X, f32x4 (&v)[MR]) {
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    i32x4 t[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) t[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(W.d[m][i], X, W.c[m][i], 0, 0, 0);
    float w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float u = fmaf((float)t[0][i], 65536.0f, (float)(t[1][i] * 256 + t[2][i]));
      w[i] = fmaf(W.s[m][i], u, W.b[m][i]);
    }
    silu4(w);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[m][i] = w[i];
  }
}

// Unfused conv0: a workgroup is 4 x 64 output pixels; wave w owns row w,
// 4 fragments of 16 pixels; the window loads of fragment j + 1 are in flight
// while fragment j runs.
constexpr int kC0TH = 4, kC0TW = 64;

template <int MR, bool F8 = false>
__global__ __launch_bounds__(256) void conv0_kernel(const uint8_t* __restrict__ img, int B, int H,
                                                    int W, Conv0Q q, void* __restrict__ out,
                                                    int out_cs, float s_out = 1.f) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int tiles_x = (Wo + kC0TW - 1) / kC0TW;
  const int tiles_y = (Ho + kC0TH - 1) / kC0TH;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, col = lane & 15, quad = lane >> 4;
  const int oy = ty * kC0TH + wave;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(img + (size_t)b * H * W * 3), 0, H * W * 3, kRsrcFlags);
  C0Wts<MR> Wt;
  Wt.load(q, 16 * MR, col, quad);
  C0Win win[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ox = tx * kC0TW + 16 * j + col;
    win[j] = conv0_window(r, oy, ox, quad, H, W * 3, oy < Ho && ox < Wo);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ox = tx * kC0TW + 16 * j + col;
    f32x4 v[MR];
    conv0_frag<MR>(Wt, conv0_bop(win[j]), v);
    if (oy >= Ho || ox >= Wo) continue;
    const size_t opix = (((size_t)b * Ho + oy) * Wo + ox) * out_cs;
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      if constexpr (F8) {
        const float vv[4] = {v[m][0], v[m][1], v[m][2], v[m][3]};
        *(uint32_t*)((uint8_t*)out + opix + 16 * m + 4 * quad) = f8_encode4(vv, 1.0f / s_out);
      } else {
        *(uint2*)((uint16_t*)out + opix + 16 * m + 4 * quad) =
            make_uint2(pack_bf16x2(v[m][0], v[m][1]), pack_bf16x2(v[m][2], v[m][3]));
      }
    }
  }
}

template <bool F8>
static int launch_conv0_t(const uint8_t* img, int B, int H, int W, const Conv0Q& q, int C0,
                          void* out, int out_cs, float s_out, hipStream_t s) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int blocks = B * ceil_div(Ho, kC0TH) * ceil_div(Wo, kC0TW);
  switch (C0) {
    case 16: conv0_kernel<1, F8><<<blocks, 256, 0, s>>>(img, B, H, W, q, out, out_cs, s_out); break;
    case 32: conv0_kernel<2, F8><<<blocks, 256, 0, s>>>(img, B, H, W, q, out, out_cs, s_out); break;
    case 48: conv0_kernel<3, F8><<<blocks, 256, 0, s>>>(img, B, H, W, q, out, out_cs, s_out); break;
    case 64: conv0_kernel<4, F8><<<blocks, 256, 0, s>>>(img, B, H, W, q, out, out_cs, s_out); break;
    case 80: conv0_kernel<5, F8><<<blocks, 256, 0, s>>>(img, B, H, W, q, out, out_cs, s_out); break;
    default:
      set_error("conv0 C0=%d unsupported", C0);
      return RV_EINVAL;
  }
  return launch_status(F8 ? "conv0_fp8" : "conv0");
}

int launch_conv0(const uint8_t* img, int B, int H, int W, const Conv0Q& q, int C0, bf16_t* out,
                 int out_cs, hipStream_t s) {
  return launch_conv0_t<false>(img, B, H, W, q, C0, out, out_cs, 1.f, s);
}

int launch_conv0_fp8(const uint8_t* img, int B, int H, int W, const Conv0Q& q, int C0,
                     uint8_t* out, int out_cs, float s_out, hipStream_t s) {
  return launch_conv0_t<true>(img, B, H, W, q, C0, out, out_cs, s_out, s);
}

// ---------------------------------------------------------------------------
// Fused stem: conv0 (3 -> C0 = 16, k3 s2, from the u8 letterbox), model.1
// (16 -> 32, k3 s2) and model.2.cv1 (32 -> 32 1x1) in one kernel.  The P1
// map (X0, the network's largest activation) only ever lives in LDS: each
// workgroup computes the X0 pixels its X1 tile needs (halo recomputed,
// 8 %) with the conv0 fragments above (window bytes straight from L2; no
// letterbox staging), then convolves them from LDS.
//
// X0 tile in LDS: 17 rows x (33 even + 32 odd columns) of 32-B pixels, the
// even tile columns first, then the odd ones (stored column of tile column
// xr: xr / 2, or 33 + xr / 2), rows 72 stored pixels apart.  model.1 runs on
// "tap pairs": a 32-deep MFMA k-step takes the 16 channels of two taps --
// (kx 0, kx 1) = (even c, odd c) for X1 column c, then (kx 2, phantom) =
// even c + 1 with zero weights for the phantom -- so 16 consecutive X1
// pixels read 16 consecutive 32-B stored pixels of one region.
// Swizzle: 16-B half h of stored pixel s sits at s * 32 + 16 (h ^ bit 2 of
// s).  conv0 writes a pixel's half as one 16-B store (the two fragments
// of a pair exchange their quad 0/1 and 2/3 channel quarters with
// v_permlane16_swap first), and 8 consecutive pixels of a ds_write_b128 lane
// group then cover all 32 banks; in model.1's ds_read_b128 lane groups the
// 16 lanes hit 16 distinct 16-B bank slots for any row (72 = 0 mod 8 keeps
// bit 2 per row).  (r03 stored 8-B quarters with ds_write_b64: 4-way
// conflicts, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.57.)  A fragments
// come from the standard packed weights [Cout][ky][kx][32] and are held in
// registers for the whole kernel.
//
// With model.2.cv1 fused, model.1's output channels are computed in the
// order that leaves lane quad q holding channels 8q .. 8q+7 of its pixel
// (fragment m, row 4q'+i = channel 8q' + 4m + i): exactly the B operand of
// a K = 32 MFMA in natural k order, so cv1 runs straight from the registers
// with the operands (and k order) of the unfused 1x1 kernels --
// bit-identical -- and X1 never reaches HBM (out == nullptr; out !=
// nullptr still writes it, for parity tests).
constexpr int kStR = 8, kStC = 32;           // X1 tile
constexpr int kStXR = 2 * kStR + 1;          // X0 tile rows (17)
constexpr int kStXE = kStC + 1;              // even X0 tile columns (33)
constexpr int kStXW = 2 * kStC + 1;          // X0 pixels per tile row (33 even + 32 odd)
constexpr int kStXS = 72;                    // stored pixel slots per row (a multiple of 8)
constexpr int kStRowB = kStXS * 32;          // 2304 B per X0 tile row
constexpr int kStXB = kStXR * kStRowB;       // 39,168 B (4 blocks / CU)
constexpr int kStNpx = kStXR * kStXW;        // 1105 X0 pixels per tile: 70 conv0 fragments
static_assert(kStXE == 33 && kStXW - kStXE == 32 && kStXR % 2 == 1,
              "conv0 strips: 2 x 16 even + 2 x 16 odd columns, 9 row pairs");

__global__ __launch_bounds__(256) void stem_kernel(const uint8_t* __restrict__ img, int B, int H,
                                                   int W, Conv0Q q0,
                                                   const uint16_t* __restrict__ w1,
                                                   const float* __restrict__ b1,
                                                   uint16_t* __restrict__ out, int out_cs,
                                                   const uint16_t* __restrict__ w2,
                                                   const float* __restrict__ b2,
                                                   uint16_t* __restrict__ out2, int out2_cs) {
  __shared__ __attribute__((aligned(16))) uint8_t xs[kStXB];
  const int H0 = (H + 1) / 2, W0 = (W + 1) / 2;     // X0 map
  const int H1 = (H0 + 1) / 2, W1 = (W0 + 1) / 2;   // X1 map
  const int tiles_x = (W1 + kStC - 1) / kStC, tiles_y = (H1 + kStR - 1) / kStR;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * kStR, ox0 = tx * kStC;        // X1 tile origin
  const int xy0 = 2 * oy0 - 1, xx0 = 2 * ox0 - 1;    // X0 tile origin
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, col = lane & 15, quad = lane >> 4;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(img + (size_t)b * H * W * 3), 0, H * W * 3, kRsrcFlags);

  // ---- 1. conv0 over the X0 tile.  Wave w owns one 16-column strip of
  //      the tile for all 17 rows: stored columns 16 w + col (w = 0, 1: even
  //      X0 columns, xr = 2 j) or 33 + 16 (w - 2) + col (w = 2, 3: odd, xr =
  //      2 (j - 33) + 1).  Pair i = tile rows 2 i (fragment a) and 2 i + 1
  //      (b).  The strip's column, window alignment and column checks are lane
  //      constants and a pair's rows are wave-uniform, so a window costs a
  //      compare, an add and two selects, and the unrolled pairs store at
  //      immediate offsets.  Pair 8 holds row 16 only; its b fragment is the
  //      17 pixels of even stored column 32 (xr = 64): rows 0-15 on wave 0,
  //      row 16 on wave 1 (per-lane rows: conv0_window).  Each lane stores its
  //      pixel's 16-B half (see the swizzle): fragment a's in quads 0 and 2,
  //      b's in quads 1 and 3.
  {
    C0Wts<1> Wt;
    Wt.load(q0, 16, col, quad);
    const int rowb = W * 3;
    const int jl = (wave < 2 ? 16 * wave : kStXE + 16 * (wave - 2)) + col;  // stored column
    const int X = xx0 + (wave < 2 ? 2 * jl : 2 * (jl - kStXE) + 1);
    const bool xin = (unsigned)X < (unsigned)W0;
    const int start = 6 * X - 3;
    const int sh = start & 3;
    const uint32_t vl = (uint32_t)(quad * rowb + start - sh);  // + (2 Y - 1) rowb
    const bool lq = xin && quad < 3, lx = X > 0;
    // out of range for every window dword (+ 0, 4, 8: no 32-bit wrap) and an
    // inline constant (-16), unlike kOOB, which costs a v_bfrev per select
    constexpr uint32_t kOOBi = 0xFFFFFFF0u;
    // the window of strip pixel (Y, X), Y wave-uniform (conv0_window's bytes)
    auto strip_win = [&](int Y) {
      C0Win w;
      w.sh = sh;
      const bool ok = lq && (unsigned)Y < (unsigned)H0 && (unsigned)(2 * Y - 1 + quad) < (unsigned)H;
      const uint32_t vb = ok ? vl + (uint32_t)((2 * Y - 1) * rowb) : kOOBi;
      w.w0 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)(lx ? vb : kOOBi), 0, 0);
      w.w1 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)(vb + 4u), 0, 0);
      w.w2 = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)(vb + 8u), 0, 0);
      return w;
    };
    // pair 8's b fragment: wave 0 rows 0-15, wave 1 row 16 (lane 0)
    const int ye = wave == 0 ? col : kStXR - 1;
    const int Ye = xy0 + ye, Xe = xx0 + 2 * (kStXE - 1);
    const bool ve = wave == 0 || (wave == 1 && col == 0);
    const bool ine = ve && (unsigned)Ye < (unsigned)H0 && (unsigned)Xe < (unsigned)W0;
    // store address of this lane's pixel in pair 0 (+ 2 rows per pair);
    // bit 2 of a stored slot is bit 2 of its column (72 = 0 mod 8)
    const int sbase = ((quad & 1) * kStXS + jl) * 32 + (((quad >> 1) ^ ((jl >> 2) & 1)) << 4);
    const int se = (ye * kStXS + kStXE - 1) * 32 + ((quad >> 1) << 4);
    C0Win na = strip_win(xy0), nb = strip_win(xy0 + 1);
#pragma unroll
    for (int i = 0; i < (kStXR + 1) / 2; ++i) {
      const C0Win ca = na, cb = nb;
      const bool last = 2 * i + 1 == kStXR;
      const int Ya = xy0 + 2 * i;
      const bool cka = xin && (unsigned)Ya < (unsigned)H0;
      const bool ckb = last ? ine : xin && (unsigned)(Ya + 1) < (unsigned)H0;
      if (2 * i + 3 < kStXR) {
        na = strip_win(Ya + 2);
        nb = strip_win(Ya + 3);
      } else if (2 * i + 3 == kStXR) {
        na = strip_win(Ya + 2);
        nb = conv0_window(r, Ye, Xe, quad, H, rowb, ine);
      }
      f32x4 va[1], vb[1];
      conv0_frag<1>(Wt, conv0_bop(ca), va);
      conv0_frag<1>(Wt, conv0_bop(cb), vb);
      // outside the X0 map the value is model.1's zero padding
      uint32_t a0 = cka ? pack_bf16x2(va[0][0], va[0][1]) : 0u;
      uint32_t a1 = cka ? pack_bf16x2(va[0][2], va[0][3]) : 0u;
      uint32_t b0 = ckb ? pack_bf16x2(vb[0][0], vb[0][1]) : 0u;
      uint32_t b1 = ckb ? pack_bf16x2(vb[0][2], vb[0][3]) : 0u;
      // lanes 16-31 (48-63) of a <-> lanes 0-15 (32-47) of b: quad q then
      // holds channels 8 (q >> 1) .. +7 of its pixel in (a0, a1, b0, b1)
      const auto x0v = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
      const auto x1v = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
      const uint4 px = make_uint4(x0v[0], x1v[0], x0v[1], x1v[1]);
      if (!last) {
        *(uint4*)(xs + sbase + i * 2 * kStRowB) = px;
      } else if (!(quad & 1)) {
        *(uint4*)(xs + sbase + i * 2 * kStRowB) = px;
      } else if (ve) {
        *(uint4*)(xs + se) = px;
      }
    }
  }
  // model.1 A fragments (all 6 k-steps, L2-resident weights) while the
  // conv0 stores drain
  constexpr int MR = 2, NR = 4;
  bf16x8 A[3][2][MR];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int kx = 2 * p + (quad >> 1);  // quads 0,1: tap 2p; quads 2,3: tap 2p+1
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const int co = 8 * (col >> 2) + 4 * m + (col & 3);  // row col of fragment m
        uint4 v = make_uint4(0, 0, 0, 0);
        if (kx < 3) v = *(const uint4*)(w1 + ((size_t)co * 9 + ky * 3 + kx) * 32 + (quad & 1) * 8);
        A[ky][p][m] = __builtin_bit_cast(bf16x8, v);
      }
    }
  __syncthreads();

  // ---- 2. model.1 (C0 = 16 -> 32, k3 s2) on tap pairs from the X0 tile
  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's B column: X1 pixel (row 2 wave + n / 2, col (n & 1) 16 + col)
  int bb0[NR], bb1[NR];
  // byte address of half h of stored pixel s (the swizzle above)
  auto xaddr = [](int s_, int h) { return s_ * 32 + ((h ^ ((s_ >> 2) & 1)) << 4); };
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    const int rr = 2 * wave + (n >> 1), c = (n & 1) * 16 + col;
    const int rs = 2 * rr * kStXS;
    // pair 0: quads 0,1 tap kx 0 (even c), quads 2,3 tap kx 1 (odd c)
    bb0[n] = quad < 2 ? xaddr(rs + c, quad) : xaddr(rs + kStXE + c, quad - 2);
    // pair 1: tap kx 2 (even c + 1); quads 2,3 (phantom tap) read the same
    bb1[n] = xaddr(rs + c + 1, quad & 1);
  }
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      bf16x8 Bf[NR];
#pragma unroll
      for (int n = 0; n < NR; ++n)
        Bf[n] = __builtin_bit_cast(bf16x8, *(const uint4*)(xs + (p ? bb1[n] : bb0[n]) + ky * kStRowB));
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ky][p][m], Bf[n], acc[m][n], 0, 0, 0);
    }
  // epilogue: bias + SiLU -> X1 values (bf16); lane quad q of fragment m
  // holds channels 8q + 4m .. 8q + 4m + 3
  bf16x8 x1[NR];
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    const f32x4 bb = *(const f32x4*)(b1 + 8 * quad + 4 * m);
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      float w[4] = {acc[m][n][0] + bb[0], acc[m][n][1] + bb[1], acc[m][n][2] + bb[2],
                    acc[m][n][3] + bb[3]};
      silu4(w);
      const uint32_t lo = pack_bf16x2(w[0], w[1]);
      const uint32_t hi = pack_bf16x2(w[2], w[3]);
      x1[n][4 * m] = __builtin_bit_cast(__bf16, (uint16_t)(lo & 0xFFFF));
      x1[n][4 * m + 1] = __builtin_bit_cast(__bf16, (uint16_t)(lo >> 16));
      x1[n][4 * m + 2] = __builtin_bit_cast(__bf16, (uint16_t)(hi & 0xFFFF));
      x1[n][4 * m + 3] = __builtin_bit_cast(__bf16, (uint16_t)(hi >> 16));
    }
  }
  // this lane's first X1 pixel (fragment n: + (n >> 1) rows, + 16 (n & 1)
  // columns; the row / column steps are wave-uniform)
  const int oyl = oy0 + 2 * wave, oxl = ox0 + col;
  const size_t pix0 = ((size_t)b * H1 + oyl) * W1 + oxl;
  if (out) {  // X1 (bf16 NHWC, channel stride out_cs)
    uint16_t* o0 = out + pix0 * out_cs + 8 * quad;
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      if (oyl + (n >> 1) >= H1 || oxl + (n & 1) * 16 >= W1) continue;
      *(uint4*)(o0 + ((n >> 1) * W1 + (n & 1) * 16) * out_cs) = __builtin_bit_cast(uint4, x1[n]);
    }
  }
  if (out2) {  // the fused 1x1 conv (32 -> 32) from the registers
    bf16x8 A2[2];
    f32x4 bb2[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      A2[m] = __builtin_bit_cast(bf16x8, *(const uint4*)(w2 + (m * 16 + col) * 32 + quad * 8));
      bb2[m] = *(const f32x4*)(b2 + m * 16 + quad * 4);
    }
    uint16_t* const o0 = out2 + pix0 * out2_cs + (quad & 1) * 16 + (quad >> 1) * 8;
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      f32x4 d[2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
        d[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A2[m], x1[n], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if (oyl + (n >> 1) >= H1 || oxl + (n & 1) * 16 >= W1) continue;
      uint16_t* o = o0 + ((n >> 1) * W1 + (n & 1) * 16) * out2_cs;
      // the two fragments as one 16-B store per lane: after the swap quad q
      // holds channels 8 (q >> 1) .. +7 of fragment q & 1 (as conv0 above)
      uint32_t pk[2][2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        float w[4] = {d[m][0] + bb2[m][0], d[m][1] + bb2[m][1], d[m][2] + bb2[m][2],
                      d[m][3] + bb2[m][3]};
        silu4(w);
        pk[m][0] = pack_bf16x2(w[0], w[1]);
        pk[m][1] = pack_bf16x2(w[2], w[3]);
      }
      const auto y0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
      const auto y1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
      *(uint4*)o = make_uint4(y0[0], y1[0], y0[1], y1[1]);
    }
  }
}

int launch_stem(const uint8_t* img, int B, int H, int W, const Conv0Q& q0, int C0,
                const bf16_t* w1, const float* b1, int C1, bf16_t* out, int out_cs,
                hipStream_t s, const bf16_t* w2, const float* b2, bf16_t* out2, int out2_cs) {
  if (C0 != 16 || C1 != 32 || (!out && !out2) || (out2 && (!w2 || !b2))) {
    set_error("stem: C0=%d C1=%d (fused stem needs 16 -> 32) / outputs", C0, C1);
    return RV_EINVAL;
  }
  const int H0 = (H + 1) / 2, W0 = (W + 1) / 2;
  const int H1 = (H0 + 1) / 2, W1 = (W0 + 1) / 2;
  const int blocks = B * ceil_div(H1, kStR) * ceil_div(W1, kStC);
  stem_kernel<<<blocks, 256, 0, s>>>(img, B, H, W, q0, (const uint16_t*)w1, b1, (uint16_t*)out,
                                     out_cs, (const uint16_t*)w2, b2, (uint16_t*)out2, out2_cs);
  return launch_status("stem");
}

}  // namespace rv
