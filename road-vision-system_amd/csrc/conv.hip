// YOLOv8 conv / pooling / head-decode kernels for gfx950.
//
// Reference: the YOLOv8 graph Ultralytics runs inside model.predict
// (src/detect/yolo_ultralytics.py:28-35; Conv = conv + fused BN + SiLU,
// C2f, SPPF, Detect with DFL).  Layout: NHWC bf16 activations, weights packed
// [Cout_pad16][ky][kx][Cin_pad32] bf16 so every MFMA operand fragment is one
// 16-byte load.
//
// conv_mfma_kernel is an implicit GEMM  D[cout][pixel] = W[cout][k] * X[k][pixel]
// on v_mfma_f32_16x16x32_bf16 with A = weights (staged through LDS, shared by
// the 4 waves of a workgroup) and B = input pixels (16 B per lane straight from
// HBM/L2: lane l reads 8 channels of pixel l&15).  The accumulator layout puts
// 4 consecutive output channels of one pixel in each lane, so the epilogue
// (bias, SiLU, residual add, bf16 pack) stores 8 contiguous bytes per lane into
// each destination view (concat slice and/or nearest-2x upsampled copy).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include "conv.h"

namespace rv {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ float silu(float v) { return v / (1.0f + __expf(-v)); }

// Wave tile: MR x NR fragments of 16x16 (16*MR output channels x 16*NR
// pixels).  A workgroup is 4 waves arranged WP (pixel groups) x WC (channel
// groups); every wave streams its own A (weights, L1/L2-resident, shared by
// the WP waves of a channel group) and B (input pixels) fragments straight
// into VGPRs, double-buffered one k-step ahead, so there is no LDS and no
// barrier in the K loop: the loads of k-step s+1 are in flight while the
// MFMAs of k-step s issue.
template <int MR, int NR, int WC>
__global__ __launch_bounds__(256, 2) void conv_mfma_kernel(ConvArgs a) {
  constexpr int WP = 4 / WC;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, quad = lane >> 4;
  const int wp = wave % WP, wc = wave / WP;
  const int cout_pad = (a.Cout + 15) & ~15;
  const int cout0 = (blockIdx.y * WC + wc) * (16 * MR);
  const int HWo = a.Ho * a.Wo;
  const int M = a.B * HWo;
  const int pix0 = (blockIdx.x * WP + wp) * (16 * NR);
  if (cout0 >= cout_pad || pix0 >= M) return;  // whole-wave early exit (no barriers below)

  const int cin_pad = (a.Cin + 31) & ~31;
  const int kspt = cin_pad >> 5;  // k-steps per tap
  const int Kp = a.k * a.k * cin_pad;
  const int nks = a.k * kspt;     // k-steps per kernel row
  const int total = a.k * nks;

  const bf16_t* wrow[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    int r = cout0 + m * 16 + col;
    r = r < cout_pad ? r : cout_pad - 1;
    wrow[m] = a.w + (size_t)r * Kp + quad * 8;
  }
  int iy0[NR], ix0[NR], pb[NR];
  bool pv[NR];
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    const int p = pix0 + n * 16 + col;
    pv[n] = p < M;
    const int pp = pv[n] ? p : 0;
    const int b = pp / HWo;
    const int r = pp - b * HWo;
    const int oy = r / a.Wo;
    const int ox = r - oy * a.Wo;
    iy0[n] = oy * a.stride - a.pad;
    ix0[n] = ox * a.stride - a.pad;
    pb[n] = b * a.Hin * a.Win * a.in_cs + a.in_co + quad * 8;
  }

  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint4 zero4 = make_uint4(0, 0, 0, 0);
  // k-step s <-> (ky, kx, cs); weights column = s*32
  auto load = [&](int s, bf16x8 (&A)[MR], bf16x8 (&Bf)[NR]) {
    const int ky = s / nks;
    const int r = s - ky * nks;
    const int kx = r / kspt;
    const int cs = r - kx * kspt;
    const int kcol = s * 32;
#pragma unroll
    for (int m = 0; m < MR; ++m) A[m] = __builtin_bit_cast(bf16x8, *(const uint4*)(wrow[m] + kcol));
    const bool cvalid = cs * 32 + quad * 8 < a.Cin;
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      const int iy = iy0[n] + ky, ix = ix0[n] + kx;
      const bool ok = pv[n] && cvalid && (unsigned)iy < (unsigned)a.Hin &&
                      (unsigned)ix < (unsigned)a.Win;
      uint4 v = zero4;
      if (ok)
        v = *(const uint4*)(a.in + (size_t)pb[n] + ((size_t)iy * a.Win + ix) * a.in_cs + cs * 32);
      Bf[n] = __builtin_bit_cast(bf16x8, v);
    }
  };
  auto mma = [&](const bf16x8 (&A)[MR], const bf16x8 (&Bf)[NR]) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int n = 0; n < NR; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[m], Bf[n], acc[m][n], 0, 0, 0);
  };
  bf16x8 A0[MR], B0[NR], A1[MR], B1[NR];
  load(0, A0, B0);
  for (int s = 0; s < total; s += 2) {
    if (s + 1 < total) load(s + 1, A1, B1);
    mma(A0, B0);
    if (s + 1 >= total) break;
    if (s + 2 < total) load(s + 2, A0, B0);
    mma(A1, B1);
  }

  // epilogue: lane holds couts cout0 + m*16 + quad*4 + i of pixel pix0 + n*16 + col
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    if (!pv[n]) continue;
    const int p = pix0 + n * 16 + col;
    const int b = p / HWo;
    const int r = p - b * HWo;
    const int oy = r / a.Wo;
    const int ox = r - oy * a.Wo;
    const size_t opix = (size_t)p;  // == (b*Ho + oy)*Wo + ox
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const int co = cout0 + m * 16 + quad * 4;
      if (co >= a.Cout) continue;
      float v[4];
      const float4 bb = *(const float4*)(a.bias + co);
      v[0] = acc[m][n][0] + bb.x;
      v[1] = acc[m][n][1] + bb.y;
      v[2] = acc[m][n][2] + bb.z;
      v[3] = acc[m][n][3] + bb.w;
      if (a.act) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = silu(v[i]);
      }
      if (a.res) {
        const uint2 rr = *(const uint2*)(a.res + opix * a.res_cs + a.res_co + co);
        v[0] += bf2f(rr.x & 0xFFFF);
        v[1] += bf2f(rr.x >> 16);
        v[2] += bf2f(rr.y & 0xFFFF);
        v[3] += bf2f(rr.y >> 16);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        void* outp = d == 0 ? a.out0 : a.out1;
        if (!outp) continue;
        const int cs_ = d == 0 ? a.out0_cs : a.out1_cs;
        const int co_ = (d == 0 ? a.out0_co : a.out1_co) + co;
        const int up = d == 0 ? a.out0_up : a.out1_up;
        if (a.out_f32) {
          float* o = (float*)outp;
          const float4 pk = make_float4(v[0], v[1], v[2], v[3]);
          if (!up) {
            *(float4*)(o + opix * cs_ + co_) = pk;
          } else {
            for (int dy = 0; dy < 2; ++dy)
              for (int dx = 0; dx < 2; ++dx) {
                const size_t q = ((size_t)(b * 2 * a.Ho + 2 * oy + dy) * (2 * a.Wo) + 2 * ox + dx);
                *(float4*)(o + q * cs_ + co_) = pk;
              }
          }
        } else {
          uint16_t* o = (uint16_t*)outp;
          const uint2 pk = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                      (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
          if (!up) {
            *(uint2*)(o + opix * cs_ + co_) = pk;
          } else {
            for (int dy = 0; dy < 2; ++dy)
              for (int dx = 0; dx < 2; ++dx) {
                const size_t q = ((size_t)(b * 2 * a.Ho + 2 * oy + dy) * (2 * a.Wo) + 2 * ox + dx);
                *(uint2*)(o + q * cs_ + co_) = pk;
              }
          }
        }
      }
    }
  }
}

template <int MR, int NR, int WC>
static void launch_t(const ConvArgs& a, hipStream_t s) {
  constexpr int WP = 4 / WC;
  const int M = a.B * a.Ho * a.Wo;
  const int T = (a.Cout + 15) / 16;
  dim3 grid(ceil_div(M, 16 * NR * WP), ceil_div(T, MR * WC));
  conv_mfma_kernel<MR, NR, WC><<<grid, 256, 0, s>>>(a);
}

// Tile choice: the largest wave tile (MR*NR fragments, i.e. MFMAs per
// k-step) that leaves >= ~2048 busy waves (8 per CU), with no more than one
// padded 16-channel tile; the 4 waves of a workgroup split channels first
// (WC) when the layer has few pixels.
static int try_launch_patch(const ConvArgs& a, hipStream_t s, int* st);

int launch_conv(const ConvArgs& a, hipStream_t s) {
  int st = 0;
  if (try_launch_patch(a, s, &st)) return st;
  const int T = (a.Cout + 15) / 16;
  const long M = (long)a.B * a.Ho * a.Wo;
  struct Cand {
    int mr, nr;
  };
  static const Cand cands[] = {{4, 4}, {2, 8}, {4, 2}, {2, 4}, {1, 8}, {4, 1}, {2, 2},
                               {1, 4}, {2, 1}, {1, 2}, {1, 1}};
  int MR = 1, NR = 1;
  for (const Cand& c : cands) {
    if (c.mr > T) continue;
    const int waste = ceil_div(T, c.mr) * c.mr - T;
    if (waste > 1 && c.mr > 1) continue;
    const long waves = (long)ceil_div((int)((M + 16 * c.nr - 1) / (16 * c.nr)), 1) * ceil_div(T, c.mr);
    MR = c.mr;
    NR = c.nr;
    if (waves >= 2048) break;
  }
  const int groups_c = ceil_div(T, MR);
  const int WC = groups_c >= 4 ? 4 : (groups_c >= 2 ? 2 : 1);
#define RV_CONV_WC(mr, nr)                                           \
  if (MR == mr && NR == nr) {                                        \
    if (WC == 4) launch_t<mr, nr, 4>(a, s);                          \
    else if (WC == 2) launch_t<mr, nr, 2>(a, s);                     \
    else launch_t<mr, nr, 1>(a, s);                                  \
    return launch_status("conv_mfma");                               \
  }
  RV_CONV_WC(4, 4) RV_CONV_WC(2, 8) RV_CONV_WC(4, 2) RV_CONV_WC(2, 4) RV_CONV_WC(1, 8)
  RV_CONV_WC(4, 1) RV_CONV_WC(2, 2) RV_CONV_WC(1, 4) RV_CONV_WC(2, 1) RV_CONV_WC(1, 2)
  RV_CONV_WC(1, 1)
#undef RV_CONV_WC
  set_error("no conv variant for MR=%d NR=%d", MR, NR);
  return RV_EINVAL;
}

// ---------------------------------------------------------------------------
// conv_patch_kernel: LDS-staged implicit GEMM for k in {1,3}, s in {1,2}.
//
// A workgroup owns an R x C tile of output pixels of one image (flattened
// into 64*NR pixel slots, 16*NR per wave) and 16*MR output channels.  The K
// loop walks the input channels in 32-channel chunks; per chunk the input
// halo patch ((R-1)*S+K rows x (C-1)*S+K cols x 32 ch) and the chunk's
// weights (16*MR rows x K*K taps x 32 ch) are DMA'd HBM/L2 -> LDS with
// global_load_lds_dwordx4 (no VGPR round trip), double-buffered so chunk c+1
// streams in while chunk c's K*K taps run on MFMA from LDS.  Every input
// pixel is fetched once per chunk and reused K*K times from LDS.
// LDS images are lane-linear per DMA instruction (16 B per lane); bank
// conflicts on the 16-B fragment reads are removed by an XOR swizzle of the
// 16-B quarter inside each 64-B pixel/tap row, applied on the DMA source
// address and on the read address (the same involution on both sides).
// Out-of-image pixels and channels >= Cin DMA from a zero block.
// ---------------------------------------------------------------------------
__device__ __attribute__((aligned(64))) uint4 g_zero16[4];

struct PatchGeo {
  int C, R;        // output tile cols / rows (R*C <= 64*NR)
  int PH, PW;      // input patch rows / cols
  int npix16;      // DMA instructions for the patch (16 pixels each)
  int tiles_x, tiles_y;
  int p_bytes;     // npix16 * 1024
};

__device__ __forceinline__ int swz(int i) { return (i >> 2) & 3; }

template <int MR, int NR>
__device__ __forceinline__ void epilogue(const ConvArgs& a, f32x4 (&acc)[MR][NR], int cout0,
                                         const bool (&pv)[NR], const int (&pb)[NR],
                                         const int (&py)[NR], const int (&px)[NR], int quad) {
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    if (!pv[n]) continue;
    const int b = pb[n], oy = py[n], ox = px[n];
    const size_t opix = ((size_t)b * a.Ho + oy) * a.Wo + ox;
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const int co = cout0 + m * 16 + quad * 4;
      if (co >= a.Cout) continue;
      float v[4];
      const float4 bb = *(const float4*)(a.bias + co);
      v[0] = acc[m][n][0] + bb.x;
      v[1] = acc[m][n][1] + bb.y;
      v[2] = acc[m][n][2] + bb.z;
      v[3] = acc[m][n][3] + bb.w;
      if (a.act) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = silu(v[i]);
      }
      if (a.res) {
        const uint2 rr = *(const uint2*)(a.res + opix * a.res_cs + a.res_co + co);
        v[0] += bf2f(rr.x & 0xFFFF);
        v[1] += bf2f(rr.x >> 16);
        v[2] += bf2f(rr.y & 0xFFFF);
        v[3] += bf2f(rr.y >> 16);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        void* outp = d == 0 ? a.out0 : a.out1;
        if (!outp) continue;
        const int cs_ = d == 0 ? a.out0_cs : a.out1_cs;
        const int co_ = (d == 0 ? a.out0_co : a.out1_co) + co;
        const int up = d == 0 ? a.out0_up : a.out1_up;
        if (a.out_f32) {
          float* o = (float*)outp;
          const float4 pk = make_float4(v[0], v[1], v[2], v[3]);
          if (!up) {
            *(float4*)(o + opix * cs_ + co_) = pk;
          } else {
            for (int dy = 0; dy < 2; ++dy)
              for (int dx = 0; dx < 2; ++dx) {
                const size_t q = ((size_t)(b * 2 * a.Ho + 2 * oy + dy) * (2 * a.Wo) + 2 * ox + dx);
                *(float4*)(o + q * cs_ + co_) = pk;
              }
          }
        } else {
          uint16_t* o = (uint16_t*)outp;
          const uint2 pk = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                      (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
          if (!up) {
            *(uint2*)(o + opix * cs_ + co_) = pk;
          } else {
            for (int dy = 0; dy < 2; ++dy)
              for (int dx = 0; dx < 2; ++dx) {
                const size_t q = ((size_t)(b * 2 * a.Ho + 2 * oy + dy) * (2 * a.Wo) + 2 * ox + dx);
                *(uint2*)(o + q * cs_ + co_) = pk;
              }
          }
        }
      }
    }
  }
}

template <int MR, int NR, int K, int S>
__global__ __launch_bounds__(256) void conv_patch_kernel(ConvArgs a, PatchGeo g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int T2 = K * K;
  constexpr int BC = 16 * MR;
  constexpr int W_BYTES = BC * T2 * 64;
  const int stage_bytes = g.p_bytes + W_BYTES;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, quad = lane >> 4;
  int bid = blockIdx.x;
  const int tx = bid % g.tiles_x;
  bid /= g.tiles_x;
  const int ty = bid % g.tiles_y;
  const int b = bid / g.tiles_y;
  const int x0 = tx * g.C, y0 = ty * g.R;
  const int cout0 = blockIdx.y * BC;
  const int cout_pad = (a.Cout + 15) & ~15;
  const int cin_pad = (a.Cin + 31) & ~31;
  const int Kp = T2 * cin_pad;
  const int nch = cin_pad >> 5;
  const int pad = K / 2;

  bool pv[NR];
  int pbase[NR], pbv[NR], pyv[NR], pxv[NR];
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    const int q = wave * (NR * 16) + n * 16 + col;
    const int r = q / g.C, cc = q - (q / g.C) * g.C;
    pv[n] = q < g.R * g.C && y0 + r < a.Ho && x0 + cc < a.Wo;
    pbase[n] = pv[n] ? (r * S) * g.PW + cc * S : 0;
    pbv[n] = b;
    pyv[n] = y0 + r;
    pxv[n] = x0 + cc;
  }
  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int npp = g.PH * g.PW;
  const bf16_t* img = a.in + (size_t)b * a.Hin * a.Win * a.in_cs + a.in_co;
  auto stage = [&](int c, int buf) {
    uint8_t* P = smem + buf * stage_bytes;
    uint8_t* Wl = P + g.p_bytes;
    const int slot = lane & 3;
    for (int j = wave; j < g.npix16; j += 4) {
      const int pp = j * 16 + (lane >> 2);
      const int q = slot ^ swz(pp);
      const int py = pp / g.PW, px = pp - (pp / g.PW) * g.PW;
      const int iy = y0 * S - pad + py, ix = x0 * S - pad + px;
      const bool ok = pp < npp && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win &&
                      c * 32 + q * 8 < a.Cin;
      const void* src = ok ? (const void*)(img + ((size_t)iy * a.Win + ix) * a.in_cs + c * 32 + q * 8)
                           : (const void*)g_zero16;
      __builtin_amdgcn_global_load_lds(src, (void*)(P + j * 1024), 16, 0, 0);
    }
    for (int j = wave; j < BC * T2 / 16; j += 4) {
      const int pr = j * 16 + (lane >> 2);
      const int row = pr / T2, tap = pr - (pr / T2) * T2;
      const int q = slot ^ swz(row);
      const int co = cout0 + row;
      const void* src = co < cout_pad
                            ? (const void*)(a.w + (size_t)co * Kp + tap * cin_pad + c * 32 + q * 8)
                            : (const void*)g_zero16;
      __builtin_amdgcn_global_load_lds(src, (void*)(Wl + j * 1024), 16, 0, 0);
    }
  };
  auto compute = [&](int buf) {
    const uint8_t* P = smem + buf * stage_bytes;
    const uint8_t* Wl = P + g.p_bytes;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int tap = ky * K + kx;
        bf16x8 A[MR], Bf[NR];
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          const int row = m * 16 + col;
          A[m] = __builtin_bit_cast(
              bf16x8, *(const uint4*)(Wl + (row * T2 + tap) * 64 + ((quad ^ swz(row)) << 4)));
        }
#pragma unroll
        for (int n = 0; n < NR; ++n) {
          const int pp = pbase[n] + ky * g.PW + kx;
          Bf[n] = __builtin_bit_cast(bf16x8, *(const uint4*)(P + pp * 64 + ((quad ^ swz(pp)) << 4)));
        }
#pragma unroll
        for (int m = 0; m < MR; ++m)
#pragma unroll
          for (int n = 0; n < NR; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[m], Bf[n], acc[m][n], 0, 0, 0);
      }
  };
  stage(0, 0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch && !(a.dbg & 2)) stage(c + 1, (c + 1) & 1);
    if (!(a.dbg & 1)) compute(c & 1);
    __syncthreads();
  }
  epilogue<MR, NR>(a, acc, cout0, pv, pbv, pyv, pxv, quad);
}

static bool patch_geo(const ConvArgs& a, int NR, int MR, PatchGeo& g, size_t& smem) {
  if (!((a.k == 1 || a.k == 3) && (a.stride == 1 || a.stride == 2) && a.pad == a.k / 2)) return false;
  const int P = 64 * NR;
  int C;
  if (a.Wo <= P && a.Wo <= 64) {
    C = a.Wo;
  } else {
    C = 16;
    for (int c : {64, 32, 16})
      if (c <= P && a.Wo % c == 0) {
        C = c;
        break;
      }
    if (a.Wo % C != 0) C = P >= 32 ? 32 : 16;
  }
  g.C = C;
  g.R = P / C;
  if (g.R < 1) return false;
  g.PH = (g.R - 1) * a.stride + a.k;
  g.PW = (g.C - 1) * a.stride + a.k;
  g.npix16 = (g.PH * g.PW + 15) / 16;
  g.p_bytes = g.npix16 * 1024;
  g.tiles_x = ceil_div(a.Wo, g.C);
  g.tiles_y = ceil_div(a.Ho, g.R);
  const int nch = ((a.Cin + 31) & ~31) / 32;
  // double-buffer only when there is a next chunk to overlap
  smem = (nch > 1 ? 2 : 1) * ((size_t)g.p_bytes + (size_t)16 * MR * a.k * a.k * 64);
  return smem <= 160 * 1024;
}

template <int MR, int NR, int K, int S>
static int launch_patch_t(const ConvArgs& a, const PatchGeo& g, size_t smem, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_patch_kernel<MR, NR, K, S>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      set_error("hipFuncSetAttribute: %s", hipGetErrorString(e));
      return -(int)e;
    }
    attr = true;
  }
  const int T = (a.Cout + 15) / 16;
  dim3 grid(a.B * g.tiles_x * g.tiles_y, ceil_div(T, MR));
  conv_patch_kernel<MR, NR, K, S><<<grid, 256, smem, s>>>(a, g);
  return launch_status("conv_patch");
}

template <int MR, int NR>
static int launch_patch_ks(const ConvArgs& a, const PatchGeo& g, size_t smem, hipStream_t s) {
  if (a.k == 3 && a.stride == 1) return launch_patch_t<MR, NR, 3, 1>(a, g, smem, s);
  if (a.k == 3 && a.stride == 2) return launch_patch_t<MR, NR, 3, 2>(a, g, smem, s);
  if (a.k == 1 && a.stride == 1) return launch_patch_t<MR, NR, 1, 1>(a, g, smem, s);
  return launch_patch_t<MR, NR, 1, 2>(a, g, smem, s);
}

// returns 1 if launched (status in *st), 0 if the patch kernel does not apply
static int try_launch_patch(const ConvArgs& a_in, hipStream_t s, int* st) {
  ConvArgs a = a_in;
  static const int ablate = getenv("RV_CONV_ABLATE") ? atoi(getenv("RV_CONV_ABLATE")) : 0;
  a.dbg = ablate;
  static const char* force = getenv("RV_CONV_FORCE");  // "direct" or "MR,NR" (experiments)
  const int T = (a.Cout + 15) / 16;
  if (force && strcmp(force, "direct") == 0) return 0;
  struct Cand {
    int mr, nr;
  };
  static const Cand cands[] = {{4, 4}, {8, 2}, {4, 2}, {2, 4}, {8, 1}, {4, 1}, {2, 2}, {1, 4},
                               {2, 1}, {1, 2}, {1, 1}};
  // Largest wave tile that still fills the machine: blocks >= 3/4 of the
  // CUs x co-resident blocks per CU (LDS-limited, at most 4); otherwise the
  // candidate with the best fill.
  int best = -1;
  double best_fill = -1.0;
  PatchGeo bg{};
  size_t bsm = 0;
  for (int i = 0; i < (int)(sizeof(cands) / sizeof(cands[0])); ++i) {
    const Cand& c = cands[i];
    if (c.mr > T && c.mr > 1) continue;
    if (ceil_div(T, c.mr) * c.mr - T > (c.mr > 1 ? 1 : 0)) continue;
    if (a.k == 3 && c.mr > 4) continue;  // keep 3x3 weight stages <= 37 KB
    PatchGeo g;
    size_t sm;
    if (!patch_geo(a, c.nr, c.mr, g, sm)) continue;
    if (force) {
      int fm = 0, fn = 0;
      if (sscanf(force, "%d,%d", &fm, &fn) == 2 && (fm != c.mr || fn != c.nr)) continue;
    }
    const long blocks = (long)a.B * g.tiles_x * g.tiles_y * ceil_div(T, c.mr);
    const int bpc = std::max(1, std::min(4, (int)((160 * 1024) / sm)));
    const double fill = (double)blocks / (256.0 * bpc);
    if (fill >= 0.75) {
      best = i;
      bg = g;
      bsm = sm;
      break;
    }
    if (fill > best_fill) {
      best_fill = fill;
      best = i;
      bg = g;
      bsm = sm;
    }
  }
  if (best < 0) return 0;
  const int MR = cands[best].mr, NR = cands[best].nr;
  static const int dbg = getenv("RV_CONV_DEBUG") ? atoi(getenv("RV_CONV_DEBUG")) : 0;
  if (dbg) {
    const long blocks = (long)a.B * bg.tiles_x * bg.tiles_y * ceil_div(T, MR);
    fprintf(stderr, "[conv] %dx%d k%d s%d Cin %d Cout %d -> patch MR=%d NR=%d tile %dx%d patch %dx%d smem %zu blocks %ld\n",
            a.Ho, a.Wo, a.k, a.stride, a.Cin, a.Cout, MR, NR, bg.R, bg.C, bg.PH, bg.PW, bsm, blocks);
  }
#define RV_PATCH(mr, nr) \
  if (MR == mr && NR == nr) { *st = launch_patch_ks<mr, nr>(a, bg, bsm, s); return 1; }
  RV_PATCH(4, 4) RV_PATCH(8, 2) RV_PATCH(4, 2) RV_PATCH(2, 4) RV_PATCH(8, 1) RV_PATCH(4, 1)
  RV_PATCH(2, 2) RV_PATCH(1, 4) RV_PATCH(2, 1) RV_PATCH(1, 2) RV_PATCH(1, 1)
#undef RV_PATCH
  return 0;
}

// ---------------------------------------------------------------------------
// conv0: 3 -> C0, k3 s2 p1, from letterboxed u8 BGR, f32 math, SiLU, bf16 out.
// ---------------------------------------------------------------------------
// One workgroup per 8 x 32 output tile: the (17 x 65) x 3 u8 input window
// is staged in LDS as f32 (x / 255, RGB order) with coalesced byte loads,
// then each thread computes all C0 channels of one output pixel.
template <int C0>
__global__ __launch_bounds__(256) void conv0_kernel(const uint8_t* __restrict__ img, int B, int H,
                                                    int W, const float* __restrict__ w,
                                                    const float* __restrict__ bias,
                                                    uint16_t* __restrict__ out, int out_cs) {
  constexpr int TH = 8, TW = 32, IH = 2 * TH + 1, IW = 2 * TW + 1;
  __shared__ float ws[C0 * 27];
  __shared__ float bs[C0];
  __shared__ float xin[3][IH][IW + 1];
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int tiles_x = (Wo + TW - 1) / TW;
  const int tiles_y = (Ho + TH - 1) / TH;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * 2 - 1, ix0 = ox0 * 2 - 1;
  for (int i = threadIdx.x; i < C0 * 27; i += 256) ws[i] = w[i];
  for (int i = threadIdx.x; i < C0; i += 256) bs[i] = bias[i];
  const uint8_t* frame = img + (size_t)b * H * W * 3;
  for (int i = threadIdx.x; i < IH * IW * 3; i += 256) {
    const int r = i / (IW * 3);
    const int rem = i - r * (IW * 3);
    const int cx = rem / 3, ch = rem - (rem / 3) * 3;  // ch: BGR byte index
    const int iy = iy0 + r, ix = ix0 + cx;
    float v = 0.f;
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
      v = (float)frame[((size_t)iy * W + ix) * 3 + ch] / 255.0f;
    xin[2 - ch][r][cx] = v;  // RGB plane order of the reference input
  }
  __syncthreads();
  const int ly = threadIdx.x / TW, lx = threadIdx.x % TW;
  const int oy = oy0 + ly, ox = ox0 + lx;
  if (oy >= Ho || ox >= Wo) return;
  float x[27];
#pragma unroll
  for (int ci = 0; ci < 3; ++ci)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) x[ci * 9 + ky * 3 + kx] = xin[ci][2 * ly + ky][2 * lx + kx];
  uint16_t* o = out + (((size_t)b * Ho + oy) * Wo + ox) * out_cs;
#pragma unroll
  for (int c8 = 0; c8 < C0; c8 += 8) {
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      float v2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = c8 + j + u;
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < 27; ++t) acc += ws[c * 27 + t] * x[t];
        v2[u] = silu(acc + bs[c]);
      }
      pk[j / 2] = (uint32_t)f2bf(v2[0]) | ((uint32_t)f2bf(v2[1]) << 16);
    }
    *(uint4*)(o + c8) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }
}

int launch_conv0(const uint8_t* img, int B, int H, int W, const float* w, const float* bias,
                 int C0, bf16_t* out, int out_cs, hipStream_t s) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int blocks = B * ceil_div(Ho, 8) * ceil_div(Wo, 32);
  if (C0 == 16) conv0_kernel<16><<<blocks, 256, 0, s>>>(img, B, H, W, w, bias, out, out_cs);
  else if (C0 == 32) conv0_kernel<32><<<blocks, 256, 0, s>>>(img, B, H, W, w, bias, out, out_cs);
  else if (C0 == 48) conv0_kernel<48><<<blocks, 256, 0, s>>>(img, B, H, W, w, bias, out, out_cs);
  else if (C0 == 64) conv0_kernel<64><<<blocks, 256, 0, s>>>(img, B, H, W, w, bias, out, out_cs);
  else {
    set_error("conv0 C0=%d unsupported", C0);
    return RV_EINVAL;
  }
  return launch_status("conv0");
}

// ---------------------------------------------------------------------------
// SPPF: three chained MaxPool2d(5, 1, 2) == clipped 5/9/13 windows.
// One thread per (pixel, 8-channel group).
// ---------------------------------------------------------------------------
// One workgroup per (image, 32-channel group): the H x W x 32 slice of x is
// staged in LDS, every (pixel, 8-channel chunk) item then takes the clipped
// 5/9/13 window maxima from LDS (bf16 max is exact).
constexpr int kSppfLds = 64 * 1024;

__global__ __launch_bounds__(256) void sppf_pool_kernel(uint16_t* __restrict__ buf, int B, int H,
                                                        int W, int c) {
  extern __shared__ __attribute__((aligned(16))) uint4 xs[];  // [H*W][4] (32 ch)
  const int groups = c / 32;
  const int b = blockIdx.x / groups, g = blockIdx.x % groups;
  const int cs = 4 * c;
  const int HW = H * W;
  uint16_t* img = buf + (size_t)b * HW * cs;
  for (int i = threadIdx.x; i < HW * 4; i += 256) {
    const int p = i >> 2, q = i & 3;
    xs[i] = *(const uint4*)(img + (size_t)p * cs + g * 32 + q * 8);
  }
  __syncthreads();
  for (int it = threadIdx.x; it < HW * 4; it += 256) {
    const int p = it >> 2, q = it & 3;
    const int y = p / W, x = p - (p / W) * W;
    float m5[8], m9[8], m13[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m5[j] = m9[j] = m13[j] = -INFINITY;
    const int y0 = max(y - 6, 0), y1 = min(y + 6, H - 1);
    const int x0 = max(x - 6, 0), x1 = min(x + 6, W - 1);
    for (int yy = y0; yy <= y1; ++yy) {
      const int ady = yy < y ? y - yy : yy - y;
      for (int xx = x0; xx <= x1; ++xx) {
        const int adx = xx < x ? x - xx : xx - x;
        const int rad = ady > adx ? ady : adx;
        const uint4 v = xs[(yy * W + xx) * 4 + q];
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f((uint16_t)(wv[j / 2] >> ((j & 1) * 16)));
          m13[j] = fmaxf(m13[j], f);
          if (rad <= 4) m9[j] = fmaxf(m9[j], f);
          if (rad <= 2) m5[j] = fmaxf(m5[j], f);
        }
      }
    }
    uint16_t* o = img + (size_t)p * cs + g * 32 + q * 8;
    const float* src[3] = {m5, m9, m13};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      uint32_t pk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        pk[j] = (uint32_t)f2bf(src[s][2 * j]) | ((uint32_t)f2bf(src[s][2 * j + 1]) << 16);
      *(uint4*)(o + (s + 1) * c) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    }
  }
}

int launch_sppf_pool(bf16_t* buf, int B, int H, int W, int c, hipStream_t s) {
  const size_t smem = (size_t)H * W * 64;
  if (c % 32 != 0 || smem > kSppfLds) {
    set_error("sppf: c=%d / map %dx%d unsupported by the LDS pool", c, H, W);
    return RV_EINVAL;
  }
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)sppf_pool_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        kSppfLds);
    (void)hipGetLastError();
    attr = true;
  }
  sppf_pool_kernel<<<B * (c / 32), 256, smem, s>>>(buf, B, H, W, c);
  return launch_status("sppf_pool");
}

// ---------------------------------------------------------------------------
// Detect head decode: DFL softmax-expectation, dist2bbox (xywh) * stride,
// class sigmoid; Ultralytics non_max_suppression candidate filter.
// ---------------------------------------------------------------------------
struct HeadLevels {
  HeadLevel lv[4];
  int start[5];  // first anchor of each level
  int blk[5];    // first 64-anchor block of each level
  int nlv;
};

// One wave per 64 consecutive anchors of one level: their (64 x cs) f32
// head logits are one contiguous span, staged into LDS with coalesced 16-B
// loads; then each lane decodes its anchor from LDS.
template <int REG>
__global__ __launch_bounds__(64) void detect_decode_kernel(HeadLevels h, int B, int nc,
                                                           float conf, float* __restrict__ raw,
                                                           Cand* __restrict__ cand, int cap,
                                                           int* __restrict__ cand_n) {
  extern __shared__ __attribute__((aligned(16))) float lg[];  // [64][cs]
  const int A = h.start[h.nlv];
  const int b = blockIdx.y;
  // block -> (level, first anchor in level)
  int blk = blockIdx.x, l = 0;
  while (l + 1 < h.nlv && blk >= h.blk[l + 1]) ++l;
  const HeadLevel& L = h.lv[l];
  const int HW = L.H * L.W;
  const int r0 = (blk - h.blk[l]) * 64;
  const int na = min(64, HW - r0);
  const int lane = threadIdx.x;
  const float* src = L.logits + ((size_t)b * HW + r0) * L.cs;
  const int n4 = na * L.cs / 4;  // cs is a multiple of 4
  for (int i = lane; i < n4; i += 64) ((float4*)lg)[i] = ((const float4*)src)[i];
  __syncthreads();
  if (lane >= na) return;
  const int r = r0 + lane;
  const int a = h.start[l] + r;
  const int y = r / L.W, x = r - (r / L.W) * L.W;
  const float* px = lg + lane * L.cs;
  float d[4];
#pragma unroll
  for (int sd = 0; sd < 4; ++sd) {
    float v[REG];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < REG; ++i) {
      v[i] = px[sd * REG + i];
      mx = fmaxf(mx, v[i]);
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < REG; ++i) {
      v[i] = __expf(v[i] - mx);
      sum += v[i];
    }
    float e = 0.f;
#pragma unroll
    for (int i = 0; i < REG; ++i) e += (float)i * (v[i] / sum);
    d[sd] = e;
  }
  const float ax = (float)x + 0.5f, ay = (float)y + 0.5f;
  const float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
  const float cx = (x1 + x2) / 2.0f * L.stride, cy = (y1 + y2) / 2.0f * L.stride;
  const float w = (x2 - x1) * L.stride, hh = (y2 - y1) * L.stride;
  float best = -1.f;
  int bc = 0;
  const float* pc = px + 4 * REG;
  for (int c = 0; c < nc; ++c) {
    const float sg = 1.0f / (1.0f + __expf(-pc[c]));
    if (raw) raw[((size_t)b * (4 + nc) + 4 + c) * A + a] = sg;
    if (sg > best) {
      best = sg;
      bc = c;
    }
  }
  if (raw) {
    raw[((size_t)b * (4 + nc) + 0) * A + a] = cx;
    raw[((size_t)b * (4 + nc) + 1) * A + a] = cy;
    raw[((size_t)b * (4 + nc) + 2) * A + a] = w;
    raw[((size_t)b * (4 + nc) + 3) * A + a] = hh;
  }
  if (cand && best > conf) {
    const int i = atomicAdd(&cand_n[b], 1);
    if (i < cap) {
      const float hw = w / 2.0f, hh2 = hh / 2.0f;  // xywh2xyxy
      Cand c;
      c.x1 = cx - hw;
      c.y1 = cy - hh2;
      c.x2 = cx + hw;
      c.y2 = cy + hh2;
      c.score = best;
      c.cls = bc;
      c.anchor = a;
      c.pad = 0;
      cand[(size_t)b * cap + i] = c;
    }
  }
}

int launch_detect_decode(const HeadLevel* lv, int nlv, int B, int nc, int reg_max, float conf,
                         float* raw, Cand* cand, int cand_cap, int* cand_n, hipStream_t s) {
  if (nlv < 1 || nlv > 4 || reg_max != 16) {
    set_error("detect decode: nlv=%d reg_max=%d unsupported", nlv, reg_max);
    return RV_EINVAL;
  }
  HeadLevels h;
  h.nlv = nlv;
  h.start[0] = 0;
  h.blk[0] = 0;
  int cs = lv[0].cs;
  for (int i = 0; i < nlv; ++i) {
    h.lv[i] = lv[i];
    h.start[i + 1] = h.start[i] + lv[i].H * lv[i].W;
    h.blk[i + 1] = h.blk[i] + ceil_div(lv[i].H * lv[i].W, 64);
    if (lv[i].cs != cs || cs % 4 != 0) {
      set_error("detect decode: head channel strides differ / not a multiple of 4");
      return RV_EINVAL;
    }
  }
  const size_t smem = (size_t)64 * cs * 4;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)detect_decode_kernel<16>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
    attr = true;
  }
  detect_decode_kernel<16><<<dim3(h.blk[nlv], B), 64, smem, s>>>(h, B, nc, conf, raw, cand,
                                                                 cand_cap, cand_n);
  return launch_status("detect_decode");
}

}  // namespace rv
