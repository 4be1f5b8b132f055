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
#include "conv_common.h"

namespace rv {

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
        silu4(v);
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
          const uint2 pk = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
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

// a virtual concat / upsampled input (ConvArgs::split, in_up) is read by
// the direct 1x1 kernel only
static bool vcat(const ConvArgs& a) { return a.split > 0 || a.in_up; }

int launch_conv(const ConvArgs& a, hipStream_t s) {
  int st = 0;
  if (vcat(a)) {  // the direct 1x1 kernel: the widest channel tile that divides Cout and fits
    const int T = (a.Cout + 15) / 16;
    ConvCfg c{1, 1, 1, 1, 1, 1};
    for (const int mr : {8, 4, 2})
      if (T % mr == 0 && conv_cfg_ok(a, ConvCfg{mr, 1, 1, 1, 1, 1})) {
        c.mr = mr;
        break;
      }
    if (!conv_cfg_ok(a, c)) {
      set_error("virtual concat input (split %d, up %d) needs a bf16 1x1 conv", a.split, a.in_up);
      return RV_EINVAL;
    }
    return launch_conv_cfg(a, c, s);
  }
  if (try_launch_patch(a, s, &st)) return st;
  if (a.ch_w) {
    set_error("chained 1x1 conv (Cout %d, k%d s%d) has no patch-kernel configuration", a.Cout, a.k,
              a.stride);
    return RV_EINVAL;
  }
  if (a.in8) {
    set_error("fp8 conv (Cin %d, Cout %d, k%d s%d) has no patch-kernel configuration", a.Cin,
              a.Cout, a.k, a.stride);
    return RV_EINVAL;
  }
  if (a.g2_cout0 > 0) {
    set_error("grouped conv (Cout %d, split %d) has no patch-kernel configuration", a.Cout,
              a.g2_cout0);
    return RV_EINVAL;
  }
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
#ifdef RV_PHASE_PROF
// Timing build (-DRV_PHASE_PROF): s_memtime cycles per phase of
// conv_patch_kernel summed over every wave of every launch: 0 prologue
// (resident weights + first stage + barrier), 1 next-step DMA issue (incl.
// the tile's offset prep), 2 compute, 3 epilogue, 4 end-of-step barrier
// (incl. the vmcnt wait for the next stage), 5 steps, 6 waves.
__device__ unsigned long long g_conv_phase[8];
#define RV_PH_T() __builtin_amdgcn_s_memtime()
#endif

// XCD-aware pixel-tile walk.  Workgroups are dispatched to the 8 XCDs
// round-robin by linear id, so with gridDim.x a multiple of 8 (the host
// rounds it: xcd_grid) every cout tile blockIdx.y of blockIdx.x lands on
// XCD blockIdx.x % 8.  XCD j then owns one contiguous run of pixel tiles
// [j * chunk, (j + 1) * chunk) and its gridDim.x / 8 walkers step through it
// together: the cout tiles of a pixel tile, and neighbouring tiles' shared
// halo rows, are read from that XCD's L2 instead of being fetched into up
// to 8 L2s (MI355X_MICROARCH.md: per-XCD L2s).  Other grids: plain stride.
struct TileWalk {
  int t0, step, end;
  __device__ __forceinline__ int count() const { return t0 < end ? (end - t0 + step - 1) / step : 0; }
};
__device__ __forceinline__ TileWalk tile_walk(int ntiles) {
  const int gx = gridDim.x, bx = blockIdx.x;
  if ((gx & 7) == 0) {
    const int chunk = (ntiles + 7) >> 3, j = bx & 7;
    return TileWalk{j * chunk + (bx >> 3), gx >> 3, min(ntiles, (j + 1) * chunk)};
  }
  return TileWalk{bx, gx, ntiles};
}
// host side: a persistent grid of `want` walkers per cout tile, rounded down
// to a multiple of 8 (at least 8 when there are that many tiles); a
// one-block-per-tile grid rounded up (the surplus walkers get no tile)
static inline int xcd_grid(int want, int ntiles, bool persist) {
  if (!persist) return ntiles >= 8 ? (ntiles + 7) & ~7 : ntiles;
  const int g = std::min(want, ntiles);
  return g >= 8 ? g & ~7 : g;
}

// cache-policy bits of the activation-patch DMA (A/B builds: 2 = nt)
#ifndef RV_CONV_IN_AUX
#define RV_CONV_IN_AUX 0
#endif
template <int AUX = 0>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           (int)voff, soff, 0, AUX);
}

// Detect-head class score: exp + one v_rcp_f32 (no IEEE division
// sequence); the decode, its raw output and the chained head epilogue
// (conv_patch_kernel CHM = 3) all use this one function.
__device__ __forceinline__ float head_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}

struct PatchGeo {
  int C, R;        // output tile cols / rows (R*C <= 64*NR)
  int G;           // input-channel chunks per pipeline stage
  int PH, PW;      // input patch rows / cols
  int pinst;       // DMA instructions for the patch (64 x 16-B slots each)
  int tiles_x, tiles_y;
  int p_bytes;     // pinst * 1024
  int fast;        // epilogue_fast applies (epi_fast)
  int stagger;     // 8-wave form: waves 4-7 run each tile's epilogue one step late
};

// The common epilogue (one bf16 output view, no upsampled copy, optional
// bf16 residual, Cout a multiple of 16, every byte offset < 2^31) runs
// epilogue_fast: buffer stores / loads whose per-lane byte offsets are one
// 24-bit multiply per pixel, each 16-channel fragment m in the instruction's
// immediate offset -- no 64-bit address arithmetic per (pixel, fragment).
static bool epi_fast(const ConvArgs& a) {
  static const bool off = getenv("RV_EPI_SLOW") != nullptr;  // A/B: the generic epilogue
  const double px = (double)a.B * a.Ho * a.Wo;
  return !off && !a.out_f32 && !a.out1 && !a.out0_up && !a.in8 && a.Cout % 16 == 0 && px < (1 << 23) &&
         a.out0_cs < 2048 && px * a.out0_cs * 2 < 2147483647.0 &&
         (!a.res || (a.res_cs < 2048 && px * a.res_cs * 2 < 2147483647.0));
}

// lane pixel opx (output pixel index b*Ho*Wo + y*Wo + x; valid = pv) of
// each n; cout0 the block's first output channel.  Fragments are stored in
// pairs (m, m+1) as 16-B stores: lane quad q holds channels 4q .. 4q+3 of
// both; one v_permlane16_swap per packed dword gives quad q the 8
// consecutive channels 8 (q >> 1) .. +7 of fragment m + (q & 1) (the stem's
// exchange), so a pair is one buffer_store_dwordx4 instead of two dwordx2 --
// half the store instructions of the tile's epilogue.  Stores of invalid
// pixels or of a fragment beyond Cout go to an out-of-range offset (dropped).
template <int MR, int NR>
__device__ __forceinline__ void epilogue_fast(const ConvArgs& a, f32x4 (&acc)[MR][NR], int cout0,
                                              const bool (&pv)[NR], const uint32_t (&opx)[NR],
                                              int quad, const f32x4 (&bias)[MR]) {
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(a.out0, 0, 0x7FFFFFFF, kRsrcFlags);
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.res, 0, 0x7FFFFFFF, kRsrcFlags);
  const int cq = cout0 + quad * 4;
  constexpr uint32_t kDrop = 0x80000000u;
  auto value = [&](int m, int n, uint32_t vr, uint32_t& lo, uint32_t& hi) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[m][n][i] + bias[m][i];
    if (a.act) {
      silu4(v);
    }
    if (a.res) {
      // a fragment at or beyond Cout (the pair's second when Cout % 32 == 16)
      // reads from an out-of-range offset: dropped, returns 0
      const uint32_t roff = cout0 + m * 16 < a.Cout ? vr + m * 32 : kDrop;
      const uint2 q = __builtin_bit_cast(
          uint2, __builtin_amdgcn_raw_buffer_load_b64(rr, (int)roff, 0, 0));
      v[0] += bf2f(q.x & 0xFFFF);
      v[1] += bf2f(q.x >> 16);
      v[2] += bf2f(q.y & 0xFFFF);
      v[3] += bf2f(q.y >> 16);
    }
    lo = pack_bf16x2(v[0], v[1]);
    hi = pack_bf16x2(v[2], v[3]);
  };
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    if (!pv[n]) continue;  // all four quads of a pixel share pv: swap partners agree
    const uint32_t vo = (__umul24(opx[n], (uint32_t)a.out0_cs) + a.out0_co + cq) * 2;
    const uint32_t vr = a.res ? (__umul24(opx[n], (uint32_t)a.res_cs) + a.res_co + cq) * 2 : 0u;
    // quad q's 16-B slot of pair (m, m+1): fragment m + (q & 1), channels
    // 8 (q >> 1) .. +7, i.e. (16 (q & 1) + 8 (q >> 1) - 4 q) channels from
    // its own dwordx2 slot
    const uint32_t vo16 = vo + (16 * (quad & 1) + 8 * (quad >> 1) - 4 * quad) * 2;
#pragma unroll
    for (int m = 0; m + 1 < MR; m += 2) {
      if (cout0 + m * 16 >= a.Cout) continue;  // block-uniform (Cout % 16 == 0)
      uint32_t a0, a1, b0, b1;
      value(m, n, vr, a0, a1);
      value(m + 1, n, vr, b0, b1);
      const auto x0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
      const auto x1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
      const bool ok = cout0 + (m + (quad & 1)) * 16 < a.Cout;
      const uint32_t off = ok ? vo16 + m * 32 : kDrop;
      const v4u32 pk = {x0[0], x1[0], x0[1], x1[1]};
      __builtin_amdgcn_raw_buffer_store_b128(pk, ro, (int)off, 0, 0);
    }
    if constexpr (MR & 1) {  // the last, unpaired fragment: one dwordx2 per lane
      constexpr int m = MR - 1;
      if (cout0 + m * 16 < a.Cout) {
        uint32_t lo, hi;
        value(m, n, vr, lo, hi);
        __builtin_amdgcn_raw_buffer_store_b64(v2u32{lo, hi}, ro, (int)(vo + m * 32), 0, 0);
      }
    }
  }
}

// The patch kernel's form of epilogue_fast, split in two: epi_pack computes
// the tile's packed bf16 outputs and their store offsets into registers
// (the same values and store layout as epilogue_fast; invalid pixels and
// fragments beyond Cout get the dropped offset, so every lane issues every
// store), epi_store issues the stores.  The patch kernel packs before its
// end-of-step barrier and stores after it, so the stores drain under the
// next step's MFMAs instead of being waited for at that barrier
// (s_waitcnt vmcnt(0) counts stores too: tools/conv_phase.py put 26 % of the
// patch kernel's wave time in that wait).
template <int MR, int NR>
struct EpiPend {
  v4u32 pk[MR / 2 > 0 ? MR / 2 : 1][NR];
  uint32_t off[MR / 2 > 0 ? MR / 2 : 1][NR];
  v2u32 pk1[NR];
  uint32_t off1[NR];
};

template <int MR, int NR>
__device__ __forceinline__ void epi_pack(const ConvArgs& a, f32x4 (&acc)[MR][NR], int cout0,
                                         const bool (&pv)[NR], const uint32_t (&opx)[NR], int quad,
                                         const f32x4 (&bias)[MR], EpiPend<MR, NR>& ep) {
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.res, 0, 0x7FFFFFFF, kRsrcFlags);
  const int cq = cout0 + quad * 4;
  constexpr uint32_t kDrop = 0x80000000u;
  // residual: every fragment's 8-B load issued up front, one wait for all
  // (a load then wait per fragment paid a full memory latency each, behind
  // the next stage's DMA in the same in-order counter)
  uint2 rq[MR][NR];
  if (a.res) {
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      const uint32_t vr = (__umul24(opx[n], (uint32_t)a.res_cs) + a.res_co + cq) * 2;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        // invalid pixels (past the map's end on the last image's bottom
        // tile row) and fragments beyond Cout read the dropped offset
        const uint32_t roff = pv[n] && cout0 + m * 16 < a.Cout ? vr + m * 32 : kDrop;
        rq[m][n] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rr, (int)roff, 0, 0));
      }
    }
  }
  auto value = [&](int m, int n, uint32_t vr, uint32_t& lo, uint32_t& hi) {
    (void)vr;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[m][n][i] + bias[m][i];
    if (a.act) silu4(v);
    if (a.res) {
      const uint2 q = rq[m][n];
      v[0] += bf2f(q.x & 0xFFFF);
      v[1] += bf2f(q.x >> 16);
      v[2] += bf2f(q.y & 0xFFFF);
      v[3] += bf2f(q.y >> 16);
    }
    lo = pack_bf16x2(v[0], v[1]);
    hi = pack_bf16x2(v[2], v[3]);
  };
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    const uint32_t vo = (__umul24(opx[n], (uint32_t)a.out0_cs) + a.out0_co + cq) * 2;
    const uint32_t vr = a.res ? (__umul24(opx[n], (uint32_t)a.res_cs) + a.res_co + cq) * 2 : 0u;
    const uint32_t vo16 = vo + (16 * (quad & 1) + 8 * (quad >> 1) - 4 * quad) * 2;
#pragma unroll
    for (int m = 0; m + 1 < MR; m += 2) {
      uint32_t a0, a1, b0, b1;
      value(m, n, vr, a0, a1);
      value(m + 1, n, vr, b0, b1);
      const auto x0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
      const auto x1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
      const bool ok = pv[n] && cout0 + (m + (quad & 1)) * 16 < a.Cout;
      ep.off[m / 2][n] = ok ? vo16 + m * 32 : kDrop;
      ep.pk[m / 2][n] = v4u32{x0[0], x1[0], x0[1], x1[1]};
    }
    if constexpr (MR & 1) {
      constexpr int m = MR - 1;
      uint32_t lo, hi;
      value(m, n, vr, lo, hi);
      ep.off1[n] = pv[n] && cout0 + m * 16 < a.Cout ? vo + m * 32 : kDrop;
      ep.pk1[n] = v2u32{lo, hi};
    }
  }
}

template <int MR, int NR>
__device__ __forceinline__ void epi_store(const ConvArgs& a, const EpiPend<MR, NR>& ep) {
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(a.out0, 0, 0x7FFFFFFF, kRsrcFlags);
#pragma unroll
  for (int n = 0; n < NR; ++n) {
#pragma unroll
    for (int m = 0; m + 1 < MR; m += 2)
      __builtin_amdgcn_raw_buffer_store_b128(ep.pk[m / 2][n], ro, (int)ep.off[m / 2][n], 0, 0);
    if constexpr (MR & 1) __builtin_amdgcn_raw_buffer_store_b64(ep.pk1[n], ro, (int)ep.off1[n], 0, 0);
  }
}

// LDS quarter swizzle of 64-B pixel / weight-row slots: slot quarter q of
// slot i holds source quarter q ^ swzq(i).  bf16 fragments are read with
// ds_read_b128, serviced in four 16-lane groups ({0-3,12-15,20-27},
// {4-11,16-19,28-31} and the same +32; MI355X_MICROARCH.md SLDS): with
// (i >> 1) & 2 the 16 lanes of every group hit 16 distinct 16-B bank slots
// for ANY alignment of the fragment's 16 consecutive slots (searched
// exhaustively); (i >> 2) & 3 collides 2-way in each group.  fp8 fragments
// (ds_read_b64, two 32-lane groups, 8 B per lane) need slots i, i+4, i+8,
// i+12 on distinct quarters: (i >> 2) & 3.
template <bool F8>
__device__ __forceinline__ int swzq(int i) {
  return F8 ? (i >> 2) & 3 : (i >> 1) & 2;
}

// bias: the lane's 4 channels per m-fragment, loaded once per block (a
// global load in the epilogue would make the compiler wait vmcnt(0), i.e.
// drain the next stage's LDS-DMA, before every tile's epilogue)
template <int MR, int NR>
__device__ __forceinline__ void epilogue(const ConvArgs& a, f32x4 (&acc)[MR][NR], int cout0,
                                         const bool (&pv)[NR], const int (&pb)[NR],
                                         const int (&py)[NR], const int (&px)[NR], int quad,
                                         const f32x4 (&bias)[MR]) {
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
      v[0] = acc[m][n][0] + bias[m][0];
      v[1] = acc[m][n][1] + bias[m][1];
      v[2] = acc[m][n][2] + bias[m][2];
      v[3] = acc[m][n][3] + bias[m][3];
      if (a.act) {
        silu4(v);
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
          const uint2 pk = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
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

// Patch layout in LDS.  Stride-1 convs: pixel pp of the halo patch owns 64
// bytes at pp * 64 (its 32 channels = 4 x 16-B quarters); LDS slot quarter
// q of a pixel in patch column px holds source quarter q ^ swzq(px), so the
// 16 consecutive pixels of a B fragment (one patch row) are conflict-free
// in every ds_read_b128 lane group.  The swizzle depends on the column only, so a
// kernel-row step (ky) moves every address by the same PW * 64 and the
// per-lane tap addresses are precomputed once per block (NR x K values).
// Stride-2 convs store the patch columns de-interleaved (even columns, then
// odd ones: stored column sc of column px = px/2 or HE + px/2, HE = the even
// count), so the 16 output pixels of a fragment -- patch columns two apart --
// read 16 consecutive stored columns at every tap (kx = 0: sc = c, 1: HE + c,
// 2: c + 1) and the same swizzle, on the stored column, keeps them
// conflict-free.  The DMA stays lane-linear: lane l of DMA instruction j
// fills slot L = 64 j + l, i.e. stored pixel L / 4, slot quarter L % 4.
template <int S>
constexpr int patch_pixb() {
  return 64;
}
// stored column of patch column px (S = 2: de-interleaved)
template <int S>
__device__ __forceinline__ int patch_scol(int px, int PW) {
  return S == 1 ? px : ((px & 1) ? (PW + 1) / 2 + (px >> 1) : (px >> 1));
}

// Per-lane DMA source offsets of one patch (elements from the image base,
// -1 = zero block), at most patch_maxit(NR, S) DMA instructions per wave.
template <int NR, int S>
constexpr int patch_maxit() {
  return (S == 2 ? 6 : 2) * NR + 2;
}

template <int MR, int NR>
__device__ __forceinline__ void epilogue8(const ConvArgs& a, f32x4 (&acc)[MR][NR], int cout0,
                                          const bool (&pv)[NR], const int (&pb)[NR],
                                          const int (&py)[NR], const int (&px)[NR], int quad,
                                          const f32x4 (&bias)[MR], const f32x4 (&dq)[MR]) {
  const float inv0 = 1.0f / a.s_out0, inv1 = 1.0f / a.s_out1;
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
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[m][n][i] * dq[m][i] + bias[m][i];
      if (a.act) {
        silu4(v);
      }
      if (a.res) {
        const uint32_t rr = *(const uint32_t*)((const uint8_t*)a.res + opix * a.res_cs + a.res_co + co);
        v[0] += __builtin_amdgcn_cvt_f32_fp8((int)rr, 0) * a.s_res;
        v[1] += __builtin_amdgcn_cvt_f32_fp8((int)rr, 1) * a.s_res;
        v[2] += __builtin_amdgcn_cvt_f32_fp8((int)rr, 2) * a.s_res;
        v[3] += __builtin_amdgcn_cvt_f32_fp8((int)rr, 3) * a.s_res;
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        void* outp = d == 0 ? a.out0 : a.out1;
        if (!outp) continue;
        const int cs_ = d == 0 ? a.out0_cs : a.out1_cs;
        const int co_ = (d == 0 ? a.out0_co : a.out1_co) + co;
        const int up = d == 0 ? a.out0_up : a.out1_up;
        const int o8 = d == 0 ? a.out0_8 : a.out1_8;
        const int ny = up ? 2 : 1;
        for (int dy = 0; dy < ny; ++dy)
          for (int dx = 0; dx < ny; ++dx) {
            const size_t q = up ? ((size_t)(b * 2 * a.Ho + 2 * oy + dy) * (2 * a.Wo) + 2 * ox + dx) : opix;
            if (o8) {
              *(uint32_t*)((uint8_t*)outp + q * cs_ + co_) = f8_encode4(v, d == 0 ? inv0 : inv1);
            } else if (a.out_f32) {
              *(float4*)((float*)outp + q * cs_ + co_) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
              *(uint2*)((uint16_t*)outp + q * cs_ + co_) =
                  make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
            }
          }
      }
    }
  }
}

// Persistent, software-pipelined form: the block owns cout tile blockIdx.y
// and walks pixel tiles blockIdx.x, +gridDim.x, ...  A step is (tile, group
// of G input-channel chunks); the DMA of step s+1 -- the next group or the
// next tile's first group -- streams in while step s runs on MFMA and while
// the previous tile's epilogue stores drain.  G > 1 cuts the number of
// dependent DMA round trips per tile (a deep-K layer with few tiles is a
// chain of nch / G latencies, not nch).  RESW: the block's whole weight slab
// (nch chunks) is DMA'd into LDS once at kernel start and stays resident, so
// a step only moves its input patch.  Per-lane DMA offsets are computed once
// per tile (no integer division in the chunk loop).
//
// Grouped form (ConvArgs::g2_*): cout tiles at or above g2_cout0 read their
// own input channel slice / weights / bias (a block-diagonal conv: the
// Detect head's cv2 and cv3 branches in one launch).  The host keeps every
// tile inside one group.
// F8 = true: fp8 e4m3 inputs / weights (ConvArgs::in8).  A pipeline chunk
// is 64 channels (64 B per pixel slot, the same LDS image as the bf16
// kernel's 32-channel chunk); each tap runs two v_mfma_f32_16x16x32_fp8_fp8
// per chunk (channels 0-31 and 32-63), each lane reading 8 of its 16-B
// quarter pair (logical quarter 2h + quad/2, byte (quad & 1) * 8).
// NW = 8 (kind 2): one 512-thread workgroup per CU instead of two of 256,
// so a resident weight slab (or a staged chunk of weights) is shared by 8
// waves and the pixel tile is twice as large -- half the LDS-DMA bytes per
// MFMA of the 4-wave form at the same occupancy (2 waves per SIMD).
// CHM > 0 (ConvArgs::ch_w / ch_mode): a chained 1x1 conv Cout -> Cout on
// the tile's output in LDS (bf16, one cout tile covering Cout): CHM 1 = a
// C2f cv1 (SiLU, stored), 2 = a Detect box branch's last conv + DFL (four
// distances per pixel stored), 3 = a Detect class branch's last conv +
// sigmoid + first maximum (score, class per pixel stored): see chain_tile.
template <int MR, int NR, int K, int S, bool RESW, bool F8, int NW = 4, int CHM = 0>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void conv_patch_kernel(ConvArgs a, PatchGeo g) {
  constexpr bool CH = CHM != 0;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int T2 = K * K;
  constexpr int BC = 16 * MR;
  constexpr int W_BYTES = BC * T2 * 64;
  constexpr int MAXP = patch_maxit<NR, S>();
  static_assert(MAXP <= 32, "tail mask is 32 bits");
  constexpr int WJ = BC * T2 / 16;            // weight DMA instructions per chunk
  constexpr int MAXW = (WJ + NW - 1) / NW;
  constexpr int EB = F8 ? 1 : 2;              // bytes per element
  constexpr int CC = F8 ? 64 : 32;            // channels per chunk (64 B per pixel)
  const int tid = threadIdx.x;
  // the wave index as a scalar: every per-wave DMA test below is then a
  // scalar branch, not an exec-mask region inside the MFMA stream
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int col = lane & 15, quad = lane >> 4;
  const int cout0 = blockIdx.y * BC;  // first output channel of the tile (output numbering)
  // the tile's group: its input slice, weights, bias and weight row base wc0
  int wc0 = cout0, gcout = a.g2_cout0 > 0 ? a.g2_cout0 : a.Cout;
  int in_co = a.in_co, Cin = a.Cin;
  const uint8_t* wts = (const uint8_t*)a.w;
  const float* bias_p = a.bias;
  const float* wsc_p = a.wscale;
  if (a.g2_cout0 > 0 && cout0 >= a.g2_cout0) {
    wc0 = cout0 - a.g2_cout0;
    gcout = a.Cout - a.g2_cout0;
    in_co = a.g2_in_co;
    Cin = a.g2_Cin;
    wts = (const uint8_t*)a.g2_w;
    bias_p = a.g2_bias;
    wsc_p = a.g2_wscale;
  }
  const int wcout_pad = (gcout + 15) & ~15;
  const int cin_pad = (Cin + CC - 1) & ~(CC - 1);
  const int Kp = T2 * cin_pad;                // weight row length (elements)
  const int nch = cin_pad / CC;
  const int G = g.G < nch ? g.G : nch;
  const int ngrp = (nch + G - 1) / G;
  const int chunk_bytes = g.p_bytes + (RESW ? 0 : W_BYTES);
  const int stage_bytes = G * chunk_bytes;
  uint8_t* const stages = smem + (RESW ? nch * W_BYTES : 0);
  constexpr int pad = K / 2;
  const int tiles_img = g.tiles_x * g.tiles_y;
  const int ntiles = a.B * tiles_img;
  const TileWalk walk = tile_walk(ntiles);
  const int nsteps = walk.count() * ngrp;
  const int npp = g.PH * g.PW;
  const float inv_pw = 1.0f / (float)g.PW;

  // block-constant: output slots -> (r, cc) of the tile, patch byte base
  constexpr int PB = patch_pixb<S>(), SL = PB / 16;
  // fp8: lane quad reads channel half 0 at logical quarter quad / 2; half 1
  // (quarter + 2) is the same address XOR 32 (the swizzle XORs the quarter)
  int orow[NR], ocol[NR], boff[NR][K];
  bool oin[NR];
#pragma unroll
  for (int n = 0; n < NR; ++n) {
    const int q = wave * (NR * 16) + n * 16 + col;
    orow[n] = q / g.C;
    ocol[n] = q - orow[n] * g.C;
    oin[n] = q < g.R * g.C;
    // per-lane LDS byte address of tap (0, kx) for output slot n
    const int pr = oin[n] ? orow[n] * S : 0, pc = oin[n] ? ocol[n] * S : 0;
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      const int sc = patch_scol<S>(pc + kx, g.PW);
      const int lq = F8 ? quad >> 1 : quad;
      if constexpr (F8 && K == 3)  // tap-pair path: pixel slot base | swizzle (low bits)
        boff[n][kx] = (pr * g.PW + sc) * 64 + swzq<true>(sc);
      else
        boff[n][kx] = (pr * g.PW + sc) * 64 + ((lq ^ swzq<F8>(sc)) << 4) + (F8 ? (quad & 1) * 8 : 0);
    }
  }
  // fp8 3x3 convs run v_mfma_scale_f32_16x16x128_f8f6f4 (unit scales) on tap
  // pairs: k-slots 32q .. 32q+31 of lane quad q = channels 32 (q & 1) ..
  // +31 of tap t + (q >> 1) -- two 16-B quarters of that tap's 64-B slot.
  // aoff: this lane's two weight-quarter offsets within a (row, tap) slot
  // pair, per m (row = m*16 + col; the swizzle of the row picks the order)
  int aoff[F8 && K == 3 ? MR : 1][2];
  if constexpr (F8 && K == 3) {
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const int row = m * 16 + col, sw = swzq<true>(row);
      const int base = (row * T2 + (quad >> 1)) * 64;
      aoff[m][0] = base + (((2 * (quad & 1)) ^ sw) << 4);
      aoff[m][1] = base + (((2 * (quad & 1) + 1) ^ sw) << 4);
    }
  }
  // bf16: the block's bias lives in LDS (BC floats after the two stages;
  // patch_geo sizes it) and is read back per tile in the epilogue, so its
  // 4 * MR registers are free during the MFMA loop.  fp8 keeps bias and
  // dequantisation scales in registers.
  float* const bias_lds = (float*)(stages + 2 * stage_bytes);
  f32x4 bias[F8 ? MR : 1], dq[F8 ? MR : 1];
  if constexpr (F8) {
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const int co = wc0 + m * 16 + quad * 4;  // bias is padded to Cout_pad16
      bias[m] = co < wcout_pad ? *(const f32x4*)(bias_p + co) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 ws = co < wcout_pad ? *(const f32x4*)(wsc_p + co) : f32x4{0.f, 0.f, 0.f, 0.f};
      dq[m] = ws * a.s_in;
    }
  } else {
    for (int i = tid; i < BC; i += 64 * NW) bias_lds[i] = wc0 + i < wcout_pad ? bias_p[wc0 + i] : 0.f;
  }
  auto bias_tile = [&](f32x4 (&bl)[MR]) {
#pragma unroll
    for (int m = 0; m < MR; ++m) bl[m] = *(const f32x4*)(bias_lds + m * 16 + quad * 4);
  };
  // CH: the chained 1x1's weights (chunk-major [c][row][64 B], the quarter
  // swizzle of conv1x1_direct_kernel), its bias, and one x tile per wave
  // (the wave's 16 NR pixels x Cout channels of the producer's bf16 output,
  // chunk-major [c][pixel][64 B], quarter swizzle by pixel)
  constexpr int CHN = (MR + 1) / 2;                 // 32-channel chunks of the chained input
  constexpr int CHF = BC + 4;                       // CHM 2: floats per pixel row of the logit tile
  uint8_t* const ch_w_lds = (uint8_t*)(bias_lds + BC);
  float* const ch_b_lds = (float*)(ch_w_lds + (CH ? CHN * BC * 64 : 0));
  uint8_t* const ch_x_lds = (uint8_t*)(ch_b_lds + (CH ? BC : 0)) + wave * (CH ? CHN * NR * 16 * 64 : 0);
  float* const ch_f_lds = (float*)((uint8_t*)(ch_b_lds + (CH ? BC : 0)) + NW * (CH ? CHN * NR * 16 * 64 : 0)) +
                          wave * (CHM == 2 ? NR * 16 * CHF : 0);
  if constexpr (CH) {
    static_assert(!F8 && K == 3, "chained 1x1: bf16 behind a 3x3 conv");
    // BC / 16 DMA instructions per chunk (16 rows x 64 B each); the packed
    // 1x1 rows are CHN * 32 channels long (zero beyond Cout)
    for (int j = wave; j < CHN * (BC / 16); j += NW) {
      const int c = j / (BC / 16), jr = j - c * (BC / 16);
      const int row = jr * 16 + (lane >> 2);
      const int q = (lane & 3) ^ swzq<false>(row);
      __builtin_amdgcn_global_load_lds((const void*)(a.ch_w + (size_t)row * (CHN * 32) + c * 32 + q * 8),
                                       (void*)(ch_w_lds + c * BC * 64 + jr * 1024), 16, 0, 0);
    }
    for (int i = tid; i < BC; i += 64 * NW) ch_b_lds[i] = a.ch_b[i];
    if constexpr (MR % 2) {  // odd MR: the last chunk's upper half is k-padding, zero for good
      for (int px = lane; px < NR * 16; px += 64) {
        uint8_t* sl = ch_x_lds + ((CHN - 1) * NR * 16 + px) * 64;
        *(uint4*)(sl + ((2 ^ swzq<false>(px)) << 4)) = make_uint4(0, 0, 0, 0);
        *(uint4*)(sl + ((3 ^ swzq<false>(px)) << 4)) = make_uint4(0, 0, 0, 0);
      }
    }
  }
  // Patch and weight DMA through buffer resources (buffer_load ... lds):
  // every DMA instruction's per-lane byte offset is computed once -- per
  // tile for the patch, per kernel for the weights --, the chunk offset
  // rides in the scalar soffset, and out-of-image pixels / rows beyond Cout
  // read zeros from the range check (voffset kOOB).  So a chunk step issues
  // its DMA with no address VALU; the tile-invariant lane geometry (patch
  // row, column, source quarter of every slot) is computed once per kernel.
  uint32_t tailbad = 0;  // bit it: this lane's quarter is >= Cin in the last chunk
  // slot it's patch row / column / source quarter: py | px << 12 | sq << 24;
  // a slot beyond the patch gets row 4095, which no map reaches (range check)
  int lgeo[MAXP];
#pragma unroll
  for (int it = 0; it < MAXP; ++it) {
    const int L = 64 * (wave + NW * it) + lane;
    const int pix = L / SL, q = L - SL * pix;
    const int py = (int)(((float)pix + 0.5f) * inv_pw);
    const int sc = pix - py * g.PW;  // stored column
    const int he = (g.PW + 1) >> 1;
    const int px = S == 1 ? sc : (sc < he ? 2 * sc : 2 * (sc - he) + 1);
    const int sq = q ^ swzq<F8>(sc);  // source quarter of slot q
    lgeo[it] = (pix < npp ? py : 4095) | (px << 12) | (sq << 24);
    if ((nch - 1) * CC + sq * (16 / EB) >= Cin) tailbad |= 1u << it;
  }
  const bool has_tail = Cin % CC != 0;
  uint32_t voff[MAXP];
  __amdgpu_buffer_rsrc_t img_rsrc;
  const int pix_bytes = a.in_cs * EB;
  auto prep_tile = [&](int ti) {
    const int b = ti / tiles_img;
    const int r = ti - b * tiles_img;
    const int ty = r / g.tiles_x, tx = r - (r / g.tiles_x) * g.tiles_x;
    const int iy0 = ty * g.R * S - pad, ix0 = tx * g.C * S - pad;
    const uint8_t* base = (const uint8_t*)a.in + ((size_t)b * a.Hin * a.Win * a.in_cs + in_co) * EB;
    img_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0,
                                                 (a.Hin * a.Win * a.in_cs - in_co) * EB, kRsrcFlags);
#pragma unroll
    for (int it = 0; it < MAXP; ++it) {
      const int gg = lgeo[it];
      const int iy = iy0 + (gg & 4095), ix = ix0 + ((gg >> 12) & 4095);
      const bool ok = (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
      // branchless select: an out-of-image slot reads zeros (kOOB)
      // 24-bit multiplies (full rate): a map pixel index and the pixel
      // stride are < 2^24 and the in-image byte offset < 2^31, so the low 32
      // bits are the product (an out-of-image slot's garbage is masked)
      const uint32_t off = __umul24((uint32_t)(__umul24(iy, a.Win) + ix), (uint32_t)pix_bytes) +
                           ((gg >> 24) & 3) * 16;
      const uint32_t m = ok ? 0u : 0xFFFFFFFFu;
      voff[it] = (off & ~m) | (kOOB & m);
    }
  };
  // weight DMA: instruction j moves (row, tap) pairs 16 j .. 16 j + 15, a
  // 16-B quarter of chunk c per lane
  const __amdgpu_buffer_rsrc_t w_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(wts + (size_t)wc0 * Kp * EB), 0, (wcout_pad - wc0) * Kp * EB, kRsrcFlags);
  uint32_t wvoff[MAXW];
#pragma unroll
  for (int it = 0; it < MAXW; ++it) {
    const int j = wave + NW * it;
    const int pr = j * 16 + (lane >> 2);
    const int row = pr / T2, tap = pr - (pr / T2) * T2;
    const int q = (lane & 3) ^ swzq<F8>(row);
    wvoff[it] = wc0 + row < wcout_pad ? (uint32_t)((row * Kp + tap * cin_pad) * EB + q * 16) : kOOB;
  }
  auto dma_weights = [&](int c, uint8_t* Wl) {
#pragma unroll
    for (int it = 0; it < MAXW; ++it) {
      const int j = wave + NW * it;
      if (j < WJ) dma16(w_rsrc, Wl + j * 1024, wvoff[it], c * 64);
    }
  };
  auto stage = [&](int grp, int buf) {
    for (int gi = 0; gi < G; ++gi) {
      const int c = grp * G + gi;
      if (c >= nch) break;
      uint8_t* P = stages + buf * stage_bytes + gi * chunk_bytes;
      const bool tail = has_tail && c == nch - 1;  // block-uniform
      // Two paths: a select feeding every DMA (tail chunk only) made the
      // compiler route all of them through ONE address VGPR, and each
      // v_cndmask into it then waited for the previous buffer_load to read
      // its operand (a VMEM-read / VALU-write interlock per DMA); the common
      // path issues straight from the per-slot offset registers.
#ifdef RV_DMA_SELECT_ALWAYS  // A/B: the r05 single path
      if (true) {
#else
      if (tail) {
#endif
#pragma unroll
        for (int it = 0; it < MAXP; ++it) {
          const int j = wave + NW * it;
          if (j < g.pinst)
            dma16<RV_CONV_IN_AUX>(img_rsrc, P + j * 1024,
                                  tail && ((tailbad >> it) & 1) ? kOOB : voff[it], c * 64);
        }
      } else {
#pragma unroll
        for (int it = 0; it < MAXP; ++it) {
          const int j = wave + NW * it;
          if (j < g.pinst) dma16<RV_CONV_IN_AUX>(img_rsrc, P + j * 1024, voff[it], c * 64);
        }
      }
      if constexpr (!RESW) dma_weights(c, P + g.p_bytes);
    }
  };
  f32x4 acc[MR][NR];
  auto compute = [&](int grp, int buf) {
    for (int gi = 0; gi < G; ++gi) {
      const int c = grp * G + gi;
      if (c >= nch) break;
      const uint8_t* P = stages + buf * stage_bytes + gi * chunk_bytes;
      const uint8_t* Wl = RESW ? smem + c * W_BYTES : P + g.p_bytes;
      if constexpr (F8 && K == 3) {
        const int rowb = g.PW * PB;
#pragma unroll
        for (int t = 0; t < 9; t += 2) {
          const bool odd = t + 1 >= 9;  // the last tap pairs with zeros
          const int ky0 = t / 3, kx0 = t % 3;
          const int ky1 = odd ? ky0 : (t + 1) / 3, kx1 = odd ? kx0 : (t + 1) % 3;
          const bool hi = (quad >> 1) != 0;
          i32x8 A[MR], Bv[NR];
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            const uint4 lo = *(const uint4*)(Wl + aoff[m][0] + t * 64);
            const uint4 up = *(const uint4*)(Wl + aoff[m][1] + t * 64);
            A[m] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w,
                         (int)up.x, (int)up.y, (int)up.z, (int)up.w};
            if (odd && hi) A[m] = i32x8{0, 0, 0, 0, 0, 0, 0, 0};
          }
#pragma unroll
          for (int n = 0; n < NR; ++n) {
            const int v = hi ? boff[n][kx1] + ky1 * rowb : boff[n][kx0] + ky0 * rowb;
            const int sw = v & 3, base = v & ~63;
            const uint4 lo = *(const uint4*)(P + base + (((2 * (quad & 1)) ^ sw) << 4));
            const uint4 up = *(const uint4*)(P + base + (((2 * (quad & 1) + 1) ^ sw) << 4));
            Bv[n] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w,
                          (int)up.x, (int)up.y, (int)up.z, (int)up.w};
          }
#pragma unroll
          for (int m = 0; m < MR; ++m)
#pragma unroll
            for (int n = 0; n < NR; ++n)
              acc[m][n] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                  A[m], Bv[n], acc[m][n], 0, 0, 0, 127, 0, 127);
        }
        continue;
      }
      if constexpr (!F8 && MR * NR < 16) {
        // bf16: the taps' fragment reads are software-pipelined one tap
        // ahead -- tap t + 1's A / B fragments are read into the other
        // register set before tap t's MFMAs issue, so the MFMAs of a tap
        // never wait on the LDS reads issued right before them
        bf16x8 Af[2][MR], Bq[2][NR];
        auto ld = [&](int tap, int sl) {
          const int ky = tap / K, kx = tap - (tap / K) * K;
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            const int row = m * 16 + col;
            Af[sl][m] = __builtin_bit_cast(
                bf16x8, *(const uint4*)(Wl + (row * T2 + tap) * 64 + ((quad ^ swzq<false>(row)) << 4)));
          }
#pragma unroll
          for (int n = 0; n < NR; ++n)
            Bq[sl][n] = __builtin_bit_cast(bf16x8, *(const uint4*)(P + ky * g.PW * PB + boff[n][kx]));
        };
        ld(0, 0);
#pragma unroll
        for (int t = 0; t < T2; ++t) {
          // hard fences pin the order (the scheduler otherwise sinks each
          // read next to its first use): tap t + 1's reads, then tap t's
          // MFMAs, which wait only for the reads issued one tap earlier
          if (t + 1 < T2) ld(t + 1, (t + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int m = 0; m < MR; ++m)
#pragma unroll
            for (int n = 0; n < NR; ++n)
              acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[t & 1][m], Bq[t & 1][n],
                                                                  acc[m][n], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
        continue;
      }
      // (fp8, and the largest bf16 tiles, whose fragments of all taps in
      // flight would exceed the register file: kernel rows not unrolled)
#pragma unroll(F8 || MR * NR >= 16 ? 1 : K)
      for (int ky = 0; ky < K; ++ky) {
        const uint8_t* Prow = P + ky * g.PW * PB;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int tap = ky * K + kx;
          if constexpr (F8) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              long A[MR], Bf[NR];
#pragma unroll
              for (int m = 0; m < MR; ++m) {
                const int row = m * 16 + col;
                A[m] = *(const long*)(Wl + (((row * T2 + tap) * 64 +
                                             (((quad >> 1) ^ swzq<true>(row)) << 4) + (quad & 1) * 8) ^
                                            (hh << 5)));
              }
#pragma unroll
              for (int n = 0; n < NR; ++n) Bf[n] = *(const long*)(Prow + (boff[n][kx] ^ (hh << 5)));
              // every read of the tap issued before its MFMAs (left alone,
              // the scheduler waits for each A fragment right before its
              // MFMAs: one LDS round trip per m)
              __builtin_amdgcn_sched_barrier(0);
#pragma unroll
              for (int m = 0; m < MR; ++m)
#pragma unroll
                for (int n = 0; n < NR; ++n)
                  acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(A[m], Bf[n], acc[m][n], 0, 0, 0);
            }
          } else {
            bf16x8 A[MR], Bf[NR];
#pragma unroll
            for (int m = 0; m < MR; ++m) {
              const int row = m * 16 + col;
              A[m] = __builtin_bit_cast(
                  bf16x8, *(const uint4*)(Wl + (row * T2 + tap) * 64 + ((quad ^ swzq<false>(row)) << 4)));
            }
#pragma unroll
            for (int n = 0; n < NR; ++n)
              Bf[n] = __builtin_bit_cast(bf16x8, *(const uint4*)(Prow + boff[n][kx]));
            // every read of the tap issued before its MFMAs (left alone, the
            // scheduler waits for each A fragment right before its MFMAs:
            // one LDS round trip per m)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < MR; ++m)
#pragma unroll
              for (int n = 0; n < NR; ++n)
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[m], Bf[n], acc[m][n], 0, 0, 0);
          }
        }
      }
    }
  };

  if (nsteps == 0) return;
#ifdef RV_PHASE_PROF
  unsigned long long ph[5] = {0, 0, 0, 0, 0}, t_ph = RV_PH_T();
#define RV_PH(i)                             \
  {                                          \
    const unsigned long long t_ = RV_PH_T(); \
    ph[i] += t_ - t_ph;                      \
    t_ph = t_;                               \
  }
#else
#define RV_PH(i)
#endif
  int ti = walk.t0;  // tile of the current step
  int grp = 0;       // chunk group of the current step
  // Stagger (8-wave form): the two waves of a SIMD are wave w and w + 4 of
  // this block, and with one barrier per step they reach their MFMAs and
  // their epilogue VALU together.  Waves 4-7 ("late") instead finish each
  // tile at the start of the NEXT step, right after the barrier, with the
  // sums still in their accumulators: on every SIMD one wave's epilogue
  // (bias, SiLU, pack, stores) then runs beside its partner's MFMAs
  // (MI355X_MICROARCH.md "Two waves per SIMD" item 9).  Same values, same
  // stores: outputs are bit-identical.
  // (not built for the 5x2 / 2x4 tiles: their extra epilogue site spills)
  constexpr bool kStagger = NW == 8 && !(MR == 5 && NR == 2) && !(MR == 2 && NR == 4);
  const bool late = kStagger && g.stagger && wave >= 4;  // wave is a scalar
  bool pend = false;  // late waves: a finished tile (ptile) awaits its epilogue
  int ptile = 0;
  constexpr bool kDefer = !F8 && !CH && MR * NR <= 10;
  // epilogue of tile `tile` from acc; `pk`: pack only (stores after the
  // barrier, epi_store)
  // CH: the finished tile's producer values (bias, SiLU, bf16 -- what the
  // unfused conv stores) go to this wave's x tile instead of HBM, then the
  // chained 1x1 runs on them: per 32-channel chunk c ascending, A = its
  // weights, B = the wave's pixels (the k order of conv1x1_direct_kernel and
  // of the patch kernel's 1x1 form: bit-identical to the unfused launch),
  // and its epilogue (bias, SiLU) stores the output views.  Each wave reads
  // only the pixels it wrote (in-order LDS, no barrier).
  auto chain_tile = [&](const bool (&pv)[NR], const uint32_t (&opx)[NR]) {
    if constexpr (CH) {
      f32x4 bl[MR];
      bias_tile(bl);
      if constexpr (MR % 2) {  // odd MR: each lane stores its 4 channels (8 B) of every fragment
#pragma unroll
        for (int n = 0; n < NR; ++n) {
          const int px = n * 16 + col;
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = acc[m][n][i] + bl[m][i];
            if (a.act) silu4(v);
            const int qq = 2 * (m & 1) + (quad >> 1);  // channels 16 (m & 1) + 4 quad of chunk m / 2
            *(v2u32*)(ch_x_lds + ((m / 2) * NR * 16 + px) * 64 + ((qq ^ swzq<false>(px)) << 4) +
                      (quad & 1) * 8) = v2u32{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
          }
        }
      } else {
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        const int px = n * 16 + col;
#pragma unroll
        for (int m = 0; m < MR; m += 2) {
          uint32_t v0[2], v1[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = acc[m + h][n][i] + bl[m + h][i];
            if (a.act) silu4(v);
            v0[h] = pack_bf16x2(v[0], v[1]);
            v1[h] = pack_bf16x2(v[2], v[3]);
          }
          // quad q: channels 16 (q & 1) + 8 (q >> 1) .. +7 of chunk m / 2
          const auto x0 = __builtin_amdgcn_permlane16_swap(v0[0], v0[1], false, false);
          const auto x1 = __builtin_amdgcn_permlane16_swap(v1[0], v1[1], false, false);
          const int qq = 2 * (quad & 1) + (quad >> 1);
          *(v4u32*)(ch_x_lds + ((m / 2) * NR * 16 + px) * 64 + ((qq ^ swzq<false>(px)) << 4)) =
              v4u32{x0[0], x1[0], x0[1], x1[1]};
        }
      }
      }
      f32x4 acc2[MR][NR];
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n) acc2[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < CHN; ++c) {
        bf16x8 A2[MR], B2[NR];
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          const int row = m * 16 + col;
          A2[m] = __builtin_bit_cast(
              bf16x8, *(const uint4*)(ch_w_lds + c * BC * 64 + row * 64 + ((quad ^ swzq<false>(row)) << 4)));
        }
#pragma unroll
        for (int n = 0; n < NR; ++n) {
          const int px = n * 16 + col;
          B2[n] = __builtin_bit_cast(
              bf16x8, *(const uint4*)(ch_x_lds + (c * NR * 16 + px) * 64 + ((quad ^ swzq<false>(px)) << 4)));
        }
#pragma unroll
        for (int m = 0; m < MR; ++m)
#pragma unroll
          for (int n = 0; n < NR; ++n)
            acc2[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A2[m], B2[n], acc2[m][n], 0, 0, 0);
      }
      f32x4 bl2[MR];
#pragma unroll
      for (int m = 0; m < MR; ++m) bl2[m] = *(const f32x4*)(ch_b_lds + m * 16 + quad * 4);
      if constexpr (CHM == 1) {
        ConvArgs a2 = a;
        a2.act = 1;
        a2.res = nullptr;
        epilogue_fast<MR, NR>(a2, acc2, 0, pv, opx, quad, bl2);
      } else if constexpr (CHM == 2) {
        // box branch: 4 sides x 16 DFL bins (fragment m = side m).  The f32
        // logits go to this wave's LDS rows, then 4 lanes per pixel take a
        // side each: softmax expectation over its bins exactly as
        // detect_decode_kernel computes it (same op order), and the pixel's
        // four distances are stored as one f32x4
        static_assert(MR == 4, "box branch: 4 sides of 16 bins");
#pragma unroll
        for (int n = 0; n < NR; ++n)
#pragma unroll
          for (int m = 0; m < MR; ++m)
            *(f32x4*)(ch_f_lds + (n * 16 + col) * CHF + m * 16 + quad * 4) = acc2[m][n] + bl2[m];
        const int pxl = lane >> 2, part = lane & 3;
#pragma unroll
        for (int n = 0; n < NR; ++n) {
          const float* row = ch_f_lds + (n * 16 + pxl) * CHF + part * 16;
          float v[16];
#pragma unroll
          for (int i = 0; i < 16; i += 4) {
            const f32x4 q4 = *(const f32x4*)(row + i);
            v[i] = q4[0];
            v[i + 1] = q4[1];
            v[i + 2] = q4[2];
            v[i + 3] = q4[3];
          }
          float mx = -INFINITY;
#pragma unroll
          for (int i = 0; i < 16; ++i) mx = fmaxf(mx, v[i]);
          float sum = 0.f;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            v[i] = __expf(v[i] - mx);
            sum += v[i];
          }
          const float rs = __builtin_amdgcn_rcpf(sum);
          float e = 0.f;
#pragma unroll
          for (int i = 0; i < 16; ++i) e += (float)i * (v[i] * rs);
          const int base = lane & ~3;
          const float d0 = __shfl(e, base), d1 = __shfl(e, base + 1), d2 = __shfl(e, base + 2),
                      d3 = __shfl(e, base + 3);
          // pixel pxl of fragment n: lane pxl holds its validity and index
          const uint32_t o = (uint32_t)__shfl((int)opx[n], pxl);
          const bool ok = __shfl((int)pv[n], pxl) != 0;
          if (part == 0 && ok) *(f32x4*)((float*)a.out0 + (size_t)o * 4) = f32x4{d0, d1, d2, d3};
        }
      } else {
        // class branch: sigmoid of every class, the first maximum in class
        // order (lane scan over its classes m * 16 + 4 quad + i ascending,
        // then the larger score / smaller class across the quads) -- the
        // fixed decode's head_mfma_fixed selection; (score, class) stored
#pragma unroll
        for (int n = 0; n < NR; ++n) {
          float best = -1.f;
          int bc = 0;
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            const int co = m * 16 + quad * 4;
            const f32x4 v = acc2[m][n] + bl2[m];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float sg = head_sigmoid(v[i]);
              if (co + i < a.Cout && sg > best) {
                best = sg;
                bc = co + i;
              }
            }
          }
#pragma unroll
          for (int off = 16; off < 64; off <<= 1) {
            const float ob = __shfl_xor(best, off);
            const int oc = __shfl_xor(bc, off);
            if (ob > best || (ob == best && oc < bc)) {
              best = ob;
              bc = oc;
            }
          }
          if (quad == 0 && pv[n])
            *(v2u32*)((float*)a.out0 + (size_t)opx[n] * 2) =
                v2u32{__float_as_uint(best), (uint32_t)bc};
        }
      }
    }
  };
  auto finish = [&](int tile, EpiPend<MR, NR>& ep, bool pk) {
    const int b = tile / tiles_img;
    const int r = tile - b * tiles_img;
    const int ty = r / g.tiles_x, tx = r - (r / g.tiles_x) * g.tiles_x;
    bool pv[NR];
    int pb[NR], py[NR], px[NR];
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      pb[n] = b;
      py[n] = ty * g.R + orow[n];
      px[n] = tx * g.C + ocol[n];
      pv[n] = oin[n] && py[n] < a.Ho && px[n] < a.Wo;
    }
#ifdef RV_EPI_SKIP
    if (a.Cout == 12345) {  // timing experiment: keep the MFMAs live, skip the epilogue
      float t = 0.f;
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n) t += acc[m][n][0] + acc[m][n][3];
      ((float*)a.out0)[tid] = t;
    }
    if (true) {
    } else
#endif
    if constexpr (F8) {
      epilogue8<MR, NR>(a, acc, cout0, pv, pb, py, px, quad, bias, dq);
    } else if constexpr (CH) {
      uint32_t opx[NR];
#pragma unroll
      for (int n = 0; n < NR; ++n) opx[n] = (uint32_t)((b * a.Ho + py[n]) * a.Wo + px[n]);
      chain_tile(pv, opx);
    } else if (g.fast) {
      uint32_t opx[NR];  // < 2^23 (epi_fast): 24-bit multiplies
#pragma unroll
      for (int n = 0; n < NR; ++n) opx[n] = __umul24((uint32_t)(b * a.Ho + py[n]), (uint32_t)a.Wo) + px[n];
      f32x4 bl[MR];
      bias_tile(bl);
      if constexpr (kDefer) {
        if (pk)
          epi_pack<MR, NR>(a, acc, cout0, pv, opx, quad, bl, ep);
        else
          epilogue_fast<MR, NR>(a, acc, cout0, pv, opx, quad, bl);
      } else {
        epilogue_fast<MR, NR>(a, acc, cout0, pv, opx, quad, bl);
      }
    } else {
      f32x4 bl[MR];
      bias_tile(bl);
      epilogue<MR, NR>(a, acc, cout0, pv, pb, py, px, quad, bl);
    }
  };
  if constexpr (RESW)
    for (int c = 0; c < nch; ++c) dma_weights(c, smem + c * W_BYTES);
  prep_tile(ti);
  stage(0, 0);
  __syncthreads();
  RV_PH(0);
  for (int s = 0; s < nsteps; ++s) {
    EpiPend<MR, NR> ep;
    if (kStagger && pend) {  // late waves: the previous tile, before its accumulators are reset
      finish(ptile, ep, false);
      pend = false;
    }
    if (grp == 0) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // issue step s+1
    const bool last = grp + 1 == ngrp;
    if (s + 1 < nsteps) {
      if (last) prep_tile(ti + walk.step);
      stage(last ? 0 : grp + 1, (s + 1) & 1);
    }
    RV_PH(1);
    compute(grp, s & 1);
    RV_PH(2);
    // a finished tile's packed outputs, stored after the barrier (tiles whose
    // pack registers fit beside the compute registers without spills)
    if (last) {
      if (late) {
        pend = true;
        ptile = ti;
      } else {
        finish(ti, ep, true);
      }
      ti += walk.step;
      grp = 0;
      RV_PH(3);
    } else {
      ++grp;
    }
    __syncthreads();
    if constexpr (kDefer) {
      if (last && g.fast && !late) epi_store<MR, NR>(a, ep);  // the finished tile's stores (epi_pack)
    }
    RV_PH(4);
  }
  if (kStagger && pend) {
    EpiPend<MR, NR> ep;
    finish(ptile, ep, false);
  }
#ifdef RV_PHASE_PROF
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i) atomicAdd(&g_conv_phase[i], ph[i]);
    atomicAdd(&g_conv_phase[5], (unsigned long long)nsteps);
    atomicAdd(&g_conv_phase[6], 1ull);
  }
#endif
#undef RV_PH
}


// ---------------------------------------------------------------------------
// conv1x1_direct_kernel: 1x1 stride-1 convs without LDS staging of the
// pixels.  A 1x1 conv has no halo, so an input pixel feeds exactly one B
// fragment column: each lane loads its 16-B fragment slice straight from
// HBM/L2 into VGPRs (global_load_dwordx4), and chunk c+1's loads are in
// flight while chunk c runs on MFMA -- no LDS round trip and no barrier in
// the K loop.  The block's weights (16*MR couts x Cin) are DMA'd into LDS
// once (same per-chunk layout and quarter swizzle as the patch kernel) and
// stay resident while a persistent block walks its pixel tiles (64*NR
// consecutive NHWC pixels of the flattened B x H x W range).  The k order
// (chunks ascending, 32 channels per MFMA) equals the patch kernel's, so the
// two are bit-identical.
// ---------------------------------------------------------------------------
template <int MR, int NR>
__global__ __launch_bounds__(256, 2) void conv1x1_direct_kernel(ConvArgs a, int fast) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int BC = 16 * MR;
  constexpr int W_BYTES = BC * 64;  // one 32-channel chunk of the block's weights
  constexpr int WJ = BC / 16;       // its DMA instructions (16 rows x 64 B each)
  constexpr int MAXW = (WJ + 3) / 4;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, quad = lane >> 4;
  const int cout0 = blockIdx.y * BC;
  const int wcout_pad = (a.Cout + 15) & ~15;
  const int cin_pad = (a.Cin + 31) & ~31;
  const int nch = cin_pad >> 5;
  const int HW = a.Ho * a.Wo;
  const int npix = a.B * HW;
  const int ntiles = (npix + 64 * NR - 1) / (64 * NR);
  for (int c = 0; c < nch; ++c) {
#pragma unroll
    for (int it = 0; it < MAXW; ++it) {
      const int j = wave + 4 * it;
      if (j < WJ) {
        const int row = j * 16 + (lane >> 2);
        const int q = (lane & 3) ^ swzq<false>(row);
        const int co = cout0 + row;
        const void* src = co < wcout_pad ? (const void*)(a.w + (size_t)co * cin_pad + q * 8 + c * 32)
                                         : (const void*)g_zero16;
        __builtin_amdgcn_global_load_lds(src, (void*)(smem + c * W_BYTES + j * 1024), 16, 0, 0);
      }
    }
  }
  __syncthreads();
  f32x4 bias[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    const int co = cout0 + m * 16 + quad * 4;  // bias is padded to Cout_pad16
    bias[m] = co < wcout_pad ? *(const f32x4*)(a.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // per-lane A fragment offsets within a chunk
  int aoff[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    const int row = m * 16 + col;
    aoff[m] = row * 64 + ((quad ^ swzq<false>(row)) << 4);
  }
  // (b, y, x) of a pixel only where it is used: the upsampled view and the
  // generic epilogue (integer divisions are long VALU sequences)
  const bool need_geo = a.in_up || !fast;
  const TileWalk walk = tile_walk(ntiles);
  // a tile's lane pixels: source pointers of both input views and validity
  struct Geo {
    const bf16_t* src[NR];
    const bf16_t* src2[NR];
    bool pv[NR];
    int pb[NR], py[NR], px[NR];
  };
  auto geo = [&](int t, Geo& G) {
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      const int p = t * 64 * NR + wave * 16 * NR + n * 16 + col;
      G.pv[n] = t < walk.end && p < npix;
      const int pp = G.pv[n] ? p : 0;
      G.pb[n] = G.py[n] = G.px[n] = 0;
      if (need_geo) {
        G.pb[n] = pp / HW;
        const int r = pp - G.pb[n] * HW;
        G.py[n] = r / a.Wo;
        G.px[n] = r - G.py[n] * a.Wo;
      }
      // the `in` view's pixel: itself, or (y/2, x/2) of the half-resolution map
      const size_t ps = a.in_up ? ((size_t)G.pb[n] * (a.Ho >> 1) + (G.py[n] >> 1)) * (a.Wo >> 1) +
                                      (G.px[n] >> 1)
                                : (size_t)pp;
      G.src[n] = a.in + ps * a.in_cs + a.in_co + quad * 8;
      // the in2 view, addressed by logical channel (chunks at or above split)
      G.src2[n] = a.in2 + (size_t)pp * a.in2_cs + a.in2_co + quad * 8 - a.split;
    }
  };
  // the B fragments of chunk c of tile G (unconditional loads: invalid
  // pixels / channels read the zero block; a branch around a load would make
  // the compiler drain vmcnt to 0 before the MFMAs, i.e. wait for the
  // prefetched chunks as well)
  auto load = [&](const Geo& G, int c, uint4 (&B)[NR]) {
    const bool kin = c * 32 + quad * 8 < a.Cin;
    const bool second = a.split > 0 && c * 32 >= a.split;
#pragma unroll
    for (int n = 0; n < NR; ++n)
      B[n] = *(const uint4*)((G.pv[n] && kin) ? (const void*)((second ? G.src2[n] : G.src[n]) + c * 32)
                                              : (const void*)g_zero16);
  };
  auto mma = [&](int c, const uint4 (&B)[NR], f32x4 (&acc)[MR][NR]) {
    const uint8_t* Wl = smem + c * W_BYTES;
    bf16x8 A[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) A[m] = __builtin_bit_cast(bf16x8, *(const uint4*)(Wl + aoff[m]));
    // all MR weight reads in flight before the first MFMA (left alone, the
    // scheduler waits for each A fragment right before its MFMAs)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int n = 0; n < NR; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[m], __builtin_bit_cast(bf16x8, B[n]),
                                                            acc[m][n], 0, 0, 0);
  };
  auto finish = [&](int t, const Geo& G, f32x4 (&acc)[MR][NR]) {
    if (fast) {
      uint32_t opx[NR];
#pragma unroll
      for (int n = 0; n < NR; ++n) opx[n] = (uint32_t)(t * 64 * NR + wave * 16 * NR + n * 16 + col);
      epilogue_fast<MR, NR>(a, acc, cout0, G.pv, opx, quad, bias);
    } else {
      epilogue<MR, NR>(a, acc, cout0, G.pv, G.pb, G.py, G.px, quad, bias);
    }
  };
  // A stream of (tile, chunk) positions with two chunk loads always in
  // flight ACROSS tile boundaries: the last chunks' MFMAs and the epilogue of
  // tile t run while tile t + step's first two chunks load (G1), so a
  // persistent block never restarts its pipeline from an empty queue, and no
  // chunk is loaded twice.  A tile spans P = nch rounded up to even positions
  // (an odd count's last position reads the zero block: the k-order and sums
  // are unchanged).
  const int P = (nch + 1) & ~1;
  uint4 B0[NR], B1[NR];
  Geo G0, G1;
  int t = walk.t0;
  geo(t, G0);
  geo(t + walk.step, G1);
  // (the last pair of positions is peeled: no branch around a load, which
  // made the compiler wait for every outstanding load at the join)
  load(G0, 0, B0);
  load(G0, 1, B1);
  for (; t < walk.end; t += walk.step) {
    f32x4 acc[MR][NR];
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < P - 2; c += 2) {  // B0: chunk c, B1: chunk c + 1 (< nch here)
      mma(c, B0, acc);
      __builtin_amdgcn_sched_barrier(0);
      load(G0, c + 2, B0);
      __builtin_amdgcn_sched_barrier(0);
      mma(c + 1, B1, acc);
      __builtin_amdgcn_sched_barrier(0);
      load(G0, c + 3, B1);
      __builtin_amdgcn_sched_barrier(0);
    }
    mma(P - 2, B0, acc);
    __builtin_amdgcn_sched_barrier(0);
    load(G1, 0, B0);
    __builtin_amdgcn_sched_barrier(0);
    if (P - 1 < nch) mma(P - 1, B1, acc);  // odd nch: position P - 1 is padding
    __builtin_amdgcn_sched_barrier(0);
    load(G1, 1, B1);
    __builtin_amdgcn_sched_barrier(0);
    finish(t, G0, acc);
    G0 = G1;
    geo(t + 2 * walk.step, G1);
  }
}

// Input-channel chunks (32 channels) of the larger group.
static int conv_nch(const ConvArgs& a) {
  int cin = a.Cin;
  if (a.g2_cout0 > 0 && a.g2_Cin > cin) cin = a.g2_Cin;
  const int cc = a.in8 ? 64 : 32;  // channels per chunk (64 B per pixel either way)
  return (cin + cc - 1) / cc;
}

static bool patch_geo(const ConvArgs& a, const ConvCfg& c, PatchGeo& g, size_t& smem) {
  if (!((a.k == 1 || a.k == 3) && (a.stride == 1 || a.stride == 2) && a.pad == a.k / 2)) return false;
  // the kernel's patch offsets use 24-bit multiplies (prep_tile)
  if ((size_t)a.Hin * a.Win >= (1u << 24) || (size_t)a.in_cs * 2 >= (1u << 24)) return false;
  const int NR = c.nr, MR = c.mr;
  const int NW = c.kind == 2 ? 8 : 4;  // waves per workgroup
  const int P = 16 * NR * NW;
  // tile width: the fewest halo-patch pixels DMA'd over the whole layer
  // (tiles x PH x PW, edge tiles included); at least 16 columns, so a B
  // fragment's 16 pixels mostly share one patch row (conflict-free reads)
  // (the search runs up to ~300 candidates with four divisions each; a plan
  // asks for the same few shapes on every forward, so the answers are kept:
  // host time per launch matters at batch 1, where the kernels are ~5 us)
  struct TileKey {
    int wo, ho, s, k, p, c;
  };
  static thread_local TileKey memo[64];
  static thread_local int memo_n = 0, memo_w = 0;
  int C = 0;
  for (int i = 0; i < memo_n && !C; ++i)
    if (memo[i].wo == a.Wo && memo[i].ho == a.Ho && memo[i].s == a.stride && memo[i].k == a.k &&
        memo[i].p == P)
      C = memo[i].c;
  if (!C) {
    long best = -1;
    for (int c = std::min(a.Wo, P); c >= std::min(16, a.Wo); --c) {
      const int r = P / c;
      const long cost = (long)ceil_div(a.Wo, c) * ceil_div(a.Ho, r) * ((r - 1) * a.stride + a.k) *
                        ((c - 1) * a.stride + a.k);
      if (best < 0 || cost < best) {
        best = cost;
        C = c;
      }
    }
    memo[memo_w++ & 63] = TileKey{a.Wo, a.Ho, a.stride, a.k, P, C};
    memo_n = std::min(memo_n + 1, 64);
  }
  g.C = C;
  g.R = P / C;
  if (g.R < 1) return false;
  g.PH = (g.R - 1) * a.stride + a.k;
  g.PW = (g.C - 1) * a.stride + a.k;
  g.pinst = ceil_div(g.PH * g.PW * 4, 64);  // 4 16-B slots per pixel (patch_pixb)
  g.p_bytes = g.pinst * 1024;
  g.tiles_x = ceil_div(a.Wo, g.C);
  g.tiles_y = ceil_div(a.Ho, g.R);
  const int nch = conv_nch(a);
  g.G = std::max(1, std::min(c.G, nch));
  g.fast = epi_fast(a) ? 1 : 0;
  // the 8-wave stagger (late waves finish a tile beside the partner's
  // MFMAs): off by default -- measured no gain when built (r06b) and
  // −1.6 % at the end of r06 (7 interleaved rounds, profiles/r06/session_ab
  // r06zh / r06zi); RV_STAGGER=1 enables it
  static const int stagger = getenv("RV_STAGGER") ? atoi(getenv("RV_STAGGER")) : 0;
  g.stagger = stagger;
  // per-lane offset registers of the kernel (patch_maxit)
  const int maxit = (a.stride == 2 ? 6 : 2) * NR + 2;
  if (ceil_div(g.pinst, NW) > maxit) return false;
  const size_t wb = (size_t)16 * MR * a.k * a.k * 64;
  // two stages: the next (tile, chunk group) streams in during the current one
  smem = (c.resw ? nch * wb : 0) + 2 * (size_t)g.G * (g.p_bytes + (c.resw ? 0 : wb)) +
         (a.in8 ? 0 : (size_t)16 * MR * 4);  // bf16: the block's bias
  if (a.ch_w) {  // chained 1x1: its weights and bias, one x tile per wave (+ logit rows)
    const size_t chn = (MR + 1) / 2;
    smem += chn * 16 * MR * 64 + (size_t)16 * MR * 4 + (size_t)NW * chn * NR * 16 * 64 +
            (a.ch_mode == 2 ? (size_t)NW * NR * 16 * (16 * MR + 4) * 4 : 0);
  }
  return smem <= 160 * 1024;
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess)
      n = p.multiProcessorCount;
    else
      n = 256;
    (void)hipGetLastError();
  }
  return n;
}

// Every instantiation gets the full 160 KB dynamic-LDS cap once; resident
// blocks per CU are cached per LDS size (per instantiation).
template <int MR, int NR, int K, int S, bool RESW, bool F8 = false, int NW = 4, int CHM = 0>
static int launch_patch_t(const ConvArgs& a, const PatchGeo& g, size_t smem, int persist,
                          hipStream_t s) {
  static bool attr = false;
  auto fn = conv_patch_kernel<MR, NR, K, S, RESW, F8, NW, CHM>;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      set_error("hipFuncSetAttribute: %s", hipGetErrorString(e));
      return -(int)e;
    }
    attr = true;
  }
  static size_t occ_smem[16] = {0};
  static int occ_val[16] = {0};
  int occ = 0;
  for (int i = 0; i < 16; ++i)
    if (occ_smem[i] == smem) occ = occ_val[i];
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 64 * NW, smem) != hipSuccess || occ < 1)
      occ = 1;
    (void)hipGetLastError();
    for (int i = 0; i < 16; ++i)
      if (occ_smem[i] == 0) {
        occ_smem[i] = smem;
        occ_val[i] = occ;
        break;
      }
  }
  const int T = (a.Cout + 15) / 16;
  const int ytiles = ceil_div(T, MR);
  const int ntiles = a.B * g.tiles_x * g.tiles_y;
  const int gx = xcd_grid(std::max(1, num_cus() * occ / ytiles), ntiles, persist != 0);
  dim3 grid(gx, ytiles);
  fn<<<grid, 64 * NW, smem, s>>>(a, g);
  return launch_status("conv_patch");
}

// 1x1 direct kernel: LDS = the block's resident weights
static size_t direct_smem(const ConvArgs& a, int MR) {
  return (size_t)((a.Cin + 31) / 32) * 16 * MR * 64;
}

template <int MR, int NR>
static int launch_direct_t(const ConvArgs& a, int persist, hipStream_t s) {
  static bool attr = false;
  auto fn = conv1x1_direct_kernel<MR, NR>;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      set_error("hipFuncSetAttribute: %s", hipGetErrorString(e));
      return -(int)e;
    }
    attr = true;
  }
  const size_t smem = direct_smem(a, MR);
  static size_t occ_smem[16] = {0};
  static int occ_val[16] = {0};
  int occ = 0;
  for (int i = 0; i < 16; ++i)
    if (occ_smem[i] == smem) occ = occ_val[i];
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, smem) != hipSuccess || occ < 1)
      occ = 1;
    (void)hipGetLastError();
    for (int i = 0; i < 16; ++i)
      if (occ_smem[i] == 0) {
        occ_smem[i] = smem;
        occ_val[i] = occ;
        break;
      }
  }
  const int ytiles = ceil_div((a.Cout + 15) / 16, MR);
  const int ntiles = ceil_div(a.B * a.Ho * a.Wo, 64 * NR);
  const int gx = xcd_grid(std::max(1, num_cus() * occ / ytiles), ntiles, persist != 0);
  fn<<<dim3(gx, ytiles), 256, smem, s>>>(a, epi_fast(a) ? 1 : 0);
  return launch_status("conv1x1_direct");
}

static bool direct_ok(const ConvArgs& a, const ConvCfg& c) {
  const int T = (a.Cout + 15) / 16;
  const bool vcat_ok = (a.split == 0 && !a.in_up) ||
                       (a.split % 32 == 0 && a.split <= a.Cin && (!a.in_up || (a.Ho % 2 == 0 && a.Wo % 2 == 0)) &&
                        (a.split == a.Cin || (a.in2 && a.in2_cs % 8 == 0 && a.in2_co % 8 == 0)));
  return a.k == 1 && a.stride == 1 && a.pad == 0 && a.g2_cout0 <= 0 && a.Hin == a.Ho &&
         a.Win == a.Wo && (c.mr <= T || c.mr == 1) && a.in_cs % 8 == 0 && a.in_co % 8 == 0 &&
         !a.in8 && vcat_ok && direct_smem(a, c.mr) <= 160 * 1024;
}


// stride-2 patches are ~4x the tile: only tiles whose offset registers and
// accumulators fit without spills (NR <= 2, MR * NR <= 8) are built for S = 2
template <int MR, int NR>
constexpr bool patch_s2_ok() {
  return NR <= 2 && MR * NR <= 8;
}

// Staged-weight (non-RESW) 3x3 variants with the biggest tiles exceed the
// register file (scratch spills); they are not built.
constexpr bool patch_spills(int MR, int NR, int K, int S, bool RESW) {
  return !RESW && K == 3 && ((S == 1 && MR * NR > 16) || (S == 2 && MR * NR >= 8));
}

// fp8 instantiations: MR, NR in {1, 2, 4}; the 3x3 ones that exceed the
// register file (4x4, 2x4 stride 1, 1x2 stride 2 with staged weights) are
// not built
template <int MR, int NR>
constexpr bool tile8_built() {
  return (MR == 1 || MR == 2 || MR == 4) && (NR == 1 || NR == 2 || NR == 4);
}
constexpr bool patch_spills8(int MR, int NR, int K, int S, bool RESW) {
  return K == 3 && (MR * NR >= 16 || (S == 1 && MR == 2 && NR == 4) ||
                    (S == 2 && !RESW && MR == 1 && NR == 2));
}

// chained-1x1 (CHM) instantiations: C2f cv1 behind a 64-channel 3x3 conv
// (YOLOv8n model.3 -> model.4.cv1, mode 1, stride 2), the Detect box /
// class branches' last convs behind their 3x3 (.1 -> .2: mode 2 with 64
// channels, mode 3 with 80, stride 1); ch_tile_ok is the host-side check
template <int MR, int NR, int CHM>
constexpr bool ch_built() {
  return NR <= 2 && ((CHM <= 2 && MR == 4) || (CHM == 3 && MR == 5));
}
static bool ch_tile_ok(int mr, int nr, int mode) {
  return nr <= 2 && ((mode <= 2 && mr == 4) || (mode == 3 && mr == 5));
}
template <int MR, int NR, bool RESW, int NW>
static int launch_patch_ch(const ConvArgs& a, const PatchGeo& g, size_t smem, int persist,
                           hipStream_t s) {
  if constexpr (ch_built<MR, NR, 1>()) {
    if (a.ch_mode == 1 && a.k == 3 && a.stride == 2)
      return launch_patch_t<MR, NR, 3, 2, RESW, false, NW, 1>(a, g, smem, persist, s);
    if (a.ch_mode == 1 && a.k == 3 && a.stride == 1)
      return launch_patch_t<MR, NR, 3, 1, RESW, false, NW, 1>(a, g, smem, persist, s);
  }
  if constexpr (ch_built<MR, NR, 2>())
    if (a.ch_mode == 2 && a.k == 3 && a.stride == 1)
      return launch_patch_t<MR, NR, 3, 1, RESW, false, NW, 2>(a, g, smem, persist, s);
  if constexpr (ch_built<MR, NR, 3>())
    if (a.ch_mode == 3 && a.k == 3 && a.stride == 1)
      return launch_patch_t<MR, NR, 3, 1, RESW, false, NW, 3>(a, g, smem, persist, s);
  set_error("conv_patch (chained 1x1 mode %d): no variant MR=%d NR=%d k=%d s=%d", a.ch_mode, MR, NR,
            a.k, a.stride);
  return RV_EINVAL;
}

template <int MR, int NR, bool RESW>
static int launch_patch_ks(const ConvArgs& a, const PatchGeo& g, size_t smem, int persist,
                           hipStream_t s) {
  if (a.ch_w) return launch_patch_ch<MR, NR, RESW, 4>(a, g, smem, persist, s);
  if (a.in8) {
    if constexpr (tile8_built<MR, NR>()) {
      if constexpr (!patch_spills(MR, NR, 3, 1, RESW) && !patch_spills8(MR, NR, 3, 1, RESW))
        if (a.k == 3 && a.stride == 1)
          return launch_patch_t<MR, NR, 3, 1, RESW, true>(a, g, smem, persist, s);
      if (a.k == 1 && a.stride == 1)
        return launch_patch_t<MR, NR, 1, 1, RESW, true>(a, g, smem, persist, s);
      if constexpr (patch_s2_ok<MR, NR>() && !patch_spills(MR, NR, 3, 2, RESW) &&
                    !patch_spills8(MR, NR, 3, 2, RESW)) {
        if (a.k == 3 && a.stride == 2)
          return launch_patch_t<MR, NR, 3, 2, RESW, true>(a, g, smem, persist, s);
      }
    }
    set_error("conv_patch (fp8): no variant MR=%d NR=%d k=%d s=%d", MR, NR, a.k, a.stride);
    return RV_EINVAL;
  }
  if constexpr (!patch_spills(MR, NR, 3, 1, RESW))
    if (a.k == 3 && a.stride == 1) return launch_patch_t<MR, NR, 3, 1, RESW>(a, g, smem, persist, s);
  if (a.k == 1 && a.stride == 1) return launch_patch_t<MR, NR, 1, 1, RESW>(a, g, smem, persist, s);
  if constexpr (patch_s2_ok<MR, NR>() && !patch_spills(MR, NR, 3, 2, RESW)) {
    if (a.k == 3 && a.stride == 2) return launch_patch_t<MR, NR, 3, 2, RESW>(a, g, smem, persist, s);
  }
  set_error("conv_patch: no variant MR=%d NR=%d k=%d s=%d", MR, NR, a.k, a.stride);
  return RV_EINVAL;
}

// 8-wave patch kernel (kind 2): bf16 3x3 layers; 2 waves per SIMD leave
// 256 VGPRs per lane, so no tile is excluded for register pressure
template <int MR, int NR>
constexpr bool tile_w8_built() {
  return (MR == 8 && NR <= 2) || (MR == 5 && NR <= 2) || (MR == 4 && NR <= 4 && NR != 3) ||
         (MR == 2 && (NR == 2 || NR == 4));
}
template <int MR, int NR, bool RESW>
static int launch_patch8_ks(const ConvArgs& a, const PatchGeo& g, size_t smem, int persist,
                            hipStream_t s) {
  if (a.ch_w) return launch_patch_ch<MR, NR, RESW, 8>(a, g, smem, persist, s);
  if constexpr (tile_w8_built<MR, NR>()) {
    if (!a.in8 && a.k == 3 && a.stride == 1)
      return launch_patch_t<MR, NR, 3, 1, RESW, false, 8>(a, g, smem, persist, s);
    if constexpr (patch_s2_ok<MR, NR>())
      if (!a.in8 && a.k == 3 && a.stride == 2)
        return launch_patch_t<MR, NR, 3, 2, RESW, false, 8>(a, g, smem, persist, s);
  }
  set_error("conv_patch (8 waves): no variant MR=%d NR=%d k=%d s=%d", MR, NR, a.k, a.stride);
  return RV_EINVAL;
}
static bool w8_tile(int mr, int nr) {
  return (mr == 8 && nr <= 2) || (mr == 5 && nr <= 2) || (mr == 4 && (nr == 1 || nr == 2 || nr == 4)) ||
         (mr == 2 && (nr == 2 || nr == 4));
}

// (MR, NR) tiles built for the patch kernel
static const int kTiles[][2] = {{8, 2}, {8, 1}, {5, 2}, {5, 1}, {4, 4}, {4, 2}, {4, 1},
                                {2, 4}, {2, 2}, {2, 1}, {1, 4}, {1, 2}, {1, 1}};

bool conv_cfg_ok(const ConvArgs& a, const ConvCfg& c) {
  if (a.ch_w &&  // chained 1x1: the patch kernel's CHM form, one cout tile covering Cout
      (c.kind == 1 || a.in8 || !ch_tile_ok(c.mr, c.nr, a.ch_mode) || 16 * c.mr < a.Cout || 16 * c.mr - a.Cout >= 16 || a.k != 3 || a.res || a.out1 || a.out0_up || a.g2_cout0 > 0 ||
       vcat(a) || (a.ch_mode == 1 ? !epi_fast(a) : (!a.out_f32 || a.stride != 1))))
    return false;
  if (c.kind == 1) return !a.in8 && direct_ok(a, c);
  if ((c.kind != 0 && c.kind != 2) || vcat(a)) return false;
  if (c.kind == 2 && (a.in8 || a.k != 3 || !w8_tile(c.mr, c.nr))) return false;
  if (a.in8 && !((c.mr == 1 || c.mr == 2 || c.mr == 4) && (c.nr == 1 || c.nr == 2 || c.nr == 4)))
    return false;
  if (a.in8 && (a.Cin % 16 || a.in_co % 16 || a.in_cs % 16 ||
                 (a.g2_cout0 > 0 && (a.g2_Cin % 16 || a.g2_in_co % 16))))
    return false;  // whole 16-B quarters of fp8 channels
  const int T = (a.Cout + 15) / 16;
  if (c.mr > T && c.mr > 1) return false;
  if (a.stride == 2 && (c.nr > 2 || c.mr * c.nr > 8 || a.k != 3)) return false;  // patch_s2_ok
  if (a.g2_cout0 > 0 && a.g2_cout0 % (16 * c.mr) != 0) return false;  // tiles inside one group
  if (c.kind == 0 && patch_spills(c.mr, c.nr, a.k, a.stride, c.resw != 0)) return false;
  if (a.in8 && patch_spills8(c.mr, c.nr, a.k, a.stride, c.resw != 0)) return false;
  PatchGeo g;
  size_t sm;
  return patch_geo(a, c, g, sm);
}

#ifdef RV_PHASE_PROF
}  // namespace rv
// Timing build only (not in include/rvhip.h): read (and with reset != 0
// clear) the conv_patch_kernel phase sums, 8 x u64.
extern "C" int rv_conv_phase_read(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rv::g_conv_phase), 8 * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  if (reset) {
    static const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rv::g_conv_phase), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
namespace rv {
#endif
int launch_conv_cfg(const ConvArgs& a, const ConvCfg& c, hipStream_t s) {
  PatchGeo g;
  size_t sm;
  if (!conv_cfg_ok(a, c) || (c.kind != 1 && !patch_geo(a, c, g, sm))) {
    set_error("conv config MR=%d NR=%d G=%d resw=%d not valid for this layer", c.mr, c.nr, c.G,
              c.resw);
    return RV_EINVAL;
  }
#define RV_PATCH(M_, N_)                                                                     \
  if (c.mr == M_ && c.nr == N_)                                                              \
    return c.kind == 1 ? launch_direct_t<M_, N_>(a, c.persist, s)                            \
           : c.kind == 2 ? (c.resw ? launch_patch8_ks<M_, N_, true>(a, g, sm, c.persist, s)    \
                                   : launch_patch8_ks<M_, N_, false>(a, g, sm, c.persist, s))  \
           : c.resw    ? launch_patch_ks<M_, N_, true>(a, g, sm, c.persist, s)               \
                       : launch_patch_ks<M_, N_, false>(a, g, sm, c.persist, s);
  RV_PATCH(8, 2) RV_PATCH(8, 1) RV_PATCH(5, 2) RV_PATCH(5, 1) RV_PATCH(4, 4) RV_PATCH(4, 2)
  RV_PATCH(4, 1) RV_PATCH(2, 4) RV_PATCH(2, 2) RV_PATCH(2, 1) RV_PATCH(1, 4) RV_PATCH(1, 2)
  RV_PATCH(1, 1)
#undef RV_PATCH
  set_error("no conv_patch tile MR=%d NR=%d", c.mr, c.nr);
  return RV_EINVAL;
}

// Every valid configuration of this layer (the autotuner's search space):
// each tile with resident weights (largest G that fits) and with staged
// weights (the largest G that fits, and G = 1); persistent grid or one
// block per pixel tile.
int conv_candidates(const ConvArgs& a, ConvCfg* out, int cap) {
  int n = 0;
  const int nch = conv_nch(a);
  for (const auto& t : kTiles) {
    for (int kind = 0; kind <= 2; kind += 2)  // 4- and 8-wave patch kernels
      for (int resw = 1; resw >= 0; --resw) {
        int gbest = 0;
        for (int G = nch; G >= 1 && !gbest; --G)
          if (conv_cfg_ok(a, ConvCfg{t[0], t[1], G, resw, 1, kind})) gbest = G;
        if (!gbest) continue;
        // persistent grid, and (for layers with few tiles) one block per tile
        for (int persist = 1; persist >= 0; --persist) {
          if (n < cap) out[n] = ConvCfg{t[0], t[1], gbest, resw, persist, kind};
          ++n;
          if (!resw && gbest > 1) {
            if (n < cap) out[n] = ConvCfg{t[0], t[1], 1, resw, persist, kind};
            ++n;
          }
        }
      }
    // 1x1 layers: the direct-B kernel
    for (int persist = 1; persist >= 0; --persist) {
      const ConvCfg d{t[0], t[1], 1, 1, persist, 1};
      if (!a.in8 && direct_ok(a, d)) {
        if (n < cap) out[n] = d;
        ++n;
      }
    }
  }
  return n;
}

// Default (untuned) choice: the largest wave tile that still fills the
// machine (blocks >= 3/4 of CUs x co-resident blocks), resident weights and
// the largest chunk group that fit.
static bool default_cfg(const ConvArgs& a, ConvCfg& best) {
  const int T = (a.Cout + 15) / 16;
  double best_fill = -1.0;
  bool found = false;
  for (const auto& t : kTiles) {
    if (ceil_div(T, t[0]) * t[0] - T > (t[0] > 1 ? 1 : 0)) continue;
    if (a.k == 3 && t[0] > 5) continue;  // keep 3x3 weight stages modest
    ConvCfg cand{0, 0, 0, 0, 1};
    bool ok = false;
    for (int resw = 1; resw >= 0 && !ok; --resw)
      for (int G = conv_nch(a); G >= 1 && !ok; --G) {
        cand = ConvCfg{t[0], t[1], G, resw, 1};
        ok = conv_cfg_ok(a, cand);
      }
    if (!ok) continue;
    PatchGeo g;
    size_t sm = 0;
    patch_geo(a, cand, g, sm);
    const long blocks = (long)a.B * g.tiles_x * g.tiles_y * ceil_div(T, t[0]);
    const int bpc = std::max(1, std::min(4, (int)((160 * 1024) / sm)));
    const double fill = (double)blocks / (256.0 * bpc);
    if (fill >= 0.75) {
      best = cand;
      return true;
    }
    if (fill > best_fill) {
      best_fill = fill;
      best = cand;
      found = true;
    }
  }
  return found;
}

// returns 1 if launched (status in *st), 0 if the patch kernel does not apply
static int try_launch_patch(const ConvArgs& a, hipStream_t s, int* st) {
  static const char* force = getenv("RV_CONV_FORCE");  // "direct" or "MR,NR[,G,resw]"
  if (force && strcmp(force, "direct") == 0) return 0;
  ConvCfg c{0, 0, 1, 0, 1};
  if (force) {
    int fm = 0, fn = 0, fg = 1, fr = 0;
    if (sscanf(force, "%d,%d,%d,%d", &fm, &fn, &fg, &fr) >= 2) {
      c = ConvCfg{fm, fn, fg, fr, 1};
      if (conv_cfg_ok(a, c)) {
        *st = launch_conv_cfg(a, c, s);
        return 1;
      }
    }
  }
  if (!default_cfg(a, c)) return 0;
  static const int persist = getenv("RV_CONV_PERSIST") ? atoi(getenv("RV_CONV_PERSIST")) : 1;
  c.persist = persist;
  static const int dbg = getenv("RV_CONV_DEBUG") ? atoi(getenv("RV_CONV_DEBUG")) : 0;
  if (dbg)
    fprintf(stderr, "[conv] %dx%d k%d s%d Cin %d Cout %d -> MR=%d NR=%d G=%d resw=%d\n", a.Ho, a.Wo,
            a.k, a.stride, a.Cin, a.Cout, c.mr, c.nr, c.G, c.resw);
  *st = launch_conv_cfg(a, c, s);
  return 1;
}

// ---------------------------------------------------------------------------
// SPPF: three chained MaxPool2d(5, 1, 2) == clipped 5/9/13 windows.
// One thread per (pixel, 8-channel group).
// ---------------------------------------------------------------------------
// One workgroup per (image, 8-channel group).  The clipped k x k max is
// separable (the clipped window is a rectangle), so a horizontal pass writes
// the row maxima for k = 5/9/13 to LDS and a vertical pass finishes them;
// one thread per pixel, 8 channels (one 16-B vector) each.  bf16 max is
// exact, so values stay bf16 throughout.
constexpr int kSppfLds = 160 * 1024;

__device__ __forceinline__ void bf8_to_f(const uint4 v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(w[j] << 16);
    f[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
  }
}
__device__ __forceinline__ uint4 f_to_bf8(const float (&f)[8]) {
  // inputs are bf16 values: truncation is exact
  uint32_t w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = (__float_as_uint(f[2 * j]) >> 16) | (__float_as_uint(f[2 * j + 1]) & 0xFFFF0000u);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// 16-B vector <-> its lanes as f32: 8 bf16 values, or 16 fp8 codes (one
// buffer scale, so the max over codes' values re-encodes exactly).
template <bool F8>
struct SppfVec {
  static constexpr int N = F8 ? 16 : 8;
  __device__ static void dec(const uint4 v, float (&f)[N]) {
    if constexpr (F8) {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[4 * j] = __builtin_amdgcn_cvt_f32_fp8((int)w[j], 0);
        f[4 * j + 1] = __builtin_amdgcn_cvt_f32_fp8((int)w[j], 1);
        f[4 * j + 2] = __builtin_amdgcn_cvt_f32_fp8((int)w[j], 2);
        f[4 * j + 3] = __builtin_amdgcn_cvt_f32_fp8((int)w[j], 3);
      }
    } else {
      bf8_to_f(v, f);
    }
  }
  __device__ static uint4 enc(const float (&f)[N]) {
    if constexpr (F8) {
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float q[4] = {f[4 * j], f[4 * j + 1], f[4 * j + 2], f[4 * j + 3]};
        w[j] = f8_encode4(q, 1.f);
      }
      return make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      return f_to_bf8(f);
    }
  }
};

template <bool F8>
__global__ __launch_bounds__(256) void sppf_pool_kernel(uint8_t* __restrict__ buf, int B, int H,
                                                        int W, int c) {
  using V = SppfVec<F8>;
  constexpr int NV = V::N, EB = F8 ? 1 : 2;
  extern __shared__ __attribute__((aligned(16))) uint4 sp[];  // x, h5, h9, h13: [H*W] uint4 each
  const int groups = c / NV;
  const int b = blockIdx.x / groups, g = blockIdx.x - (blockIdx.x / groups) * groups;
  const int cs = 4 * c * EB;  // pixel stride, bytes
  const int HW = H * W;
  uint4* xs = sp;
  uint4* h5 = sp + HW;
  uint4* h9 = sp + 2 * HW;
  uint4* h13 = sp + 3 * HW;
  uint8_t* img = buf + (size_t)b * HW * cs + g * 16;
  for (int p = threadIdx.x; p < HW; p += 256) xs[p] = *(const uint4*)(img + (size_t)p * cs);
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += 256) {
    const int y = p / W, x = p - (p / W) * W;
    float a5[NV], a9[NV], a13[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) a5[j] = a9[j] = a13[j] = -INFINITY;
    // the taps' LDS reads issued in two groups (7 + 6) ahead of their max
    // chains (a branch around each read made every one a separate LDS round
    // trip; all 13 at once doubled the VGPRs, which cost more beside the
    // forward's other kernels than the round trips saved); out-of-map taps
    // read the edge pixel instead, which the window always holds, so the
    // max (the -inf padding of MaxPool2d) is unchanged
#pragma unroll
    for (int d0 = -6; d0 <= 6; d0 += 7) {
      uint4 raw[7];
#pragma unroll
      for (int d = d0; d < d0 + 7 && d <= 6; ++d) raw[d - d0] = xs[y * W + min(max(x + d, 0), W - 1)];
#pragma unroll
      for (int d = d0; d < d0 + 7 && d <= 6; ++d) {
        float f[NV];
        V::dec(raw[d - d0], f);
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          a13[j] = fmaxf(a13[j], f[j]);
          if (d >= -4 && d <= 4) a9[j] = fmaxf(a9[j], f[j]);
          if (d >= -2 && d <= 2) a5[j] = fmaxf(a5[j], f[j]);
        }
      }
    }
    h5[p] = V::enc(a5);
    h9[p] = V::enc(a9);
    h13[p] = V::enc(a13);
  }
  __syncthreads();
  for (int p = threadIdx.x; p < HW; p += 256) {
    const int y = p / W, x = p - (p / W) * W;
    float a5[NV], a9[NV], a13[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) a5[j] = a9[j] = a13[j] = -INFINITY;
    // column pass, the same way: each map's taps read first, edge rows
    // standing in for the out-of-map ones
    auto col_max = [&](const uint4* hm, int r, float (&acc)[NV]) {
#pragma unroll
      for (int d0 = -r; d0 <= r; d0 += 7) {
        uint4 rv[7];
#pragma unroll
        for (int d = d0; d < d0 + 7 && d <= r; ++d) rv[d - d0] = hm[min(max(y + d, 0), H - 1) * W + x];
#pragma unroll
        for (int d = d0; d < d0 + 7 && d <= r; ++d) {
          float f[NV];
          V::dec(rv[d - d0], f);
#pragma unroll
          for (int j = 0; j < NV; ++j) acc[j] = fmaxf(acc[j], f[j]);
        }
      }
    };
    col_max(h13, 6, a13);
    col_max(h9, 4, a9);
    col_max(h5, 2, a5);
    uint8_t* o = img + (size_t)p * cs;
    *(uint4*)(o + c * EB) = V::enc(a5);
    *(uint4*)(o + 2 * c * EB) = V::enc(a9);
    *(uint4*)(o + 3 * c * EB) = V::enc(a13);
  }
}

template <bool F8>
static int launch_sppf_t(uint8_t* buf, int B, int H, int W, int c, hipStream_t s) {
  const size_t smem = (size_t)H * W * 64;  // 4 x 16 B per pixel
  const int nv = F8 ? 16 : 8;
  if (c % nv != 0 || smem > kSppfLds) {
    set_error("sppf: c=%d / map %dx%d unsupported by the LDS pool", c, H, W);
    return RV_EINVAL;
  }
  static bool attr = false;
  if (!attr && smem > 64 * 1024) {  // only raise the cap when a map needs it
    // best effort: a failure surfaces as the launch error reported below
    (void)hipFuncSetAttribute((const void*)sppf_pool_kernel<F8>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kSppfLds);
    (void)hipGetLastError();
    attr = true;
  }
  sppf_pool_kernel<F8><<<B * (c / nv), 256, smem, s>>>(buf, B, H, W, c);
  return launch_status("sppf_pool");
}

int launch_sppf_pool(bf16_t* buf, int B, int H, int W, int c, hipStream_t s) {
  return launch_sppf_t<false>((uint8_t*)buf, B, H, W, c, s);
}

int launch_sppf_pool_fp8(uint8_t* buf, int B, int H, int W, int c, hipStream_t s) {
  return launch_sppf_t<true>(buf, B, H, W, c, s);
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

// One 256-thread workgroup per 64 consecutive anchors of one level: their
// (64 x cs) f32 head logits are one contiguous span, staged into LDS with
// coalesced 16-B loads at a padded row stride (cs + 4 floats: rows 20 banks
// apart, conflict-free fragment reads).  Four lanes share an anchor: lane
// part p takes the DFL side p (softmax expectation over REG bins) and the
// classes p, p+4, ...; the quad then combines the four sides and the
// first-max class with lane shuffles.
//
// FUSED: the head's last 1x1 convs (cv2.i.2: 4*REG box logits, cv3.i.2: nc
// class logits, no activation) run here on MFMA from the level's bf16
// features (L.feat, [box feats | class feats]) straight into the LDS logits
// tile, so the f32 logits never touch HBM (L.logits, when non-null, still
// receives them: the parity tests read it).  Wave w computes anchors
// 16w..16w+15 of the block: box fragments m = 0..REG/4-1, class fragments
// after them; B fragments are 16-B loads of one anchor's 8 channels, A
// fragments 16-B loads of the packed [cout][cin_pad32] weights (L2-resident).
// Class score: exp + one v_rcp_f32 (no IEEE division sequence).  The raw
// output and the candidate filter use this same function, so the scores NMS
// sees are the scores in `raw`.
// (head_sigmoid: defined with the patch kernel's chained head epilogue)

// The fused head's MFMA section with compile-time trip counts (KB box /
// KC class 32-channel k-steps, NCF class fragments: YOLOv8n's head is
// KB = 2, KC = 3, NCF = 5): every A / B fragment load of the wave is issued
// before the first MFMA, so the wave waits out one L2 latency instead of
// one per (fragment, k-step) -- the runtime-bound loops compiled to a
// load / s_waitcnt vmcnt(0) / MFMA chain.  Same k order and sums as the
// generic loops (bit-identical logits).  The weight fragments (23 x 16 B
// per lane) are loaded by head_weights once per level and stay in VGPRs
// while the block walks its anchor tiles: per 16-anchor wave tile they were
// 4.6x the feature bytes, all of it L2 -> CU traffic.
template <int REG, int KB, int KC, int NCF>
__device__ __forceinline__ void head_weights(const HeadLevel& L, uint4 (&Ab)[KB][REG / 4],
                                             uint4 (&Ac)[KC][NCF]) {
  constexpr int MB = REG / 4;
  const int lane = threadIdx.x & 63, col = lane & 15, quad = lane >> 4;
  constexpr int cinb = KB * 32, cinc = KC * 32;
#pragma unroll
  for (int k = 0; k < KB; ++k)
#pragma unroll
    for (int m = 0; m < MB; ++m)
      Ab[k][m] = *(const uint4*)(L.w_box + (size_t)(m * 16 + col) * cinb + k * 32 + quad * 8);
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int m = 0; m < NCF; ++m)
      Ac[k][m] = *(const uint4*)(L.w_cls + (size_t)(m * 16 + col) * cinc + k * 32 + quad * 8);
}

// one 16-anchor wave tile's feature fragments (B operands): box channels,
// then class channels of anchor r0 + 16 wave + col
template <int REG, int KB, int KC>
__device__ __forceinline__ void head_feats(const HeadLevel& L, int b, int HW, int r0, int na,
                                           uint4 (&Bb)[KB], uint4 (&Bc)[KC]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, quad = lane >> 4;
  const int an0 = wave * 16 + col;
  const bool ok = an0 < na;
  const bf16_t* fp = L.feat + ((size_t)b * HW + r0 + (ok ? an0 : 0)) * L.feat_cs + quad * 8;
#pragma unroll
  for (int k = 0; k < KB; ++k)
    Bb[k] = ok && k * 32 + quad * 8 < L.cin_b ? *(const uint4*)(fp + k * 32) : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < KC; ++k)
    Bc[k] = ok && k * 32 + quad * 8 < L.cin_c ? *(const uint4*)(fp + 4 * REG + k * 32)
                                              : make_uint4(0, 0, 0, 0);
}

template <int REG, int KB, int KC, int NCF>
__device__ __forceinline__ void head_mfma_fixed(const HeadLevel& L, const uint4 (&Ab)[KB][REG / 4],
                                                const uint4 (&Ac)[KC][NCF], const uint4 (&Bb)[KB],
                                                const uint4 (&Bc)[KC], float* lg, int nc,
                                                float& best_out, int& bc_out) {
  constexpr int MB = REG / 4;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, col = lane & 15, quad = lane >> 4;
  float* row = lg + (size_t)(wave * 16 + col) * (L.cs + 4);
  {
    f32x4 acc[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KB; ++k)
#pragma unroll
      for (int m = 0; m < MB; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, Ab[k][m]),
                                                         __builtin_bit_cast(bf16x8, Bb[k]), acc[m], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const int co = m * 16 + quad * 4;
      *(f32x4*)(row + co) = acc[m] + *(const f32x4*)(L.b_box + co);
    }
  }
  {
    f32x4 acc[NCF];
#pragma unroll
    for (int m = 0; m < NCF; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int m = 0; m < NCF; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, Ac[k][m]),
                                                         __builtin_bit_cast(bf16x8, Bc[k]), acc[m], 0, 0, 0);
    // the class scores never go to LDS: lane quad q holds classes
    // m * 16 + 4 q + i of its anchor (ascending in (m, i)), so a scan keeps
    // the lane's first maximum and two cross-quad steps (larger score, then
    // smaller class) give the anchor's first maximum -- the (score, class)
    // of a scan over all nc in order.  Same value per class as the LDS path
    // (acc + bias, then head_sigmoid).
    float best = -1.f;
    int bc = 0;
#pragma unroll
    for (int m = 0; m < NCF; ++m) {
      const int co = m * 16 + quad * 4;
      const f32x4 v = acc[m] + *(const f32x4*)(L.b_cls + co);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float sg = head_sigmoid(v[i]);
        if (co + i < nc && sg > best) {
          best = sg;
          bc = co + i;
        }
      }
    }
#pragma unroll
    for (int off = 16; off < 64; off <<= 1) {
      const float ob = __shfl_xor(best, off);
      const int oc = __shfl_xor(bc, off);
      if (ob > best || (ob == best && oc < bc)) {
        best = ob;
        bc = oc;
      }
    }
    best_out = best;
    bc_out = bc;
  }
}


template <int REG, bool FUSED, int KB = 0, int KC = 0, int NCF = 0, int NCT = 0>
__global__ __launch_bounds__(256) void detect_decode_kernel(HeadLevels h, int B, int nc,
                                                            float conf, float* __restrict__ raw,
                                                            Cand* __restrict__ cand, int cap,
                                                            int* __restrict__ seg_n, int nblk,
                                                            int tpb) {
  extern __shared__ __attribute__((aligned(16))) float lg[];  // [64][cs + 4]
  __shared__ int wcnt[4];
  const int b = blockIdx.y;
  constexpr bool kFixed = FUSED && KC > 0;
  uint4 Ab[kFixed ? KB : 1][REG / 4], Ac[kFixed ? KC : 1][kFixed ? NCF : 1];
  uint4 Bb[kFixed ? KB : 1], Bc[kFixed ? KC : 1];  // the current tile's features
  int wl = -1;       // level whose head weights are in Ab / Ac
  bool pre = false;  // Bb / Bc already hold this tile's features
  float hbest = -1.f;  // fixed head: the lane's anchor's best class score / class
  int hbc = 0;
  // The block walks anchor tiles blockIdx.x * tpb .. + tpb - 1 (64 anchors
  // each; tpb > 1 only for the fixed fused head, whose weight fragments then
  // stay in registers).  Every lg read of a tile precedes the block barrier
  // before its candidate write-out, and a wave writes only its own 16 rows,
  // so the next tile's MFMA section may overwrite the tile in place.
  for (int t = 0; t < tpb; ++t) {
    // block -> (level, first anchor in level).  Only compile-time indices
    // into the by-value argument: a dynamic index would copy it to scratch.
    const int blk = blockIdx.x * tpb + t;
    if (blk >= nblk) break;  // block-uniform
    int l = 0, A = h.start[1], lstart = 0, lblk = 0;
    HeadLevel L = h.lv[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      if (i < h.nlv) A = h.start[i + 1];
      if (i < h.nlv && blk >= h.blk[i]) {
        l = i;
        L = h.lv[i];
        lstart = h.start[i];
        lblk = h.blk[i];
      }
    }
    const int HW = L.H * L.W;
    const int r0 = (blk - lblk) * 64;
    const int na = min(64, HW - r0);
    const int tid = threadIdx.x;
    const int cs4 = L.cs / 4, ls4 = cs4 + 1;  // row length / LDS row stride in float4
    if constexpr (kFixed) {
      if (l != wl) {
        head_weights<REG, KB, KC, NCF>(L, Ab, Ac);
        wl = l;
      }
      if (!pre) head_feats<REG, KB, KC>(L, b, HW, r0, na, Bb, Bc);
      head_mfma_fixed<REG, KB, KC, NCF>(L, Ab, Ac, Bb, Bc, lg, nc, hbest, hbc);
      // the next tile's features stream in under this tile's decode (same
      // level only; a level change loads them at the top of its iteration)
      pre = t + 1 < tpb && blk + 1 < nblk && r0 + 64 < HW;
      if (pre) head_feats<REG, KB, KC>(L, b, HW, r0 + 64, min(64, HW - r0 - 64), Bb, Bc);
      __syncthreads();
    } else if constexpr (FUSED) {
      constexpr int MB = REG / 4;  // box fragments (4*REG couts)
      const int wave = tid >> 6, lane = tid & 63, col = lane & 15, quad = lane >> 4;
      const int an0 = wave * 16 + col;  // this lane's anchor (B column / D column)
      const bool ok = an0 < na;
      const bf16_t* fp = L.feat + ((size_t)b * HW + r0 + (ok ? an0 : 0)) * L.feat_cs + quad * 8;
      const int ncf = (nc + 15) / 16;  // class fragments
      float* lrow = lg + (size_t)an0 * (L.cs + 4);
      // box: K = cin_b (multiple of 32)
      {
        f32x4 acc[MB];
#pragma unroll
        for (int m = 0; m < MB; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int cinp = (L.cin_b + 31) & ~31;
        for (int k = 0; k < cinp; k += 32) {
          const bool kv = ok && k + quad * 8 < L.cin_b;
          const uint4 bv = kv ? *(const uint4*)(fp + k) : make_uint4(0, 0, 0, 0);
          const bf16x8 Bf = __builtin_bit_cast(bf16x8, bv);
#pragma unroll
          for (int m = 0; m < MB; ++m) {
            const bf16x8 Af = __builtin_bit_cast(
                bf16x8, *(const uint4*)(L.w_box + (size_t)(m * 16 + col) * cinp + k + quad * 8));
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af, Bf, acc[m], 0, 0, 0);
          }
        }
        // lane holds couts m*16 + quad*4 + i of anchor `col` of this wave
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          const int co = m * 16 + quad * 4;
          const f32x4 bb = *(const f32x4*)(L.b_box + co);
          *(f32x4*)(lg + (size_t)(wave * 16 + col) * (L.cs + 4) + co) = acc[m] + bb;
        }
      }
      // classes: K = cin_c, couts nc (padded to 16)
      {
        const int cinp = (L.cin_c + 31) & ~31;
        for (int m0 = 0; m0 < ncf; m0 += 5) {  // up to 5 fragments (80 classes) per pass
          f32x4 acc[5];
#pragma unroll
          for (int m = 0; m < 5; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int k = 0; k < cinp; k += 32) {
            const bool kv = ok && k + quad * 8 < L.cin_c;
            const uint4 bv = kv ? *(const uint4*)(fp + 4 * REG + k) : make_uint4(0, 0, 0, 0);
            const bf16x8 Bf = __builtin_bit_cast(bf16x8, bv);
#pragma unroll
            for (int m = 0; m < 5; ++m) {
              if (m0 + m >= ncf) break;
              const bf16x8 Af = __builtin_bit_cast(
                  bf16x8,
                  *(const uint4*)(L.w_cls + (size_t)((m0 + m) * 16 + col) * cinp + k + quad * 8));
              acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af, Bf, acc[m], 0, 0, 0);
            }
          }
#pragma unroll
          for (int m = 0; m < 5; ++m) {
            if (m0 + m >= ncf) break;
            const int co = (m0 + m) * 16 + quad * 4;  // class index (bias padded to 16)
            const f32x4 bb = *(const f32x4*)(L.b_cls + co);
            float* d = lg + (size_t)(wave * 16 + col) * (L.cs + 4) + 4 * REG + co;
            const f32x4 v = acc[m] + bb;
            // the last fragment may run past nc: keep the padding out of the row
            if (co + 3 < nc) {
              *(f32x4*)d = v;
            } else {
              for (int i = 0; i < 4; ++i)
                if (co + i < nc) d[i] = v[i];
            }
          }
        }
      }
      (void)lrow;
      __syncthreads();
      if (L.logits_out) {  // parity/debug copy of the logits (coalesced rows)
        f32x4* dst = (f32x4*)(L.logits_out + ((size_t)b * HW + r0) * L.cs);
        for (int i = tid; i < na * cs4; i += 256) {
          const int row = i / cs4, c4 = i - (i / cs4) * cs4;
          dst[i] = ((const f32x4*)lg)[row * ls4 + c4];
        }
      }
    } else {
      const f32x4* src = (const f32x4*)(L.logits + ((size_t)b * HW + r0) * L.cs);
      // 8 loads in flight per thread before any LDS store (a plain copy loop
      // would wait out one HBM latency per element)
      for (int i0 = tid; i0 < na * cs4; i0 += 8 * 256) {
        f32x4 v[8];  // native vectors (a float4 struct array would live in scratch)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u * 256;
          v[u] = i < na * cs4 ? src[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u * 256;
          if (i < na * cs4) {
            const int row = i / cs4, c4 = i - (i / cs4) * cs4;
            ((f32x4*)lg)[row * ls4 + c4] = v[u];
          }
        }
      }
      __syncthreads();
    }
    const int an = tid >> 2, part = tid & 3;
    const bool live = an < na;
    const float* px = lg + (live ? an : 0) * (L.cs + 4);
    // DFL side `part`
    float d;
    {
      float v[REG];
      float mx = -INFINITY;
      // the side's REG logits are 16-B aligned in the row (cs + 4 floats,
      // a multiple of 4): ds_read_b128s
#pragma unroll
      for (int i = 0; i < REG; i += 4) {
        const f32x4 q = *(const f32x4*)(px + part * REG + i);
        v[i] = q[0];
        v[i + 1] = q[1];
        v[i + 2] = q[2];
        v[i + 3] = q[3];
      }
#pragma unroll
      for (int i = 0; i < REG; ++i) mx = fmaxf(mx, v[i]);
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < REG; ++i) {
        v[i] = __expf(v[i] - mx);
        sum += v[i];
      }
      // softmax probabilities by one reciprocal (v_rcp_f32, <= 1 ulp from
      // v / sum; the decode tolerance is 2e-3 px)
      const float rs = __builtin_amdgcn_rcpf(sum);
      float e = 0.f;
#pragma unroll
      for (int i = 0; i < REG; ++i) e += (float)i * (v[i] * rs);
      d = e;
    }
    // first maximum of the sigmoid scores.  The fixed head (NCT > 0) found
    // it in registers (head_mfma_fixed: lane (col, quad) of the MFMA layout
    // holds anchor col's result); otherwise lane part scans classes part,
    // part + 4, ... in LDS and the quad reduction picks the larger score,
    // then the smaller class.
    const float* pc = px + 4 * REG;
    float best = -1.f;
    int bc = 0;
    if constexpr (NCT > 0) {
      best = __shfl(hbest, (tid & 63) >> 2);
      bc = __shfl(hbc, (tid & 63) >> 2);
    } else {
      for (int c = part; c < nc; c += 4) {
        const float sg = head_sigmoid(pc[c]);
        if (sg > best) {
          best = sg;
          bc = c;
        }
      }
#pragma unroll
      for (int off = 1; off < 4; off <<= 1) {
        const float ob = __shfl_xor(best, off);
        const int oc = __shfl_xor(bc, off);
        if (ob > best || (ob == best && oc < bc)) {
          best = ob;
          bc = oc;
        }
      }
    }
    const int base = tid & ~3;
    const float d0 = __shfl(d, base), d1 = __shfl(d, base + 1), d2 = __shfl(d, base + 2),
                d3 = __shfl(d, base + 3);
    const int r = r0 + (live ? an : 0);
    const int a = lstart + r;
    const int y = r / L.W, x = r - (r / L.W) * L.W;
    const float ax = (float)x + 0.5f, ay = (float)y + 0.5f;
    const float x1 = ax - d0, y1 = ay - d1, x2 = ax + d2, y2 = ay + d3;
    const float cx = (x1 + x2) / 2.0f * L.stride, cy = (y1 + y2) / 2.0f * L.stride;
    const float w = (x2 - x1) * L.stride, hh = (y2 - y1) * L.stride;
    if (NCT == 0 && raw && live) {  // (the fixed head runs without raw / logits_out)
      for (int c = part; c < nc; c += 4)
        raw[((size_t)b * (4 + nc) + 4 + c) * A + a] = head_sigmoid(pc[c]);
      const float bxv = part == 0 ? cx : (part == 1 ? cy : (part == 2 ? w : hh));
      raw[((size_t)b * (4 + nc) + part) * A + a] = bxv;
    }
    // Candidates go to this block's own 64-slot segment of the image's list
    // (slot = segment * 64 + rank, ranks in anchor order) and the segment's
    // count to seg_n: no cross-block atomics (same-address device atomics
    // from thousands of waves serialise for ~100 us).
    const bool pass = live && part == 0 && cand && best > conf;
    const unsigned long long m = __ballot(pass);
    const int wave = tid >> 6;
    if ((tid & 63) == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    if (!cand) continue;
    int base0 = blk * 64;
    for (int w2 = 0; w2 < wave; ++w2) base0 += wcnt[w2];
    if (tid == 0) seg_n[(size_t)b * nblk + blk] = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (pass) {
      const int i = base0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
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
}

// The chained head's last step (ConvArgs::ch_mode 2 / 3 wrote, per level
// pixel, the four DFL distances and the best class (score, class)): one
// wave per 64-anchor segment of one image -- dist2bbox * stride,
// xywh2xyxy and the conf filter with the expressions of
// detect_decode_kernel, candidates in the same segmented layout and anchor
// order (ballot ranks), so its output equals the fixed decode's.
__global__ __launch_bounds__(256) void head_combine_kernel(HeadCombine h, int B, float conf,
                                                           Cand* __restrict__ cand, int cap,
                                                           int* __restrict__ seg_n, int nblk) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);  // wave-uniform
  if (blk >= nblk) return;
  int l = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < h.nlv && blk >= h.blk[i]) l = i;
  // compile-time selection of the level's fields (no dynamic index into
  // the by-value argument)
  const float* bx = h.bx[0];
  const float* sc = h.sc[0];
  int W = h.W[0], HW = h.H[0] * h.W[0], lstart = h.start[0], lblk = h.blk[0];
  float stride = h.stride[0];
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i == l) {
      bx = h.bx[i];
      sc = h.sc[i];
      W = h.W[i];
      HW = h.H[i] * h.W[i];
      lstart = h.start[i];
      lblk = h.blk[i];
      stride = h.stride[i];
    }
  const int r0 = (blk - lblk) * 64;
  const bool live = r0 + lane < HW;
  const int r = r0 + (live ? lane : 0);
  const f32x4 d = *(const f32x4*)(bx + ((size_t)b * HW + r) * 4);
  const v2u32 q = *(const v2u32*)(sc + ((size_t)b * HW + r) * 2);
  const float best = __uint_as_float(q[0]);
  const int bc = (int)q[1];
  const int a = lstart + r;
  const int y = r / W, x = r - (r / W) * W;
  const float ax = (float)x + 0.5f, ay = (float)y + 0.5f;
  const float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
  const float cx = (x1 + x2) / 2.0f * stride, cy = (y1 + y2) / 2.0f * stride;
  const float w = (x2 - x1) * stride, hh = (y2 - y1) * stride;
  const bool pass = live && best > conf;
  const unsigned long long m = __ballot(pass);
  if (lane == 0) seg_n[(size_t)b * nblk + blk] = __popcll(m);
  if (pass) {
    const int i = blk * 64 + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
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

int launch_head_combine(const HeadCombine& h, int B, float conf, Cand* cand, int cand_cap,
                        int* cand_n, hipStream_t s) {
  const int nblk = h.blk[h.nlv];
  if (!cand || !cand_n || cand_cap < nblk * 64) {
    set_error("head combine: candidate buffers (cap %d < %d segments x 64)", cand_cap, nblk);
    return RV_EINVAL;
  }
  head_combine_kernel<<<dim3(ceil_div(nblk, 4), B), 256, 0, s>>>(h, B, conf, cand, cand_cap, cand_n, nblk);
  return launch_status("head_combine");
}

int decode_segments(const HeadLevel* lv, int nlv) {
  int n = 0;
  for (int i = 0; i < nlv; ++i) n += ceil_div(lv[i].H * lv[i].W, 64);
  return n;
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
  const size_t smem = (size_t)64 * (cs + 4) * 4;
  const bool fused = lv[0].feat != nullptr;
  // YOLOv8n's fused head (every level: box 64 -> 64, class 80 -> 80): the
  // compile-time MFMA section
  // (it keeps the class scores in registers: no raw output, no logits copy)
  bool fixed = fused && nc == 80 && raw == nullptr;
  for (int i = 0; i < nlv && fixed; ++i)
    fixed = lv[i].cin_b == 64 && lv[i].cin_c == 80 && lv[i].logits_out == nullptr;
  static const bool fixed_env = !getenv("RV_DECODE_FIXED") || atoi(getenv("RV_DECODE_FIXED")) != 0;
  fixed = fixed && fixed_env;
  if (smem > 64 * 1024) {  // only raise the cap when the head needs it (large nc)
    // best effort: a failure surfaces as the launch error reported below
    (void)hipFuncSetAttribute(fused ? (const void*)detect_decode_kernel<16, true>
                              : (const void*)detect_decode_kernel<16, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
  }
  const int nblk = h.blk[nlv];
  if (cand && cand_cap < nblk * 64) {
    set_error("detect decode: cand_cap %d < %d segments x 64", cand_cap, h.blk[nlv]);
    return RV_EINVAL;
  }
  if (fused) {
    for (int i = 0; i < nlv; ++i)
      if (lv[i].cs != 4 * reg_max + nc || lv[i].cin_b % 8 || lv[i].cin_c % 8 || lv[i].feat_cs % 8) {
        set_error("fused head: bad level %d geometry", i);
        return RV_EINVAL;
      }
    if (fixed) {
      // anchor tiles per block: enough blocks to fill the chip several times
      static const int tpb_env = getenv("RV_DECODE_TPB") ? atoi(getenv("RV_DECODE_TPB")) : 0;
      int tpb = tpb_env > 0 ? tpb_env : 4;
      while (tpb > 1 && (long)ceil_div(nblk, tpb) * B < 4L * num_cus()) --tpb;
      detect_decode_kernel<16, true, 2, 3, 5, 80><<<dim3(ceil_div(nblk, tpb), B), 256, smem, s>>>(
          h, B, nc, conf, raw, cand, cand_cap, cand_n, nblk, tpb);
    } else {
      detect_decode_kernel<16, true><<<dim3(nblk, B), 256, smem, s>>>(h, B, nc, conf, raw, cand,
                                                                      cand_cap, cand_n, nblk, 1);
    }
  } else {
    detect_decode_kernel<16, false><<<dim3(nblk, B), 256, smem, s>>>(h, B, nc, conf, raw, cand,
                                                                     cand_cap, cand_n, nblk, 1);
  }
  return launch_status("detect_decode");
}


// One bf16 conv (k 1 or 3, pad k / 2, SiLU optional, optional bf16 residual
// of the output's shape) through the production launcher, for layer tests:
// the weights packed as yolo.hip packs them ([Cout_pad16][k*k][Cin_pad32]
// bf16), the bias padded to Cout_pad16.  cfg6 (nullable): an explicit
// {MR, NR, G, resw, persist, kind} configuration.
}  // namespace rv
extern "C" int rv_conv_bf16(const void* in, int B, int Hin, int Win, int Cin, int in_cs,
                            const void* w, const float* bias, int Cout, int k, int stride, void* out,
                            int out_cs, const void* res, int res_cs, int act, const int* cfg6,
                            void* stream) {
  using namespace rv;
  RV_CHECK_ARG(in && w && bias && out, "null pointer");
  RV_CHECK_ARG(B >= 1 && Hin >= 1 && Win >= 1 && Cin >= 1 && Cout >= 1, "bad shape");
  RV_CHECK_ARG((k == 1 || k == 3) && (stride == 1 || stride == 2), "k %d stride %d", k, stride);
  RV_CHECK_ARG(in_cs >= Cin && out_cs >= Cout && (!res || res_cs >= Cout), "channel strides");
  ConvArgs a;
  memset(&a, 0, sizeof(a));
  a.in = (const bf16_t*)in;
  a.in_cs = in_cs;
  a.Hin = Hin;
  a.Win = Win;
  a.Cin = Cin;
  a.w = (const bf16_t*)w;
  a.bias = bias;
  a.Cout = Cout;
  a.k = k;
  a.stride = stride;
  a.pad = k / 2;
  a.Ho = (Hin + 2 * a.pad - k) / stride + 1;
  a.Wo = (Win + 2 * a.pad - k) / stride + 1;
  a.B = B;
  a.out0 = out;
  a.out0_cs = out_cs;
  a.res = (const bf16_t*)res;
  a.res_cs = res_cs;
  a.act = act ? 1 : 0;
  const hipStream_t s = (hipStream_t)stream;
  if (cfg6) {
    const ConvCfg c{cfg6[0], cfg6[1], cfg6[2], cfg6[3], cfg6[4], cfg6[5]};
    return launch_conv_cfg(a, c, s);
  }
  return launch_conv(a, s);
}
namespace rv {
}  // namespace rv
