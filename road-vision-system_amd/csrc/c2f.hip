// Fused C2f bottleneck chain + cv2 for the narrow (C <= 32) C2f blocks of
// YOLOv8 (Ultralytics C2f / Bottleneck; oracle/yolo_ref.py YoloRef.c2f):
//
//   y0, y1 = cv1(x).chunk(2)          (cv1 runs before, as a normal 1x1 conv,
//                                      into the block's concat buffer)
//   z_i = [y_in +] cvb_i(cva_i(y_in))  (3x3 C -> C twice, residual if shortcut;
//                                      y_in = y1 for i = 0, z_{i-1} after)
//   out = cv2(cat(y0, y1, z_0 .. z_{N-1}))   (1x1 (2+N)C -> 2C)
//
// One workgroup (8 waves) per TR x TC output tile of one image.  y1 is read
// with a halo of 2N pixels (each 3x3 conv eats one), y0 at the tile only;
// every intermediate (t_i = cva_i(.), z_i) lives in LDS only and never
// touches HBM -- the unfused form writes and re-reads all of them, one
// launch per conv.  Out-of-image pixels of every LDS map are zero (the next
// 3x3 conv's padding).
//
// Bit-identical to the unfused kernels (conv_patch_kernel /
// conv1x1_direct_kernel): the same v_mfma_f32_16x16x32_bf16 k-order (taps
// (ky, kx) ascending with one 32-channel k-step each -- channels >= C are
// zero in both operands -- and cv2's 32-channel chunks ascending), the same
// epilogue (bias, SiLU, residual add of the bf16 input, round to bf16).
//
// LDS maps are pixel-major and linear: PB = 2C bytes per pixel (C channels
// of bf16), quarter q of pixel p at p*PB + 16q.  With the region widths
// compile-time, every tap of a 3x3 conv is one ds_read_b128 at a constant
// offset from the lane's base address: no per-tap address VALU (the XOR
// swizzle this replaced cost ~5 VALU per tap and pair, and the chain loops
// were VALU-issue-bound).  gfx950 ds_read_b128 lane groups ({0-3,12-15,
// 20-27}, {4-11,16-19,28-31}, +32): PB = 32 is conflict-free for 16
// consecutive pixels, PB = 64 at most 2-way.  At C = 16 the k-padding
// quarters (2, 3) of a B fragment read a zeroed LDS span instead of a
// branch per tap.
#include "conv.h"
#include "conv_common.h"

namespace rv {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8c;
typedef __attribute__((ext_vector_type(4))) float f32x4c;
typedef __attribute__((ext_vector_type(2))) float f32x2c;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2c;

__device__ __forceinline__ uint32_t c2f_pack(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2c{lo, hi}, bf16x2c));
}
__device__ __forceinline__ float c2f_bf2f(uint32_t h) { return __uint_as_float(h << 16); }

template <int C>
struct C2fGeo {
  static constexpr int PB = 2 * C;      // bytes per pixel
  static constexpr int NQ = PB / 16;    // 16-B quarters per pixel
  static constexpr int MR = C / 16;     // 16-cout fragments of a C-out conv
  __device__ static __forceinline__ int addr(int p, int q) { return p * PB + (q << 4); }
};

template <int TR, int TC>
struct C2fTile {
  __host__ __device__ static constexpr int rh(int e) { return TR + 2 * e; }
  __host__ __device__ static constexpr int rw(int e) { return TC + 2 * e; }
  __host__ __device__ static constexpr int rp(int e) { return rh(e) * rw(e); }
};

template <int C, int N, int TR, int TC>
struct C2fLds {
  using G = C2fGeo<C>;
  using T = C2fTile<TR, TC>;
  static constexpr int h = 2 * N;
  static constexpr int Y = 0;                                  // y1, halo h
  static constexpr int Tb = Y + T::rp(h) * G::PB;              // t_i (largest: halo h-1)
  static constexpr int Z0 = Tb + T::rp(h - 1) * G::PB;         // z_0, halo h-2
  static constexpr int Z1 = Z0 + T::rp(h - 2) * G::PB;         // z_1, halo h-4 (N = 2)
  static constexpr int Y0 = Z1 + (N == 2 ? T::rp(0) * G::PB : 0);  // y0, halo 0
  // zeros read by the k-padding quarters at C = 16: the largest tap offset
  // span (2 rows + 2 pixels of the widest input region) + one quarter
  static constexpr int ZR = Y0 + T::rp(0) * G::PB;
  static constexpr int ZBYTES = G::NQ < 4 ? (2 * T::rw(h) + 3) * G::PB : 0;
  static constexpr int BYTES = ZR + ZBYTES;
};

// 3x3 C -> C conv from an LDS map at halo e_out + 1 into one at halo e_out
// (+ residual from an LDS map at halo e_res), zero outside the image.
template <int C, int TR, int TC, bool RES, int EO, int ER>
__device__ __forceinline__ void c2f_conv3(const uint8_t* __restrict__ in, uint8_t* __restrict__ outb,
                                          const bf16_t* __restrict__ w,
                                          const float* __restrict__ bias,
                                          const uint8_t* __restrict__ res, int oy0, int ox0, int H,
                                          int W, const uint8_t* __restrict__ zeros, bool pairs) {
  using G = C2fGeo<C>;
  using T = C2fTile<TR, TC>;
  constexpr int MR = G::MR;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, quad = lane >> 4;
  constexpr int e_out = EO, e_res = ER;
  constexpr int rwo = T::rw(e_out), rpo = T::rp(e_out), rwi = rwo + 2, rwr = T::rw(e_res);
  // A fragments of all 9 taps: packed [Cout_pad16][3][3][32] (Cin zero-padded to 32)
  bf16x8c A[9][MR];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int m = 0; m < MR; ++m)
      A[t][m] = __builtin_bit_cast(bf16x8c,
                                   *(const uint4*)(w + ((size_t)(m * 16 + col) * 9 + t) * 32 + quad * 8));
  f32x4c bv[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) bv[m] = *(const f32x4c*)(bias + m * 16 + quad * 4);
  const int nfrag = (rpo + 15) / 16;
  if (C == 16 && pairs) {  // block-uniform
    // Tap pairs (the stem's model.1 form): a 32-deep k-step takes the 16
    // channels of two taps -- quads 0, 1 tap 2p, quads 2, 3 tap 2p + 1 (the
    // last, tap 8, pairs with zero weights) -- so a 16-channel 3x3 conv is 5
    // MFMAs and 5 B reads per fragment instead of 9 half-zero ones.  The sums
    // differ from the unfused per-tap k-steps by rounding only (1 bf16 ulp:
    // tests/test_yolo_layers_gpu.py).  Pair p's second tap is tap 2p + 1:
    // the next pixel for p = 0, 2, 3, the next row's first for p = 1.
    bf16x8c Ap[5];
#pragma unroll
    for (int p = 0; p < 5; ++p) {
      const int t = 2 * p + (quad >> 1);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (t < 9) v = *(const uint4*)(w + ((size_t)col * 9 + t) * 32 + (quad & 1) * 8);
      Ap[p] = __builtin_bit_cast(bf16x8c, v);
    }
    const bool hiq = quad >= 2;
    for (int f0 = wave * 2; f0 < nfrag; f0 += 16) {
      f32x4c acc[2];
      int o[2];
      const uint8_t* b1[2];  // pairs 0, 2, 3: tap 2p + (quad >> 1)
      const uint8_t* b2[2];  // pair 1: taps 2 (0, 2) and 3 (1, 0)
      const uint8_t* b4[2];  // tap 8 (quads 0, 1) or zeros
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        o[n] = (f0 + n) * 16 + col;
        const int oo = o[n] < rpo ? o[n] : 0;
        const int r = oo / rwo, c = oo - r * rwo;
        const uint8_t* bp = in + G::addr(r * rwi + c, quad & 1);
        b1[n] = bp + (hiq ? G::PB : 0);
        b2[n] = bp + (hiq ? (rwi - 2) * G::PB : 0) + (2 * G::PB);
        b4[n] = hiq ? zeros : bp + (2 * rwi + 2) * G::PB;
        acc[n] = f32x4c{0.f, 0.f, 0.f, 0.f};
      }
      bf16x8c Bp[5][2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        Bp[0][n] = __builtin_bit_cast(bf16x8c, *(const uint4*)(b1[n]));
        Bp[1][n] = __builtin_bit_cast(bf16x8c, *(const uint4*)(b2[n]));
        Bp[2][n] = __builtin_bit_cast(bf16x8c, *(const uint4*)(b1[n] + (rwi + 1) * G::PB));
        Bp[3][n] = __builtin_bit_cast(bf16x8c, *(const uint4*)(b1[n] + (2 * rwi) * G::PB));
        Bp[4][n] = __builtin_bit_cast(bf16x8c, *(const uint4*)(b4[n]));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < 5; ++p)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ap[p], Bp[p][n], acc[n], 0, 0, 0);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if (o[n] >= rpo) continue;
        const int r = o[n] / rwo, c = o[n] - (o[n] / rwo) * rwo;
        const int gy = oy0 - e_out + r, gx = ox0 - e_out + c;
        const bool inside = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[n][i] + bv[0][i];
        silu4(v);
        const int lq = (quad * 4) >> 3, half = (quad & 1) * 8;
        if (RES) {
          const int d = e_res - e_out;
          const int pr = (r + d) * rwr + c + d;
          const uint2 rr = *(const uint2*)(res + G::addr(pr, lq) + half);
          v[0] += c2f_bf2f(rr.x & 0xFFFF);
          v[1] += c2f_bf2f(rr.x >> 16);
          v[2] += c2f_bf2f(rr.y & 0xFFFF);
          v[3] += c2f_bf2f(rr.y >> 16);
        }
        const uint2 pk = inside ? make_uint2(c2f_pack(v[0], v[1]), c2f_pack(v[2], v[3]))
                                : make_uint2(0, 0);
        *(uint2*)(outb + G::addr(o[n], lq) + half) = pk;
      }
    }
    return;
  }
  for (int f0 = wave * 2; f0 < nfrag; f0 += 16) {
    f32x4c acc[2][MR];
    int o[2];
    const uint8_t* bp[2];  // this lane's quarter of the tap-(0,0) pixel
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      o[n] = (f0 + n) * 16 + col;
      const int oo = o[n] < rpo ? o[n] : 0;
      const int r = oo / rwo, c = oo - r * rwo;
      bp[n] = quad < G::NQ ? in + G::addr(r * rwi + c, quad) : zeros;
#pragma unroll
      for (int m = 0; m < MR; ++m) acc[n][m] = f32x4c{0.f, 0.f, 0.f, 0.f};
    }
    // B fragments read D - 1 taps ahead into a ring of registers, the order
    // pinned by sched_barrier fences: left to the scheduler, every tap's
    // ds_read_b128 landed in one register right before its MFMA with an
    // lgkmcnt(0) wait in between -- 18 serial LDS round trips per fragment
    // pair.  The MFMA order (taps ascending, then n, then m) is unchanged.
    constexpr int D = 4;
    bf16x8c Bq[D][2];
    auto ld = [&](int t, int sl) {
      const int ky = t / 3, kx = t - (t / 3) * 3;
#pragma unroll
      for (int n = 0; n < 2; ++n)
        Bq[sl][n] = __builtin_bit_cast(bf16x8c, *(const uint4*)(bp[n] + (ky * rwi + kx) * G::PB));
    };
#pragma unroll
    for (int t = 0; t < D - 1; ++t) ld(t, t);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + D - 1 < 9) ld(t + D - 1, (t + D - 1) % D);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int m = 0; m < MR; ++m)
          acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[t][m], Bq[t % D][n], acc[n][m], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      if (o[n] >= rpo) continue;
      const int r = o[n] / rwo, c = o[n] - (o[n] / rwo) * rwo;
      const int gy = oy0 - e_out + r, gx = ox0 - e_out + c;
      const bool inside = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[n][m][i] + bv[m][i];
        silu4(v);
        const int lq = (m * 16 + quad * 4) >> 3, half = (quad & 1) * 8;
        if (RES) {
          const int d = e_res - e_out;
          const int pr = (r + d) * rwr + c + d;
          const uint2 rr = *(const uint2*)(res + G::addr(pr, lq) + half);
          v[0] += c2f_bf2f(rr.x & 0xFFFF);
          v[1] += c2f_bf2f(rr.x >> 16);
          v[2] += c2f_bf2f(rr.y & 0xFFFF);
          v[3] += c2f_bf2f(rr.y >> 16);
        }
        const uint2 pk = inside ? make_uint2(c2f_pack(v[0], v[1]), c2f_pack(v[2], v[3]))
                                : make_uint2(0, 0);
        *(uint2*)(outb + G::addr(o[n], lq) + half) = pk;
      }
    }
  }
}

template <int C, int N, bool SC, int TR, int TC>
__global__ __launch_bounds__(512) void c2f_chain_kernel(C2fArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  using G = C2fGeo<C>;
  using T = C2fTile<TR, TC>;
  using L = C2fLds<C, N, TR, TC>;
  constexpr int h = 2 * N;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, quad = lane >> 4;
  const int tiles_x = (a.W + TC - 1) / TC, tiles_y = (a.H + TR - 1) / TR;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int oy0 = ty * TR, ox0 = tx * TC;
  const bf16_t* img = a.cat + (size_t)b * a.H * a.W * a.cat_cs + a.cat_co;

  // ---- 1. y1 (halo h) and y0 (tile) from the concat buffer, zero outside.
  //      Element i of a map is its 16-B quarter i % NQ of pixel i / NQ, stored
  //      at byte 16 i (PB = 16 NQ); the map widths are compile-time, so the
  //      pixel's (row, column) is a division by a constant, and every load of
  //      a thread is issued before the first LDS store.
  {
    constexpr int NY = T::rp(h) * G::NQ, N0 = T::rp(0) * G::NQ;
    constexpr int U1 = (NY + 511) / 512, U0 = (N0 + 511) / 512;
    auto fetch = [&](int i, int n, int e, int rwe, int ch) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (i < n) {
        const int p = i / G::NQ, q = i - p * G::NQ;
        const int r = p / rwe, c = p - r * rwe;
        const int gy = oy0 - e + r, gx = ox0 - e + c;
        if ((unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W)
          // the pixel index (< H * W) widened before the channel-stride multiply
          v = *(const uint4*)(img + ((size_t)gy * a.W + gx) * a.cat_cs + ch + q * 8);
      }
      return v;
    };
    uint4 v1[U1], v0[U0];
#pragma unroll
    for (int u = 0; u < U1; ++u) v1[u] = fetch(tid + 512 * u, NY, h, T::rw(h), C);
#pragma unroll
    for (int u = 0; u < U0; ++u) v0[u] = fetch(tid + 512 * u, N0, 0, T::rw(0), 0);
#pragma unroll
    for (int u = 0; u < U1; ++u)
      if (tid + 512 * u < NY) *(uint4*)(smem + L::Y + 16 * (tid + 512 * u)) = v1[u];
#pragma unroll
    for (int u = 0; u < U0; ++u)
      if (tid + 512 * u < N0) *(uint4*)(smem + L::Y0 + 16 * (tid + 512 * u)) = v0[u];
    for (int i = tid; i < L::ZBYTES / 16; i += 512) *(uint4*)(smem + L::ZR + 16 * i) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  // ---- 2. bottlenecks: t = cva(y_in) at halo e-1, z = [y_in +] cvb(t) at e-2
  const uint8_t* zeros = smem + L::ZR;
  c2f_conv3<C, TR, TC, false, h - 1, 0>(smem + L::Y, smem + L::Tb, a.wa[0], a.ba[0], nullptr, oy0,
                                        ox0, a.H, a.W, zeros, a.tap_pairs != 0);
  __syncthreads();
  c2f_conv3<C, TR, TC, SC, h - 2, h>(smem + L::Tb, smem + L::Z0, a.wb[0], a.bb[0], smem + L::Y, oy0,
                                     ox0, a.H, a.W, zeros, a.tap_pairs != 0);
  __syncthreads();
  if constexpr (N == 2) {
    c2f_conv3<C, TR, TC, false, h - 3, 0>(smem + L::Z0, smem + L::Tb, a.wa[1], a.ba[1], nullptr, oy0,
                                          ox0, a.H, a.W, zeros, a.tap_pairs != 0);
    __syncthreads();
    c2f_conv3<C, TR, TC, SC, h - 4, h - 2>(smem + L::Tb, smem + L::Z1, a.wb[1], a.bb[1],
                                           smem + L::Z0, oy0, ox0, a.H, a.W, zeros, a.tap_pairs != 0);
    __syncthreads();
  }

  // ---- 3. cv2: 1x1 over cat(y0, y1, z_0 .. z_{N-1}) at the tile -> HBM
  constexpr int KC = (2 + N) * C;        // concat channels
  constexpr int NCH = (KC + 31) / 32;    // 32-channel k-steps
  constexpr int MR2 = 2 * C / 16;        // cv2 cout fragments (2C couts)
  static_assert(MR2 % 2 == 0, "cv2 stores fragment pairs");
  constexpr int KP = NCH * 32;           // packed Cin (padded to 32)
  bf16x8c A2[NCH][MR2];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int m = 0; m < MR2; ++m)
      A2[j][m] = __builtin_bit_cast(bf16x8c,
                                    *(const uint4*)(a.w2 + (size_t)(m * 16 + col) * KP + j * 32 + quad * 8));
  f32x4c bv2[MR2];
#pragma unroll
  for (int m = 0; m < MR2; ++m) bv2[m] = *(const f32x4c*)(a.b2 + m * 16 + quad * 4);
  // segment s of the concat: 0 = y0 (halo 0), 1 = y1 (halo h), 2 + i = z_i
  auto seg_buf = [&](int s) -> int {
    return s == 0 ? L::Y0 : (s == 1 ? L::Y : (s == 2 ? L::Z0 : L::Z1));
  };
  auto seg_halo = [&](int s) -> int { return s == 0 ? 0 : (s == 1 ? h : h - 2 * (s - 1)); };
  constexpr int RP0 = T::rp(0);
  constexpr int NFR = RP0 / 16;
  for (int f0 = wave * 2; f0 < NFR; f0 += 16) {
    f32x4c acc[2][MR2];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int m = 0; m < MR2; ++m) acc[n][m] = f32x4c{0.f, 0.f, 0.f, 0.f};
    // every k-step's B fragments first (NCH x 2 ds_read_b128 in flight),
    // then the MFMAs in the same order as before
    bf16x8c B2[NCH][2];
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int k0 = j * 32 + quad * 8;  // first concat channel of this lane's k-slice
      const int s = k0 / C, qq = (k0 - s * C) >> 3;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int o = (f0 + n) * 16 + col;
        const int r = o / TC, c = o - (o / TC) * TC;
        uint4 bq = make_uint4(0, 0, 0, 0);
        if (s < 2 + N) {
          const int e = seg_halo(s);
          const int p = (r + e) * T::rw(e) + c + e;
          bq = *(const uint4*)(smem + seg_buf(s) + G::addr(p, qq));
        }
        B2[j][n] = __builtin_bit_cast(bf16x8c, bq);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int m = 0; m < MR2; ++m)
          acc[n][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A2[j][m], B2[j][n], acc[n][m], 0, 0, 0);
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int o = (f0 + n) * 16 + col;
      const int r = o / TC, c = o - (o / TC) * TC;
      const int gy = oy0 + r, gx = ox0 + c;
      if (gy >= a.H || gx >= a.W) continue;
      uint16_t* dst = a.out + ((size_t)(b * a.H + gy) * a.W + gx) * a.out_cs + a.out_co;
      // fragment pairs (m, m+1) as 16-B stores: after one v_permlane16_swap
      // per packed dword quad q holds channels 8 (q >> 1) .. +7 of fragment
      // m + (q & 1) (conv.hip epilogue_fast); all quads of a pixel share
      // the bounds test above
#pragma unroll
      for (int m = 0; m < MR2; m += 2) {
        uint32_t pk[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = acc[n][m + h][i] + bv2[m + h][i];
          silu4(v);
          pk[h][0] = c2f_pack(v[0], v[1]);
          pk[h][1] = c2f_pack(v[2], v[3]);
        }
        const auto x0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
        const auto x1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
        *(uint4*)(dst + (m + (quad & 1)) * 16 + (quad >> 1) * 8) = make_uint4(x0[0], x1[0], x0[1], x1[1]);
      }
    }
  }
}

template <int C, int N, bool SC, int TR, int TC>
static int launch_c2f_t(const C2fArgs& a, hipStream_t s) {
  using L = C2fLds<C, N, TR, TC>;
  static_assert(L::BYTES <= 160 * 1024, "C2f tile exceeds LDS");
  static_assert((TR * TC) % 32 == 0, "tile must hold whole fragment pairs");
  auto fn = c2f_chain_kernel<C, N, SC, TR, TC>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       L::BYTES);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      set_error("hipFuncSetAttribute(c2f): %s", hipGetErrorString(e));
      return -(int)e;
    }
    attr = true;
  }
  const int blocks = a.B * ceil_div(a.H, TR) * ceil_div(a.W, TC);
  fn<<<blocks, 512, L::BYTES, s>>>(a);
  return launch_status("c2f_chain");
}

bool c2f_fusable(int C, int N, int cat_cs, int cat_co, int out_cs, int out_co) {
  return (C == 16 || C == 32) && (N == 1 || N == 2) && !(C == 16 && N == 2) && cat_cs % 8 == 0 &&
         cat_co % 8 == 0 && out_cs % 4 == 0 && out_co % 4 == 0;
}

int launch_c2f_chain(const C2fArgs& a, int C, int N, bool shortcut, hipStream_t s) {
  if (!c2f_fusable(C, N, a.cat_cs, a.cat_co, a.out_cs, a.out_co)) {
    set_error("c2f_chain: C=%d N=%d unsupported", C, N);
    return RV_EINVAL;
  }
  // tiles: 16 x 32 at C = 16 (P2 maps), 16 x 16 at C = 32 (P3 maps divide)
  if (C == 16) return shortcut ? launch_c2f_t<16, 1, true, 16, 32>(a, s)
                               : launch_c2f_t<16, 1, false, 16, 32>(a, s);
  if (N == 1) return shortcut ? launch_c2f_t<32, 1, true, 16, 16>(a, s)
                              : launch_c2f_t<32, 1, false, 16, 16>(a, s);
  return shortcut ? launch_c2f_t<32, 2, true, 16, 16>(a, s) : launch_c2f_t<32, 2, false, 16, 16>(a, s);
}

}  // namespace rv
