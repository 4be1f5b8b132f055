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

constexpr int KB = 128;        // k per LDS weight stage (4 MFMA k-steps)
constexpr int WROW = KB + 8;   // LDS row stride in bf16 (272 B: conflict-free rows)

template <int MR, int NR>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
  constexpr int BC = 16 * MR;
  __shared__ __attribute__((aligned(16))) uint16_t wl[BC * WROW];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, quad = lane >> 4;
  const int cout0 = blockIdx.y * BC;
  const int HWo = a.Ho * a.Wo;
  const int M = a.B * HWo;
  const int pix0 = blockIdx.x * (64 * NR) + wave * (16 * NR);

  const int cin_pad = (a.Cin + 31) & ~31;
  const int kspt = cin_pad >> 5;  // k-steps per tap
  const int taps = a.k * a.k;
  const int nks = taps * kspt;
  const int Kp = taps * cin_pad;
  const int cout_pad = (a.Cout + 15) & ~15;

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
  for (int kb0 = 0; kb0 < nks; kb0 += KB / 32) {
    __syncthreads();
    for (int i = tid; i < BC * (KB / 8); i += 256) {
      const int row = i / (KB / 8);
      const int q = i - row * (KB / 8);
      const int kcol = kb0 * 32 + q * 8;
      const int co = cout0 + row;
      uint4 v = zero4;
      if (co < cout_pad && kcol < Kp) v = *(const uint4*)(a.w + (size_t)co * Kp + kcol);
      *(uint4*)&wl[row * WROW + q * 8] = v;
    }
    __syncthreads();
    const int kend = min(KB / 32, nks - kb0);
    for (int ks = 0; ks < kend; ++ks) {
      const int kstep = kb0 + ks;
      const int tap = kstep / kspt;
      const int cs = kstep - tap * kspt;
      const int ky = tap / a.k;
      const int kx = tap - ky * a.k;
      const bool cvalid = cs * 32 + quad * 8 < a.Cin;
      bf16x8 bfr[NR];
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        const int iy = iy0[n] + ky, ix = ix0[n] + kx;
        const bool ok = pv[n] && cvalid && (unsigned)iy < (unsigned)a.Hin &&
                        (unsigned)ix < (unsigned)a.Win;
        uint4 v = zero4;
        if (ok) v = *(const uint4*)(a.in + (size_t)pb[n] + ((size_t)iy * a.Win + ix) * a.in_cs +
                                    cs * 32);
        bfr[n] = __builtin_bit_cast(bf16x8, v);
      }
      bf16x8 afr[MR];
#pragma unroll
      for (int m = 0; m < MR; ++m)
        afr[m] = __builtin_bit_cast(
            bf16x8, *(const uint4*)&wl[(m * 16 + col) * WROW + ks * 32 + quad * 8]);
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[m], bfr[n], acc[m][n], 0, 0, 0);
    }
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

template <int MR, int NR>
static void launch_t(const ConvArgs& a, hipStream_t s) {
  const int M = a.B * a.Ho * a.Wo;
  dim3 grid(ceil_div(M, 64 * NR), ceil_div(a.Cout, 16 * MR));
  conv_mfma_kernel<MR, NR><<<grid, 256, 0, s>>>(a);
}

int launch_conv(const ConvArgs& a, hipStream_t s) {
  const int T = (a.Cout + 15) / 16;  // 16-channel output tiles
  const int M = a.B * a.Ho * a.Wo;
  // channel-tile grouping: the MR in {8,6,5,4,3,2,1} with the least padded
  // output tiles, the largest such MR on ties
  static const int kMR[] = {8, 6, 5, 4, 3, 2, 1};
  int MR = 1, best_waste = 1 << 30;
  for (int mr : kMR) {
    const int waste = ceil_div(T, mr) * mr - T;
    if (waste < best_waste) {
      best_waste = waste;
      MR = mr;
    }
  }
  // pixel tile: keep >= ~1024 workgroups when the layer allows
  const int blocks_c = ceil_div(T, MR);
  int NR = 4;
  if ((long)ceil_div(M, 64 * 4) * blocks_c < 1024) NR = 2;
  if ((long)ceil_div(M, 64 * 2) * blocks_c < 512) NR = 1;
#define RV_CONV_MR(mr)                                                   \
  if (MR == mr) {                                                        \
    if (NR == 4) launch_t<mr, 4>(a, s);                                  \
    else if (NR == 2) launch_t<mr, 2>(a, s);                             \
    else launch_t<mr, 1>(a, s);                                          \
    return launch_status("conv_mfma");                                   \
  }
  RV_CONV_MR(8) RV_CONV_MR(6) RV_CONV_MR(5) RV_CONV_MR(4) RV_CONV_MR(3) RV_CONV_MR(2)
  RV_CONV_MR(1)
#undef RV_CONV_MR
  set_error("no conv variant for MR=%d NR=%d", MR, NR);
  return RV_EINVAL;
}

// ---------------------------------------------------------------------------
// conv0: 3 -> C0, k3 s2 p1, from letterboxed u8 BGR, f32 math, SiLU, bf16 out.
// ---------------------------------------------------------------------------
template <int C0>
__global__ __launch_bounds__(256) void conv0_kernel(const uint8_t* __restrict__ img, int B, int H,
                                                    int W, const float* __restrict__ w,
                                                    const float* __restrict__ bias,
                                                    uint16_t* __restrict__ out, int out_cs) {
  __shared__ float ws[C0 * 27];
  __shared__ float bs[C0];
  for (int i = threadIdx.x; i < C0 * 27; i += 256) ws[i] = w[i];
  for (int i = threadIdx.x; i < C0; i += 256) bs[i] = bias[i];
  __syncthreads();
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= B * Ho * Wo) return;
  const int b = p / (Ho * Wo);
  const int r = p - b * Ho * Wo;
  const int oy = r / Wo, ox = r - (r / Wo) * Wo;
  float x[27];  // [ci(rgb)][ky][kx]
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int iy = oy * 2 - 1 + ky, ix = ox * 2 - 1 + kx;
      const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const uint8_t* px = img + (((size_t)b * H + (ok ? iy : 0)) * W + (ok ? ix : 0)) * 3;
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) x[ci * 9 + ky * 3 + kx] = ok ? (float)px[2 - ci] / 255.0f : 0.f;
    }
  uint16_t* o = out + (size_t)p * out_cs;
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
  const int blocks = ceil_div(B * Ho * Wo, 256);
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
__global__ __launch_bounds__(256) void sppf_pool_kernel(uint16_t* __restrict__ buf, int B, int H,
                                                        int W, int c) {
  const int groups = c / 8;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * H * W * groups) return;
  const int g = idx % groups;
  const int p = idx / groups;
  const int b = p / (H * W);
  const int r = p - b * H * W;
  const int y = r / W, x = r - (r / W) * W;
  const int cs = 4 * c;
  float m5[8], m9[8], m13[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m5[j] = m9[j] = m13[j] = -INFINITY;
  for (int dy = -6; dy <= 6; ++dy) {
    const int yy = y + dy;
    if (yy < 0 || yy >= H) continue;
    for (int dx = -6; dx <= 6; ++dx) {
      const int xx = x + dx;
      if (xx < 0 || xx >= W) continue;
      const uint4 v = *(const uint4*)(buf + ((size_t)(b * H + yy) * W + xx) * cs + g * 8);
      const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
      const int ady = dy < 0 ? -dy : dy, adx = dx < 0 ? -dx : dx;
      const int rad = ady > adx ? ady : adx;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = bf2f((uint16_t)(wv[j / 2] >> ((j & 1) * 16)));
        m13[j] = fmaxf(m13[j], f);
        if (rad <= 4) m9[j] = fmaxf(m9[j], f);
        if (rad <= 2) m5[j] = fmaxf(m5[j], f);
      }
    }
  }
  uint16_t* o = buf + (size_t)p * cs + g * 8;
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

int launch_sppf_pool(bf16_t* buf, int B, int H, int W, int c, hipStream_t s) {
  const int total = B * H * W * (c / 8);
  sppf_pool_kernel<<<ceil_div(total, 256), 256, 0, s>>>(buf, B, H, W, c);
  return launch_status("sppf_pool");
}

// ---------------------------------------------------------------------------
// Detect head decode: DFL softmax-expectation, dist2bbox (xywh) * stride,
// class sigmoid; Ultralytics non_max_suppression candidate filter.
// ---------------------------------------------------------------------------
struct HeadLevels {
  HeadLevel lv[4];
  int start[5];
  int nlv;
};

template <int REG>
__global__ __launch_bounds__(256) void detect_decode_kernel(HeadLevels h, int B, int nc,
                                                            float conf, float* __restrict__ raw,
                                                            Cand* __restrict__ cand, int cap,
                                                            int* __restrict__ cand_n) {
  const int A = h.start[h.nlv];
  const int a = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (a >= A) return;
  int l = 0;
  while (l + 1 < h.nlv && a >= h.start[l + 1]) ++l;
  const HeadLevel& L = h.lv[l];
  const int r = a - h.start[l];
  const int y = r / L.W, x = r - (r / L.W) * L.W;
  const float* px = L.logits + ((size_t)(b * L.H + y) * L.W + x) * L.cs;
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
  for (int i = 0; i < nlv; ++i) {
    h.lv[i] = lv[i];
    h.start[i + 1] = h.start[i] + lv[i].H * lv[i].W;
  }
  const int A = h.start[nlv];
  detect_decode_kernel<16><<<dim3(ceil_div(A, 256), B), 256, 0, s>>>(h, B, nc, conf, raw, cand,
                                                                      cand_cap, cand_n);
  return launch_status("detect_decode");
}

}  // namespace rv
