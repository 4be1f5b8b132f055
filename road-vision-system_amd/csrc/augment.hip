// Fog + rain synthetic-input generator on device (the
// config-5 "fog/rain-augmented frames").  Restates the scattering core of
// EnhancedFogSynthesizer.synthesize (src/augment/fog.py:239-299):
//   depth proxy            fog.py:141-163  (per-row terms precomputed on host)
//   beta map (value noise) fog.py:8-45, 166-169
//   transmission           fog.py:172-173  (t = clip(exp(-beta d), .05, 1))
//   airlight map           fog.py:128-138  (vertical x horizontal gradient)
//   I = J t + A (1 - t)    fog.py:271
//   global veil            fog.py:274-275
//   colour tint / gamma    fog.py:291-296
// plus rain streaks (the reference has fog only).  The OpenCV
// filters of the reference (guided / bilateral filters, glow, depth blur,
// local contrast fade) are not restated; DESIGN.md §"Fog generator" says why.
//
// HBM-bound elementwise work: 3 B read + 3 B written per pixel.  One thread
// handles 4 pixels (12 B: three dword loads / stores) when the row layout
// allows it.  The value noise needs a per-frame min/max before it can be
// normalised (fog.py:43), so a first pass reduces it (ALU only, no frame
// bytes read, partials per workgroup, no atomics) and the second pass does
// the per-pixel work.  The per-pixel pass is VALU-bound, so its exp, pow and
// divides use the hardware instructions (v_exp_f32 / v_log_f32 / v_rcp_f32,
// about 1 ulp) instead of the IEEE library sequences; the oracle's bar (u8
// |d| <= 1, >= 99 % exact) covers that.  The noise range pass keeps exact
// divides.
#include "common.h"

namespace rv {

namespace {

constexpr int kFogMaxOct = 4;
constexpr int kGridLds = 2048;  // noise grid floats staged in LDS (8 KB)

struct FogConsts {
  float vx, vy, dv_max, d_min, d_range, veil_unused, rain_p, rain_len;
  int n_oct;
  int gh[kFogMaxOct], gw[kFogMaxOct];
  float amp[kFogMaxOct];
  int goff[kFogMaxOct];
  float norm;
  int grid_stride;
  uint32_t rain_thresh;
};

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Raw (un-normalised) fBM value noise at pixel (y, x): rand_perlin
// (fog.py:8-41) with ys = (y*gh)/h in f32, bilinear on the per-frame grid.
// The per-axis sample taps (y0, y1, wy) / (x0, x1, wx) of every octave are
// resolution-only, so the host computes them once (same f32 values) and the
// kernel reads them from the scene buffer: no divides or floors per pixel.
__device__ __forceinline__ float noise_at(const FogConsts& c, const float* __restrict__ g,
                                          const float* __restrict__ taps, int y, int x, int H,
                                          int W) {
  float base = 0.f;
  for (int j = 0; j < c.n_oct; ++j) {
    const float* ty = taps + (size_t)j * 3 * (H + W);
    const float* tx = ty + 3 * H;
    const int y0 = (int)ty[y], y1 = (int)ty[H + y];
    const float wy = ty[2 * H + y];
    const int x0 = (int)tx[x], x1 = (int)tx[W + x];
    const float wx = tx[2 * W + x];
    const float* gj = g + c.goff[j];
    const int rw = c.gw[j] + 1;
    const float g00 = gj[y0 * rw + x0], g01 = gj[y0 * rw + x1];
    const float g10 = gj[y1 * rw + x0], g11 = gj[y1 * rw + x1];
    const float top = g00 * (1.f - wx) + g01 * wx;
    const float bot = g10 * (1.f - wx) + g11 * wx;
    const float val = top * (1.f - wy) + bot * wy;
    base = base + c.amp[j] * val;
  }
  return base / fmaxf(1e-6f, c.norm);
}

// Per-frame noise range in two steps with no atomics: each of the
// kRangeBlocks workgroups of a frame stores its partial min / max (vector
// stores), then one workgroup per frame folds them.  (A device-scope atomic
// per workgroup serialises across the 8 XCDs' L2s: 1600 of them on one
// address cost ~0.45 ms per batch.)
constexpr int kRangeBlocks = 256;

__global__ __launch_bounds__(256) void fog_range_kernel(const float* __restrict__ grids,
                                                        const float* __restrict__ taps,
                                                        FogConsts c, int H, int W,
                                                        float* __restrict__ part) {
  __shared__ float sgrid[kGridLds];  // this frame's value-noise grids
  const int b = blockIdx.y;
  const bool grid_lds = c.grid_stride <= kGridLds;
  if (grid_lds)
    for (int i = threadIdx.x; i < c.grid_stride; i += blockDim.x)
      sgrid[i] = grids[(size_t)b * c.grid_stride + i];
  __syncthreads();
  const float* g = grid_lds ? sgrid : grids + (size_t)b * c.grid_stride;
  float mn = INFINITY, mx = -INFINITY;
  for (int y = blockIdx.x; y < H; y += gridDim.x)  // whole rows: no index divides
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
      const float v = noise_at(c, g, taps, y, x, H, W);
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o));
    mx = fmaxf(mx, __shfl_xor(mx, o));
  }
  __shared__ float smn[4], smx[4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smn[wv] = mn;
    smx[wv] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) {
      mn = fminf(mn, smn[k]);
      mx = fmaxf(mx, smx[k]);
    }
    float* p = part + ((size_t)b * gridDim.x + blockIdx.x) * 2;
    p[0] = mn;
    p[1] = mx;
  }
}

__global__ __launch_bounds__(256) void fog_range_finish(const float* __restrict__ part,
                                                        int nblk, float* __restrict__ range) {
  const int b = blockIdx.x;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
    mn = fminf(mn, part[((size_t)b * nblk + i) * 2]);
    mx = fmaxf(mx, part[((size_t)b * nblk + i) * 2 + 1]);
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o));
    mx = fmaxf(mx, __shfl_xor(mx, o));
  }
  __shared__ float smn[4], smx[4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smn[wv] = mn;
    smx[wv] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) {
      mn = fminf(mn, smn[k]);
      mx = fmaxf(mx, smx[k]);
    }
    range[2 * b] = mn;
    range[2 * b + 1] = mx;
  }
}

// Hardware transcendentals (about 1 ulp): 2^x, log2 x, 1/x.
__device__ __forceinline__ float hw_exp(float x) {
  return __builtin_amdgcn_exp2f(x * 1.44269504088896341f);
}
__device__ __forceinline__ float hw_pow01(float h, float g) {  // h in [0, 1]
  return __builtin_amdgcn_exp2f(g * __builtin_amdgcn_logf(h));
}
__device__ __forceinline__ float hw_div(float a, float b) {
  return a * __builtin_amdgcn_rcpf(b);
}

// One output channel value, fog.py:271-296 (f32, contract off).
__device__ __forceinline__ int fog_channel(float v, float t, float A, float gv, float tint,
                                           float gamma, bool rain) {
  float h = v * t + A * (1.f - t);
  h = fminf(fmaxf(h * (1.f - gv) + A * gv, 0.f), 1.f);
  h = fminf(fmaxf(h * tint, 0.f), 1.f);
  if (gamma != 1.f) h = fminf(fmaxf(hw_pow01(h, gamma), 0.f), 1.f);
  if (rain) h = h + (1.f - h) * 0.45f;
  return (int)(h * 255.f + 0.5f);
}

template <int V>
__global__ __launch_bounds__(256) void fog_apply_kernel(
    const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int H, int W, int pitch,
    const float* __restrict__ scene, const float* __restrict__ fparams,
    const float* __restrict__ grids, FogConsts c, const float* __restrict__ range) {
  __shared__ float inv255[256];  // u / 255.f, exactly as the scalar divide
  __shared__ float sgrid[kGridLds];  // this frame's value-noise grids
  const int b = blockIdx.y;
  inv255[threadIdx.x] = (float)threadIdx.x / 255.f;
  const bool grid_lds = c.grid_stride <= kGridLds;
  if (grid_lds)
    for (int i = threadIdx.x; i < c.grid_stride; i += blockDim.x)
      sgrid[i] = grids[(size_t)b * c.grid_stride + i];
  __syncthreads();
  const float* fp = fparams + (size_t)b * RV_FOG_NPARAM;
  const float beta0 = fp[0], Ab = fp[1], Ag = fp[2], Ar = fp[3], Asc = fp[4];
  const float tb = fp[5], tg = fp[6], tr = fp[7], gamma = fp[8];
  const uint32_t rseed = (uint32_t)fp[9];
  const float mn = range[2 * b], mx = range[2 * b + 1];
  const float* g = grid_lds ? sgrid : grids + (size_t)b * c.grid_stride;
  const float* row_dp = scene;
  const float* row_fac = scene + H;
  const float* row_gv = scene + 2 * H;
  const float* row_vg = scene + 3 * H;
  const float* col_xg = scene + 4 * H;
  const float* taps = scene + 4 * H + W;
  const int gpr = W / V;  // pixel groups per row
  const size_t fofs = (size_t)b * H * pitch;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < H * gpr;
       i += gridDim.x * blockDim.x) {
    const int y = i / gpr, x0 = (i - y * gpr) * V;
    const uint8_t* src = in + fofs + (size_t)y * pitch + 3 * x0;
    uint8_t* dst = out + fofs + (size_t)y * pitch + 3 * x0;
    uint8_t px[3 * V];
    if (V == 4) {
      const uint32_t* s32 = (const uint32_t*)src;
      uint32_t w0 = s32[0], w1 = s32[1], w2 = s32[2];
      for (int k = 0; k < 4; ++k) {
        px[k] = (w0 >> (8 * k)) & 255;
        px[4 + k] = (w1 >> (8 * k)) & 255;
        px[8 + k] = (w2 >> (8 * k)) & 255;
      }
    } else {
      for (int k = 0; k < 3 * V; ++k) px[k] = src[k];
    }
    const float dp = row_dp[y], fac = row_fac[y], gv = row_gv[y], vg = row_vg[y];
    const float dy = (float)y - c.vy;
    const int seg = y / (int)c.rain_len;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int x = x0 + k;
      const float n = noise_at(c, g, taps, y, x, H, W);
      const float nn = hw_div(n - mn, fmaxf(1e-6f, mx - mn));
      const float beta = beta0 * (0.85f + 0.35f * nn);
      const float dx = (float)x - c.vx;
      const float dv = __builtin_amdgcn_rcpf(sqrtf(dx * dx + dy * dy) + 1.f);
      float d = dp + 0.3f * hw_div(dv, c.dv_max);
      d = hw_div(d - c.d_min, c.d_range);
      d = fminf(fmaxf(d * fac, 0.f), 1.f);
      const float t = fminf(fmaxf(hw_exp(-beta * d), 0.05f), 1.f);
      const float xg = col_xg[x];
      const float Ab_ = fminf(fmaxf(fminf(fmaxf(Ab * vg * xg, 0.7f), 1.f) * Asc, 0.75f), 1.f);
      const float Ag_ = fminf(fmaxf(fminf(fmaxf(Ag * vg * xg, 0.7f), 1.f) * Asc, 0.75f), 1.f);
      const float Ar_ = fminf(fmaxf(fminf(fmaxf(Ar * vg * xg, 0.7f), 1.f) * Asc, 0.75f), 1.f);
      bool rain = false;
      if (c.rain_thresh) {
        const uint32_t col = (uint32_t)(x + (y >> 2));
        const uint32_t hsh =
            lowbias32(rseed ^ lowbias32(col * 0x9E3779B1u + lowbias32((uint32_t)seg)));
        rain = hsh < c.rain_thresh;
      }
      px[3 * k + 0] = (uint8_t)fog_channel(inv255[px[3 * k + 0]], t, Ab_, gv, tb, gamma, rain);
      px[3 * k + 1] = (uint8_t)fog_channel(inv255[px[3 * k + 1]], t, Ag_, gv, tg, gamma, rain);
      px[3 * k + 2] = (uint8_t)fog_channel(inv255[px[3 * k + 2]], t, Ar_, gv, tr, gamma, rain);
    }
    if (V == 4) {
      uint32_t* d32 = (uint32_t*)dst;
      uint32_t w0 = 0, w1 = 0, w2 = 0;
      for (int k = 0; k < 4; ++k) {
        w0 |= (uint32_t)px[k] << (8 * k);
        w1 |= (uint32_t)px[4 + k] << (8 * k);
        w2 |= (uint32_t)px[8 + k] << (8 * k);
      }
      d32[0] = w0;
      d32[1] = w1;
      d32[2] = w2;
    } else {
      for (int k = 0; k < 3 * V; ++k) dst[k] = px[k];
    }
  }
}

}  // namespace

extern "C" size_t rv_fog_ws_bytes(int B) {
  return B <= 0 ? 0 : (size_t)B * (2 + 2 * kRangeBlocks) * sizeof(float);
}

extern "C" int rv_fog_rain_u8(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                              const float* consts, int n_consts, const float* scene,
                              const float* frame_params, const float* grids, int grid_stride,
                              void* ws, size_t ws_bytes, void* stream) {
  RV_CHECK_ARG(in != nullptr && out != nullptr && consts != nullptr && scene != nullptr &&
                   frame_params != nullptr && grids != nullptr && ws != nullptr,
               "null pointer");
  RV_CHECK_ARG(B >= 0 && H > 0 && W > 0 && pitch >= 3 * W, "bad frame shape");
  RV_CHECK_ARG((const void*)in != (const void*)out, "in and out must not alias");
  RV_CHECK_ARG(n_consts == RV_FOG_NCONST, "n_consts %d != %d", n_consts, RV_FOG_NCONST);
  FogConsts c{};
  c.vx = consts[0];
  c.vy = consts[1];
  c.dv_max = consts[2];
  c.d_min = consts[3];
  c.d_range = consts[4];
  c.rain_p = consts[6];
  c.rain_len = consts[7];
  c.n_oct = (int)consts[8];
  RV_CHECK_ARG(c.n_oct >= 1 && c.n_oct <= kFogMaxOct, "octaves %d out of [1,4]", c.n_oct);
  RV_CHECK_ARG(c.rain_len >= 1.f && c.rain_p >= 0.f && c.rain_p <= 1.f, "bad rain params");
  RV_CHECK_ARG(c.dv_max > 0.f && c.d_range > 0.f, "bad depth constants");
  int off = 0;
  for (int j = 0; j < c.n_oct; ++j) {
    c.gh[j] = (int)consts[9 + 4 * j];
    c.gw[j] = (int)consts[10 + 4 * j];
    c.amp[j] = consts[11 + 4 * j];
    RV_CHECK_ARG(c.gh[j] >= 1 && c.gw[j] >= 1 && c.gh[j] <= H && c.gw[j] <= W,
                 "octave %d grid %dx%d", j, c.gh[j], c.gw[j]);
    c.goff[j] = off;
    off += (c.gh[j] + 1) * (c.gw[j] + 1);
  }
  c.norm = consts[25];
  RV_CHECK_ARG(grid_stride >= off, "grid_stride %d < %d", grid_stride, off);
  c.grid_stride = grid_stride;
  // exact on both sides of the parity test: double product, truncation
  c.rain_thresh = (uint32_t)fmin((double)c.rain_p * 4294967296.0, 4294967295.0);
  if (B == 0) return RV_OK;
  RV_CHECK_ARG(ws_bytes >= rv_fog_ws_bytes(B), "workspace %zu < %zu bytes", ws_bytes,
               rv_fog_ws_bytes(B));
  hipStream_t s = as_stream(stream);
  float* range = (float*)ws;
  float* part = range + 2 * (size_t)B;
  const int rblocks = min(kRangeBlocks, ceil_div(H * W, 256));
  fog_range_kernel<<<dim3(rblocks, B), 256, 0, s>>>(grids, scene + 4 * H + W, c, H, W,
                                                      part);
  fog_range_finish<<<B, 256, 0, s>>>(part, rblocks, range);
  const bool vec = (W % 4 == 0) && (pitch % 4 == 0) && (((uintptr_t)in | (uintptr_t)out) % 4 == 0);
  if (vec) {
    const int blocks = min(4096, ceil_div(H * (W / 4), 256));
    fog_apply_kernel<4><<<dim3(blocks, B), 256, 0, s>>>(in, out, H, W, pitch, scene,
                                                         frame_params, grids, c, range);
  } else {
    const int blocks = min(4096, ceil_div(H * W, 256));
    fog_apply_kernel<1><<<dim3(blocks, B), 256, 0, s>>>(in, out, H, W, pitch, scene,
                                                         frame_params, grids, c, range);
  }
  return launch_status("rv_fog_rain_u8");
}

}  // namespace rv
