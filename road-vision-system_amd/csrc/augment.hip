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


// ===========================================================================
// Full synthesize: every filter of EnhancedFogSynthesizer.synthesize
// (fog.py:227-299), restated as opencv-python runs it (no cv2.ximgproc, so
// _guided_filter is its bilateralFilter fallback, fog.py:61-67).
//   fog_air_kernel      image airlight: band luminance 0.9-quantile (radix
//                       select, bit-exact to np.quantile), masked mean,
//                       tint + clip (fog.py:120-130)
//   fog_t_kernel        t0 = clip(exp(-beta d), .05, 1) (fog.py:173-175) and
//                       the partial sums of the filtered airlight map's mean
//   fog_tbil_kernel     bilateralFilter(t0, 17, 12, 12) (fog.py:176-178)
//   fog_scatter_kernel  I = J t + A (1 - t), global veil (fog.py:266-270),
//                       the glow's gray plane and its mean / std partials
//   fog_sep_h/v<GLOW>   _glow: GaussianBlur of the bright mask and of the
//                       image, composite (fog.py:182-191)
//   fog_sep_h/v<BAND>   _depth_blur, one launch pair per depth band
//                       (fog.py:194-214)
//   fog_fade_kernel     _local_contrast_fade: YCrCb, 8U bilateral on Y,
//                       addWeighted, back to BGR (fog.py:217-224), then
//                       tint, gamma, sensor noise, rain and the u8 store
//                       (fog.py:284-293)
// The airlight map's filter: A_map[c] = a_c * vgrad(y) * xgrad(x) is a
// smooth rank-1 map whose values differ by < 0.25 anywhere, so the bilateral
// colour weight exp(-d^2 / 288) is >= 0.9998 for every pair and the filter
// is its normalised spatial disk filter to < 1e-5 absolute; that filter of
// vgrad x xgrad (per resolution) comes from the host as `amap_unit` and the
// device scales it by a_c.  tests/test_fog.py pins the bound against the
// literal bilateral restatement.
// ===========================================================================

constexpr int kSepRMax = 31;   // Gaussian kernels up to 63 taps
constexpr int kFadeRMax = 7;   // contrast-fade bilateral up to d = 15
// per-frame filter table offsets (floats; fog_taps_kernel)
constexpr int kTabGlowA = 0, kTabGlowB = 32, kTabBand = 64, kTabCw = 160, kTabSw = 416,
              kTabTbil = 480, kTabStride = 576;

struct FogFull {
  int band_h, q_k, edge_guided, nblk;
  float q_t;
};

__device__ __forceinline__ float u8f(int v) { return (float)v / 255.f; }

// 0.299 R + 0.587 G + 0.114 B in f32, numpy's order (fog.py:124).
__device__ __forceinline__ float band_lum(const uint8_t* p) {
  return __fadd_rn(__fadd_rn(__fmul_rn(0.299f, u8f(p[2])), __fmul_rn(0.587f, u8f(p[1]))),
                   __fmul_rn(0.114f, u8f(p[0])));
}

__device__ double block_sum_f64(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// Image airlight (fog.py:120-130) over all frames' bands at once: the k-th
// smallest band luminance by a 3-pass radix select on the f32 bit patterns
// (non-negative floats order as integers; 11 / 11 / 10 bits), the (k+1)-th
// as the minimum key above it, numpy's f32 lerp, then the per-channel mean
// of the band pixels at or above the threshold (all of them if fewer than
// 100).  Workgroups keep LDS histograms and flush their non-zero bins.
struct AirState {
  uint32_t pref, mask, k, eq, min_gt, pad[3];
  double sum[12];  // gt b/g/r/count, eq b/g/r/count, all b/g/r, 0
};
constexpr int kAirPerBlock = 2048;

__global__ __launch_bounds__(256) void fog_lum_kernel(const uint8_t* __restrict__ in, int W,
                                                      int pitch, size_t fstride, int n,
                                                      uint32_t* __restrict__ keys,
                                                      uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[2048];
  const int b = blockIdx.y;
  for (int i = threadIdx.x; i < 2048; i += 256) h[i] = 0;
  __syncthreads();
  const uint8_t* src = in + (size_t)b * fstride;
  const int i0 = blockIdx.x * kAirPerBlock;
  for (int i = i0 + threadIdx.x; i < min(n, i0 + kAirPerBlock); i += 256) {
    const int y = i / W, x = i - y * W;
    const uint32_t key = __float_as_uint(band_lum(src + (size_t)y * pitch + 3 * x));
    keys[(size_t)b * n + i] = key;
    atomicAdd(&h[key >> 21], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 256)
    if (h[i]) atomicAdd(&hist[(size_t)b * 2048 + i], h[i]);
}

__global__ __launch_bounds__(256) void fog_hist_kernel(const uint32_t* __restrict__ keys, int n,
                                                       int shift, int nb,
                                                       const AirState* __restrict__ st,
                                                       uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[2048];
  const int b = blockIdx.y;
  for (int i = threadIdx.x; i < nb; i += 256) h[i] = 0;
  __syncthreads();
  const uint32_t pref = st[b].pref, msk = st[b].mask;
  const int i0 = blockIdx.x * kAirPerBlock;
  for (int i = i0 + threadIdx.x; i < min(n, i0 + kAirPerBlock); i += 256) {
    const uint32_t key = keys[(size_t)b * n + i];
    if ((key & msk) == pref) atomicAdd(&h[(key >> shift) & (nb - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += 256)
    if (h[i]) atomicAdd(&hist[(size_t)b * 2048 + i], h[i]);
}

// One workgroup per frame: the bin holding the k-th key; clears the
// histogram for the next pass.
__global__ __launch_bounds__(256) void fog_sel_kernel(uint32_t* __restrict__ hist, int shift,
                                                      int nb, int first, int q_k,
                                                      AirState* __restrict__ st) {
  __shared__ uint32_t part[256];
  const int b = blockIdx.x;
  uint32_t* hb = hist + (size_t)b * 2048;
  const int per = nb / 256;
  uint32_t v = 0;
  for (int i = 0; i < per; ++i) v += hb[threadIdx.x * per + i];
  part[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t k = first ? (uint32_t)q_k : st[b].k;
    uint32_t cum = 0;
    int t = 255;
    for (int i = 0; i < 256; ++i) {
      if (cum + part[i] > k) {
        t = i;
        break;
      }
      cum += part[i];
    }
    int bin = t * per + per - 1;
    for (int i = t * per; i < t * per + per; ++i) {
      if (cum + hb[i] > k) {
        bin = i;
        break;
      }
      cum += hb[i];
    }
    const uint32_t pref = first ? 0u : st[b].pref, msk = first ? 0u : st[b].mask;
    st[b].k = k - cum;
    st[b].eq = hb[bin];
    st[b].pref = pref | ((uint32_t)bin << shift);
    st[b].mask = msk | ((uint32_t)(nb - 1) << shift);
    if (first) st[b].min_gt = 0xffffffffu;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += 256) hb[i] = 0;
}

__global__ __launch_bounds__(256) void fog_airsum_kernel(const uint8_t* __restrict__ in, int W,
                                                         int pitch, size_t fstride, int n,
                                                         const uint32_t* __restrict__ keys,
                                                         AirState* __restrict__ st) {
  __shared__ double red[4];
  __shared__ uint32_t s_min;
  const int b = blockIdx.y;
  const uint32_t lo = st[b].pref;
  if (threadIdx.x == 0) s_min = 0xffffffffu;
  double a[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t mgt = 0xffffffffu;
  const uint8_t* src = in + (size_t)b * fstride;
  const int i0 = blockIdx.x * kAirPerBlock;
  for (int i = i0 + threadIdx.x; i < min(n, i0 + kAirPerBlock); i += 256) {
    const int y = i / W, x = i - y * W;
    const uint8_t* p = src + (size_t)y * pitch + 3 * x;
    const float vb = u8f(p[0]), vg = u8f(p[1]), vr = u8f(p[2]);
    const uint32_t key = keys[(size_t)b * n + i];
    const int o = key > lo ? 0 : (key == lo ? 4 : -1);
    if (o >= 0) {
      a[o] += vb;
      a[o + 1] += vg;
      a[o + 2] += vr;
      a[o + 3] += 1.0;
    }
    if (key > lo) mgt = min(mgt, key);
    a[8] += vb;
    a[9] += vg;
    a[10] += vr;
  }
  __syncthreads();
  atomicMin(&s_min, mgt);
  for (int k = 0; k < 11; ++k) {
    const double v = block_sum_f64(a[k], red);
    if (threadIdx.x == 0 && v != 0.0) atomicAdd(&st[b].sum[k], v);
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicMin(&st[b].min_gt, s_min);
}

__global__ void fog_airfin_kernel(const AirState* __restrict__ st, FogFull f, int n,
                                  const float* __restrict__ fparams, float* __restrict__ air) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= (int)gridDim.x * (int)blockDim.x) return;
  const AirState& s = st[b];
  const bool same = s.k + 1 < s.eq || f.q_k + 1 >= n;
  const float a = __uint_as_float(s.pref), bq = same ? a : __uint_as_float(s.min_gt);
  const float d = __fsub_rn(bq, a);
  const float thr = f.q_t >= 0.5f ? __fsub_rn(bq, __fmul_rn(d, __fsub_rn(1.f, f.q_t)))
                                  : __fadd_rn(a, __fmul_rn(d, f.q_t));
  // mask = lum >= thr: keys above lo, plus those equal to lo when thr == lo
  const bool with_eq = thr <= a;
  double m[4];
  for (int c = 0; c < 4; ++c) m[c] = s.sum[c] + (with_eq ? s.sum[4 + c] : 0.0);
  const bool all = m[3] < 100.0;
  const double nn = all ? (double)n : m[3];
  const float* fp = fparams + (size_t)b * RV_FOG_NPARAM_FULL;
  for (int c = 0; c < 3; ++c) {
    const float mean = (float)((all ? s.sum[8 + c] : m[c]) / nn);
    air[4 * b + c] = fminf(fmaxf(mean + fp[1 + c], 0.7f), 1.f);
  }
  air[4 * b + 3] = thr;
}

// t0 and the airlight-map mean partials.
__global__ __launch_bounds__(256) void fog_t_kernel(
    const float* __restrict__ grids, const float* __restrict__ taps, FogConsts c, FogFull f,
    int H, int W, const float* __restrict__ depth, const float* __restrict__ amap_unit,
    const float* __restrict__ fparams, const float* __restrict__ range,
    const float* __restrict__ air, float* __restrict__ t0, double* __restrict__ apart) {
  __shared__ float sgrid[kGridLds];
  __shared__ double red[4];
  const int b = blockIdx.y;
  const bool grid_lds = c.grid_stride <= kGridLds;
  if (grid_lds)
    for (int i = threadIdx.x; i < c.grid_stride; i += blockDim.x)
      sgrid[i] = grids[(size_t)b * c.grid_stride + i];
  __syncthreads();
  const float* g = grid_lds ? sgrid : grids + (size_t)b * c.grid_stride;
  const float beta0 = fparams[(size_t)b * RV_FOG_NPARAM_FULL];
  const float mn = range[2 * b], mx = range[2 * b + 1];
  const float ab = air[4 * b], ag = air[4 * b + 1], ar = air[4 * b + 2];
  float acc = 0.f;
  double accd = 0.0;
  int cnt = 0;
  float* tb = t0 + (size_t)b * H * W;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < H * W; i += gridDim.x * blockDim.x) {
    const int y = i / W, x = i - y * W;
    const float nz = noise_at(c, g, taps, y, x, H, W);
    const float nn = (nz - mn) / fmaxf(1e-6f, mx - mn);
    const float beta = beta0 * (0.85f + 0.35f * nn);
    tb[i] = fminf(fmaxf(expf(-beta * depth[i]), 0.05f), 1.f);
    const float r = amap_unit[i];
    acc += fminf(fmaxf(ab * r, 0.7f), 1.f) + fminf(fmaxf(ag * r, 0.7f), 1.f) +
           fminf(fmaxf(ar * r, 0.7f), 1.f);
    if (++cnt == 64) {
      accd += acc;
      acc = 0.f;
      cnt = 0;
    }
  }
  accd += acc;
  accd = block_sum_f64(accd, red);
  if (threadIdx.x == 0) apart[(size_t)b * f.nblk + blockIdx.x] = accd;
}

// Per frame: airlight scale a_target / mean(A_map) (fog.py:257) into air[4b+3]
// is kept for the threshold, so the scale goes to scl[b].
__global__ __launch_bounds__(256) void fog_sum_finish(const double* __restrict__ part, int nblk,
                                                      int parts_per, double count,
                                                      const float* __restrict__ fparams,
                                                      int mode, float* __restrict__ outv) {
  __shared__ double red[4];
  const int b = blockIdx.x;
  double s = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
    s += part[((size_t)b * nblk + i) * parts_per];
    if (parts_per > 1) s2 += part[((size_t)b * nblk + i) * parts_per + 1];
  }
  s = block_sum_f64(s, red);
  s2 = block_sum_f64(s2, red);
  if (threadIdx.x == 0) {
    const float mean = (float)(s / count);
    if (mode == 0) {  // airlight scale (f32 division, as numpy's weak scalar)
      const float tgt = fparams[(size_t)b * RV_FOG_NPARAM_FULL + 4];
      outv[b] = tgt / fmaxf(1e-6f, mean);
    } else {  // glow threshold clip(mean + 0.6 std, .65, .9) (fog.py:184)
      const double var = fmax(0.0, s2 / count - (s / count) * (s / count));
      const float sd = (float)sqrt(var);
      outv[b] = fminf(fmaxf(mean + 0.6f * sd, 0.65f), 0.9f);
    }
  }
}

// bilateralFilter(t0, d = 17, 12, 12), BORDER_REFLECT_101; 64 x 16 outputs
// per workgroup, the tile + radius-8 halo in LDS, two horizontally adjacent
// outputs per lane as packed f32 pairs (v_pk_mul / v_pk_add / v_pk_fma).
// Tap order and the (sum + centre) / (wsum + 1) form follow
// bilateralFilterInvoker_32f.  The colour weight exp(-d^2 / 288), d <= 0.95
// (t in [0.05, 1]), is 1 + x + x^2 / 2 (x = -d^2 / 288 >= -0.0032: the
// dropped x^3 / 6 is < 6e-9, under half an f32 ulp of 1), which OpenCV
// approximates by its 4096-bin interpolated LUT instead.
constexpr int kTbR = 8, kTbW = 64, kTbH = 16;
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void fog_tbil_kernel(const float* __restrict__ t0, int H, int W,
                                                       const float* __restrict__ tab,
                                                       float* __restrict__ tf) {
  __shared__ float tile[kTbH + 2 * kTbR][kTbW + 2 * kTbR];
  __shared__ float sw[kTbR * kTbR + 1];
  const int b = blockIdx.z;
  const int x0 = blockIdx.x * kTbW, y0 = blockIdx.y * kTbH;
  const float* src = t0 + (size_t)b * H * W;
  for (int i = threadIdx.x; i < (kTbH + 2 * kTbR) * (kTbW + 2 * kTbR); i += blockDim.x) {
    const int ty = i / (kTbW + 2 * kTbR), tx = i - ty * (kTbW + 2 * kTbR);
    const int yy = reflect101(y0 + ty - kTbR, H), xx = reflect101(x0 + tx - kTbR, W);
    tile[ty][tx] = src[(size_t)yy * W + xx];
  }
  if (threadIdx.x <= kTbR * kTbR) sw[threadIdx.x] = tab[kTabTbil + threadIdx.x];
  __syncthreads();
  const f32x2 cc = (f32x2)(-1.f / 288.f), half = (f32x2)(0.5f), one = (f32x2)(1.f);
  const int tx = 2 * (threadIdx.x & 31);
  for (int r = threadIdx.x >> 5; r < kTbH; r += 8) {
    const int y = y0 + r, x = x0 + tx;
    if (y >= H || x >= W) continue;
    const f32x2 c0 = {tile[r + kTbR][tx + kTbR], tile[r + kTbR][tx + kTbR + 1]};
    f32x2 s = (f32x2)(0.f), ws = (f32x2)(0.f);
#pragma unroll
    for (int i = -kTbR; i <= kTbR; ++i)
#pragma unroll
      for (int j = -kTbR; j <= kTbR; ++j) {
        const int r2 = i * i + j * j;
        if (r2 > kTbR * kTbR || r2 == 0) continue;
        const f32x2 v = {tile[r + kTbR + i][tx + kTbR + j], tile[r + kTbR + i][tx + kTbR + j + 1]};
        const f32x2 dd = v - c0;
        const f32x2 xx = dd * dd * cc;
        const f32x2 wc = __builtin_elementwise_fma(__builtin_elementwise_fma(half, xx, one), xx, one);
        const f32x2 w = (f32x2)(sw[r2]) * wc;
        ws = ws + w;
        s = s + v * w;
      }
    const f32x2 res = (s + c0) / (ws + one);
    float* d = tf + (size_t)b * H * W + (size_t)y * W + x;
    d[0] = fminf(fmaxf(res.x, 0.05f), 1.f);
    if (x + 1 < W) d[1] = fminf(fmaxf(res.y, 0.05f), 1.f);
  }
}

// Scattering + veil -> H1 (b, g, r, gray u8 of the truncated result), with
// the gray plane's sum / sum of squares partials for the glow threshold.
__global__ __launch_bounds__(256) void fog_scatter_kernel(
    const uint8_t* __restrict__ in, int H, int W, int pitch, size_t fstride,
    const float* __restrict__ scene, const float* __restrict__ amap_unit,
    const float* __restrict__ tf, const float* __restrict__ air, const float* __restrict__ ascale,
    FogFull f, float4* __restrict__ h1, double* __restrict__ gpart) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  const float ab = air[4 * b], ag = air[4 * b + 1], ar = air[4 * b + 2], sc = ascale[b];
  const float* row_gv = scene + 2 * H;
  const uint8_t* src = in + (size_t)b * fstride;
  const float* tb = tf + (size_t)b * H * W;
  float4* ob = h1 + (size_t)b * H * W;
  double g1 = 0.0, g2 = 0.0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < H * W; i += gridDim.x * blockDim.x) {
    const int y = i / W, x = i - y * W;
    const uint8_t* p = src + (size_t)y * pitch + 3 * x;
    const float r = amap_unit[i], t = tb[i], gv = row_gv[y];
    const float A[3] = {fminf(fmaxf(fminf(fmaxf(ab * r, 0.7f), 1.f) * sc, 0.75f), 1.f),
                        fminf(fmaxf(fminf(fmaxf(ag * r, 0.7f), 1.f) * sc, 0.75f), 1.f),
                        fminf(fmaxf(fminf(fmaxf(ar * r, 0.7f), 1.f) * sc, 0.75f), 1.f)};
    float h[3];
    int q[3];
    for (int ch = 0; ch < 3; ++ch) {
      const float v = u8f(p[ch]) * t + A[ch] * (1.f - t);
      h[ch] = fminf(fmaxf(v * (1.f - gv) + A[ch] * gv, 0.f), 1.f);
      q[ch] = (int)(h[ch] * 255.f);
    }
    const int gy = bgr_to_y(q[0], q[1], q[2]);
    ob[i] = make_float4(h[0], h[1], h[2], (float)gy);
    const float gf = u8f(gy);
    g1 += gf;
    g2 += (double)gf * gf;
  }
  g1 = block_sum_f64(g1, red);
  g2 = block_sum_f64(g2, red);
  if (threadIdx.x == 0) {
    gpart[((size_t)b * f.nblk + blockIdx.x) * 2] = g1;
    gpart[((size_t)b * f.nblk + blockIdx.x) * 2 + 1] = g2;
  }
}

// Per-frame filter tables (one workgroup per frame, computed once):
//   getGaussianKernel(k, sigma, CV_32F) half kernels (centre + right half;
//   double exp / sum, cast to f32) for the glow image (k2, 0.25 k2), the glow
//   mask (k, 0.35 k) and the three depth bands (rad, 0.5 rad); the contrast
//   fade's 8U bilateral colour weights (256) and space weights (by r^2); the
//   transmission bilateral's space weights (by r^2, sigma 12).
__device__ void gauss_table(int k, double sigma, float* out) {
  __shared__ double tmp[2 * kSepRMax + 1];
  __shared__ double inv;
  const int r = k / 2;
  __syncthreads();
  if ((int)threadIdx.x < k) {
    const double x = (double)threadIdx.x - (k - 1) * 0.5;
    tmp[threadIdx.x] = exp((-0.5 / (sigma * sigma)) * x * x);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sum = 0.0;
    for (int i = 0; i < k; ++i) sum += tmp[i];
    inv = 1.0 / sum;
  }
  __syncthreads();
  if ((int)threadIdx.x <= kSepRMax)
    out[threadIdx.x] = (int)threadIdx.x <= r ? (float)(tmp[r + threadIdx.x] * inv) : 0.f;
}

__global__ __launch_bounds__(256) void fog_taps_kernel(const float* __restrict__ fparams,
                                                       float* __restrict__ tab) {
  const int b = blockIdx.x;
  const float* fp = fparams + (size_t)b * RV_FOG_NPARAM_FULL;
  float* t = tab + (size_t)b * kTabStride;
  const int k2 = min((int)fp[17], 2 * kSepRMax + 1), k = min((int)fp[16], 2 * kSepRMax + 1);
  gauss_table(k2, k2 * 0.25, t + kTabGlowA);
  gauss_table(k, k * 0.35, t + kTabGlowB);
  for (int i = 0; i < 3; ++i) {
    const int rad = min(max((int)fp[13 + i], 1), 2 * kSepRMax + 1);
    gauss_table(rad, rad * 0.5, t + kTabBand + 32 * i);
  }
  const double sig = 25.0 + (double)fp[11] * 50.0;
  const double coef = -0.5 / (sig * sig);
  t[kTabCw + threadIdx.x] = (float)exp((double)threadIdx.x * threadIdx.x * coef);
  if (threadIdx.x <= kFadeRMax * kFadeRMax)
    t[kTabSw + threadIdx.x] = (float)exp((double)threadIdx.x * coef);
  if (threadIdx.x <= 64)
    t[kTabTbil + threadIdx.x] = (float)exp((double)threadIdx.x * (-0.5 / (12.0 * 12.0)));
}

enum { kSepGlow = 0, kSepBand = 1 };

// Kernel sizes of a pass: A for the colour channels, B for the mask channel.
__device__ __forceinline__ void sep_sizes(int mode, int band, const float* fp, int& ka, double& sa,
                                          int& kb, double& sb) {
  if (mode == kSepGlow) {
    kb = (int)fp[16];  // bright mask: k = int(9 + 20 s) | 1, sigma 0.35 k
    sb = kb * 0.35;
    ka = (int)fp[17];  // image: k2, sigma 0.25 k2
    sa = ka * 0.25;
  } else {
    ka = kb = (int)fp[13 + band];  // depth band: rad, sigma 0.5 rad
    sa = sb = ka * 0.5;
  }
  ka = min(ka, 2 * kSepRMax + 1);
  kb = min(kb, 2 * kSepRMax + 1);
}

// Row pass: one workgroup per 256-pixel row segment, float4 row + halo in
// LDS.  GLOW: xyz = H1 colour, w = gray/255 > thr; BAND: xyz = H2 colour,
// w = (band map == band).  s = k_c S_0 + sum_i k_{c+i} (S_-i + S_i).
template <int MODE>
__global__ __launch_bounds__(256) void fog_sep_h(const float4* __restrict__ src, int H, int W,
                                                 const float* __restrict__ fparams,
                                                 const float* __restrict__ tab,
                                                 const float* __restrict__ thr,
                                                 const uint8_t* __restrict__ bands, int band,
                                                 float4* __restrict__ dst) {
  __shared__ float4 row[256 + 2 * kSepRMax];
  __shared__ float kA[kSepRMax + 1], kB[kSepRMax + 1];
  const int b = blockIdx.z, y = blockIdx.y, x0 = blockIdx.x * 256;
  const float* fp = fparams + (size_t)b * RV_FOG_NPARAM_FULL;
  int ka, kb;
  double sa, sb;
  sep_sizes(MODE, band, fp, ka, sa, kb, sb);
  if (MODE == kSepBand && ka <= 1) return;
  {
    const float* tb = tab + (size_t)b * kTabStride;
    const int oa = MODE == kSepGlow ? kTabGlowA : kTabBand + 32 * band;
    const int ob = MODE == kSepGlow ? kTabGlowB : kTabBand + 32 * band;
    if (threadIdx.x <= kSepRMax) {
      kA[threadIdx.x] = tb[oa + threadIdx.x];
      kB[threadIdx.x] = tb[ob + threadIdx.x];
    }
  }
  const int ra = ka / 2, rb = kb / 2, R = max(ra, rb);
  const float4* s = src + (size_t)b * H * W + (size_t)y * W;
  const float th = MODE == kSepGlow ? thr[b] : 0.f;
  for (int i = threadIdx.x; i < 256 + 2 * R; i += blockDim.x) {
    const int xx = reflect101(x0 + i - R, W);
    float4 v = s[xx];
    if (MODE == kSepGlow)
      v.w = u8f((int)v.w) > th ? 1.f : 0.f;
    else
      v.w = bands[(size_t)y * W + xx] == band ? 1.f : 0.f;
    row[i] = v;
  }
  __syncthreads();
  const int x = x0 + threadIdx.x;
  if (x >= W) return;
  const int c = threadIdx.x + R;
  float4 o;
  o.x = kA[0] * row[c].x;
  o.y = kA[0] * row[c].y;
  o.z = kA[0] * row[c].z;
  for (int i = 1; i <= ra; ++i) {
    o.x = o.x + kA[i] * (row[c - i].x + row[c + i].x);
    o.y = o.y + kA[i] * (row[c - i].y + row[c + i].y);
    o.z = o.z + kA[i] * (row[c - i].z + row[c + i].z);
  }
  o.w = kB[0] * row[c].w;
  for (int i = 1; i <= rb; ++i) o.w = o.w + kB[i] * (row[c - i].w + row[c + i].w);
  dst[(size_t)b * H * W + (size_t)y * W + x] = o;
}

// Column pass + composite.  32 columns x 32 rows per workgroup, the column
// strip + halo in LDS.  GLOW: soft = clip(blur(mask)), H2 = H1 (in-place
// copy too) = clip(h (1 - soft) + (h + s blur) soft); BAND: H1 = H1 (1 - m)
// + blur m.
constexpr int kVCols = 32, kVRows = 32;
template <int MODE>
__global__ __launch_bounds__(256) void fog_sep_v(const float4* __restrict__ tmp, int H, int W,
                                                 const float* __restrict__ fparams,
                                                 const float* __restrict__ tab, int band,
                                                 float4* __restrict__ h1, float4* __restrict__ h2) {
  extern __shared__ float4 col[];  // [(kVRows + 2 R) * kVCols]
  __shared__ float kA[kSepRMax + 1], kB[kSepRMax + 1];
  const int b = blockIdx.z, x0 = blockIdx.x * kVCols, y0 = blockIdx.y * kVRows;
  const float* fp = fparams + (size_t)b * RV_FOG_NPARAM_FULL;
  int ka, kb;
  double sa, sb;
  sep_sizes(MODE, band, fp, ka, sa, kb, sb);
  if (MODE == kSepBand && ka <= 1) return;
  {
    const float* tb = tab + (size_t)b * kTabStride;
    const int oa = MODE == kSepGlow ? kTabGlowA : kTabBand + 32 * band;
    const int ob = MODE == kSepGlow ? kTabGlowB : kTabBand + 32 * band;
    if (threadIdx.x <= kSepRMax) {
      kA[threadIdx.x] = tb[oa + threadIdx.x];
      kB[threadIdx.x] = tb[ob + threadIdx.x];
    }
  }
  const int ra = ka / 2, rb = kb / 2, R = max(ra, rb);
  const float4* s = tmp + (size_t)b * H * W;
  for (int i = threadIdx.x; i < (kVRows + 2 * R) * kVCols; i += blockDim.x) {
    const int ty = i / kVCols, tx = i - ty * kVCols;
    const int yy = reflect101(y0 + ty - R, H), xx = min(x0 + tx, W - 1);
    col[i] = s[(size_t)yy * W + xx];
  }
  __syncthreads();
  const int tx = threadIdx.x & (kVCols - 1), x = x0 + tx;
  if (x >= W) return;
  const float strength = fp[10];
  for (int r = threadIdx.x / kVCols; r < kVRows; r += blockDim.x / kVCols) {
    const int y = y0 + r;
    if (y >= H) break;
    const int c = (r + R) * kVCols + tx;
    float bx = kA[0] * col[c].x, by = kA[0] * col[c].y, bz = kA[0] * col[c].z;
    for (int i = 1; i <= ra; ++i) {
      const float4 u = col[c - i * kVCols], d = col[c + i * kVCols];
      bx = bx + kA[i] * (u.x + d.x);
      by = by + kA[i] * (u.y + d.y);
      bz = bz + kA[i] * (u.z + d.z);
    }
    float m = kB[0] * col[c].w;
    for (int i = 1; i <= rb; ++i) m = m + kB[i] * (col[c - i * kVCols].w + col[c + i * kVCols].w);
    const size_t o = (size_t)b * H * W + (size_t)y * W + x;
    const float4 h = h1[o];
    float4 v;
    if (MODE == kSepGlow) {
      const float soft = fminf(fmaxf(m, 0.f), 1.f);
      v.x = fminf(fmaxf(h.x * (1.f - soft) + (h.x + strength * bx) * soft, 0.f), 1.f);
      v.y = fminf(fmaxf(h.y * (1.f - soft) + (h.y + strength * by) * soft, 0.f), 1.f);
      v.z = fminf(fmaxf(h.z * (1.f - soft) + (h.z + strength * bz) * soft, 0.f), 1.f);
      v.w = 0.f;
      h2[o] = v;
    } else {
      v.x = h.x * (1.f - m) + bx * m;
      v.y = h.y * (1.f - m) + by * m;
      v.z = h.z * (1.f - m) + bz * m;
      v.w = 0.f;
    }
    h1[o] = v;
  }
}

// _local_contrast_fade + the sensor stage: 64 x 16 outputs per workgroup,
// the Y plane of the tile + halo in LDS (computed from the clipped,
// truncated u8 of H1, as (img * 255).astype(uint8) then cvtColor).
constexpr int kFW = 64, kFH = 16;
__global__ __launch_bounds__(256) void fog_fade_kernel(
    const float4* __restrict__ h1, int H, int W, const float* __restrict__ fparams,
    const float* __restrict__ noise, const float* __restrict__ tab, FogConsts c,
    uint8_t* __restrict__ out, int pitch, size_t fstride) {
  __shared__ int ytile[(kFH + 2 * kFadeRMax) * (kFW + 2 * kFadeRMax)];
  __shared__ float cw[256];
  __shared__ float sw[kFadeRMax * kFadeRMax + 1];
  const int b = blockIdx.z, x0 = blockIdx.x * kFW, y0 = blockIdx.y * kFH;
  const float* fp = fparams + (size_t)b * RV_FOG_NPARAM_FULL;
  const float amount = fp[11];
  const int rad = min(max((int)fp[18] / 2, 1), kFadeRMax);
  const float* tb = tab + (size_t)b * kTabStride;
  cw[threadIdx.x] = tb[kTabCw + threadIdx.x];
  if ((int)threadIdx.x <= rad * rad) sw[threadIdx.x] = tb[kTabSw + threadIdx.x];
  const int TW = kFW + 2 * rad, TH = kFH + 2 * rad;
  const float4* src = h1 + (size_t)b * H * W;
  for (int i = threadIdx.x; i < TW * TH; i += blockDim.x) {
    const int ty = i / TW, tx = i - ty * TW;
    const float4 v = src[(size_t)reflect101(y0 + ty - rad, H) * W + reflect101(x0 + tx - rad, W)];
    ytile[i] = bgr_to_y((int)(fminf(fmaxf(v.x, 0.f), 1.f) * 255.f),
                        (int)(fminf(fmaxf(v.y, 0.f), 1.f) * 255.f),
                        (int)(fminf(fmaxf(v.z, 0.f), 1.f) * 255.f));
  }
  __syncthreads();
  const float alpha = (float)(1.0 - (double)amount), beta = amount;
  const float tint[3] = {fp[5], fp[6], fp[7]};
  const float gamma = fp[8];
  const bool has_noise = fp[12] != 0.f && noise != nullptr;
  const uint32_t rseed = (uint32_t)fp[9];
  const int tx = threadIdx.x & 63;
  for (int r = threadIdx.x >> 6; r < kFH; r += 4) {
    const int y = y0 + r, x = x0 + tx;
    if (y >= H || x >= W) continue;
    const int ci = (r + rad) * TW + tx + rad;
    const int y_c = ytile[ci];
    float s = 0.f, ws = 0.f;
    for (int i = -rad; i <= rad; ++i)
      for (int j = -rad; j <= rad; ++j) {
        const int r2 = i * i + j * j;
        if (r2 > rad * rad) continue;
        const int v = ytile[ci + i * TW + j];
        const float w = sw[r2] * cw[abs(v - y_c)];
        ws = ws + w;
        s = s + (float)v * w;
      }
    const int ys = __float2int_rn(s / ws);
    const int ymix = sat_u8(__float2int_rn((float)y_c * alpha + (float)ys * beta));
    const float4 v = src[(size_t)y * W + x];
    const int qb = (int)(fminf(fmaxf(v.x, 0.f), 1.f) * 255.f);
    const int qg = (int)(fminf(fmaxf(v.y, 0.f), 1.f) * 255.f);
    const int qr = (int)(fminf(fmaxf(v.z, 0.f), 1.f) * 255.f);
    int Y, Cr, Cb, ob, og, orr;
    bgr_to_ycrcb(qb, qg, qr, Y, Cr, Cb);
    ycrcb_to_bgr(ymix, Cr, Cb, ob, og, orr);
    const int q3[3] = {ob, og, orr};
    bool rain = false;
    if (c.rain_thresh) {
      const uint32_t colv = (uint32_t)(x + (y >> 2));
      const uint32_t seg = (uint32_t)(y / (int)c.rain_len);
      rain = lowbias32(rseed ^ lowbias32(colv * 0x9E3779B1u + lowbias32(seg))) < c.rain_thresh;
    }
    uint8_t* d = out + (size_t)b * fstride + (size_t)y * pitch + 3 * x;
    const float* nz = has_noise ? noise + (((size_t)b * H + y) * W + x) * 3 : nullptr;
    for (int ch = 0; ch < 3; ++ch) {
      float h = fminf(fmaxf(u8f(q3[ch]) * tint[ch], 0.f), 1.f);
      if (gamma != 1.f) h = fminf(fmaxf(powf(h, gamma), 0.f), 1.f);
      if (has_noise) h = fminf(fmaxf(h + nz[ch], 0.f), 1.f);
      if (rain) h = h + (1.f - h) * 0.45f;
      d[ch] = (uint8_t)(int)(h * 255.f + 0.5f);
    }
  }
}

// _airlight_from_image's band rows, max(10, int(0.12 h)) (fog.py:122).
inline int air_band_rows(int H) { return max(10, (int)(0.12 * H)); }

// Workspace layout of rv_fog_full_u8.
struct FullWs {
  float *range, *part, *air, *ascale, *gthr, *tab;
  uint32_t *keys, *hist;
  AirState* st;
  double *apart, *gpart;
  float *t0, *tf;
  float4 *h1, *tmp, *h2;
  size_t bytes;
};
constexpr int kFullNblk = 512;
FullWs full_ws(void* base, int B, int H, int W) {
  FullWs w{};
  size_t off = 0;
  auto take = [&](size_t n) {
    off = (off + 255) & ~(size_t)255;
    char* p = (char*)base + off;
    off += n;
    return (void*)p;
  };
  const size_t px = (size_t)B * H * W;
  w.range = (float*)take((size_t)B * 2 * sizeof(float));
  w.part = (float*)take((size_t)B * 2 * kRangeBlocks * sizeof(float));
  w.air = (float*)take((size_t)B * 4 * sizeof(float));
  w.ascale = (float*)take((size_t)B * sizeof(float));
  w.gthr = (float*)take((size_t)B * sizeof(float));
  w.tab = (float*)take((size_t)B * kTabStride * sizeof(float));
  w.hist = (uint32_t*)take((size_t)B * 2048 * sizeof(uint32_t));
  w.st = (AirState*)take((size_t)B * sizeof(AirState));
  w.keys = (uint32_t*)take((size_t)B * air_band_rows(H) * W * sizeof(uint32_t));
  w.apart = (double*)take((size_t)B * kFullNblk * sizeof(double));
  w.gpart = (double*)take((size_t)B * kFullNblk * 2 * sizeof(double));
  w.t0 = (float*)take(px * sizeof(float));
  w.tf = (float*)take(px * sizeof(float));
  w.h1 = (float4*)take(px * sizeof(float4));
  w.tmp = (float4*)take(px * sizeof(float4));
  w.h2 = (float4*)take(px * sizeof(float4));
  w.bytes = off;
  return w;
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


extern "C" size_t rv_fog_full_ws_bytes(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  return full_ws(nullptr, B, H, W).bytes;
}

extern "C" int rv_fog_full_u8(const uint8_t* in, uint8_t* out, int B, int H, int W, int pitch,
                              const float* consts, int n_consts, const float* full,
                              int n_full, const float* scene, const float* depth,
                              const float* amap_unit, const uint8_t* bands,
                              const float* frame_params, const float* grids, int grid_stride,
                              const float* noise, void* ws, size_t ws_bytes, void* stream) {
  RV_CHECK_ARG(in != nullptr && out != nullptr && consts != nullptr && full != nullptr &&
                   scene != nullptr && depth != nullptr && amap_unit != nullptr &&
                   bands != nullptr && frame_params != nullptr && grids != nullptr &&
                   ws != nullptr,
               "null pointer");
  RV_CHECK_ARG(B >= 0 && H >= 2 * kSepRMax + 2 && W >= 2 * kSepRMax + 2 && pitch >= 3 * W,
               "bad frame shape (H, W >= %d)", 2 * kSepRMax + 2);
  RV_CHECK_ARG((const void*)in != (const void*)out, "in and out must not alias");
  RV_CHECK_ARG(n_consts == RV_FOG_NCONST, "n_consts %d != %d", n_consts, RV_FOG_NCONST);
  RV_CHECK_ARG(n_full == RV_FOG_NFULL, "n_full %d != %d", n_full, RV_FOG_NFULL);
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
  c.rain_thresh = (uint32_t)fmin((double)c.rain_p * 4294967296.0, 4294967295.0);
  FogFull f{};
  f.band_h = (int)full[0];
  f.q_k = (int)full[1];
  f.q_t = full[2];
  f.edge_guided = full[3] != 0.f;
  f.nblk = min(kFullNblk, ceil_div(H * W, 256));
  RV_CHECK_ARG(f.band_h >= 1 && f.band_h <= H && f.band_h <= air_band_rows(H) && f.q_k >= 0 && f.q_k < f.band_h * W &&
                   f.q_t >= 0.f && f.q_t < 1.f,
               "bad airlight band constants");
  if (B == 0) return RV_OK;
  RV_CHECK_ARG(ws_bytes >= rv_fog_full_ws_bytes(B, H, W), "workspace %zu < %zu bytes", ws_bytes,
               rv_fog_full_ws_bytes(B, H, W));
  hipStream_t s = as_stream(stream);
  FullWs w = full_ws(ws, B, H, W);
  const size_t fstride = (size_t)H * pitch;
  const float* taps = scene + 4 * H + W;
  const int rblocks = min(kRangeBlocks, ceil_div(H * W, 256));
  fog_range_kernel<<<dim3(rblocks, B), 256, 0, s>>>(grids, taps, c, H, W, w.part);
  fog_range_finish<<<B, 256, 0, s>>>(w.part, rblocks, w.range);
  fog_taps_kernel<<<B, 256, 0, s>>>(frame_params, w.tab);
  {  // image airlight: band quantile + masked mean (fog.py:120-130)
    const int n = f.band_h * W;
    const dim3 ga(ceil_div(n, kAirPerBlock), B);
    int rc = hip_check(hipMemsetAsync(w.hist, 0, (size_t)B * 2048 * sizeof(uint32_t), s),
                       "hipMemsetAsync(hist)");
    if (rc == RV_OK)
      rc = hip_check(hipMemsetAsync(w.st, 0, (size_t)B * sizeof(AirState), s),
                     "hipMemsetAsync(air state)");
    if (rc != RV_OK) return rc;
    fog_lum_kernel<<<ga, 256, 0, s>>>(in, W, pitch, fstride, n, w.keys, w.hist);
    fog_sel_kernel<<<B, 256, 0, s>>>(w.hist, 21, 2048, 1, f.q_k, w.st);
    fog_hist_kernel<<<ga, 256, 0, s>>>(w.keys, n, 10, 2048, w.st, w.hist);
    fog_sel_kernel<<<B, 256, 0, s>>>(w.hist, 10, 2048, 0, f.q_k, w.st);
    fog_hist_kernel<<<ga, 256, 0, s>>>(w.keys, n, 0, 1024, w.st, w.hist);
    fog_sel_kernel<<<B, 256, 0, s>>>(w.hist, 0, 1024, 0, f.q_k, w.st);
    fog_airsum_kernel<<<ga, 256, 0, s>>>(in, W, pitch, fstride, n, w.keys, w.st);
    fog_airfin_kernel<<<B, 1, 0, s>>>(w.st, f, n, frame_params, w.air);
  }
  fog_t_kernel<<<dim3(f.nblk, B), 256, 0, s>>>(grids, taps, c, f, H, W, depth, amap_unit,
                                               frame_params, w.range, w.air, w.t0, w.apart);
  fog_sum_finish<<<B, 256, 0, s>>>(w.apart, f.nblk, 1, 3.0 * H * W, frame_params, 0, w.ascale);
  const float* tf = w.t0;
  if (f.edge_guided) {
    fog_tbil_kernel<<<dim3(ceil_div(W, kTbW), ceil_div(H, kTbH), B), 256, 0, s>>>(w.t0, H, W,
                                                                                w.tab, w.tf);
    tf = w.tf;
  }
  fog_scatter_kernel<<<dim3(f.nblk, B), 256, 0, s>>>(in, H, W, pitch, fstride, scene, amap_unit,
                                                     tf, w.air, w.ascale, f, w.h1, w.gpart);
  fog_sum_finish<<<B, 256, 0, s>>>(w.gpart, f.nblk, 2, (double)H * W, frame_params, 1, w.gthr);
  const dim3 gh(ceil_div(W, 256), H, B), gv(ceil_div(W, kVCols), ceil_div(H, kVRows), B);
  const size_t vlds = (size_t)(kVRows + 2 * kSepRMax) * kVCols * sizeof(float4);
  fog_sep_h<kSepGlow><<<gh, 256, 0, s>>>(w.h1, H, W, frame_params, w.tab, w.gthr, bands, 0,
                                         w.tmp);
  fog_sep_v<kSepGlow><<<gv, 256, vlds, s>>>(w.tmp, H, W, frame_params, w.tab, 0, w.h1, w.h2);
  for (int band = 0; band < 3; ++band) {
    fog_sep_h<kSepBand><<<gh, 256, 0, s>>>(w.h2, H, W, frame_params, w.tab, w.gthr, bands, band,
                                           w.tmp);
    fog_sep_v<kSepBand><<<gv, 256, vlds, s>>>(w.tmp, H, W, frame_params, w.tab, band, w.h1,
                                              w.h2);
  }
  fog_fade_kernel<<<dim3(ceil_div(W, kFW), ceil_div(H, kFH), B), 256, 0, s>>>(
      w.h1, H, W, frame_params, noise, w.tab, c, out, pitch, fstride);
  return launch_status("rv_fog_full_u8");
}

}  // namespace rv
