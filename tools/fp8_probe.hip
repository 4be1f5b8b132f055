// Probe of the gfx950 fp8 (OCP e4m3fn) primitives the fp8 conv path uses:
//  1. v_cvt_pk_fp8_f32 (f32 -> e4m3, as __builtin_amdgcn_cvt_pk_fp8_f32)
//     against a host round-to-nearest-even reference, on values clamped to
//     +-448 (normals, subnormals, ties, zero);
//  2. v_cvt_f32_fp8 (decode) for all 256 codes (NaN codes skipped);
//  3. v_mfma_f32_16x16x32_fp8_fp8 lane layout with exact small integers:
//     lane l holds A[l & 15][8 (l >> 4) + j] and B[8 (l >> 4) + j][l & 15]
//     (j = byte 0..7 of its 64-bit operand), C/D as bf16 16x16x32;
//  4. its accumulation precision on random codes over the whole e4m3 range:
//     max |D - exact| relative to sum |products| (and to |exact|).
// Build: hipcc --offload-arch=gfx950 -O2 tools/fp8_probe.hip -o tools/fp8_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void cvt_kernel(const float* in, uint8_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = fminf(fmaxf(in[i], -448.f), 448.f);
  const int p = __builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false);
  out[i] = (uint8_t)(p & 255);
}

__global__ void dec_kernel(float* out) {
  const int i = threadIdx.x;
  out[i] = __builtin_amdgcn_cvt_f32_fp8(i, 0);
}

__global__ void mfma_raw_kernel(const uint8_t* A, const uint8_t* B, float* D, int nk) {
  // D = A (16 x 32 nk) * B (32 nk x 16), codes, nk chained MFMAs
  const int l = threadIdx.x, col = l & 15, q = l >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < nk; ++k) {
    uint64_t a = 0, b = 0;
    for (int j = 0; j < 8; ++j) {
      a |= (uint64_t)A[col * 32 * nk + 32 * k + 8 * q + j] << (8 * j);
      b |= (uint64_t)B[(32 * k + 8 * q + j) * 16 + col] << (8 * j);
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8((long)a, (long)b, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) D[(q * 4 + i) * 16 + col] = acc[i];
}

__global__ void mfma_kernel(const int8_t* A, const int8_t* B, float* D, const uint8_t* code) {
  // A 16x32, B 32x16 small integers encoded as e4m3 codes via `code`
  const int l = threadIdx.x, col = l & 15, q = l >> 4;
  uint64_t a = 0, b = 0;
  for (int j = 0; j < 8; ++j) {
    a |= (uint64_t)code[A[col * 32 + 8 * q + j] + 8] << (8 * j);
    b |= (uint64_t)code[B[(8 * q + j) * 16 + col] + 8] << (8 * j);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8((long)a, (long)b, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[(q * 4 + i) * 16 + col] = acc[i];
}

// host e4m3fn: RNE, |v| <= 448 (no overflow), subnormals 2^-9 steps
static double e4m3_value(int code) {
  const int s = code >> 7, e = (code >> 3) & 15, m = code & 7;
  double v = e == 0 ? ldexp(m, -9) : ldexp(1.0 + m / 8.0, e - 7);
  return s ? -v : v;
}
static int host_e4m3(float f) {
  const int s = f < 0 || (f == 0 && signbit(f));
  double a = fabs((double)f);
  int best = 0;
  double bd = 1e30;
  for (int c = 0; c < 127; ++c) {  // 0x7f = NaN
    const double d = fabs(e4m3_value(c) - a);
    if (d < bd || (d == bd && (c & 1) == 0)) {
      bd = d;
      best = c;
    }
  }
  return (s << 7) | best;
}

int main() {
  // 1. conversion
  std::vector<float> v;
  for (int c = 0; c < 127; ++c) {  // every code, midpoints, and nudges
    const double x = e4m3_value(c), y = e4m3_value(c + 1 < 127 ? c + 1 : c);
    v.push_back((float)x);
    v.push_back((float)((x + y) / 2));
    v.push_back(nextafterf((float)((x + y) / 2), 1e9f));
    v.push_back(nextafterf((float)((x + y) / 2), -1e9f));
  }
  srand(1);
  for (int i = 0; i < 20000; ++i) v.push_back((float)(((rand() / (double)RAND_MAX) * 2 - 1) * 500));
  for (int i = 0; i < 20000; ++i) v.push_back((float)(((rand() / (double)RAND_MAX) * 2 - 1) * 0.02));
  const int n0 = (int)v.size();
  for (int i = 0; i < n0; ++i) v.push_back(-v[i]);
  const int n = (int)v.size();
  float* din;
  uint8_t* dout;
  hipMalloc(&din, n * 4);
  hipMalloc(&dout, n);
  hipMemcpy(din, v.data(), n * 4, hipMemcpyHostToDevice);
  cvt_kernel<<<(n + 255) / 256, 256>>>(din, dout, n);
  std::vector<uint8_t> got(n);
  hipMemcpy(got.data(), dout, n, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    const float c = fminf(fmaxf(v[i], -448.f), 448.f);
    const int want = host_e4m3(c);
    if (got[i] != want && !(c == 0 && (got[i] & 127) == 0)) {
      if (bad < 10) printf("cvt mismatch v=%.9g got 0x%02x want 0x%02x\n", c, got[i], want);
      ++bad;
    }
  }
  printf("cvt_pk_fp8_f32: %d / %d mismatches vs host RNE\n", bad, n);
  // 2. decode
  float* ddec;
  hipMalloc(&ddec, 256 * 4);
  dec_kernel<<<1, 256>>>(ddec);
  std::vector<float> dec(256);
  hipMemcpy(dec.data(), ddec, 1024, hipMemcpyDeviceToHost);
  int badd = 0;
  for (int c = 0; c < 256; ++c) {
    if ((c & 127) == 127) continue;
    if (dec[c] != (float)e4m3_value(c)) ++badd;
  }
  printf("cvt_f32_fp8: %d / 254 mismatches\n", badd);
  // 3. MFMA layout
  std::vector<int8_t> A(16 * 32), B(32 * 16);
  for (int i = 0; i < 16 * 32; ++i) A[i] = (int8_t)(rand() % 9 - 4);
  for (int i = 0; i < 32 * 16; ++i) B[i] = (int8_t)(rand() % 9 - 4);
  uint8_t code[17];
  for (int k = -8; k <= 8; ++k) code[k + 8] = (uint8_t)host_e4m3((float)k);
  int8_t *dA, *dB;
  uint8_t* dcode;
  float* dD;
  hipMalloc(&dA, A.size());
  hipMalloc(&dB, B.size());
  hipMalloc(&dcode, 17);
  hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipMemcpy(dcode, code, 17, hipMemcpyHostToDevice);
  mfma_kernel<<<1, 64>>>(dA, dB, dD, dcode);
  std::vector<float> D(256);
  hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
  int badm = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      int s = 0;
      for (int k = 0; k < 32; ++k) s += A[i * 32 + k] * B[k * 16 + j];
      if (D[i * 16 + j] != (float)s) ++badm;
    }
  printf("mfma_f32_16x16x32_fp8_fp8 layout: %d / 256 mismatches\n", badm);
  // 4. accumulation precision
  for (int nk : {1, 9, 36}) {
    double worst_abs = 0, worst_ex = 0;
    for (int trial = 0; trial < 200; ++trial) {
      std::vector<uint8_t> a8(16 * 32 * nk), b8(32 * nk * 16);
      for (auto& x : a8) { do x = (uint8_t)(rand() & 255); while ((x & 127) == 127); }
      for (auto& x : b8) { do x = (uint8_t)(rand() & 255); while ((x & 127) == 127); }
      uint8_t *da, *db;
      float* dd;
      hipMalloc(&da, a8.size());
      hipMalloc(&db, b8.size());
      hipMalloc(&dd, 1024);
      hipMemcpy(da, a8.data(), a8.size(), hipMemcpyHostToDevice);
      hipMemcpy(db, b8.data(), b8.size(), hipMemcpyHostToDevice);
      mfma_raw_kernel<<<1, 64>>>(da, db, dd, nk);
      std::vector<float> o(256);
      hipMemcpy(o.data(), dd, 1024, hipMemcpyDeviceToHost);
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          double ex = 0, sa = 0;
          for (int k = 0; k < 32 * nk; ++k) {
            const double p = e4m3_value(a8[i * 32 * nk + k]) * e4m3_value(b8[k * 16 + j]);
            ex += p;
            sa += fabs(p);
          }
          const double err = fabs(o[i * 16 + j] - ex);
          worst_abs = std::max(worst_abs, err / sa);
          worst_ex = std::max(worst_ex, err / std::max(fabs(ex), 1e-30));
        }
      hipFree(da);
      hipFree(db);
      hipFree(dd);
    }
    printf("fp8 MFMA accumulation, K = %d: max |err| / sum|p| = %.3g (2^%.1f), / |exact| = %.3g\n",
           32 * nk, worst_abs, log2(worst_abs), worst_ex);
  }
  return (bad || badd || badm) ? 1 : 0;
}
