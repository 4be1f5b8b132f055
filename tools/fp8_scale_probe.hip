// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 operands (gfx950):
//  1. the A/B lane -> k map (candidate maps tried on exact small integers);
//  2. accumulation precision on random codes over the whole e4m3 range, as
//     fp8_probe.hip measures for v_mfma_f32_16x16x32_fp8_fp8.
// Build: hipcc --offload-arch=gfx950 -O2 tools/fp8_scale_probe.hip -o tools/fp8_scale_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;

__global__ void mfma_scale_kernel(const uint8_t* Al, const uint8_t* Bl, float* D, int nk) {
  // Al / Bl: per k-step, per lane 32 bytes (already in register order)
  const int l = threadIdx.x, col = l & 15, q = l >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < nk; ++k) {
    i32x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = *(const int*)(Al + ((size_t)k * 64 + l) * 32 + 4 * j);
      b[j] = *(const int*)(Bl + ((size_t)k * 64 + l) * 32 + 4 * j);
    }
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, 127, 0, 127);
  }
  for (int i = 0; i < 4; ++i) D[(q * 4 + i) * 16 + col] = acc[i];
}

static double e4m3_value(int code) {
  const int s = code >> 7, e = (code >> 3) & 15, m = code & 7;
  double v = e == 0 ? ldexp(m, -9) : ldexp(1.0 + m / 8.0, e - 7);
  return s ? -v : v;
}
static int host_e4m3(double a) {  // exact small values only
  int best = 0;
  double bd = 1e30;
  for (int c = 0; c < 255; ++c) {
    if ((c & 127) == 127) continue;
    const double d = fabs(e4m3_value(c) - a);
    if (d < bd) { bd = d; best = c; }
  }
  return best;
}

// candidate maps: k index of byte j (0..31) of lane-group q (= lane >> 4)
static int kmap(int hyp, int q, int j) {
  switch (hyp) {
    case 0: return 32 * q + j;                                   // contiguous 32
    case 1: return (j < 16) ? 16 * q + j : 64 + 16 * q + (j - 16);  // two 64-halves
    case 2: return 8 * q + (j & 7) + 32 * (j >> 3);              // 8-byte groups strided
    case 3: return (j < 8) ? 8 * q + j : 32 + 32 * ((j - 8) / 8) + 8 * q + (j & 7) - 0;
    default: return -1;
  }
}

static void pack_lanes(int hyp, const std::vector<uint8_t>& A, const std::vector<uint8_t>& B,
                       int K, std::vector<uint8_t>& Al, std::vector<uint8_t>& Bl) {
  const int nk = K / 128;
  Al.assign((size_t)nk * 64 * 32, 0);
  Bl.assign((size_t)nk * 64 * 32, 0);
  for (int s = 0; s < nk; ++s)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int k = 128 * s + kmap(hyp, l >> 4, j);
        Al[((size_t)s * 64 + l) * 32 + j] = A[(size_t)(l & 15) * K + k];
        Bl[((size_t)s * 64 + l) * 32 + j] = B[(size_t)k * 16 + (l & 15)];
      }
}

static std::vector<float> run(const std::vector<uint8_t>& Al, const std::vector<uint8_t>& Bl,
                              int nk) {
  uint8_t *da, *db;
  float* dd;
  (void)hipMalloc(&da, Al.size());
  (void)hipMalloc(&db, Bl.size());
  (void)hipMalloc(&dd, 1024);
  (void)hipMemcpy(da, Al.data(), Al.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(db, Bl.data(), Bl.size(), hipMemcpyHostToDevice);
  mfma_scale_kernel<<<1, 64>>>(da, db, dd, nk);
  std::vector<float> o(256);
  (void)hipMemcpy(o.data(), dd, 1024, hipMemcpyDeviceToHost);
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dd);
  return o;
}

int main() {
  srand(3);
  // 1. layout: exact small integers (each k distinct enough)
  const int K = 128;
  std::vector<int> Ai(16 * K), Bi(K * 16);
  for (auto& x : Ai) x = rand() % 9 - 4;
  for (auto& x : Bi) x = rand() % 9 - 4;
  std::vector<uint8_t> A(16 * K), B(K * 16);
  for (size_t i = 0; i < A.size(); ++i) A[i] = (uint8_t)host_e4m3(Ai[i]);
  for (size_t i = 0; i < B.size(); ++i) B[i] = (uint8_t)host_e4m3(Bi[i]);
  int good = -1;
  for (int hyp = 0; hyp < 4; ++hyp) {
    std::vector<uint8_t> Al, Bl;
    pack_lanes(hyp, A, B, K, Al, Bl);
    auto o = run(Al, Bl, 1);
    int bad = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        int s = 0;
        for (int k = 0; k < K; ++k) s += Ai[i * K + k] * Bi[k * 16 + j];
        if (o[i * 16 + j] != (float)s) ++bad;
      }
    printf("map %d: %d / 256 mismatches\n", hyp, bad);
    if (!bad && good < 0) good = hyp;
  }
  if (good < 0) return 1;
  // 2. accumulation precision with the working map
  for (int nk : {1, 3, 9}) {
    const int KK = 128 * nk;
    double worst = 0;
    for (int t = 0; t < 200; ++t) {
      std::vector<uint8_t> a8(16 * KK), b8(KK * 16);
      for (auto& x : a8) { do x = (uint8_t)(rand() & 255); while ((x & 127) == 127); }
      for (auto& x : b8) { do x = (uint8_t)(rand() & 255); while ((x & 127) == 127); }
      std::vector<uint8_t> Al, Bl;
      pack_lanes(good, a8, b8, KK, Al, Bl);
      auto o = run(Al, Bl, nk);
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          double ex = 0, sa = 0;
          for (int k = 0; k < KK; ++k) {
            const double p = e4m3_value(a8[i * KK + k]) * e4m3_value(b8[k * 16 + j]);
            ex += p;
            sa += fabs(p);
          }
          worst = std::max(worst, fabs(o[i * 16 + j] - ex) / sa);
        }
    }
    printf("scaled fp8 MFMA accumulation, K = %d: max |err| / sum|p| = %.3g (2^%.1f)\n", KK, worst,
           log2(worst));
  }
  return 0;
}
