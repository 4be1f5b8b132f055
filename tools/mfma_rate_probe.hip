// Cycles per MFMA on one SIMD (one wave, 4 independent accumulators),
// s_memtime around a back-to-back loop: v_mfma_f32_16x16x32_bf16 against
// v_mfma_f32_16x16x16_bf16 (the K = 16 form a 16-channel tail chunk could
// use instead of a zero-padded K = 32 step).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_rate_probe tools/mfma_rate_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int KIND>
__global__ void probe(float* out, unsigned long long* cyc, int n) {
  f32x4 acc[4] = {};
  bf16x8 a8, b8;
  bf16x4 a4, b4;
  for (int i = 0; i < 8; ++i) {
    a8[i] = (__bf16)(threadIdx.x * 0.001f + i);
    b8[i] = (__bf16)(i * 0.5f);
  }
  for (int i = 0; i < 4; ++i) {
    a4[i] = a8[i];
    b4[i] = b8[i];
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (KIND == 0)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[j], 0, 0, 0);
      else
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[j], 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 64 * sizeof(float));
  hipMalloc(&cyc, sizeof(unsigned long long));
  const int n = 4096;
  for (int k = 0; k < 2; ++k) {
    for (int rep = 0; rep < 3; ++rep) {
      if (k == 0) probe<0><<<1, 64>>>(out, cyc, n);
      else probe<1><<<1, 64>>>(out, cyc, n);
      hipDeviceSynchronize();
    }
    unsigned long long c;
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%s: %.2f cycles per MFMA\n", k == 0 ? "16x16x32_bf16" : "16x16x16_bf16",
           (double)c / (4.0 * n));
  }
  return 0;
}
