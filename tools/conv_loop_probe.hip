// Ceiling of conv_patch_kernel's inner loop on gfx950: MR x NR fragments of
// v_mfma_f32_16x16x32_bf16 per wave and tap, A (weights) and B (patch)
// fragments read from LDS with ds_read_b128 exactly as the kernel reads them
// (64-B slots, quarter swizzle), the next tap's reads issued before this
// tap's MFMAs, optionally a workgroup barrier every 9 taps (a chunk step).
// No DMA, no epilogue.  Reports TFLOP/s and the fraction of the bf16 peak.
//   hipcc --offload-arch=gfx950 -O3 -o conv_loop_probe tools/conv_loop_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ int swz(int i) { return (i >> 1) & 2; }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff, 0, 0, 0);
}

// NDMA > 0: each chunk step also LDS-DMAs NDMA 1-KB pieces per wave (the
// next step's patch) from a streamed global buffer into the other stage,
// then s_waitcnt vmcnt(0) + barrier (the kernel's step structure)
template <int MR, int NR, int NW, bool BAR, int NDMA = 0, int AHEAD = 1, bool SPREAD = false>
__global__ __launch_bounds__(64 * NW, 1) void probe(float* out, int iters, int PW, const uint8_t* src,
                                                    uint32_t src_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int BC = 16 * MR, T2 = 9;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 15, quad = lane >> 4;
  uint8_t* Wl = smem;                          // weights [BC][9][64 B]
  uint8_t* P = smem + BC * T2 * 64;           // patch (stage 0; stage 1 follows)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, src_bytes, 0x00020000);
  for (int i = tid; i < (BC * T2 * 64 + 12 * PW * 64) / 16; i += 64 * NW)
    ((uint4*)smem)[i] = make_uint4(0x3c003c00u ^ i, 0x3c003c00u, 0x3c003c00u, 0x3c003c00u);
  __syncthreads();
  int boff[NR][3];
  for (int n = 0; n < NR; ++n) {
    const int q = wave * NR * 16 + n * 16 + col;
    const int r = q / 32, c = q % 32;
    for (int kx = 0; kx < 3; ++kx) {
      const int sc = c + kx;
      boff[n][kx] = (r * PW + sc) * 64 + ((quad ^ swz(sc)) << 4);
    }
  }
  f32x4 acc[MR][NR];
  for (int m = 0; m < MR; ++m)
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
    bf16x8 Af[2][MR], Bq[2][NR];
    uint8_t* P1 = P + 12 * PW * 64;
    auto dma = [&](int i) {
      const uint32_t piece = ((uint32_t)(blockIdx.x * iters + it) * NW * NDMA + wave * NDMA + i) * 1024u;
      dma16(rs, P1 + ((wave * NDMA + i) % 22) * 1024, (piece + lane * 16) % src_bytes);
    };
    if constexpr (NDMA > 0 && !SPREAD) {
#pragma unroll
      for (int i = 0; i < NDMA; ++i) dma(i);
    }
    auto ld = [&](int tap, int sl) {
      const int ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const int row = m * 16 + col;
        Af[sl][m] = __builtin_bit_cast(bf16x8, *(const uint4*)(Wl + (row * T2 + tap) * 64 + ((quad ^ swz(row)) << 4)));
      }
#pragma unroll
      for (int n = 0; n < NR; ++n)
        Bq[sl][n] = __builtin_bit_cast(bf16x8, *(const uint4*)(P + ky * PW * 64 + boff[n][kx]));
    };
    ld(0, 0);
#pragma unroll
    for (int t = 0; t < T2; ++t) {
      if (t + 1 < T2) ld(t + 1, (t + 1) & 1);
      if constexpr (NDMA > 0 && SPREAD) {
        for (int i = t; i < NDMA; i += T2) dma(i);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[t & 1][m], Bq[t & 1][n], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (BAR) {
      if constexpr (NDMA > 0) {
        if constexpr (AHEAD == 1) __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
        else if constexpr (NDMA <= 15) __builtin_amdgcn_s_waitcnt(0x3f70 | (NDMA & 15) | ((NDMA >> 4) << 14));  // vmcnt(NDMA)
      }
      __syncthreads();
    }
  }
  float s = 0.f;
  for (int m = 0; m < MR; ++m)
    for (int n = 0; n < NR; ++n) s += acc[m][n][0] + acc[m][n][3];
  out[blockIdx.x * 64 * NW + tid] = s;
}

static uint8_t* g_src = nullptr;
static const uint32_t kSrcBytes = 256u << 20;

static uint32_t g_src_bytes = 256u << 20;
template <int MR, int NR, int NW, bool BAR, int NDMA = 0, int AHEAD = 1, bool SPREAD = false>
void run(int ncu, int iters) {
  const int PW = 34;
  const size_t sm = 16 * MR * 9 * 64 + 2 * 12 * PW * 64;
  auto fn = probe<MR, NR, NW, BAR, NDMA, AHEAD, SPREAD>;
  hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  float* out;
  hipMalloc(&out, (size_t)ncu * 2 * 64 * NW * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 2; ++w) fn<<<ncu, 64 * NW, sm>>>(out, iters, PW, g_src, g_src_bytes);
  hipEventRecord(a);
  fn<<<ncu, 64 * NW, sm>>>(out, iters, PW, g_src, g_src_bytes);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double flops = 2.0 * 16 * 16 * 32 * MR * NR * 9.0 * iters * NW * ncu;
  printf("MR=%d NR=%d waves=%d barrier=%d dma/wave/step=%d ahead=%d spread=%d src=%uMB: %.3f ms %.1f TFLOP/s = %.3f of 2.5 PF\n", MR, NR, NW, (int)BAR, NDMA, AHEAD, (int)SPREAD, g_src_bytes >> 20, ms,
         flops / ms * 1e-9, flops / ms * 1e-9 / 2500.0);
  hipFree(out);
}

int main(int argc, char** argv) {
  const int ncu = 256, iters = argc > 1 ? atoi(argv[1]) : 2000;
  hipMalloc(&g_src, kSrcBytes);
  hipMemset(g_src, 0, kSrcBytes);
  // the loop alone: no DMA (barrier every chunk step, or none)
  g_src_bytes = 2u << 20;
  run<4, 2, 4, false>(ncu, iters);
  run<4, 2, 4, true>(ncu, iters);
  run<5, 2, 8, true>(ncu, iters);
  run<2, 2, 8, true>(ncu, iters);
  run<2, 1, 4, true>(ncu, iters);
  for (int pass = 0; pass < 2; ++pass) {
    g_src_bytes = pass == 0 ? (256u << 20) : (2u << 20);
    run<5, 2, 8, true, 3>(ncu, iters);
    run<5, 2, 8, true, 3, 2>(ncu, iters);
    run<5, 2, 8, true, 3, 1, true>(ncu, iters);
    run<5, 2, 8, true, 3, 2, true>(ncu, iters);
    run<2, 2, 8, true, 3>(ncu, iters);
    run<2, 2, 8, true, 3, 2, true>(ncu, iters);
    run<5, 2, 8, true, 9>(ncu, iters);
    run<5, 2, 8, true, 9, 2, true>(ncu, iters);
  }
  return 0;
}
