// Microbenchmark: filling LDS from global memory, one-shot per workgroup
// (the conv kernel's "stage everything, one barrier" pattern).  Compares
// global_load_lds (LDS-DMA, 16 B/lane) with global_load_dwordx4 + ds_write,
// for data every workgroup shares (weights: L2-resident) and data distinct
// per workgroup (input patches).  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void glds_fill(const uint4* __restrict__ src, int kb, int shared,
                                                 unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int wave = threadIdx.x >> 6;
  const uint4* s = src + (shared ? 0 : (size_t)blockIdx.x * kb * 64);
  for (int j = wave; j < kb; j += 4)
    __builtin_amdgcn_global_load_lds((const void*)(s + (size_t)j * 64 + (threadIdx.x & 63)),
                                     (void*)(smem + j * 1024), 16, 0, 0);
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = smem[(blockIdx.x * 97) % (kb * 1024)];
}

__global__ __launch_bounds__(256) void vload_fill(const uint4* __restrict__ src, int kb, int shared,
                                                  unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint4* s = src + (shared ? 0 : (size_t)blockIdx.x * kb * 64);
  uint4 v[8];
  for (int j0 = threadIdx.x; j0 < kb * 64; j0 += 8 * 256) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * 256;
      v[u] = j < kb * 64 ? s[j] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * 256;
      if (j < kb * 64) ((uint4*)smem)[j] = v[u];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = smem[(blockIdx.x * 97) % (kb * 1024)];
}

int main() {
  const size_t total = (size_t)1 << 30;
  uint4* src;
  unsigned* out;
  hipMalloc(&src, total);
  hipMalloc(&out, 4 << 16);
  hipMemset(src, 1, total);
  hipFuncSetAttribute((const void*)glds_fill, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)vload_fill, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int kbs[] = {16, 32, 64, 128};
  const int grids[] = {256, 512, 1024};
  printf("%-6s %6s %6s %6s %10s %10s\n", "kind", "KB", "grid", "shared", "us", "GB/s");
  for (int kind = 0; kind < 2; ++kind)
    for (int kb : kbs)
      for (int grid : grids)
        for (int shared = 0; shared < 2; ++shared) {
          if ((size_t)grid * kb * 1024 > total) continue;
          auto launch = [&]() {
            if (kind == 0)
              glds_fill<<<grid, 256, kb * 1024>>>(src, kb, shared, out);
            else
              vload_fill<<<grid, 256, kb * 1024>>>(src, kb, shared, out);
          };
          for (int w = 0; w < 3; ++w) launch();
          hipEventRecord(e0);
          const int reps = 20;
          for (int r = 0; r < reps; ++r) launch();
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms = 0;
          hipEventElapsedTime(&ms, e0, e1);
          const double us = ms * 1e3 / reps;
          printf("%-6s %6d %6d %6d %10.2f %10.1f\n", kind ? "vload" : "glds", kb, grid, shared, us,
                 (double)grid * kb * 1024 / (us * 1e3));
        }
  hipFree(src);
  hipFree(out);
  return 0;
}
