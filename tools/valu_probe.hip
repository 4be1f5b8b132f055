// VALU issue-rate probe: wave64 integer VALU throughput per SIMD versus
// waves per SIMD, with 8 independent dependency chains per wave.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_probe tools/valu_probe.hip
// Prints instructions / cycle / SIMD (clock from the kernel's own
// s_memtime-free wall time and the nominal 2.4 GHz).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void probe(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 1) + i;
  const uint32_t k1 = seed ^ 0x55, k2 = seed ^ 0x33;
  for (int n = 0; n < iters; ++n) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (OP == 0) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(k1), "v"(k2));
        if (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(k1));
        if (OP == 2) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(k1), "v"(k2));
        if (OP == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(k1), "v"(k2));
        if (OP == 4) asm volatile("v_min3_u32 %0, %0, 5, 7" : "+v"(a[i]));
        if (OP == 5) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[i]) : "v"(k1));
        if (OP == 6) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a[i]));
        if (OP == 7) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(k1));
        if (OP == 8) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(k1));
        if (OP == 9) asm volatile("v_min3_u32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(k1));
        if (OP == 10) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "s"(k1), "v"(k2));
        if (OP == 11) asm volatile("v_cvt_f32_ubyte1 %0, %0" : "+v"(a[i]));
        if (OP == 12) asm volatile("v_min_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(a[i]) : "v"(k1));
        if (OP == 13) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(double*)&a[i & 6]) : "v"(*(double*)&a[(i + 2) & 6]));
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
static void run(const char* name, uint32_t* d, int waves_per_simd) {
  const int cus = 256, threads = 256;  // 4 waves per block = 1 per SIMD
  const int blocks = cus * waves_per_simd;
  const int iters = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<OP><<<blocks, threads>>>(d, iters, 7);
  hipEventRecord(e0);
  probe<OP><<<blocks, threads>>>(d, iters, 9);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double winstr = (double)blocks * 4 * iters * 32;  // wave-instructions
  const double cyc = ms * 1e-3 * 2.4e9;
  printf("%-14s waves/SIMD %d: %8.3f ms  %.3f instr/cycle/SIMD\n", name, waves_per_simd, ms,
         winstr / 1024.0 / cyc);
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 256 * 8 * 256 * sizeof(uint32_t));
  for (int w : {4, 8}) {
    run<0>("v_min3_u32 vvv", d, w);
    run<9>("v_min3_u32 vvc", d, w);
    run<10>("v_min3_u32 vsv", d, w);
    run<4>("v_min3_u32 vcc", d, w);
    run<1>("v_add_u32 e32", d, w);
    run<5>("v_add_u32 e64", d, w);
    run<8>("v_min_u32 e32", d, w);
    run<12>("v_min_u32 sdwa", d, w);
    run<6>("v_bfe_u32 vcc", d, w);
    run<7>("v_pk_add_u16", d, w);
    run<11>("v_cvt_f32_ubyte1", d, w);
    run<2>("v_mad_u32_u24", d, w);
    run<3>("v_perm_b32", d, w);
    run<13>("v_pk_mul_f32", d, w);
  }
  hipFree(d);
  return 0;
}
