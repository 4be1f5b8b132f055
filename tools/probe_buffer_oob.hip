// Range-check semantics of buffer_load ... lds (raw buffer, stride 0) on
// gfx950, for the conv kernels' DMA: is soffset part of the bounds check,
// and does an out-of-range voffset load zeros into LDS?
//   case A: num_records 256, voffset 0,   soffset 1024 -> data (soffset unchecked) or 0
//   case B: num_records 256, voffset 512, soffset 0    -> 0 expected (voffset checked)
//   case C: num_records 4096, voffset 0x80000000, soffset 64 -> 0 expected
//   case D: num_records 4096, voffset 16*lane, soffset 64 -> data at 64 + 16*lane
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void probe(const unsigned* src, unsigned* out, int nrec, unsigned voff, int soff) {
  __shared__ __attribute__((aligned(16))) unsigned sm[256];
  const int lane = threadIdx.x;
  for (int i = lane; i < 256; i += 64) sm[i] = 0xDEADBEEF;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nrec, 0x00020000);
  const unsigned v = voff == 0xFFFFFFFFu ? lane * 16u : voff;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)sm, 16, v,
                                           soff, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = lane; i < 256; i += 64) out[i] = sm[i];
}

int main() {
  unsigned *src, *out, h[256];
  hipMalloc(&src, 65536);
  hipMalloc(&out, 1024);
  unsigned init[16384];
  for (int i = 0; i < 16384; ++i) init[i] = 0x10000000u + i;
  hipMemcpy(src, init, 65536, hipMemcpyHostToDevice);
  struct { const char* name; int nrec; unsigned voff; int soff; } cases[] = {
      {"A nrec 256, voff 0, soff 1024", 256, 0u, 1024},
      {"B nrec 256, voff 512, soff 0", 256, 512u, 0},
      {"C nrec 4096, voff 0x80000000, soff 64", 4096, 0x80000000u, 64},
      {"D nrec 4096, voff 16*lane, soff 64", 4096, 0xFFFFFFFFu, 64}};
  for (auto& c : cases) {
    probe<<<1, 64>>>(src, out, c.nrec, c.voff, c.soff);
    hipMemcpy(h, out, 1024, hipMemcpyDeviceToHost);
    printf("%-40s lane0 %08x %08x %08x %08x  lane1 %08x  lane63 %08x\n", c.name, h[0], h[1], h[2],
           h[3], h[4], h[252]);
  }
  return 0;
}
