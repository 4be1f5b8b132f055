// Device helpers shared by the conv kernels (conv.hip) and the stem /
// conv0 kernels (stem.hip): operand vector types, bf16 packing, SiLU, the
// raw buffer-resource constants and the fp8 encoder.
#pragma once
#include "conv.h"

namespace rv {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;

typedef __attribute__((ext_vector_type(2))) float f32x2v;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;
typedef __attribute__((ext_vector_type(2))) unsigned int v2u32;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u32;

// f32 -> bf16, round to nearest even, on the hardware converter
// (v_cvt_pk_bf16_f32: two values per instruction).
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v{lo, hi}, bf16x2v));
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// SiLU x * sigmoid(x) = x * 1/(1 + e^-x) with the hardware reciprocal
// (<= 1 ulp f32; the result is stored as bf16).
__device__ __forceinline__ float silu(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
}
// The same SiLU on a pair: the scale by -log2(e) (what __expf(-v) lowers
// to: one f32 multiply, then v_exp_f32), the + 1 and the final product run
// as packed f32 pair instructions (v_pk_mul_f32 / v_pk_add_f32); element by
// element these are the same IEEE operations as silu(), so the result is
// bit-identical with half the non-transcendental instructions.
__device__ __forceinline__ f32x2v silu2(f32x2v x) {
  const float nl2e = __builtin_bit_cast(float, 0xBFB8AA3Bu);  // -log2(e) in f32
  const f32x2v t = x * f32x2v{nl2e, nl2e};
  const f32x2v d = f32x2v{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.0f;
  return x * f32x2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
// v[i] = SiLU(v[i]) for 4 values (two silu2 pairs)
__device__ __forceinline__ void silu4(float (&v)[4]) {
  const f32x2v a = silu2(f32x2v{v[0], v[1]}), b = silu2(f32x2v{v[2], v[3]});
  v[0] = a.x;
  v[1] = a.y;
  v[2] = b.x;
  v[3] = b.y;
}

// Buffer-resource LDS-DMA (conv_patch_kernel): dword3 of the descriptor
// for a raw (stride 0) buffer on gfx950, and the voffset that the range
// check (voffset + soffset against num_records, checked on the GPU:
// tools/probe_buffer_oob.hip) always rejects -- such a load writes zeros.
constexpr int kRsrcFlags = 0x00020000;
constexpr uint32_t kOOB = 0x80000000u;
// fp8 epilogue8 (ConvArgs::in8): dequantise (acc * wscale[co] * s_in), bias,
// SiLU, residual (fp8 code * s_res), then per output view fp8 codes of
// value / s_out (v_cvt_pk_fp8_f32, round to nearest even, saturated to
// +-448 first) or bf16 / f32.
__device__ __forceinline__ uint32_t f8_encode4(const float (&v)[4], float inv_s) {
  float q[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = fminf(fmaxf(v[i] * inv_s, -448.f), 448.f);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], w, true);
  return (uint32_t)w;
}

}  // namespace rv
