// Attention building blocks shared by attention.hip (the attention kernels) and gemm_p8.hip (the cross-attention
// epilogue of the q projection): transposed LDS reads, lane-group max, bf16 packing, K/V tile swizzles, raw exp2.
#pragma once
#include "vst_common.h"

namespace vst {

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x4 ds_read_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)((__attribute__((address_space(3))) char*)(uintptr_t)(p)));
}

// max over the four 16-lane groups (lanes i, i^16, i^32, i^48) with two VALU lane swaps instead of two LDS
// ds_bpermute round trips; v_max_f32 as asm keeps the compiler from adding canonicalising maxes around the swaps
__device__ __forceinline__ float vmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float group_max(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = vmax_raw(__uint_as_float(p[0]), __uint_as_float(p[1]));
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax_raw(__uint_as_float(q[0]), __uint_as_float(q[1]));
}

__device__ __forceinline__ bf16x8 cat_tr(s16x4 lo, s16x4 hi) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 pack_p8(float a0, float a1, float a2, float a3, float b0, float b1,
                                          float b2, float b3) {
  u32x4 u{pack2bf(a0, a1), pack2bf(a2, a3), pack2bf(b0, b1), pack2bf(b2, b3)};
  return __builtin_bit_cast(bf16x8, u);
}

// K tile: [64 keys][64 d] bf16, 128-B rows, GEMM swizzle (ds_read_b128 row reads)
__device__ __forceinline__ int k_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
// V tile: [64 keys][64 d], swizzle chosen for conflict-free ds_read_b64_tr_b16 over 8-row groups
__device__ __forceinline__ int v_off(int row, int chunk) { return row * 128 + ((chunk ^ (((row >> 1) & 3) << 1)) << 4); }

// Raw v_exp_f32 (2^x): the softmax arguments are <= 0, so the denormal-range fix-up that exp2f() wraps around
// it (v_ldexp + compares + selects, ~4 VALU per score) only decides whether a ~1e-38 weight is flushed to 0.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

}  // namespace vst
