// Shared device helpers for the VST (video style transfer) HIP kernels.
// gfx950 / CDNA4 only: 64-lane wavefronts, bf16 MFMA, raw buffer loads with
// hardware range checking (out-of-range offsets read as zero, which is how
// every kernel here implements zero padding and M/N/K tails without branches).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vst {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;  // storage type of a bf16 in global memory

// Offset that is always outside every buffer resource: buffer loads return 0.
constexpr int kOOB = 0x7ffffff0;

// Host side: the byte size of a buffer descriptor, with a flag for extents past 2^31 - 1 (the kernels' 32-bit
// offsets would read zeros there).  An entry point that is not chunked refuses such a call (VST_ERR_ARG) instead of
// computing on zeros.
struct Fit31 {
  bool over = false;
  uint32_t operator()(size_t bytes) {
    if (bytes > 0x7fffffffULL) {
      over = true;
      return 0x7fffffffu;
    }
    return (uint32_t)bytes;
  }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ u32x2 buf_load8(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t buf_load4(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ uint16_t buf_load2(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even f32 -> bf16 (NaN handled by the hardware cvt path)
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<uint16_t*>(&b);
}
// value of x after a bf16 store and reload (the rounding point of a bf16 tensor boundary)
__device__ __forceinline__ float round_bf(float x) { return bf2f(f2bf(x)); }
// one v_cvt_pk_bf16_f32 (RNE, lo -> bits 0-15): the scalar casts + shift + or cost 4 VALU per pair
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  typedef float vst_f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 vst_b2 __attribute__((ext_vector_type(2)));
  const vst_f2 v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, vst_b2));
}
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2bf(f[2 * i], f[2 * i + 1]);
  return r;
}

// x * sigmoid(x) on v_exp_f32 + v_rcp_f32 (the IEEE division would add a ~10-instruction fix-up sequence)
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
// erf by Abramowitz & Stegun 7.1.26 (|error| < 1.5e-7, far below the bf16 rounding of every GELU output here)
// on one v_rcp_f32 + one v_exp_f32 + 6 FMAs: erff() costs ~30 VALU, which in the GEGLU epilogue is ~10 % of the
// largest GEMM of the step (one erf per output element, not overlapped with the MFMA loop).
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float y = 1.0f - poly * __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  return copysignf(y, x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }

// h * GELU(g) for two columns at once (the GEGLU GEMM epilogues), the same A&S 7.1.26 erf on packed fp32 (v_pk_*):
//   0.5 g (1 + erf(g / sqrt2)) = 0.5 g + 0.5 |g| erf(|g| / sqrt2),  erf(z) = 1 - poly(t) exp(-z^2), t = 1 / (1 + p z)
// (erf odd: no copysign); only |g|, the rcp and the exp2 are per element.  ~10 VALU per output instead of ~18 for
// the scalar form, whose cost was ~12 % of the 16^2 GEGLU launch (tools/p8_epi_ablate.sh).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 geglu2(f32x2 h, f32x2 g) {
  const f32x2 ag = {fabsf(g.x), fabsf(g.y)};
  const f32x2 u = __builtin_elementwise_fma(ag, f32x2(0.3275911f * 0.70710678118654752f), f32x2(1.0f));
  const f32x2 t = {__builtin_amdgcn_rcpf(u.x), __builtin_amdgcn_rcpf(u.y)};
  f32x2 poly = __builtin_elementwise_fma(t, f32x2(1.061405429f), f32x2(-1.453152027f));
  poly = __builtin_elementwise_fma(poly, t, f32x2(1.421413741f));
  poly = __builtin_elementwise_fma(poly, t, f32x2(-0.284496736f));
  poly = __builtin_elementwise_fma(poly, t, f32x2(0.254829592f));
  poly = poly * t;
  const f32x2 w = (g * g) * f32x2(-0.5f * 1.4426950408889634f);
  const f32x2 e = {__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)};
  const f32x2 hag = ag * f32x2(0.5f);
  const f32x2 y = __builtin_elementwise_fma(-(poly * e), hag, hag);  // 0.5 |g| erf(|g| / sqrt2)
  return h * __builtin_elementwise_fma(g, f32x2(0.5f), y);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Bijective XCD-aware block remap (blocks b and b+8 share an XCD under
// round-robin dispatch): consecutive logical tiles land on one XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

}  // namespace vst

// C-ABI status codes (see include/vst.h)
#define VST_OK 0
#define VST_ERR_ARG 1
#define VST_ERR_LAUNCH 2
#define VST_ERR_UNSUPPORTED 3
