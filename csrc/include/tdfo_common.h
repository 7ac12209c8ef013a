// Shared device helpers for the tdfo_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 tensors are passed as raw uint16_t storage (no torch types in kernels).
//   * wave = 64 lanes; blocks are multiples of 64 threads.
//   * launchers are plain C++ functions taking a hipStream_t so they can be
//     captured in hipGraphs (no allocation / sync inside a launcher).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

#define TDFO_LDS __attribute__((address_space(3)))

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

namespace tdfo {

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even f32 -> bf16 via the native cast (v_cvt_pk_bf16_f32 on
// gfx950), which keeps NaN a NaN (MI355X_MICROARCH.md, correctness boundaries).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Full-wave sum on the DPP path (no LDS round trips): two quad swaps, the
// half-row and row mirrors leave every lane of a 16-lane row holding the row's
// sum; row_bcast15 / row_bcast31 fold rows 0..2 into row 3, and lane 63's value
// is broadcast through an SGPR. ~7 dependent VALU ops instead of 6 ds_bpermute
// round trips (the embedding update reduces once per unique row, in series).
// Summation order differs from wave_sum: same math, different rounding.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, ROWS, 0xf, false));
}

__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<0xb1, 0xf>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4e, 0xf>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141, 0xf>(v);   // row_half_mirror
  v += dpp_f<0x140, 0xf>(v);   // row_mirror
  v += dpp_f<0x142, 0xa>(v);   // row_bcast15 into rows 1, 3
  v += dpp_f<0x143, 0xc>(v);   // row_bcast31 into rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// One Adam / AdamW element update (torch.optim.Adam's L2 form, or decoupled
// weight decay), shared by the flat dense optimizer and the kernels that fuse
// the update into their epilogue (linear_xent's output layer): contraction
// off, so every caller gives the same bits. g is the gradient already
// multiplied by the loss-scale unscale factor.
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float lr,
                                          float bc1, float bc2, float b1, float b2, float eps,
                                          float wd, bool adamw) {
#pragma clang fp contract(off)
  if (adamw) p -= lr * wd * p;
  else g += wd * p;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  // hardware sqrt / reciprocal (1 ulp) and the bias corrections as uniform
  // reciprocals: ~10 VALU ops per element instead of ~35 for three IEEE
  // divisions and a scaled sqrt (the Linear+CE wgrad steps 17 M elements per
  // Bert4Rec step with it). Every optimizer path shares this function, so the
  // fused and separate steps stay bit-identical.
  const float den = __builtin_amdgcn_sqrtf(v * (1.f / bc2)) + eps;
  p -= lr * (m * (1.f / bc1)) * __builtin_amdgcn_rcpf(den);
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): consecutive remapped ids land on one XCD,
// so tiles that share an operand panel share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

}  // namespace tdfo

// Host-side HIP errors are fatal for the op: throw, so torch raises a Python
// error instead of launching dependent kernels on garbage.
#define TDFO_CHECK_HIP(expr)                                                   \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      throw std::runtime_error(std::string("HIP error ") +                     \
                               hipGetErrorString(_e) + " at " + __FILE__ +     \
                               ":" + std::to_string(__LINE__));                \
    }                                                                          \
  } while (0)
