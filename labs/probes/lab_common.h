// Shared helpers of the GEMM structure labs (labs/probes/gemm_*.hip):
// LDS-DMA pieces, swizzled fragment reads (the production layouts of
// csrc/kernels/gemm.hip), XCD remap, a naive fp32 reference GEMM.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#define LDSP __attribute__((address_space(3)))
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int BK = 64;
constexpr int IMG = 128 * BK * 2;   // one 128 x 64 bf16 image, 16 KiB

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ void glds16_asm(const void* src, LDSP char* dst) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds)
               : "memory", "m0");
}

__device__ __forceinline__ int swz_col(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// one 1-KiB piece ii (0..15) of a 128 x 64 image; row operand: 8 rows x 128 B,
// col operand: 4 k-rows x 256 B (see csrc/kernels/gemm.hip)
template <bool COL>
__device__ __forceinline__ void piece(const uint16_t* g, int64_t ld, int x0, int xs, int k0,
                                      LDSP char* img, int ii, int lane) {
  if (COL) {
    const int kr = ii * 4 + (lane >> 4);
    const int c = (lane & 15) ^ swz_col(kr);
    int gc = x0 + c * 8;
    gc = gc <= xs - 8 ? gc : xs - 8;
    glds16_asm(g + (int64_t)(k0 + kr) * ld + gc, img + ii * 1024);
  } else {
    const int r = ii * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    int gr = x0 + r;
    gr = gr < xs ? gr : xs - 1;
    glds16_asm(g + (int64_t)gr * ld + k0 + c * 8, img + ii * 1024);
  }
}

__device__ __forceinline__ bf16x8_t frag_row(const LDSP char* img, int r0, int ks, int lane) {
  const int r = r0 + (lane & 15);
  const int c = (ks * 4 + (lane >> 4)) ^ (r & 7);
  return *(const LDSP bf16x8_t*)(img + r * 128 + c * 16);
}

__device__ __forceinline__ bf16x8_t frag_col(const LDSP char* img, int c0, int ks, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, p = i & 3;
  const int m = c0 + 4 * p;
  s16x4_t v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = ks * 32 + 8 * g + 4 * h + q;
    const int off = k * 256 + (((m >> 3) ^ swz_col(k)) << 4) + ((m & 7) << 1);
    v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDSP s16x4_t*)(img + off));
  }
  s16x8_t r = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

template <bool COL>
__device__ __forceinline__ bf16x8_t frag(const LDSP char* img, int x0, int ks, int lane) {
  return COL ? frag_col(img, x0, ks, lane) : frag_row(img, x0, ks, lane);
}

struct P {
  const uint16_t *A, *B;
  uint16_t* C;
  int64_t lda, ldb, ldc;
  int M, N, K;
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// naive reference: C[m][n] = sum_k A(m,k) B(k,n) in fp32
__global__ void ref_kernel(P p, int ac, int bc, float* out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= p.N) return;
  float s = 0.f;
  for (int k = 0; k < p.K; ++k) {
    const uint16_t a = ac ? p.A[(int64_t)k * p.lda + m] : p.A[(int64_t)m * p.lda + k];
    const uint16_t b = bc ? p.B[(int64_t)k * p.ldb + n] : p.B[(int64_t)n * p.ldb + k];
    s += __uint_as_float((uint32_t)a << 16) * __uint_as_float((uint32_t)b << 16);
  }
  out[(int64_t)m * p.N + n] = s;
}

static uint16_t f2b(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

