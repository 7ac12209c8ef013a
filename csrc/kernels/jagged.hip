// Jagged <-> padded-dense conversions (fbgemm
// jagged_2d_to_dense at torchrec/models.py:167-174 and KJT.to_padded_dense at
// torchrec/models.py:210-212).
//
//   jagged_to_dense : values [nnz, D] + offsets [B+1] -> out [B, T, D]
//                     (rows past a sequence's length or T are `pad`;
//                      sequences longer than T are truncated, like fbgemm)
//   dense_to_jagged : the adjoint, grad [B, T, D] -> values_grad [nnz, D]
//                     (entries beyond T get 0)
// D is handled in 16-B chunks when D % 4 == 0 (fp32), one thread per chunk;
// the integer variant (ids, D = 1) pads sequences of int64 ids.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

__device__ __forceinline__ int64_t find_bag(const int64_t* off, int B, int64_t i) {
  int lo = 0, hi = B;   // largest b with off[b] <= i
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid;
  }
  return lo;
}

template <bool VEC>
__global__ __launch_bounds__(256) void j2d_kernel(const float* __restrict__ values,
                                                  const int64_t* __restrict__ off, int B, int T,
                                                  int D, float pad, float* __restrict__ out) {
  const int C = VEC ? D / 4 : D;
  const int64_t total = (int64_t)B * T * C;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int c = (int)(e % C);
    const int64_t bt = e / C;
    const int t = (int)(bt % T);
    const int b = (int)(bt / T);
    const int64_t s0 = off[b], len = off[b + 1] - s0;
    if (VEC) {
      float4 v = make_float4(pad, pad, pad, pad);
      if (t < len) v = *(const float4*)(values + (s0 + t) * D + c * 4);
      *(float4*)(out + bt * D + c * 4) = v;
    } else {
      out[bt * D + c] = t < len ? values[(s0 + t) * D + c] : pad;
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void d2j_kernel(const float* __restrict__ dense,
                                                  const int64_t* __restrict__ off, int B, int T,
                                                  int D, int64_t nnz, float* __restrict__ vgrad) {
  const int C = VEC ? D / 4 : D;
  const int64_t total = nnz * C;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int c = (int)(e % C);
    const int64_t i = e / C;
    const int b = (int)find_bag(off, B, i);
    const int64_t t = i - off[b];
    if (VEC) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (t < T) v = *(const float4*)(dense + ((int64_t)b * T + t) * D + c * 4);
      *(float4*)(vgrad + i * D + c * 4) = v;
    } else {
      vgrad[i * D + c] = t < T ? dense[((int64_t)b * T + t) * D + c] : 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void j2d_ids_kernel(const int64_t* __restrict__ values,
                                                      const int64_t* __restrict__ off, int B,
                                                      int T, int64_t pad,
                                                      int64_t* __restrict__ out) {
  const int64_t total = (int64_t)B * T;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e % T);
    const int b = (int)(e / T);
    const int64_t s0 = off[b], len = off[b + 1] - s0;
    out[e] = t < len ? values[s0 + t] : pad;
  }
}

int grid_of(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace

void jagged_to_dense(const float* values, const int64_t* off, int B, int T, int D, float pad,
                     float* out, hipStream_t s) {
  const bool vec = (D % 4) == 0;
  const int64_t n = (int64_t)B * T * (vec ? D / 4 : D);
  if (n == 0) return;
  if (vec)
    hipLaunchKernelGGL(j2d_kernel<true>, dim3(grid_of(n)), dim3(256), 0, s, values, off, B, T, D,
                       pad, out);
  else
    hipLaunchKernelGGL(j2d_kernel<false>, dim3(grid_of(n)), dim3(256), 0, s, values, off, B, T, D,
                       pad, out);
  TDFO_CHECK_HIP(hipGetLastError());
}

void dense_to_jagged(const float* dense, const int64_t* off, int B, int T, int D, int64_t nnz,
                     float* vgrad, hipStream_t s) {
  const bool vec = (D % 4) == 0;
  const int64_t n = nnz * (vec ? D / 4 : D);
  if (n == 0) return;
  if (vec)
    hipLaunchKernelGGL(d2j_kernel<true>, dim3(grid_of(n)), dim3(256), 0, s, dense, off, B, T, D,
                       nnz, vgrad);
  else
    hipLaunchKernelGGL(d2j_kernel<false>, dim3(grid_of(n)), dim3(256), 0, s, dense, off, B, T, D,
                       nnz, vgrad);
  TDFO_CHECK_HIP(hipGetLastError());
}

void jagged_ids_to_dense(const int64_t* values, const int64_t* off, int B, int T, int64_t pad,
                         int64_t* out, hipStream_t s) {
  const int64_t n = (int64_t)B * T;
  if (n == 0) return;
  hipLaunchKernelGGL(j2d_ids_kernel, dim3(grid_of(n)), dim3(256), 0, s, values, off, B, T, pad,
                     out);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
