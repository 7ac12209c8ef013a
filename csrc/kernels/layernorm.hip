// LayerNorm over the last n elements of each row, forward and backward
// (K13/K16 in SURVEY.md §2.3). Bert4Rec uses it twice: over E = 16 per token
// inside every pre-norm sublayer (torchrec/models.py:91-106) and jointly over
// [T, E] = 320 elements after the positional encoding (models.py:147, quirk
// Q10). One wave per row; lane l owns elements l, l+64, ... (NPL per lane) so
// the row statistics are two wave reductions. fp32 throughout.
//   fwd : y = (x - mean) * rstd * gamma + beta; saves mean, rstd per row
//   bwd : dx = rstd * (g' - mean(g') - xhat * mean(g' * xhat)), g' = g * gamma
//         dgamma / dbeta: per-block partials [block][2n] (fixed row order),
//         summed by reduce_rows -> deterministic
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int LN_WAVES = 4;

template <int NPL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int64_t M,
                                                     int n, float eps,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta,
                                                     float* __restrict__ y,
                                                     float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float invn = 1.f / (float)n;
  for (int64_t r = wave; r < M; r += nw) {
    const float* xr = x + r * n;
    float v[NPL];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int e = lane + 64 * k;
      v[k] = e < n ? xr[e] : 0.f;
      s += v[k];
    }
    const float mu = wave_sum(s) * invn;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int e = lane + 64 * k;
      const float d = e < n ? v[k] - mu : 0.f;
      q += d * d;
    }
    const float rs = rsqrtf(wave_sum(q) * invn + eps);
    float* yr = y + r * n;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int e = lane + 64 * k;
      if (e < n) yr[e] = (v[k] - mu) * rs * gamma[e] + beta[e];
    }
    if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
  }
}

template <int NPL>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x,
                                                     const float* __restrict__ g, int64_t M,
                                                     int n, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     float* __restrict__ dx,
                                                     float* __restrict__ part) {
  __shared__ float red[LN_WAVES][2 * NPL * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float invn = 1.f / (float)n;
  float dg[NPL], db[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) { dg[k] = 0.f; db[k] = 0.f; }
  for (int64_t r = wave; r < M; r += nw) {
    const float mu = mean[r], rs = rstd[r];
    float xh[NPL], gg[NPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int e = lane + 64 * k;
      const bool ok = e < n;
      const float gv = ok ? g[r * n + e] : 0.f;
      xh[k] = ok ? (x[r * n + e] - mu) * rs : 0.f;
      gg[k] = ok ? gv * gamma[e] : 0.f;
      s1 += gg[k];
      s2 += gg[k] * xh[k];
      dg[k] += gv * xh[k];
      db[k] += gv;
    }
    const float m1 = wave_sum(s1) * invn, m2 = wave_sum(s2) * invn;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int e = lane + 64 * k;
      if (e < n) dx[r * n + e] = rs * (gg[k] - m1 - xh[k] * m2);
    }
  }
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    red[w][k * 64 + lane] = dg[k];
    red[w][NPL * 64 + k * 64 + lane] = db[k];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * n; e += blockDim.x) {
    const int half = e >= n, c = half ? e - n : e;
    const int idx = half * NPL * 64 + c;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < LN_WAVES; ++q) s += red[q][idx];
    part[(int64_t)blockIdx.x * 2 * n + e] = s;
  }
}

}  // namespace

int layernorm_parts(int64_t M) {
  const int64_t b = (M + LN_WAVES - 1) / LN_WAVES;
  return (int)(b < 256 ? (b < 1 ? 1 : b) : 256);
}

#define TDFO_LN_DISPATCH(KERNEL, ...)                                               \
  {                                                                                 \
    const int npl = (n + 63) / 64;                                                  \
    if (npl <= 1) hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__);                       \
    else if (npl <= 2) hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__);                  \
    else if (npl <= 4) hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__);                  \
    else if (npl <= 8) hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__);                  \
    else if (npl <= 16) hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__);                \
    else throw std::runtime_error("layernorm: n > 1024");                           \
  }

void layernorm_fwd(const float* x, int64_t M, int n, float eps, const float* gamma,
                   const float* beta, float* y, float* mean, float* rstd, hipStream_t s) {
  if (M <= 0) return;
  const dim3 grid(layernorm_parts(M)), block(64 * LN_WAVES);
  TDFO_LN_DISPATCH(ln_fwd_kernel, grid, block, 0, s, x, M, n, eps, gamma, beta, y, mean, rstd);
  TDFO_CHECK_HIP(hipGetLastError());
}

void layernorm_bwd(const float* x, const float* g, int64_t M, int n, const float* gamma,
                   const float* mean, const float* rstd, float* dx, float* part,
                   float* dgamma_dbeta, hipStream_t s) {
  if (M <= 0) return;
  const int nb = layernorm_parts(M);
  const dim3 grid(nb), block(64 * LN_WAVES);
  TDFO_LN_DISPATCH(ln_bwd_kernel, grid, block, 0, s, x, g, M, n, gamma, mean, rstd, dx, part);
  TDFO_CHECK_HIP(hipGetLastError());
  reduce_rows(part, nb, 2 * n, 2 * n, dgamma_dbeta, 0, 1.f, s);
}
#undef TDFO_LN_DISPATCH

}  // namespace tdfo
