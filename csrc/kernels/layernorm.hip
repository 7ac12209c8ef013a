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
// Sequence prologue (PRO = true): the Bert4Rec input block
//   y = dropout(LN(x + pos))   (torchrec/models.py:147-150: item embedding +
// positional encoding, LayerNorm over [T, E], embedding dropout) in one pass;
// the dropout mask is the counter hash of encoder.hip (nothing stored, the
// backward regenerates it) and the backward also emits d_pos = sum over rows
// of dx as a third partial column block [block][3n].
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int LN_WAVES = 4;

// Optional prologue inputs of the PRO kernels.
struct ProArgs {
  const float* pos;        // [n] added to every row
  float rate;              // dropout rate on the output (0: none)
  uint32_t seed;
  const int64_t* step;     // device step counter mixed into the seed
};

__device__ __forceinline__ uint32_t pro_hash3(uint32_t a, uint32_t b, uint32_t c) {
  // the counter hash of encoder.hip / attention.hip
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

__device__ __forceinline__ float pro_mul(const ProArgs& p, uint32_t sd, int64_t r, int e) {
  if (p.rate <= 0.f) return 1.f;
  const uint32_t h = pro_hash3(sd, (uint32_t)r, (uint32_t)e);
  return (float)(h >> 8) * (1.0f / 16777216.0f) >= p.rate ? 1.f / (1.f - p.rate) : 0.f;
}

__device__ __forceinline__ uint32_t pro_seed(const ProArgs& p) {
  const uint32_t step = p.step ? (uint32_t)p.step[0] : 0u;
  return p.seed ^ (step * 0x632BE5ABu) ^ 0x51ED270Bu;
}

template <int NPL, bool PRO>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int64_t M,
                                                     int n, float eps,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta,
                                                     float* __restrict__ y,
                                                     float* __restrict__ mean,
                                                     float* __restrict__ rstd, ProArgs pa) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const float invn = 1.f / (float)n;
  const uint32_t sd = PRO ? pro_seed(pa) : 0u;
  for (int64_t r = wave; r < M; r += nw) {
    const float* xr = x + r * n;
    float v[NPL];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int e = lane + 64 * k;
      v[k] = e < n ? xr[e] + (PRO ? pa.pos[e] : 0.f) : 0.f;
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
      if (e < n) {
        const float o = (v[k] - mu) * rs * gamma[e] + beta[e];
        yr[e] = PRO ? o * pro_mul(pa, sd, r, e) : o;
      }
    }
    if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
  }
}

template <int NPL, bool PRO>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x,
                                                     const float* __restrict__ g, int64_t M,
                                                     int n, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     float* __restrict__ dx,
                                                     float* __restrict__ part, ProArgs pa,
                                                     int nb, EncRedJob job) {
  constexpr int NP = PRO ? 3 : 2;                  // partial blocks: dgamma | dbeta (| dpos)
  __shared__ float red[LN_WAVES][NP * NPL * 64];
  if ((int)blockIdx.x >= nb) {   // a parked encoder reduction's extra blocks (no barrier)
    enc_red_col(job, ((int)blockIdx.x - nb) * (int)blockDim.x + (int)threadIdx.x);
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)nb * blockDim.x) >> 6;
  const float invn = 1.f / (float)n;
  const uint32_t sd = PRO ? pro_seed(pa) : 0u;
  float dg[NPL], db[NPL], dp[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) { dg[k] = 0.f; db[k] = 0.f; dp[k] = 0.f; }
  for (int64_t r = wave; r < M; r += nw) {
    const float mu = mean[r], rs = rstd[r];
    float xh[NPL], gg[NPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int e = lane + 64 * k;
      const bool ok = e < n;
      float gv = ok ? g[r * n + e] : 0.f;
      if (PRO && ok) gv *= pro_mul(pa, sd, r, e);
      xh[k] = ok ? (x[r * n + e] + (PRO ? pa.pos[e] : 0.f) - mu) * rs : 0.f;
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
      if (e < n) {
        const float d = rs * (gg[k] - m1 - xh[k] * m2);
        dx[r * n + e] = d;
        if (PRO) dp[k] += d;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    red[w][k * 64 + lane] = dg[k];
    red[w][NPL * 64 + k * 64 + lane] = db[k];
    if (PRO) red[w][2 * NPL * 64 + k * 64 + lane] = dp[k];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NP * n; e += blockDim.x) {
    const int blk = e / n, c = e - blk * n;
    const int idx = blk * NPL * 64 + c;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < LN_WAVES; ++q) s += red[q][idx];
    part[(int64_t)blockIdx.x * NP * n + e] = s;
  }
}

}  // namespace

int layernorm_parts(int64_t M) {
  const int64_t b = (M + LN_WAVES - 1) / LN_WAVES;
  return (int)(b < 256 ? (b < 1 ? 1 : b) : 256);
}

#define TDFO_LN_DISPATCH(KERNEL, PRO, ...)                                          \
  {                                                                                 \
    const int npl = (n + 63) / 64;                                                  \
    if (npl <= 1) hipLaunchKernelGGL((KERNEL<1, PRO>), __VA_ARGS__);                \
    else if (npl <= 2) hipLaunchKernelGGL((KERNEL<2, PRO>), __VA_ARGS__);           \
    else if (npl <= 4) hipLaunchKernelGGL((KERNEL<4, PRO>), __VA_ARGS__);           \
    else if (npl <= 8) hipLaunchKernelGGL((KERNEL<8, PRO>), __VA_ARGS__);           \
    else if (npl <= 16) hipLaunchKernelGGL((KERNEL<16, PRO>), __VA_ARGS__);         \
    else throw std::runtime_error("layernorm: n > 1024");                           \
  }

void layernorm_fwd(const float* x, int64_t M, int n, float eps, const float* gamma,
                   const float* beta, float* y, float* mean, float* rstd, hipStream_t s) {
  if (M <= 0) return;
  const dim3 grid(layernorm_parts(M)), block(64 * LN_WAVES);
  TDFO_LN_DISPATCH(ln_fwd_kernel, false, grid, block, 0, s, x, M, n, eps, gamma, beta, y, mean,
                   rstd, ProArgs{});
  TDFO_CHECK_HIP(hipGetLastError());
}

void layernorm_bwd(const float* x, const float* g, int64_t M, int n, const float* gamma,
                   const float* mean, const float* rstd, float* dx, float* part,
                   float* dgamma_dbeta, hipStream_t s) {
  if (M <= 0) return;
  const int nb = layernorm_parts(M);
  const dim3 grid(nb), block(64 * LN_WAVES);
  TDFO_LN_DISPATCH(ln_bwd_kernel, false, grid, block, 0, s, x, g, M, n, gamma, mean, rstd, dx,
                   part, ProArgs{}, nb, EncRedJob{});
  TDFO_CHECK_HIP(hipGetLastError());
  reduce_rows(part, nb, 2 * n, 2 * n, dgamma_dbeta, 0, 1.f, s);
}

void seq_prologue_fwd(const float* x, const float* pos, int64_t M, int n, float eps,
                      const float* gamma, const float* beta, float rate, uint32_t seed,
                      const int64_t* step, float* y, float* mean, float* rstd, hipStream_t s) {
  if (M <= 0) return;
  const dim3 grid(layernorm_parts(M)), block(64 * LN_WAVES);
  const ProArgs pa{pos, rate, seed, step};
  TDFO_LN_DISPATCH(ln_fwd_kernel, true, grid, block, 0, s, x, M, n, eps, gamma, beta, y, mean,
                   rstd, pa);
  TDFO_CHECK_HIP(hipGetLastError());
}

void seq_prologue_bwd(const float* x, const float* pos, const float* g, int64_t M, int n,
                      const float* gamma, const float* mean, const float* rstd, float rate,
                      uint32_t seed, const int64_t* step, float* dx, float* part,
                      float* dgamma_dbeta_dpos, hipStream_t s, const int64_t* idx) {
  if (M <= 0) return;
  const int nb = layernorm_parts(M);
  // the last encoder layer's parked parameter-gradient reduction, if any,
  // rides in extra blocks of this launch
  EncRedJob job;
  const int extra = encoder_reduce_take(&job) ? (job.P + 64 * LN_WAVES - 1) / (64 * LN_WAVES) : 0;
  const dim3 grid(nb + extra), block(64 * LN_WAVES);
  const ProArgs pa{pos, rate, seed, step};
  TDFO_LN_DISPATCH(ln_bwd_kernel, true, grid, block, 0, s, x, g, M, n, gamma, mean, rstd, dx,
                   part, pa, nb, job);
  TDFO_CHECK_HIP(hipGetLastError());
  reduce_rows(part, nb, 3 * n, 3 * n, dgamma_dbeta_dpos, 0, 1.f, s, idx);
}
#undef TDFO_LN_DISPATCH

}  // namespace tdfo
