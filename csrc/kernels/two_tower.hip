// Fused TwoTower towers + row-wise dot + BCE + full backward (gfx950).
//
// Model (reference jax-flax/models.py:72-102, tensorflow2/models.py:43-71):
//   u = fc2_u(swish(fc1_u(e_user)))                       16 -> 16 -> 16
//   i = fc2_i(swish(fc1_i([e_item e_lang e_ebook e_fmt e_pub e_dec avg pages])))
//                                                          98 -> 16 -> 16
//   logit = sum(u * i); loss = BCE-with-logits(logit, label)
//
// All dense parameters are 2,400 floats, so the whole step is memory/launch
// bound, not MFMA bound (E = 16). One launch does forward, loss and the full
// backward for 128 samples per block: one thread per sample with the weights
// broadcast from LDS, then the per-sample activations / gradients are staged
// in LDS and every thread reduces float4 slices of the weight gradient over
// the block's samples. Block partials go to part[block][TT_PART_LD] and are
// reduced in a fixed order (tdfo::reduce_rows) -> deterministic, no atomics.
// Embedding gradients are written per sample (dX) for the sort-based fused
// sparse optimizer (embedding.hip).
//
// Parameter layout (flat fp32, Flax kernel convention W[in][out]):
//   [uW1 16x16 | ub1 16 | uW2 16x16 | ub2 16 | iW1 98x16 | ib1 16 | iW2 16x16 | ib2 16]
// i.e. 150 "rows" of 16; row r < 17 -> (xu,1) x dh_u, r < 34 -> (a_u,1) x du,
// r < 133 -> (xi,1) x dh_i, else (a_i,1) x di.
#include <hip/hip_fp16.h>

#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int E = 16;
constexpr int NI = 98;          // item tower input width
constexpr int SPB = 128;        // samples per block
constexpr int AROWS = 150;      // rows of the parameter matrix
constexpr int NP = AROWS * E;   // 2400

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// fp16 compute (the reference's mixed_precision path: Flax dtype=float16 on
// GPU, jax-flax/models.py:142-151): values are rounded to fp16 where a
// half-precision layer would store them; sums accumulate in fp32 like an
// fp16 MFMA / XLA dot with fp32 accumulation.
template <bool HALF>
__device__ __forceinline__ float rnd(float x) {
  if constexpr (HALF) return __half2float(__float2half(x));
  else return x;
}

template <bool TRAIN, bool HALF>
__global__ __launch_bounds__(SPB) void two_tower_kernel(TwoTowerArgs a) {
  __shared__ float Wl[NP];
  __shared__ float As[TRAIN ? SPB : 1][AROWS];
  __shared__ __attribute__((aligned(16))) float Gs[TRAIN ? SPB : 1][4 * E];
  __shared__ float red[SPB / 64];
  const int t = threadIdx.x;
  for (int k = t; k < NP; k += SPB) Wl[k] = rnd<HALF>(a.P[k]);
  __syncthreads();
  const float* uW1 = Wl;
  const float* ub1 = Wl + 16 * E;
  const float* uW2 = Wl + 17 * E;
  const float* ub2 = Wl + 33 * E;
  const float* iW1 = Wl + 34 * E;
  const float* ib1 = Wl + 132 * E;
  const float* iW2 = Wl + 133 * E;
  const float* ib2 = Wl + 149 * E;

  const int64_t s = (int64_t)blockIdx.x * SPB + t;
  const bool valid = s < a.B;
  const float* xr = a.X + (valid ? s : 0) * a.ldx;
  float xu[E], xi[NI];
#pragma unroll
  for (int k = 0; k < E; k += 4) {
    const float4 v = *(const float4*)(xr + k);
    xu[k] = rnd<HALF>(v.x); xu[k + 1] = rnd<HALF>(v.y);
    xu[k + 2] = rnd<HALF>(v.z); xu[k + 3] = rnd<HALF>(v.w);
  }
#pragma unroll
  for (int k = 0; k < 96; k += 4) {
    const float4 v = *(const float4*)(xr + E + k);
    xi[k] = rnd<HALF>(v.x); xi[k + 1] = rnd<HALF>(v.y);
    xi[k + 2] = rnd<HALF>(v.z); xi[k + 3] = rnd<HALF>(v.w);
  }
  xi[96] = rnd<HALF>(xr[E + 96]);
  xi[97] = rnd<HALF>(xr[E + 97]);

  // ---- forward
  float hu[E], au[E], u[E], hi[E], ai[E], iv[E];
#pragma unroll
  for (int o = 0; o < E; ++o) { hu[o] = ub1[o]; hi[o] = ib1[o]; }
#pragma unroll
  for (int k = 0; k < E; ++k)
#pragma unroll
    for (int o = 0; o < E; ++o) hu[o] = fmaf(xu[k], uW1[k * E + o], hu[o]);
#pragma unroll
  for (int k = 0; k < NI; ++k)
#pragma unroll
    for (int o = 0; o < E; ++o) hi[o] = fmaf(xi[k], iW1[k * E + o], hi[o]);
#pragma unroll
  for (int o = 0; o < E; ++o) {
    hu[o] = rnd<HALF>(hu[o]);
    hi[o] = rnd<HALF>(hi[o]);
    au[o] = rnd<HALF>(hu[o] * sigm(hu[o]));
    ai[o] = rnd<HALF>(hi[o] * sigm(hi[o]));
    u[o] = ub2[o];
    iv[o] = ib2[o];
  }
#pragma unroll
  for (int k = 0; k < E; ++k)
#pragma unroll
    for (int o = 0; o < E; ++o) {
      u[o] = fmaf(au[k], uW2[k * E + o], u[o]);
      iv[o] = fmaf(ai[k], iW2[k * E + o], iv[o]);
    }
  float logit = 0.f;
#pragma unroll
  for (int o = 0; o < E; ++o) {
    u[o] = rnd<HALF>(u[o]);
    iv[o] = rnd<HALF>(iv[o]);
  }
#pragma unroll
  for (int o = 0; o < E; ++o) logit = fmaf(u[o], iv[o], logit);
  logit = rnd<HALF>(logit);
  if (valid) a.logits[s] = logit;
  if constexpr (!TRAIN) return;

  // ---- loss + backward
  const float y = valid ? a.labels[s] : 0.f;
  float loss = valid ? fmaxf(logit, 0.f) - logit * y + log1pf(__expf(-fabsf(logit))) : 0.f;
  const float ls = a.loss_scale ? a.loss_scale[0] : 1.f;
  const float dl = valid ? rnd<HALF>((sigm(logit) - y) * a.inv_n * ls) : 0.f;
  float du[E], di[E], dhu[E], dhi[E];
#pragma unroll
  for (int o = 0; o < E; ++o) { du[o] = rnd<HALF>(dl * iv[o]); di[o] = rnd<HALF>(dl * u[o]); }
#pragma unroll
  for (int k = 0; k < E; ++k) {
    float gu = 0.f, gi = 0.f;
#pragma unroll
    for (int o = 0; o < E; ++o) {
      gu = fmaf(uW2[k * E + o], du[o], gu);
      gi = fmaf(iW2[k * E + o], di[o], gi);
    }
    const float su = sigm(hu[k]), si = sigm(hi[k]);
    dhu[k] = rnd<HALF>(gu * su * (1.f + hu[k] * (1.f - su)));
    dhi[k] = rnd<HALF>(gi * si * (1.f + hi[k] * (1.f - si)));
  }
  if (valid) {
    float* dxr = a.dX + s * a.lddx;
#pragma unroll
    for (int k = 0; k < E; k += 4) {
      float g[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float acc = 0.f;
#pragma unroll
        for (int o = 0; o < E; ++o) acc = fmaf(uW1[(k + q) * E + o], dhu[o], acc);
        g[q] = rnd<HALF>(acc);
      }
      *(float4*)(dxr + k) = make_float4(g[0], g[1], g[2], g[3]);
    }
#pragma unroll
    for (int k = 0; k < 96; k += 4) {
      float g[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float acc = 0.f;
#pragma unroll
        for (int o = 0; o < E; ++o) acc = fmaf(iW1[(k + q) * E + o], dhi[o], acc);
        g[q] = rnd<HALF>(acc);
      }
      *(float4*)(dxr + E + k) = make_float4(g[0], g[1], g[2], g[3]);
    }
  }
  // stage A (inputs of each weight row, 1 for biases) and G (output grads)
  float* A = As[t];
#pragma unroll
  for (int k = 0; k < E; ++k) { A[k] = xu[k]; A[17 + k] = au[k]; A[133 + k] = ai[k]; }
#pragma unroll
  for (int k = 0; k < NI; ++k) A[34 + k] = xi[k];
  const float one = valid ? 1.f : 0.f;
  A[16] = one; A[33] = one; A[132] = one; A[149] = one;
  float* G = Gs[t];
#pragma unroll
  for (int o = 0; o < E; ++o) { G[o] = dhu[o]; G[E + o] = du[o]; G[2 * E + o] = dhi[o]; G[3 * E + o] = di[o]; }
  // block loss sum
  for (int off = 32; off > 0; off >>= 1) loss += __shfl_xor(loss, off);
  if ((t & 63) == 0) red[t >> 6] = loss;
  __syncthreads();
  float* prow = a.part + (int64_t)blockIdx.x * TT_PART_LD;
  if (t == 0) {
    float l = 0.f;
    for (int w = 0; w < SPB / 64; ++w) l += red[w];
    prow[NP] = l;
  }
  // weight gradient: unit = (row r, 4 columns c4)
  for (int unit = t; unit < AROWS * 4; unit += SPB) {
    const int r = unit >> 2, c4 = (unit & 3) * 4;
    const int grp = r < 17 ? 0 : (r < 34 ? 1 : (r < 133 ? 2 : 3));
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < SPB; ++q) {
      const float av = As[q][r];
      const float4 g = *(const float4*)(&Gs[q][grp * E + c4]);
      acc.x = fmaf(av, g.x, acc.x);
      acc.y = fmaf(av, g.y, acc.y);
      acc.z = fmaf(av, g.z, acc.z);
      acc.w = fmaf(av, g.w, acc.w);
    }
    *(float4*)(prow + r * E + c4) = acc;
  }
}

}  // namespace

int two_tower_parts(int B) { return (B + SPB - 1) / SPB; }

void two_tower(const TwoTowerArgs& a, int train, hipStream_t s) {
  if (a.B <= 0) return;
  const int grid = two_tower_parts(a.B);
  if (train && a.half)
    hipLaunchKernelGGL((two_tower_kernel<true, true>), dim3(grid), dim3(SPB), 0, s, a);
  else if (train)
    hipLaunchKernelGGL((two_tower_kernel<true, false>), dim3(grid), dim3(SPB), 0, s, a);
  else if (a.half)
    hipLaunchKernelGGL((two_tower_kernel<false, true>), dim3(grid), dim3(SPB), 0, s, a);
  else
    hipLaunchKernelGGL((two_tower_kernel<false, false>), dim3(grid), dim3(SPB), 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
