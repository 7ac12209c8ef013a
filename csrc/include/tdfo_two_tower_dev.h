// Device side of the fused TwoTower step (two_tower.hip's kernel, and the
// tower blocks co-launched with the one-hot embedding sort in embedding.hip).
// See two_tower.hip for the design notes.
#pragma once
#include <hip/hip_fp16.h>

#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace tt {

constexpr int E = 16;
constexpr int NI = 98;          // item tower input width
constexpr int WS = 16;          // samples per wave
constexpr int SPB = WS;        // samples per partial row (= ops.reference.TT_SPB)
constexpr int NP = 150 * E;     // 2400 parameters
constexpr int XLD = 116;        // staged sample row (114 used)
// parameter offsets
constexpr int O_UW1 = 0, O_UB1 = 256, O_UW2 = 272, O_UB2 = 528, O_IW1 = 544, O_IB1 = 2112,
              O_IW2 = 2128, O_IB2 = 2384;

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

__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <bool HALF>
__device__ __forceinline__ f32x4_t rnd4(f32x4_t v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = rnd<HALF>(v[r]);
  return v;
}

// per-wave LDS tiles [feature][sample] of the weight-gradient operands
enum { G_AU, G_DU, G_DHU, G_AI, G_DI, G_DHI, G_N };

// LDS of one tower block of NWV waves
template <int NWV>
struct Smem {
  float Wl[NP];
  float Xs[NWV][WS][XLD];
  float Gs[NWV][G_N][E][WS];
  __attribute__((aligned(16))) float Ps[NWV][NP];
  float red[NWV];
};
// block barriers every thread of a block running tower_block passes
// (threads of the block that run no tower wave must pass as many)
template <bool TRAIN>
constexpr int tower_barriers() { return TRAIN ? 3 : 1; }

// Tower block `blk`: NWV waves (threads t < 64 * NWV) on samples
// blk * 16 * NWV + 16 w ... Partial rows: one per block, waves summed in
// fixed order (ROWS_PER_WAVE = false), or one per wave at row blk * NWV + w
// (true): with either, NWV = 1 and NWV > 1 per-wave rows are the same rows.
template <bool TRAIN, bool HALF, int NWV, bool ROWS_PER_WAVE>
__device__ __forceinline__ void tower_block(const TwoTowerArgs& a, int blk, int t,
                                            Smem<NWV>& sm) {
  float* Wl = sm.Wl;
  float(*Xs)[WS][XLD] = sm.Xs;
  float(*Gs)[G_N][E][WS] = sm.Gs;
  float(*Ps)[NP] = sm.Ps;
  float* red = sm.red;
  const int lane = t & 63, w = t >> 6;
  const int j = lane & 15, g = lane >> 4;          // sample column / feature group
  {
    // weights to LDS: every float4 load issued before the first store (a
    // scalar strided loop waited on ~38 dependent loads per lane)
    static_assert(NP % 4 == 0, "float4 weight staging");
    constexpr int NV4 = NP / 4, PER = (NV4 + 64 * NWV - 1) / (64 * NWV);
    float4 wv[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = t + 64 * NWV * i;
      wv[i] = k < NV4 ? ((const float4*)a.P)[k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int k = t + 64 * NWV * i;
      if (k < NV4) {
        Wl[4 * k] = rnd<HALF>(wv[i].x);
        Wl[4 * k + 1] = rnd<HALF>(wv[i].y);
        Wl[4 * k + 2] = rnd<HALF>(wv[i].z);
        Wl[4 * k + 3] = rnd<HALF>(wv[i].w);
      }
    }
  }
  const int64_t s0 = ((int64_t)blk * NWV + w) * WS;
  float(*X)[XLD] = Xs[w];
  if (a.emb_w != nullptr) {
    // fused lookup: (sample, table) pairs p = lane, lane + 64 of the wave's
    // 16 x 7; both ids first, then 8 independent float4 row loads (two
    // round trips), rows straight into the staged X tile
    constexpr int NT = 7, NPAIR = WS * NT;
    int64_t row[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = lane + 64 * q;
      const int r = p / NT, t = p - r * NT;
      const int64_t sr = s0 + r;
      row[q] = (p < NPAIR && sr < a.B) ? a.row_off[t] + a.ids[(int64_t)t * a.B + sr] : -1;
    }
    float4 v[2][4];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[q][u] = row[q] >= 0 ? ((const float4*)(a.emb_w + row[q] * E))[u]
                              : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = lane + 64 * q;
      if (p < NPAIR) {
        const int r = p / NT, t = p - r * NT;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          X[r][t * E + 4 * u] = rnd<HALF>(v[q][u].x);
          X[r][t * E + 4 * u + 1] = rnd<HALF>(v[q][u].y);
          X[r][t * E + 4 * u + 2] = rnd<HALF>(v[q][u].z);
          X[r][t * E + 4 * u + 3] = rnd<HALF>(v[q][u].w);
        }
      }
    }
    if (lane < 2 * WS) {
      const int r = lane >> 1, c = 112 + (lane & 1);
      const int64_t sr = s0 + r;
      X[r][c] = sr < a.B ? rnd<HALF>(a.X[sr * a.ldx + c]) : 0.f;
    }
  } else {
    for (int idx = lane; idx < WS * 114; idx += 64) {
      const int r = idx / 114, c = idx - r * 114;
      const int64_t sr = s0 + r;
      X[r][c] = sr < a.B ? rnd<HALF>(a.X[sr * a.ldx + c]) : 0.f;
    }
  }
  __syncthreads();
  const float* uW1 = Wl + O_UW1;
  const float* uW2 = Wl + O_UW2;
  const float* iW1 = Wl + O_IW1;
  const float* iW2 = Wl + O_IW2;

  // ---- forward: H^T = W1^T X^T + b1 (rows: hidden feature 4g+r, cols: sample j)
  f32x4_t hu, hi;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    hu[r] = Wl[O_UB1 + 4 * g + r];
    hi[r] = Wl[O_IB1 + 4 * g + r];
  }
#pragma unroll
  for (int k0 = 0; k0 < E; k0 += 4) hu = mfma4(uW1[(k0 + g) * E + j], X[j][k0 + g], hu);
#pragma unroll
  for (int k0 = 0; k0 < 100; k0 += 4) {
    const int k = k0 + g;
    hi = mfma4(k < NI ? iW1[k * E + j] : 0.f, k < NI ? X[j][E + k] : 0.f, hi);
  }
  hu = rnd4<HALF>(hu);
  hi = rnd4<HALF>(hi);
  f32x4_t au, ai, u, iv;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    au[r] = rnd<HALF>(hu[r] * sigm(hu[r]));
    ai[r] = rnd<HALF>(hi[r] * sigm(hi[r]));
    u[r] = Wl[O_UB2 + 4 * g + r];
    iv[r] = Wl[O_IB2 + 4 * g + r];
  }
  // fc2: k-step r takes hidden feature 4g+r from lane group g (register r)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    u = mfma4(uW2[(4 * g + r) * E + j], au[r], u);
    iv = mfma4(iW2[(4 * g + r) * E + j], ai[r], iv);
  }
  u = rnd4<HALF>(u);
  iv = rnd4<HALF>(iv);
  float dot = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) dot = fmaf(u[r], iv[r], dot);
  dot += __shfl_xor(dot, 16, 64);
  dot += __shfl_xor(dot, 32, 64);
  const float logit = rnd<HALF>(dot);
  const int64_t s = s0 + j;
  const bool valid = s < a.B;
  if (valid && g == 0) a.logits[s] = logit;
  if constexpr (TRAIN) {
    // ---- loss + backward
    const float y = valid ? a.labels[s] : 0.f;
    if (blk == 0 && t < a.bumps.n) a.bumps.p[t][1] += 1.f;
    float loss = (valid && g == 0) ? fmaxf(logit, 0.f) - logit * y + log1pf(__expf(-fabsf(logit)))
                                   : 0.f;
    const float ls = a.loss_scale ? a.loss_scale[0] : 1.f;
    const float dl = valid ? rnd<HALF>((sigm(logit) - y) * a.inv_n * ls) : 0.f;
    f32x4_t du, di;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      du[r] = rnd<HALF>(dl * iv[r]);
      di[r] = rnd<HALF>(dl * u[r]);
    }
    // dA^T = W2 dY^T (rows: hidden feature, k-step r: output feature 4g+r)
    f32x4_t dau = {0.f, 0.f, 0.f, 0.f}, dai = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dau = mfma4(uW2[j * E + 4 * g + r], du[r], dau);
      dai = mfma4(iW2[j * E + 4 * g + r], di[r], dai);
    }
    f32x4_t dhu, dhi;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float su = sigm(hu[r]), si = sigm(hi[r]);
      dhu[r] = rnd<HALF>(dau[r] * su * (1.f + hu[r] * (1.f - su)));
      dhi[r] = rnd<HALF>(dai[r] * si * (1.f + hi[r] * (1.f - si)));
    }
    // embedding gradients dX^T = W1 dH^T: lane (g, j) holds dX[s][k0 + 4g .. +3]
    {
      f32x4_t d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) d = mfma4(uW1[j * E + 4 * g + r], dhu[r], d);
      if (valid)
        *(float4*)(a.dX + s * a.lddx + 4 * g) =
            make_float4(rnd<HALF>(d[0]), rnd<HALF>(d[1]), rnd<HALF>(d[2]), rnd<HALF>(d[3]));
    }
#pragma unroll
    for (int rb = 0; rb < 6; ++rb) {
      f32x4_t d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) d = mfma4(iW1[(rb * E + j) * E + 4 * g + r], dhi[r], d);
      if (valid)
        *(float4*)(a.dX + s * a.lddx + E + rb * E + 4 * g) =
            make_float4(rnd<HALF>(d[0]), rnd<HALF>(d[1]), rnd<HALF>(d[2]), rnd<HALF>(d[3]));
    }
    // ---- weight gradients of this wave's 16 samples: dW[k][o] = sum_s A[s][k] dY[s][o]
    float(*G)[E][WS] = Gs[w];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      G[G_AU][4 * g + r][j] = au[r];
      G[G_DU][4 * g + r][j] = du[r];
      G[G_DHU][4 * g + r][j] = dhu[r];
      G[G_AI][4 * g + r][j] = ai[r];
      G[G_DI][4 * g + r][j] = di[r];
      G[G_DHI][4 * g + r][j] = dhi[r];
    }
    __syncthreads();
    float* P = Ps[w];
    // k-step m sums samples 4m + g; result row k = 4g + r, column o = j
    auto wtile = [&](auto act, int dy, int base, int krows) {
      f32x4_t d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < 4; ++m) d = mfma4(act(4 * m + g), G[dy][j][4 * m + g], d);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < krows) P[base + (4 * g + r) * E + j] = d[r];
    };
    wtile([&](int sm) { return X[sm][j]; }, G_DHU, O_UW1, E);
    wtile([&](int sm) { return G[G_AU][j][sm]; }, G_DU, O_UW2, E);
    wtile([&](int sm) { return G[G_AI][j][sm]; }, G_DI, O_IW2, E);
#pragma unroll
    for (int kb = 0; kb < 7; ++kb)
      wtile([&](int sm) { return kb * E + j < NI ? X[sm][E + kb * E + j] : 0.f; }, G_DHI,
            O_IW1 + kb * E * E, NI - kb * E);
    {   // bias grads: lane (g, j) sums tile g's feature j over the samples
      const int src = g == 0 ? G_DHU : (g == 1 ? G_DU : (g == 2 ? G_DHI : G_DI));
      const int dst = g == 0 ? O_UB1 : (g == 1 ? O_UB2 : (g == 2 ? O_IB1 : O_IB2));
      float b = 0.f;
#pragma unroll
      for (int q = 0; q < WS; ++q) b += G[src][j][q];
      P[dst + j] = b;
    }
    const float lw = wave_sum(loss);
    if (lane == 0) red[w] = lw;
    __syncthreads();
    if constexpr (ROWS_PER_WAVE) {
      // this wave's own partial row (TT_PART_LD % 4 == 0); a wave past the
      // batch (the last block's tail) has no row: the buffer holds
      // two_tower_parts(B) of them
      if (s0 < a.B) {
        float* prow = a.part + ((int64_t)blk * NWV + w) * TT_PART_LD;
        for (int k = lane; k < NP / 4; k += 64)
          *(float4*)(prow + 4 * k) = *(const float4*)&P[4 * k];
        if (lane == 0) prow[NP] = lw;
      }
    } else {
      // block partial: fixed wave order
      float* prow = a.part + (int64_t)blk * TT_PART_LD;
      for (int k = t; k < NP / 4; k += 64 * NWV) {
        float4 v = *(const float4*)&Ps[0][4 * k];
#pragma unroll
        for (int q = 1; q < NWV; ++q) {
          const float4 u = *(const float4*)&Ps[q][4 * k];
          v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
        }
        *(float4*)(prow + 4 * k) = v;
      }
      if (t == 0) {
        float l = 0.f;
#pragma unroll
        for (int q = 0; q < NWV; ++q) l += red[q];
        prow[NP] = l;
      }
    }
  }
}


}  // namespace tt
}  // namespace tdfo
