// Bert4Rec evaluation scoring + ranking metrics (K20 in SURVEY.md §2.3;
// reference torchrec/train.py:52-78: scores = h . W[cand] + b[cand] over
// 1 positive + negatives, rank of the positive, Recall@k / NDCG@k).
//
// One wave per sample: lane c gathers candidate row W[cand[b, c]] (E <= 64
// fp32, float4 loads) and scores it against the sample's hidden state, which
// every lane reads as one broadcast row. The positive's 0-based rank is the
// ballot count of negatives scoring >= it (ties rank the positive behind:
// pessimistic, the same rule as tdfo_amd.models.bert4rec.recall_ndcg_sums).
// Each block writes its metric partials [Recall@K... | NDCG@K... | count]
// in fixed sample order and reduce_rows sums the blocks in order: no
// [B, C] score tensor, no atomics, deterministic.
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {
namespace {

constexpr int RK_WAVES = 4;

template <int E>
__global__ __launch_bounds__(64 * RK_WAVES) void rank_metrics_kernel(
    const float* __restrict__ h, const float* __restrict__ W, const float* __restrict__ bias,
    const int64_t* __restrict__ cand, int B, int C, int nk, RankKs ks,
    float* __restrict__ part) {
  static_assert(E % 4 == 0 && E <= 64, "E");
  constexpr int Q = E / 4;
  __shared__ float red[RK_WAVES][2 * 8 + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc[2 * 8 + 1];
#pragma unroll
  for (int q = 0; q < 2 * 8 + 1; ++q) acc[q] = 0.f;
  const int nw = gridDim.x * RK_WAVES;
  for (int b = blockIdx.x * RK_WAVES + w; b < B; b += nw) {
    float4 hv[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) hv[q] = *(const float4*)(h + (int64_t)b * E + 4 * q);
    const int64_t* cb = cand + (int64_t)b * C;
    float s0 = 0.f;
    int ahead = 0;
    for (int c0 = 0; c0 < C; c0 += 64) {
      const int c = c0 + lane;
      float sc = -INFINITY;
      if (c < C) {
        const int64_t id = cb[c];
        const float* wr = W + id * E;
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const float4 v = *(const float4*)(wr + 4 * q);
          s = fmaf(v.x, hv[q].x, s); s = fmaf(v.y, hv[q].y, s);
          s = fmaf(v.z, hv[q].z, s); s = fmaf(v.w, hv[q].w, s);
        }
        sc = s + bias[id];
      }
      if (c0 == 0) s0 = __shfl(sc, 0);
      const bool neg_ahead = c < C && c > 0 && sc >= s0;
      ahead += __popcll(__ballot(neg_ahead));
    }
    if (lane == 0) {
      const float r = (float)ahead;
      const float g = 1.f / log2f(r + 2.f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (k < nk && ahead < ks.k[k]) {
          acc[k] += 1.f;
          acc[8 + k] += g;
        }
      }
      acc[16] += 1.f;
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < 17; ++q) red[w][q] = acc[q];
  }
  __syncthreads();
  if (threadIdx.x < 2 * nk + 1) {
    const int q = threadIdx.x;
    const int src = q < nk ? q : (q < 2 * nk ? 8 + (q - nk) : 16);
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < RK_WAVES; ++v) s += red[v][src];
    part[(int64_t)blockIdx.x * (2 * nk + 1) + q] = s;
  }
}

}  // namespace

int rank_metrics_parts(int B) {
  const int b = (B + RK_WAVES - 1) / RK_WAVES;
  return b < 1024 ? (b < 1 ? 1 : b) : 1024;
}

void rank_metrics(const float* h, const float* W, const float* bias, const int64_t* cand, int B,
                  int C, int E, const RankKs& ks, int nk, float* part, float* out,
                  hipStream_t s) {
  if (B <= 0) return;
  if (nk < 1 || nk > 8) throw std::runtime_error("rank_metrics: 1..8 cutoffs");
  const int nb = rank_metrics_parts(B);
#define TDFO_RK(EE)                                                                   \
  hipLaunchKernelGGL(rank_metrics_kernel<EE>, dim3(nb), dim3(64 * RK_WAVES), 0, s, h, W, \
                     bias, cand, B, C, nk, ks, part)
  switch (E) {
    case 16: TDFO_RK(16); break;
    case 32: TDFO_RK(32); break;
    case 64: TDFO_RK(64); break;
    default: throw std::runtime_error("rank_metrics: E must be 16, 32 or 64");
  }
#undef TDFO_RK
  TDFO_CHECK_HIP(hipGetLastError());
  reduce_rows(part, nb, 2 * nk + 1, 2 * nk + 1, out, 0, 1.f, s);
}

}  // namespace tdfo
