// Device side of tdfo::reduce_adam, shared by its own kernel (loss.hip) and
// the side blocks of the one-hot embedding sort (embedding.hip).
#pragma once
#include "tdfo_common.h"
#include "tdfo_kernels.h"

namespace tdfo {

// One thread's share of a fixed-order column sum over nparts partial rows:
// rows ph, ph + PH, ... in groups of four into s0..s3 (a partial last group
// into s0), returned as (s0 + s1) + (s2 + s3) -- reduce_rows_kernel's loop,
// with the first PRE rows loaded up front at clamped addresses and then added
// in that order, so the sums are the plain loop's with one round trip for up
// to PRE * PH = 512 partial rows (B = 8192) instead of one per group.
template <int PH>
__device__ __forceinline__ float col_phase_sum(const float* __restrict__ part, int nparts,
                                               int ld, int j, int ph) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  constexpr int PRE = 32;
  float v[PRE];
#pragma unroll
  for (int q = 0; q < PRE; ++q) {
    const int r = min(ph + q * PH, nparts - 1);
    v[q] = part[(int64_t)r * ld + j];
  }
#pragma unroll
  for (int g = 0; g < PRE / 4; ++g) {
    const int r = ph + 4 * g * PH;
    if (r + 3 * PH < nparts) {
      s0 += v[4 * g]; s1 += v[4 * g + 1]; s2 += v[4 * g + 2]; s3 += v[4 * g + 3];
    } else {
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (r + q * PH < nparts) s0 += v[4 * g + q];
    }
  }
  int r = ph + PRE * PH;
  if (r < nparts) {
    // (more than PRE * PH rows: every group above was full)
    for (; r + 3 * PH < nparts; r += 4 * PH) {
      s0 += part[(int64_t)r * ld + j];
      s1 += part[(int64_t)(r + PH) * ld + j];
      s2 += part[(int64_t)(r + 2 * PH) * ld + j];
      s3 += part[(int64_t)(r + 3 * PH) * ld + j];
    }
    for (; r < nparts; r += PH) s0 += part[(int64_t)r * ld + j];
  }
  return (s0 + s1) + (s2 + s3);
}

constexpr int RA_COLS = 16;                  // columns per 256-thread unit
constexpr int RA_PH = 256 / RA_COLS;         // row phases per column

// 256-thread work units of a reduce_adam: one per 16 columns (n + 1 of them:
// the parameters and the loss), plus one for the AUC binning
__host__ __device__ inline int reduce_adam_units(const ReduceAdamArgs& a) {
  return (a.n + 1 + RA_COLS - 1) / RA_COLS + (a.hist != nullptr ? 1 : 0);
}

// Unit `unit` run by 256 threads (ltid) of a block: 16 columns' fixed-order
// sums + Adam step (+ the loss), or the AUC binning (auc_hist_kernel's LDS
// counts, one integer atomic per non-empty bucket), or nothing (unit past the
// end). EVERY path passes exactly two block barriers, so several units can
// share a block (red: this unit's [RA_PH][RA_COLS] LDS; lh: 2 * nb LDS
// counters, used by the AUC unit only).
__device__ __forceinline__ void reduce_adam_unit(const ReduceAdamArgs& a, int unit, int ltid,
                                                 float (*red)[RA_COLS], unsigned int* lh) {
  const int ncol = (a.n + 1 + RA_COLS - 1) / RA_COLS;
  if (unit < ncol) {
    const int c = ltid % RA_COLS, ph = ltid / RA_COLS;
    const int j = unit * RA_COLS + c;
    red[ph][c] = (j <= a.n && a.nparts > 0) ? col_phase_sum<RA_PH>(a.part, a.nparts, a.ld, j, ph)
                                            : 0.f;
    __syncthreads();
    if (ph == 0 && j <= a.n) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < RA_PH; ++q) t += red[q][c];
      a.grad[j] = t;
      if (j == a.n) {
        a.loss_acc[0] += (double)t;
      } else {
        const float lr = a.hyper[0], step = a.hyper[1], gs = a.hyper[2];
        const float bc1 = 1.f - powf(a.beta1, step), bc2 = 1.f - powf(a.beta2, step);
        float p = a.p[j], m = a.m[j], v = a.v[j];
        adam_elem(p, t * gs, m, v, lr, bc1, bc2, a.beta1, a.beta2, a.eps, a.wd, a.adamw != 0);
        a.p[j] = p;
        a.m[j] = m;
        a.v[j] = v;
      }
    }
    __syncthreads();
  } else if (unit == ncol && a.hist != nullptr) {
    for (int i = ltid; i < 2 * a.nb; i += 256) lh[i] = 0;
    __syncthreads();
    for (int i = ltid; i < a.nlog; i += 256) {
      const float pr = 1.f / (1.f + __expf(-a.logits[i]));
      int bkt = (int)(pr * a.nb);
      bkt = bkt < 0 ? 0 : (bkt >= a.nb ? a.nb - 1 : bkt);
      atomicAdd(&lh[(a.labels[i] > 0.5f ? a.nb : 0) + bkt], 1u);
    }
    __syncthreads();
    for (int i = ltid; i < 2 * a.nb; i += 256)
      if (lh[i]) atomicAdd(&a.hist[i], (unsigned long long)lh[i]);
  } else {
    __syncthreads();
    __syncthreads();
  }
}

// head_reduce's work as 256-thread units (16 columns of [grad | loss] each,
// head_reduce_kernel's sums and order), for the side blocks of a GEMM launch;
// exactly one block barrier on every path
__host__ __device__ inline int head_reduce_units(const HeadReduceJob& j) {
  return (j.K + 2 + RA_COLS - 1) / RA_COLS;
}
__device__ __forceinline__ void head_reduce_unit(const HeadReduceJob& j, int unit, int ltid,
                                                 float (*red)[RA_COLS]) {
  const int ld = j.K + 2;
  const int c = ltid % RA_COLS, ph = ltid / RA_COLS;
  const int col = unit * RA_COLS + c;
  const bool live = unit < head_reduce_units(j);
  red[ph][c] = (live && col < ld && j.nparts > 0) ? col_phase_sum<RA_PH>(j.part, j.nparts, ld, col, ph)
                                                  : 0.f;
  __syncthreads();
  if (live && ph == 0 && col < ld) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < RA_PH; ++q) t += red[q][c];
    if (col <= j.K) j.grad[col] = t;
    else j.loss_acc[0] += t;
  }
  if (unit == 0 && ltid < j.bumps.n) j.bumps.p[ltid][1] += 1.f;
}

}  // namespace tdfo
