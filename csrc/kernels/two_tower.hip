// Fused TwoTower towers + row-wise dot + BCE + full backward (gfx950).
//
// Model (reference jax-flax/models.py:72-102, tensorflow2/models.py:43-71):
//   u = fc2_u(swish(fc1_u(e_user)))                       16 -> 16 -> 16
//   i = fc2_i(swish(fc1_i([e_item e_lang e_ebook e_fmt e_pub e_dec avg pages])))
//                                                          98 -> 16 -> 16
//   logit = sum(u * i); loss = BCE-with-logits(logit, label)
//
// Every product is a 16-wide fp32 matmul, run on the exact-f32 matrix cores
// (v_mfma_f32_16x16x4_f32: a k-ordered fmaf chain, cdna_hip_programming.md
// §3 'FP32-input MFMA') with one wave per 16 samples, in a transposed
// layout: every activation / gradient tile is [16 features][16 samples] in
// the accumulator (lane l: samples l&15, features 4(l>>4)+r in register r),
// which is exactly the B operand the next layer needs (register r feeds the
// MFMA of k-step r), so forward, backward and input gradients chain in
// registers with no data movement; weights are broadcast from LDS. Weight
// gradients (sums over samples) read the tiles back from a per-wave LDS
// stage, are reduced over the block's waves in LDS and written as one
// partial row per block (reduced in a fixed order by tdfo::reduce_rows:
// deterministic, no atomics). One wave per block: B = 2048 is 128 blocks
// (64-sample blocks of 4 waves: 19.7 us, 32 blocks). Embedding gradients are
// written per sample (dX) for the sort-based fused sparse optimizer
// (embedding.hip). (The one-thread-per-sample VALU kernel this replaces
// took 38.8 us at B = 2048, 16 blocks: profiles/r05/two_tower/.) Optionally
// the optimizers' step counters are bumped here too (no bump launch), and
// tdfo::reduce_adam sums the partial rows straight into the AdamW step (and
// bins the logits for the AUC in a block of its own). Binning the logits here
// with global atomics cost 7 us: at init every logit lands in one bucket.
//
// Parameter layout (flat fp32, Flax kernel convention W[in][out]):
//   [uW1 16x16 | ub1 16 | uW2 16x16 | ub2 16 | iW1 98x16 | ib1 16 | iW2 16x16 | ib2 16]
#include "tdfo_two_tower_dev.h"

namespace tdfo {
namespace {

template <bool TRAIN, bool HALF>
__global__ __launch_bounds__(64) void two_tower_kernel(TwoTowerArgs a) {
  __shared__ tt::Smem<1> sm;
  tt::tower_block<TRAIN, HALF, 1, false>(a, blockIdx.x, threadIdx.x, sm);
}

}  // namespace

int two_tower_parts(int B) { return (B + tt::SPB - 1) / tt::SPB; }

void two_tower(const TwoTowerArgs& a, int train, hipStream_t s) {
  if (a.B <= 0) return;
  const int grid = two_tower_parts(a.B);
  const dim3 blk(64);
  if (train && a.half)
    hipLaunchKernelGGL((two_tower_kernel<true, true>), dim3(grid), blk, 0, s, a);
  else if (train)
    hipLaunchKernelGGL((two_tower_kernel<true, false>), dim3(grid), blk, 0, s, a);
  else if (a.half)
    hipLaunchKernelGGL((two_tower_kernel<false, true>), dim3(grid), blk, 0, s, a);
  else
    hipLaunchKernelGGL((two_tower_kernel<false, false>), dim3(grid), blk, 0, s, a);
  TDFO_CHECK_HIP(hipGetLastError());
}

}  // namespace tdfo
