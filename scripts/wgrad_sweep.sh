#!/bin/bash
# A/B of the weight-grad variants on MI355X: fused bias column sums (csum) vs
# the bias column inside N, over split-K block targets; per-GEMM times
# (graph-replayed) and the full DLRM-1TB step.
set -u
O=gpurun_out/sweep; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > $O/t.log 2>&1 || exit 1
for cs in ${CSS:-1 0}; do for t in ${TARGETS:-256 512}; do
  export TDFO_WGRAD_CSUM=$cs TDFO_WGRAD_TARGET=$t
  timeout -k 10 200 python -u scripts/gemm_step_bench.py --policies 0 --only wgrad > $O/wg_${cs}_$t.jsonl 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > $O/b_${cs}_$t.log 2>&1 || exit 1
done; done
