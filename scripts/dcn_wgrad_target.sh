#!/bin/bash
# DCN-v2 weight-grad split targets on the real step shapes (policy 25).
set -o pipefail
mkdir -p gpurun_out/dcnwg
for t in ${TARGETS:-256 512 768 1024}; do
  TDFO_WGRAD_TARGET=$t timeout -k 10 240 python scripts/gemm_step_bench.py --model dcnv2 \
    --policies 25 --only "${ONLY:-wgrad}" > gpurun_out/dcnwg/t$t.jsonl 2>&1 || exit $?
done
