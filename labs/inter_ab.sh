#!/bin/bash
# Interaction kernel numerics + samples-per-wave A/B (MI355X).
set -u
O=gpurun_out/inter; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "interaction or dlrm" > $O/t.log 2>&1 || exit 1
for spw in ${SPWS:-1 2 4}; do
  TDFO_INTER_SPW=$spw timeout -k 10 200 python -u scripts/bench_kernels.py --only none > $O/k_$spw.jsonl 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 > $O/bench.log 2>&1
