#!/bin/bash
# Per-stream hipGraphs (TDFO_STREAM_GRAPHS=1) vs one whole-step graph:
# numerics check (GPU DLRM tests) and interleaved bench A/B.
set -u
O=gpurun_out/streams; mkdir -p $O
TDFO_STREAM_GRAPHS=${SG_TEST:-1} timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dlrm or graph" > $O/t.log 2>&1 || exit 1
rm -rf gpurun_out/ab
AB_VAR=TDFO_STREAM_GRAPHS AB_VALS="${SG_VALS:-0 1}" AB_REPS=3 bash labs/bench_ab.sh > /dev/null || exit 1
mv gpurun_out/ab gpurun_out/ab_streams
AB_VAR=TDFO_STREAM_GRAPHS AB_VALS="${SG_VALS:-0 1}" AB_REPS=2 AB_STEPS=30 AB_ARGS="--model dcnv2" bash labs/bench_ab.sh > /dev/null
