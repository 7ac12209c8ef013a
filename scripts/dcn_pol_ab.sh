#!/bin/bash
set -u
O=gpurun_out/deep; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or dcn or dlrm" > $O/t2.log 2>&1 || exit 1
rm -rf gpurun_out/ab
AB_VAR=TDFO_GEMM_POLICY AB_VALS="2 25" AB_REPS=2 AB_STEPS=30 AB_ARGS="--model dcnv2" bash scripts/bench_ab.sh
