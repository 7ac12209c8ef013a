#!/bin/bash
# Multi-rank (2 ranks sharing the GPU over gloo) tests incl. the pipelined
# input dist, DCN policy A/B, and graph-queue env A/B.
set -u
O=gpurun_out/pipe; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py > $O/t.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or dcn or dlrm" > $O/t2.log 2>&1 || exit 1
rm -rf gpurun_out/ab
AB_VAR=TDFO_GEMM_POLICY AB_VALS="2 25" AB_REPS=2 AB_STEPS=30 AB_ARGS="--model dcnv2" bash scripts/bench_ab.sh > /dev/null || exit 1
mv gpurun_out/ab gpurun_out/ab_dcnpol
AB_VAR=DEBUG_HIP_FORCE_GRAPH_QUEUES AB_VALS="0 2 4" AB_REPS=2 bash scripts/bench_ab.sh > /dev/null
