#!/bin/bash
# Deep-pipelined 128x128 GEMM: numerics, then per-GEMM step A/B on DLRM and DCN-v2.
set -u
O=gpurun_out/deep; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > $O/t.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_step_bench.py --model dcnv2 --policies 2,23,24 > $O/dcn.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_step_bench.py --policies 0,23,24 > $O/dlrm.jsonl 2>&1 || exit 1
