#!/bin/bash
# 256x128 GEMM kernel back: GEMM tests, DCN-v2 policy A/B
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for rep in 1 2; do
for p in 0 3 5; do
  TDFO_GEMM_POLICY=$p timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 > $O/dcn_p$p.log 2>&1
  echo "policy $p $(tail -1 $O/dcn_p$p.log | cut -c150-200)"
done
done
