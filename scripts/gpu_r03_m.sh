#!/bin/bash
# DCN-v2 on 256x128 tiles (policy 5): GEMM + DCN tests, same-box A/B vs round-2 tree and policy 0
set -e
export PYTHONUNBUFFERED=1
R=$PWD; O=$R/gpurun_out/r03m; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm or dcn or graph_replay" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for rep in 1 2; do
  (cd _r2 && timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 > $O/r2_dcn.log 2>&1)
  echo "r2 dcn $(tail -1 $O/r2_dcn.log | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 --data pool > $O/r3_dcn.log 2>&1
  echo "r3 dcn pool $(tail -1 $O/r3_dcn.log | grep -o '"ms_per_step": [0-9.]*')"
  TDFO_GEMM_POLICY=0 timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 --data pool > $O/r3_dcn0.log 2>&1
  echo "r3 dcn pool p0 $(tail -1 $O/r3_dcn0.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 > $O/r3_dcn_fresh.log 2>&1
echo "r3 dcn fresh $(tail -1 $O/r3_dcn_fresh.log | grep -o '"ms_per_step": [0-9.]*')"
