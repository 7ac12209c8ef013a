#!/bin/bash
# same-box A/B: round-2 tree (_r2, pool data) vs this tree (--data pool), DCN-v2 and DLRM-1TB
set -e
export PYTHONUNBUFFERED=1
R=$PWD; O=$R/gpurun_out/r03j; mkdir -p $O
for rep in 1 2; do
  (cd _r2 && timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 > $O/r2_dcn.log 2>&1)
  echo "r2 dcn $(tail -1 $O/r2_dcn.log | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 --data pool > $O/r3_dcn.log 2>&1
  echo "r3 dcn $(tail -1 $O/r3_dcn.log | grep -o '"ms_per_step": [0-9.]*')"
  (cd _r2 && timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > $O/r2_dlrm.log 2>&1)
  echo "r2 dlrm $(tail -1 $O/r2_dlrm.log | grep -o '"ms_per_step": [0-9.]*')"
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --data pool > $O/r3_dlrm.log 2>&1
  echo "r3 dlrm $(tail -1 $O/r3_dlrm.log | grep -o '"ms_per_step": [0-9.]*')"
done
