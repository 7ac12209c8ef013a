#!/bin/bash
# interaction backward rework: tests, isolated timing + LDS counters, W=1 bench
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_comm.py -x -q -k "interaction or stream_graphs or dlrm" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash scripts/inter_pmc.sh > $O/pmc.txt 2>&1
head -4 $O/pmc.txt; grep -A7 "inter_bwd" $O/pmc.txt | grep "BANK\|IDX_ACTIVE\|INSTS_VALU\|INSTS_LDS" || true
for rep in 1 2; do
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/w1.log 2>&1
echo "w1 $(tail -1 $O/w1.log | grep -o '"ms_per_step": [0-9.]*')"
done
