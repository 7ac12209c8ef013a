#!/bin/bash
# Bert4Rec: one-launch step counters; tests, bench, kernel profile
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_bert4rec.py tests/test_gpu_two_tower.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u scripts/bench_bert4rec.py --steps 50 --warmup 10 > $O/bert4rec.log 2>&1
echo "bert4rec $(tail -1 $O/bert4rec.log | cut -c1-200)"
OUT=$O/prof_bert4rec STEPS=60 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh scripts/bench_bert4rec.py --steps 50 --warmup 10 > $O/prof.txt 2>&1
grep -n "at::native\|rocclr\|total" $O/prof_bert4rec/summary.txt || true
