#!/bin/bash
# Emulated multi-rank step on one GPU (bench.py --emulate-world W) + the
# RCCL issue-cost microbench + a kernel trace of the emulated W=8 step.
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/emu; mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > $O/w1.log 2>&1
for W in 2 4 8; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --emulate-world $W > $O/w$W.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --emulate-world 8 --no-pipeline > $O/w8_nopipe.log 2>&1
timeout -k 10 120 python -u scripts/rccl_issue_cost.py > $O/rccl_cost.log 2>&1
OUT=$O/prof_w8 STEPS=20 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh bench.py --steps 20 --warmup 5 --emulate-world 8 > $O/prof_w8.txt 2>&1
