#!/bin/bash
# Native RCCL comm layer + whole-step multi-rank graph: GPU tests, 1-GPU
# bench, emulated W=2/8 (whole graph vs staged).
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_multirank.py -x -v -k "comm or data_parallel or auto" --timeout 300 --timeout-method thread > $O/t_comm.log 2>&1
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > $O/w1.log 2>&1
for W in 2 8; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --emulate-world $W > $O/w$W.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --emulate-world 8 --no-stream-graphs > $O/w8_staged.log 2>&1
OUT=gpurun_out/r03c/prof_w8 STEPS=20 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh bench.py --steps 20 --warmup 6 --emulate-world 8 > $O/prof_w8.txt 2>&1
python3 scripts/step_timeline.py $(ls gpurun_out/r03c/prof_w8/*kernel_trace.csv | head -1) > $O/timeline_w8.txt 2>&1
