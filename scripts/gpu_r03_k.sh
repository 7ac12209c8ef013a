#!/bin/bash
# kernel change check: interaction tests, W=1 bench, W=1 kernel profile
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_comm.py -x -q -k "interaction or stream_graphs" --timeout 200 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > $O/w1.log 2>&1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --emulate-world 8 > $O/w8.log 2>&1
OUT=$O/prof_w1 STEPS=20 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh bench.py --steps 20 --warmup 6 > $O/prof_w1.txt 2>&1
