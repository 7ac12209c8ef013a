#!/bin/bash
# data-source event change: data GPU tests, W=1 bench fresh/pool/host, step timeline
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_data.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for d in "--data fresh" "--data pool" "--data host"; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 $d > $O/w1_${d#--data }.log 2>&1
  echo "$d $(tail -1 $O/w1_${d#--data }.log | cut -c100-200)"
done
OUT=$O/prof_w1 STEPS=20 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh bench.py --steps 20 --warmup 6 > $O/prof_w1.txt 2>&1
python scripts/step_timeline.py $O/prof_w1/run_kernel_trace.csv -3 60 > $O/tl.txt
cat $O/tl.txt
