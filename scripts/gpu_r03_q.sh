#!/bin/bash
# interaction depth-2 prefetch A/B: correctness tests, isolated timing, W=1 bench (two library builds)
set -e
export PYTHONUNBUFFERED=1
R=$PWD; O=$R/gpurun_out/r03q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "interaction" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
cd /tmp && export TMPDIR=/tmp
for v in d2; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o run --output-format csv -- python3 $R/scripts/inter_probe.py 20 > $O/kt_$v.log 2>&1
  echo "$v"; python3 $R/scripts/prof_summary.py $(ls $O/kt_$v/*kernel_trace.csv | head -1) --steps 20 | sed -n 2,3p
done
cd $R
for r in 1 2; do timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/w1.log 2>&1; echo "w1 $(tail -1 $O/w1.log | grep -o "\"ms_per_step\": [0-9.]*")"; done
