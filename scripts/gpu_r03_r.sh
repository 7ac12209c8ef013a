#!/bin/bash
# zero-slot S operand (interaction bwd) check + one-GPU segment timeline + W=1 bench
set -e
export PYTHONUNBUFFERED=1
R=$PWD; O=$R/gpurun_out/r03r2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "interaction or graph_replay" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
(cd /tmp && TMPDIR=/tmp timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/scripts/inter_probe.py 20 > $O/kt.log 2>&1)
python3 scripts/prof_summary.py $(ls $O/kt/*kernel_trace.csv | head -1) --steps 20 | sed -n 2,3p
timeout -k 10 200 python -u scripts/w1_timeline.py > $O/tl.log 2>&1
cat $O/tl.log
for r in 1 2; do timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/w1.log 2>&1; echo "w1 $(tail -1 $O/w1.log | grep -o '"ms_per_step": [0-9.]*')"; done
