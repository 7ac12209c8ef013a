#!/bin/bash
# interaction samples-per-wave A/B (TDFO_INTER_SPW, isolated kernel trace) + W=1 bench
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ispw; mkdir -p $O
for spw in 1 2 4 8; do
  TDFO_INTER_SPW=$spw timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt$spw -o run --output-format csv -- python3 $R/scripts/inter_probe.py 20 > $O/kt$spw.log 2>&1
  echo "spw=$spw"; python3 $R/scripts/prof_summary.py $(ls $O/kt$spw/*kernel_trace.csv | head -1) --steps 20 | sed -n 2,3p
done
cd $R
for spw in 2 4; do
  TDFO_INTER_SPW=$spw timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/w1_$spw.log 2>&1
  echo "w1 spw=$spw $(tail -1 $O/w1_$spw.log | grep -o '"ms_per_step": [0-9.]*')"
done
