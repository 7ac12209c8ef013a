#!/bin/bash
# same-box kernel profiles of DCN-v2: round-2 tree vs this tree (pool data)
set -e
R=$PWD; O=gpurun_out/r03l; mkdir -p $O
(cd _r2 && OUT=../$O/prof_r2 STEPS=13 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh bench.py --model dcnv2 --steps 10 --warmup 3 > ../$O/prof_r2.txt 2>&1)
OUT=$O/prof_r3 STEPS=13 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh bench.py --model dcnv2 --steps 10 --warmup 3 --data pool > $O/prof_r3.txt 2>&1
python scripts/step_timeline.py $O/prof_r3/run_kernel_trace.csv -3 60 > $O/tl_r3.txt
python scripts/step_timeline.py $O/prof_r2/run_kernel_trace.csv -3 60 > $O/tl_r2.txt
head -3 $O/tl_r2.txt $O/tl_r3.txt
