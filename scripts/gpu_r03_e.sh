#!/bin/bash
# embedding-kernel change check: embedding GPU tests, W=1 bench, W=1 profile + step timeline
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "emb or embedding or onehot or segsort or multirun" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > $O/w1.log 2>&1
tail -1 $O/w1.log | cut -c1-160
OUT=$O/prof_w1 STEPS=20 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh bench.py --steps 20 --warmup 6 > $O/prof_w1.txt 2>&1
python scripts/step_timeline.py $O/prof_w1/run_kernel_trace.csv -3 60 > $O/tl.txt
cat $O/tl.txt
