#!/bin/bash
# staged batches in the per-stream graphs: replay tests, timeline, W=1 bench (fresh / host / pool)
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_data.py -x -q -k "graph_replay or dlrm or data" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python -u scripts/w1_timeline.py fresh > $O/tl_fresh.log 2>&1; tail -8 $O/tl_fresh.log
for r in 1 2; do for d in fresh host pool; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --data $d > $O/w1_$d.log 2>&1
  echo "w1 $d $(tail -1 $O/w1_$d.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
