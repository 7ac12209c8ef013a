#!/bin/bash
# dense-optimizer placement A/B on one GPU (side_top vs one_pass), graph-replay test
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "graph_replay_matches_eager" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python -u scripts/cfg_ab.py '{"opt_placement": "side_top"}' '{"opt_placement": "one_pass"}' > $O/ab.log 2>&1
tail -2 $O/ab.log
for d in pool fresh; do
  timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 --data $d > $O/dcn_$d.log 2>&1
  echo "dcn $d $(tail -1 $O/dcn_$d.log | cut -c150-200)"
done
