#!/bin/bash
# one-GPU config A/B with staged batches: dense-optimizer placement, deferred top wgrads
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 600 python -u scripts/cfg_ab.py '{"opt_placement": "one_pass"}' '{"opt_placement": "split_main"}' '{"defer_wgrad": true}' > $O/ab.log 2>&1
tail -3 $O/ab.log
