#!/bin/bash
# one-GPU segment timelines: fresh vs pool data, ids stream on/off
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 200 python -u scripts/w1_timeline.py fresh > $O/tl_fresh.log 2>&1; tail -9 $O/tl_fresh.log
timeout -k 10 200 python -u scripts/w1_timeline.py pool > $O/tl_pool.log 2>&1; tail -9 $O/tl_pool.log
timeout -k 10 200 python -u scripts/w1_timeline.py fresh '{"ids_stream": false}' > $O/tl_noids.log 2>&1; tail -9 $O/tl_noids.log
