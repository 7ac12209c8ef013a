#!/bin/bash
# after the DCN mixin move: DCN / DLRM GPU tests + DCN bench
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multirank.py -x -q -k "dcn or dlrm or graph_replay" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 > $O/dcn.log 2>&1
echo "dcn $(tail -1 $O/dcn.log | grep -o '"ms_per_step": [0-9.]*')"
