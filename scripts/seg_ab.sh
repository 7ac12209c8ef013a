#!/bin/bash
# 7- vs 6-bit segsort digits: numerics (new build), full-backward timing, DLRM bench, and the priority A/B.
set -u
O=gpurun_out/seg; mkdir -p $O
L=$PWD/tdfo_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "emb or embedding or dlrm" > $O/t.log 2>&1 || exit 1
TDFO_STREAM_PRIO=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dlrm or graph" > $O/t_prio.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bench_segsort.py > $O/seg7.jsonl 2>&1 || exit 1
TDFO_LIB_PATH=$L/ab/seg6.so timeout -k 10 200 python -u scripts/bench_segsort.py > $O/seg6.jsonl 2>&1 || exit 1
LIBS="seg7:$L/libtdfo_hip.so seg6:$L/ab/seg6.so" AB_REPS=2 AB_ARGS="--steps 100 --warmup 10" bash scripts/lib_ab.sh > /dev/null || exit 1
rm -rf gpurun_out/ab
AB_VAR=TDFO_STREAM_PRIO AB_VALS="0 1" AB_REPS=3 bash scripts/bench_ab.sh > /dev/null
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bert4rec.py > $O/t_b4r.log 2>&1
