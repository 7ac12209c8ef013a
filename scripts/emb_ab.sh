#!/bin/bash
# Multi-hot embedding forward: numerics + old/new library A/B + DCN-v2 step.
set -u
O=gpurun_out/emb; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "emb or embedding or dcn" > $O/t.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bench_emb_fwd.py > $O/new.jsonl 2>&1 || exit 1
TDFO_LIB_PATH=$PWD/tdfo_amd/lib/ab/libtdfo_hip_old.so timeout -k 10 200 python -u scripts/bench_emb_fwd.py > $O/old.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --model dcnv2 --steps 20 --warmup 3 > $O/dcn_new.log 2>&1 || exit 1
TDFO_LIB_PATH=$PWD/tdfo_amd/lib/ab/libtdfo_hip_old.so timeout -k 10 300 python -u bench.py --model dcnv2 --steps 20 --warmup 3 > $O/dcn_old.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_step_bench.py --model dcnv2 --policies 2,0 > $O/gemm_dcn.jsonl 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_bert4rec.py > $O/t_b4r.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_new.log 2>&1 || exit 1
TDFO_LIB_PATH=$PWD/tdfo_amd/lib/ab/libtdfo_hip_old.so timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_old.log 2>&1
