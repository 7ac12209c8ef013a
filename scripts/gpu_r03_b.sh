#!/bin/bash
# bisect of the whole-step capture crash + multi-run one-hot backward (tests, A/B)
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "onehot" --timeout 120 --timeout-method thread > $O/t_onehot.log 2>&1
timeout -k 10 200 python -u scripts/bench_segsort.py > $O/segsort_ab.log 2>&1
timeout -k 10 700 python -u scripts/whole_capture_bisect.py > $O/bisect.log 2>&1
