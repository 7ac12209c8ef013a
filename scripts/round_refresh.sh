#!/bin/bash
# Round-end style refresh on one MI355X: full GPU test suite, then the
# headline and secondary benches, then a kernel-trace profile of the step.
set -u
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/refresh}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -x -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > $O/bench_1tb.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --rows kaggle > $O/bench_kaggle.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --host-data > $O/bench_1tb_host.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --model dcnv2 > $O/bench_dcn.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/bench_two_tower.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/bench_bert4rec.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_bert4rec.py --batch 256 > $O/bench_bert4rec_b256.log 2>&1 || exit 1
for f in $O/bench_*.log; do echo "$f: $(tail -1 $f | cut -c1-220)"; done
