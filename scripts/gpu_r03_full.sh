#!/bin/bash
# full GPU suite + smoke + W=1 bench (round-end rehearsal)
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03t2; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_all.log 2>&1 || { tail -40 $O/gpu_all.log; exit 1; }
tail -3 $O/gpu_all.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1
tail -1 $O/bench_default.log | cut -c1-400
