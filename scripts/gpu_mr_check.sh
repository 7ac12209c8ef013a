#!/bin/bash
# multi-rank stream graphs: tests, emulated W=2/4/8 benches, segment timeline
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread > $O/t_comm.log 2>&1
tail -1 $O/t_comm.log
for W in 2 4 8; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --emulate-world $W > $O/emu_w$W.log 2>&1
  echo "W=$W $(tail -1 $O/emu_w$W.log | cut -c1-130)"
done
timeout -k 10 300 python -u scripts/mr_timeline.py > $O/mr_tl.log 2>&1
tail -4 $O/mr_tl.log
