#!/bin/bash
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread > $O/t_comm.log 2>&1
tail -1 $O/t_comm.log
for P in none M EC M,EC none M; do
  TDFO_MR_PRIO=$P timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --emulate-world 8 > $O/prio_$P.log 2>&1
  echo "$P $(tail -1 $O/prio_$P.log | cut -c1-120)"
done
