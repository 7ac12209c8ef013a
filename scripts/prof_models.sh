#!/bin/bash
# rocprofv3 kernel-trace passes over the secondary workloads (TwoTower,
# Bert4Rec, DCN-v2); CSVs under gpurun_out/prof_<name>/.
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$name -o run --output-format csv -- python3 "$@" > $R/gpurun_out/prof_$name.log 2>&1
  echo "$name rc=$?"
}
run two_tower $R/scripts/bench_two_tower.py --steps 50 --warmup 10 &&
run bert4rec $R/scripts/bench_bert4rec.py --steps 50 --warmup 10 &&
run dcnv2 $R/bench.py --model dcnv2 --steps 10 --warmup 3
