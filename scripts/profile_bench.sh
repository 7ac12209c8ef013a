#!/bin/bash
# rocprofv3 kernel trace of the headline bench (eager, so every kernel is a
# separate dispatch) + per-kernel summary. Run on the GPU box via gpurun.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=${OUT:-gpurun_out/prof_bench}
ARGS=${PROF_ARGS:---steps 10 --warmup 3 --no-graph}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/$OUT/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 $ROOT/scripts/prof_summary.py $(ls $ROOT/$OUT/*kernel_trace.csv | head -1) --steps ${PROF_STEPS:-13} > $ROOT/$OUT/summary.txt
cat $ROOT/$OUT/summary.txt
