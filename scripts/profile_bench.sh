#!/bin/bash
# rocprofv3 kernel trace of the headline bench (graph replays: every kernel
# node is a dispatch in the trace) + a steady-state per-step summary. Run on
# the GPU box via gpurun.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=${OUT:-gpurun_out/prof_bench}
ARGS=${PROF_ARGS:---steps 30 --warmup 10}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT -o run -- python3 $ROOT/bench.py $ARGS > $ROOT/$OUT/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
# steady state: the last PROF_LAST steps between two dispatches of the
# once-per-step head kernel (1.0 calls/step for once-per-step kernels)
python3 $ROOT/scripts/prof_summary.py $(ls $ROOT/$OUT/*kernel_trace.csv | head -1) --marker ${PROF_MARKER:-head_bce} --last ${PROF_LAST:-20} > $ROOT/$OUT/summary.txt
cat $ROOT/$OUT/summary.txt
