#!/bin/bash
# rocprofv3 kernel trace + per-kernel summary of an arbitrary python script.
# usage: OUT=gpurun_out/prof_x STEPS=N bash scripts/profile_cmd.sh script.py args...
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=${OUT:-gpurun_out/prof_cmd}
mkdir -p $OUT
SCRIPT=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT -o run -- python3 $ROOT/$SCRIPT "$@" > $ROOT/$OUT/run.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || { tail -20 $ROOT/$OUT/run.log; exit $rc; }
python3 $ROOT/scripts/prof_summary.py $(ls $ROOT/$OUT/*kernel_trace.csv | head -1) --steps ${STEPS:-1} > $ROOT/$OUT/summary.txt
head -30 $ROOT/$OUT/summary.txt
