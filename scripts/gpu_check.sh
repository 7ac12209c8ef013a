#!/bin/bash
# GPU-box check: kernel tests, short bench, optional rocprof stats.
# Stops at the first crash-like exit (fault/abort/timeout); test failures
# (exit 1) still let the bench run.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ok_or_fail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
  ok_or_fail $rc || exit $rc
fi
if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -20 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_PROF:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py ${PROF_ARGS:---steps 10 --warmup 3} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof.log
  exit $rc
fi
