set -u
O=gpurun_out/r06/fin2; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
