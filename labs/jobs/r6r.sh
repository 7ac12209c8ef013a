set -u
O=gpurun_out/r06/r; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_two_tower.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in 1 0; do
TDFO_TT_FORK=$v timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt_${v}_$k.log 2>&1 || { echo "tt rc=$?"; tail -5 $O/tt_${v}_$k.log; exit 1; }
echo "fork=$v $k $(tail -n 1 $O/tt_${v}_$k.log)"
done; done
