# Embedding-row Adam on hardware sqrt / rcp (new) vs IEEE divisions (pre).
set -u
O=gpurun_out/r06/au; rm -rf $O; mkdir -p $O
TDFO_LIB_PATH=$PWD/labs/ab/libtdfo_hip_new.so timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2 3; do
for c in pre new; do
TDFO_LIB_PATH=$PWD/labs/ab/libtdfo_hip_$c.so timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${c}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${c}_$k.log; exit 1; }
TDFO_LIB_PATH=$PWD/labs/ab/libtdfo_hip_$c.so timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt_${c}_$k.log 2>&1 || { echo "tt rc=$?"; tail -5 $O/tt_${c}_$k.log; exit 1; }
echo "$c $k b16 $(tail -n 1 $O/b4r_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*') tt $(tail -n 1 $O/tt_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
