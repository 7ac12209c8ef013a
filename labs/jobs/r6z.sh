# Narrow-row update chunk size A/B (32 default vs 16 vs 8 entries per wave).
set -u
O=gpurun_out/r06/z; rm -rf $O; mkdir -p $O
for c in 16 8; do
TDFO_LIB_PATH=$PWD/labs/ab/libtdfo_hip_ch$c.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_two_tower.py tests/test_gpu_kernels.py -k "two_tower or embedding" > $O/tests_$c.log 2>&1 || { echo "tests $c rc=$?"; tail -30 $O/tests_$c.log; exit 1; }
tail -1 $O/tests_$c.log
done
for k in 1 2; do
for c in 32 16 8; do
L=""; [ $c != 32 ] && L=$PWD/labs/ab/libtdfo_hip_ch$c.so
TDFO_LIB_PATH=$L timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt_${c}_$k.log 2>&1 || { echo "tt rc=$?"; tail -5 $O/tt_${c}_$k.log; exit 1; }
TDFO_LIB_PATH=$L timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${c}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${c}_$k.log; exit 1; }
echo "ch=$c $k tt $(tail -n 1 $O/tt_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*') b4r $(tail -n 1 $O/b4r_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
