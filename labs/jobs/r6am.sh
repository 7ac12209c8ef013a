# Encoder block kernels: 256 vs 512 vs 1024 threads per sequence.
set -u
O=gpurun_out/r06/am; rm -rf $O; mkdir -p $O
for c in 512 1024; do
TDFO_LIB_PATH=$PWD/labs/ab/libtdfo_hip_t$c.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $O/tests_$c.log 2>&1 || { echo "tests $c rc=$?"; tail -30 $O/tests_$c.log; exit 1; }
tail -1 $O/tests_$c.log
done
for k in 1 2; do
for c in 256 512 1024; do
TDFO_LIB_PATH=$PWD/labs/ab/libtdfo_hip_t$c.so timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${c}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${c}_$k.log; exit 1; }
echo "$c $k b16 $(tail -n 1 $O/b4r_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
