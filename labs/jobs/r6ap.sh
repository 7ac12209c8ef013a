# Bert4Rec: encoder reductions parked into the next backward launch (1) vs own launches (0).
set -u
O=gpurun_out/r06/ap; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bert4rec.py tests/test_gpu_attention.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2 3; do
for c in 0 1; do
TDFO_B4R_DEFER_ENC_RED=$c timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${c}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${c}_$k.log; exit 1; }
echo "defer=$c $k b16 $(tail -n 1 $O/b4r_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
