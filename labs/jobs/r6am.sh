# Bert4Rec: step counters bumped by the item lookup launch.
set -u
O=gpurun_out/r06/am; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bert4rec.py tests/test_gpu_kernels.py -k "bert4rec or embedding_bag or lookup or fwd" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in 1 0; do
TDFO_B4R_FOLD_BUMP=$v timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${v}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${v}_$k.log; exit 1; }
echo "fold=$v $k b4r $(tail -n 1 $O/b4r_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
