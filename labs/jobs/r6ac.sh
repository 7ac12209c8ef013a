# Bert4Rec: wgrad slab sum + loss in one tail launch.
set -u
O=gpurun_out/r06/ac; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bert4rec.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_$k.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_bert4rec.py --batch 256 > $O/b4r256_$k.log 2>&1 || { echo "b4r256 rc=$?"; tail -5 $O/b4r256_$k.log; exit 1; }
echo "$k b4r $(tail -n 1 $O/b4r_$k.log | grep -o '"ms_per_step": [0-9.]*') b4r256 $(tail -n 1 $O/b4r256_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done
