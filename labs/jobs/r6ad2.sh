# Linear+CE: 3-pass bf16 pass1 (impl 2) vs f32 MFMA (impl 1).
set -u
O=gpurun_out/r06/ad2; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bert4rec.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for c in 1 2; do
TDFO_XENT_IMPL=$c timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${c}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${c}_$k.log; exit 1; }
echo "impl $c $k b4r $(tail -n 1 $O/b4r_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
