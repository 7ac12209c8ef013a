# DLRM: top MLP's optimizer part as side blocks of the first bottom backward pair.
set -u
O=gpurun_out/r06/al; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "dlrm or head or optim or dense" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in 1 0; do
TDFO_OPT_SIDE=$v timeout -k 10 300 python -u bench.py --steps 300 --warmup 10 > $O/b300_${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/b300_${v}_$k.log; exit 1; }
TDFO_OPT_SIDE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/drv_${v}_$k.log 2>&1 || { echo "drv rc=$?"; tail -5 $O/drv_${v}_$k.log; exit 1; }
echo "side=$v $k 300: $(tail -n 1 $O/b300_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*') drv: $(tail -n 1 $O/drv_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
