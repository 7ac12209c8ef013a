set -u
O=gpurun_out/r06/d; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "embedding or radix" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/emb_iso.py --cases dlrm > $O/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $O/iso.log; exit 1; }
grep case $O/iso.log
for k in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/drv$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/drv$k.log; exit 1; }
echo "drv$k $(tail -n 1 $O/drv$k.log | grep -o '"ms_per_step": [0-9.]*')"
TDFO_SEG_SPLIT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/drv_old$k.log 2>&1 || { echo "bench rc=$?"; exit 1; }
echo "old$k $(tail -n 1 $O/drv_old$k.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 > $O/long.log 2>&1 || { echo "bench rc=$?"; exit 1; }
echo "long $(tail -n 1 $O/long.log | grep -o '"ms_per_step": [0-9.]*')"
OUT=$O/prof PROF_ARGS="--steps 30 --warmup 10" bash scripts/profile_bench.sh > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail $O/prof.log; exit 1; }
cat $O/prof/summary.txt
python scripts/step_lanes.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/prof/lanes.txt && cat $O/prof/lanes.txt
