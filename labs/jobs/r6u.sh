# Driver-window warm curve: per-step device times of the first 40 timed steps
# after the driver's 5 warm-ups, by pre-heat kind.
set -u
O=gpurun_out/r06/u; rm -rf $O; mkdir -p $O
for k in 1 2; do
timeout -k 10 300 env TDFO_BENCH_CURVE=1 python -u bench.py --steps 40 --warmup 5 > $O/burn_$k.log 2>&1 || { echo "rc=$?"; tail -5 $O/burn_$k.log; exit 1; }
timeout -k 10 300 env TDFO_BENCH_CURVE=1 TDFO_PREHEAT_KIND=copy python -u bench.py --steps 40 --warmup 5 > $O/copy_$k.log 2>&1 || { echo "rc=$?"; tail -5 $O/copy_$k.log; exit 1; }
timeout -k 10 300 env TDFO_BENCH_CURVE=1 python -u bench.py --steps 40 --warmup 5 --preheat-ms 0 > $O/none_$k.log 2>&1 || { echo "rc=$?"; tail -5 $O/none_$k.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/drv_$k.log 2>&1 || { echo "rc=$?"; tail -5 $O/drv_$k.log; exit 1; }
done
for f in $O/*.log; do echo "== $f"; grep -h "ms_per_step_windows" $f | cut -c1-400 || true; tail -n 1 $f | grep -o '"ms_per_step": [0-9.]*' || true; done
