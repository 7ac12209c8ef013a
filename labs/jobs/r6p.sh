set -u
O=gpurun_out/r06/p; rm -rf $O; mkdir -p $O
for k in 1 2; do
for v in one_pass top_early; do
timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 --opt-placement $v > $O/l_${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/l_${v}_$k.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --opt-placement $v > $O/d_${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/d_${v}_$k.log; exit 1; }
echo "$v $k long $(tail -n 1 $O/l_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*') drv $(tail -n 1 $O/d_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
OUT=$O/prof PROF_ARGS="--steps 30 --warmup 10 --opt-placement top_early" bash scripts/profile_bench.sh > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail $O/prof.log; exit 1; }
python scripts/step_lanes.py $(ls $O/prof/*kernel_trace.csv | head -1) > $O/prof/lanes.txt; cat $O/prof/lanes.txt
