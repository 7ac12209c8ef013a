# TwoTower: towers co-launched with the per-table sort, reduce_adam beside the update.
set -u
O=gpurun_out/r06/ae; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_two_tower.py tests/test_gpu_kernels.py -k "two_tower or embedding or reduce" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in 1 0; do
TDFO_TT_COLAUNCH=$v timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt_${v}_$k.log 2>&1 || { echo "tt rc=$?"; tail -5 $O/tt_${v}_$k.log; exit 1; }
echo "colaunch=$v $k tt $(tail -n 1 $O/tt_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_tt -o tt -- python3 $ROOT/scripts/bench_two_tower.py --steps 200 > $ROOT/$O/prof_tt.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $ROOT
python scripts/prof_summary.py $(ls $O/prof_tt/*kernel_trace.csv | head -1) --marker emb_segsort_tower --last 100 > $O/prof_tt/summary.txt; cat $O/prof_tt/summary.txt
