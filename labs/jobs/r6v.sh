# TwoTower six-launch step: tests, A/B (TDFO_TT_FUSED=1/0, x2), kernel table;
# then the DLRM driver-window warm curve (r6u).
set -u
O=gpurun_out/r06/v; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_two_tower.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in 1 0; do
TDFO_TT_FUSED=$v timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt_${v}_$k.log 2>&1 || { echo "tt rc=$?"; tail -5 $O/tt_${v}_$k.log; exit 1; }
echo "fused=$v $k $(tail -n 1 $O/tt_${v}_$k.log)"
done; done
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o tt -- python3 $ROOT/scripts/bench_two_tower.py --steps 200 > $ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $ROOT
python scripts/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) --marker two_tower_kernel --last 100 > $O/prof/summary.txt; cat $O/prof/summary.txt
for k in 1 2; do
for v in 1 0; do
TDFO_EMB_INKERNEL_COMBINE=$v timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/ttc_${v}_$k.log 2>&1 || { echo "ttc rc=$?"; tail -5 $O/ttc_${v}_$k.log; exit 1; }
TDFO_EMB_INKERNEL_COMBINE=$v timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4rc_${v}_$k.log 2>&1 || { echo "b4rc rc=$?"; tail -5 $O/b4rc_${v}_$k.log; exit 1; }
echo "inkernel_combine=$v $k tt $(tail -n 1 $O/ttc_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*') b4r $(tail -n 1 $O/b4rc_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
bash labs/jobs/r6u.sh
