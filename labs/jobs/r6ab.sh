# Linear+CE: unrolled column sums in pass1 and batched split loads in the merge (new) vs HEAD (pre).
set -u
O=gpurun_out/r06/ab; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bert4rec.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2 3; do
for c in pre new; do
TDFO_LIB_PATH=$PWD/labs/ab/libtdfo_hip_$c.so timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${c}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${c}_$k.log; exit 1; }
echo "$c $k b4r $(tail -n 1 $O/b4r_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u scripts/bench_bert4rec.py --steps 50 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -2
