set -u
O=gpurun_out/r06/n; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bert4rec.py tests/test_gpu_kernels.py -k "xent or bert4rec or embedding or dense or optim or fused_bottom or radix" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in 1 0; do
TDFO_XENT_FUSED_STEP=$v timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${v}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${v}_$k.log; exit 1; }
echo "fused=$v $k $(tail -n 1 $O/b4r_${v}_$k.log)"
done; done
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o b4r -- python3 $ROOT/scripts/bench_bert4rec.py --steps 100 > $ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $ROOT
python scripts/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) --marker xent_loss --last 50 > $O/prof/summary.txt; cat $O/prof/summary.txt
