# Linear+CE: 3-pass bf16 pass1 + wgrad (impl 2) vs f32 MFMA (impl 1); kernel table of impl 2.
set -u
O=gpurun_out/r06/ae2; rm -rf $O; mkdir -p $O
ROOT=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bert4rec.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for c in 1 2; do
TDFO_XENT_IMPL=$c timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${c}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${c}_$k.log; exit 1; }
echo "impl $c $k b4r $(tail -n 1 $O/b4r_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
TDFO_XENT_IMPL=2 timeout -k 10 300 python -u scripts/bench_bert4rec.py --batch 256 > $O/b4r256_2.log 2>&1 && TDFO_XENT_IMPL=1 timeout -k 10 300 python -u scripts/bench_bert4rec.py --batch 256 > $O/b4r256_1.log 2>&1 || { echo "b256 rc=$?"; exit 1; }
echo "B=256 impl1 $(grep -o '"ms_per_step": [0-9.]*' $O/b4r256_1.log) impl2 $(grep -o '"ms_per_step": [0-9.]*' $O/b4r256_2.log)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o b4r -- python3 $ROOT/scripts/bench_bert4rec.py --steps 200 > $ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $ROOT/$O/prof.log; exit 1; }
cd $ROOT
python scripts/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) --marker xent_pass1 --last 100 > $O/summary.txt; head -8 $O/summary.txt; tail -2 $O/summary.txt
