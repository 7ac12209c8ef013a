# Bert4Rec without the lookup clone and the backward root fill; TwoTower
# fused step; tests + benches + kernel tables.
set -u
O=gpurun_out/r06/y; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_two_tower.py tests/test_gpu_bert4rec.py tests/test_gpu_attention.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt_$k.log 2>&1 || { echo "tt rc=$?"; tail -5 $O/tt_$k.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_$k.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_bert4rec.py --batch 256 > $O/b4r256_$k.log 2>&1 || { echo "b4r256 rc=$?"; tail -5 $O/b4r256_$k.log; exit 1; }
echo "$k tt $(tail -n 1 $O/tt_$k.log | grep -o '"ms_per_step": [0-9.]*') b4r $(tail -n 1 $O/b4r_$k.log | grep -o '"ms_per_step": [0-9.]*') b4r256 $(tail -n 1 $O/b4r256_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_b4r -o b4r -- python3 $ROOT/scripts/bench_bert4rec.py --steps 100 > $ROOT/$O/prof_b4r.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $ROOT
python scripts/prof_summary.py $(ls $O/prof_b4r/*kernel_trace.csv | head -1) --marker xent_loss --last 50 > $O/prof_b4r/summary.txt; cat $O/prof_b4r/summary.txt
