# Bert4Rec: encoder / prologue gradients straight into the flat buffer (no
# index_copy / fill launches) + the TwoTower six-launch step; tests, A/Bs,
# kernel tables; then the DLRM driver-window warm curve.
set -u
O=gpurun_out/r06/${JOBTAG:-w}; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_two_tower.py tests/test_gpu_bert4rec.py tests/test_gpu_attention.py tests/test_gpu_kernels.py -k "two_tower or bert4rec or attention or embedding or xent or encoder or layernorm or prologue" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in 1 0; do
TDFO_TT_FUSED=$v timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt_${v}_$k.log 2>&1 || { echo "tt rc=$?"; tail -5 $O/tt_${v}_$k.log; exit 1; }
TDFO_B4R_DIRECT_GRADS=$v timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_${v}_$k.log 2>&1 || { echo "b4r rc=$?"; tail -5 $O/b4r_${v}_$k.log; exit 1; }
echo "new=$v $k tt $(tail -n 1 $O/tt_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*') b4r $(tail -n 1 $O/b4r_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
for k in 1 2; do
for v in 0; do
TDFO_EMB_INKERNEL_COMBINE=$v timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/ttc_${v}_$k.log 2>&1 || { echo "ttc rc=$?"; tail -5 $O/ttc_${v}_$k.log; exit 1; }
TDFO_EMB_INKERNEL_COMBINE=$v timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4rc_${v}_$k.log 2>&1 || { echo "b4rc rc=$?"; tail -5 $O/b4rc_${v}_$k.log; exit 1; }
echo "inkernel_combine=$v $k tt $(tail -n 1 $O/ttc_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*') b4r $(tail -n 1 $O/b4rc_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_tt -o tt -- python3 $ROOT/scripts/bench_two_tower.py --steps 200 > $ROOT/$O/prof_tt.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_b4r -o b4r -- python3 $ROOT/scripts/bench_bert4rec.py --steps 100 > $ROOT/$O/prof_b4r.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $ROOT
python scripts/prof_summary.py $(ls $O/prof_tt/*kernel_trace.csv | head -1) --marker two_tower_kernel --last 100 > $O/prof_tt/summary.txt; cat $O/prof_tt/summary.txt
python scripts/prof_summary.py $(ls $O/prof_b4r/*kernel_trace.csv | head -1) --marker xent_loss --last 50 > $O/prof_b4r/summary.txt; cat $O/prof_b4r/summary.txt
