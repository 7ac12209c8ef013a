set -u
O=gpurun_out/r06/q; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u scripts/gemm_vs_blas.py > $O/gemm_dlrm.log 2>&1 || { echo "gemm rc=$?"; tail -5 $O/gemm_dlrm.log; exit 1; }
timeout -k 10 300 python -u scripts/gemm_vs_blas.py --model dcnv2 > $O/gemm_dcn.log 2>&1 || { echo "gemm rc=$?"; tail -5 $O/gemm_dcn.log; exit 1; }
grep '^{' $O/gemm_dlrm.log $O/gemm_dcn.log | cut -c1-300
for k in 1 2; do
timeout -k 10 300 python -u bench.py --model dcnv2 --steps 50 --warmup 10 > $O/dcn_$k.log 2>&1 || { echo "dcn rc=$?"; tail -5 $O/dcn_$k.log; exit 1; }
echo "dcn $k $(tail -n 1 $O/dcn_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt.log 2>&1 || { echo "tt rc=$?"; tail -5 $O/tt.log; exit 1; }
tail -n 2 $O/tt.log
OUT=$O/prof_dcn PROF_ARGS="--model dcnv2 --steps 20 --warmup 10" bash scripts/profile_bench.sh > $O/prof_dcn.log 2>&1 || { echo "prof rc=$?"; tail $O/prof_dcn.log; exit 1; }
python scripts/step_lanes.py $(ls $O/prof_dcn/*kernel_trace.csv | head -1) > $O/prof_dcn/lanes.txt
head -30 $O/prof_dcn/summary.txt
