# Round-6 normalised step profiles of the DLRM-1TB headline and DCN-v2.
set -u
O=gpurun_out/r06/prof; rm -rf $O; mkdir -p $O
OUT=$O/dlrm PROF_ARGS="--steps 60 --warmup 10" PROF_LAST=40 bash scripts/profile_bench.sh > $O/dlrm.log 2>&1 || { echo "prof dlrm rc=$?"; tail $O/dlrm.log; exit 1; }
python scripts/step_lanes.py $(ls $O/dlrm/*kernel_trace.csv | head -1) > $O/dlrm/lanes.txt
OUT=$O/dcn PROF_ARGS="--model dcnv2 --steps 40 --warmup 10" PROF_LAST=20 bash scripts/profile_bench.sh > $O/dcn.log 2>&1 || { echo "prof dcn rc=$?"; tail $O/dcn.log; exit 1; }
python scripts/step_lanes.py $(ls $O/dcn/*kernel_trace.csv | head -1) > $O/dcn/lanes.txt
head -24 $O/dlrm/summary.txt; head -8 $O/dlrm/lanes.txt; head -24 $O/dcn/summary.txt
for k in 1 2; do
timeout -k 10 300 python -u bench.py --model dcnv2 --steps 50 --warmup 10 > $O/dcn_$k.log 2>&1 || { echo "dcn rc=$?"; tail -5 $O/dcn_$k.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/drv_$k.log 2>&1 || { echo "drv rc=$?"; tail -5 $O/drv_$k.log; exit 1; }
echo "$k dcn $(tail -n 1 $O/dcn_$k.log | grep -o '"ms_per_step": [0-9.]*') dlrm $(tail -n 1 $O/drv_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done
