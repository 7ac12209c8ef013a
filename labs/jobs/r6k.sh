set -u
O=gpurun_out/r06/k; rm -rf $O; mkdir -p $O
for v in r05 cur; do
if [ $v = r05 ]; then export TDFO_LIB_PATH=$PWD/ab_libs/${v}_libtdfo_hip.so; else unset TDFO_LIB_PATH; fi
OUT=$O/prof_$v PROF_ARGS="--steps 30 --warmup 10" bash scripts/profile_bench.sh > $O/prof_$v.log 2>&1 || { echo "prof rc=$?"; tail $O/prof_$v.log; exit 1; }
python scripts/step_lanes.py $(ls $O/prof_$v/*kernel_trace.csv | head -1) > $O/prof_$v/lanes.txt
python - $O/prof_$v <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/*kernel_trace.csv")[0]
seen = set()
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "emb_" in n and n not in seen:
        seen.add(n)
        print(n.split("(tdfo")[0][-60:], "vgpr", r["VGPR_Count"], "scratch", r["Scratch_Size"], "lds", r["LDS_Block_Size"])
PY
done
cat $O/prof_r05/summary.txt; cat $O/prof_cur/summary.txt
