# Bert4Rec kernel table (new lib) + PMC passes on the Linear+CE kernels.
set -u
O=gpurun_out/r06/ac; rm -rf $O; mkdir -p $O
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o b4r -- python3 $ROOT/scripts/bench_bert4rec.py --steps 200 > $ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $ROOT/$O/prof.log; exit 1; }
cd $ROOT
python scripts/prof_summary.py $(ls $O/prof/*kernel_trace.csv | head -1) --marker xent_pass1_mfma --last 100 > $O/summary.txt; cat $O/summary.txt
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "xent_(pass1|wgrad|merge)" --output-format csv -d $ROOT/$O/pmc1 -o p -- python3 $ROOT/scripts/bench_bert4rec.py --steps 20 --warmup 5 --no-graph > $ROOT/$O/pmc1.log 2>&1 || { echo "pmc1 rc=$?"; tail -5 $ROOT/$O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-include-regex "xent_(pass1|wgrad|merge)" --output-format csv -d $ROOT/$O/pmc2 -o p -- python3 $ROOT/scripts/bench_bert4rec.py --steps 20 --warmup 5 --no-graph > $ROOT/$O/pmc2.log 2>&1 || { echo "pmc2 rc=$?"; tail -5 $ROOT/$O/pmc2.log; exit 1; }
ls $ROOT/$O/pmc1 $ROOT/$O/pmc2
