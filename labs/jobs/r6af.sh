# PMC pass on the 3-pass bf16 Linear+CE kernels.
set -u
O=gpurun_out/r06/af; rm -rf $O; mkdir -p $O
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "xent_(pass1|wgrad|merge)" --output-format csv -d $ROOT/$O/pmc1 -o p -- python3 $ROOT/scripts/bench_bert4rec.py --steps 20 --warmup 5 --no-graph > $ROOT/$O/pmc1.log 2>&1 || { echo "pmc1 rc=$?"; tail -5 $ROOT/$O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAVES FETCH_SIZE --kernel-include-regex "xent_(pass1|wgrad|merge)" --output-format csv -d $ROOT/$O/pmc2 -o p -- python3 $ROOT/scripts/bench_bert4rec.py --steps 20 --warmup 5 --no-graph > $ROOT/$O/pmc2.log 2>&1 || { echo "pmc2 rc=$?"; tail -5 $ROOT/$O/pmc2.log; exit 1; }
echo done
