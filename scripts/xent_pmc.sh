#!/bin/bash
# PMC passes over the fused Linear+CE kernels (bench_xent config 0, MFMA impl).
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/xpmc; mkdir -p $O
ARGS="--cfg 0 --impls ${IMPL:-1} --no-torch"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- python3 $R/scripts/bench_xent.py $ARGS > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_MISC GRBM_COUNT -d $O/p2 -o run --output-format csv -- python3 $R/scripts/bench_xent.py $ARGS > $O/p2.log 2>&1 || exit 1
for p in p1 p2; do python3 $R/scripts/pmc_summary.py $(ls $O/$p/*counter_collection.csv | head -1) xent; done > $O/summary.txt
cat $O/summary.txt
