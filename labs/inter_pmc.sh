#!/bin/bash
# kernel trace + PMC passes (one run each) over the interaction kernels
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ipmc; mkdir -p $O
P="python3 $R/labs/inter_probe.py 20"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- $P > $O/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- $P > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES -d $O/p2 -o run --output-format csv -- $P > $O/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o run --output-format csv -- $P > $O/p3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/p4 -o run --output-format csv -- $P > $O/p4.log 2>&1
cd $R
python3 scripts/prof_summary.py $(ls $O/kt/*kernel_trace.csv | head -1) --steps 20 | head -6
for p in p1 p2 p3 p4; do python3 scripts/pmc_summary.py $(ls $O/$p/*counter_collection.csv | head -1) inter; done
