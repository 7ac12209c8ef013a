#!/bin/bash
# PMC passes over one GEMM shape per tile policy (each pass its own run).
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc; mkdir -p $O
SHAPE=${SHAPE:-"fwd 8192 1024 1024"}
for pol in ${POLS:-1 2}; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt_$pol -o run --output-format csv -- python3 $R/labs/gemm_probe.py $SHAPE $pol > $O/kt_$pol.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/p1_$pol -o run --output-format csv -- python3 $R/labs/gemm_probe.py $SHAPE $pol 20 > $O/p1_$pol.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum -d $O/p2_$pol -o run --output-format csv -- python3 $R/labs/gemm_probe.py $SHAPE $pol 20 > $O/p2_$pol.log 2>&1 || exit 1
done
echo pmc done
