#!/bin/bash
# Kernel trace + two PMC passes for a wgrad and a fwd GEMM shape (policy 0),
# summarised into gpurun_out/pmc_gemm_summary.txt.
set -u
R=$GRAFT_REPO_ROOT
SHAPE="${WSHAPE:-wgrad 8192 1024 1088}" POLS="0" bash $R/scripts/gemm_pmc.sh || exit 1
rm -rf $R/gpurun_out/pmc_wgrad; mv $R/gpurun_out/pmc $R/gpurun_out/pmc_wgrad
SHAPE="${FSHAPE:-fwd 8192 1024 1024}" POLS="0" bash $R/scripts/gemm_pmc.sh || exit 1
rm -rf $R/gpurun_out/pmc_fwd; mv $R/gpurun_out/pmc $R/gpurun_out/pmc_fwd
for d in pmc_wgrad pmc_fwd; do
  for p in kt_0 p1_0 p2_0; do
    f=$(ls $R/gpurun_out/$d/$p/*/*.csv $R/gpurun_out/$d/$p/*.csv 2>/dev/null | grep -E "counter_collection|kernel_trace" | head -1)
    echo "== $d $p"
    python3 $R/scripts/pmc_summary.py $f gemm
  done
done > $R/gpurun_out/pmc_gemm_summary.txt 2>&1
