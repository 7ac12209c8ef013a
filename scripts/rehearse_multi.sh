#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: N ranks share cuda:0 and talk over
# gloo (RCCL refuses two ranks on one device), so the staged-graph multi-rank
# DLRM step runs on the real HIP kernels. Stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TDFO_SHARE_DEVICE=1 TDFO_DIST_BACKEND=gloo
N=${N:-2}
run() {
  local tag=$1; shift
  timeout -k 10 ${STEP_TIMEOUT:-300} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port ${PORT:-29611} bench.py --gpus $N "$@" \
    > gpurun_out/rehearse_$tag.log 2>&1
  local rc=$?
  echo "== $tag rc=$rc"; tail -4 gpurun_out/rehearse_$tag.log
  return $rc
}
if [ "${SET:-full}" = "guards" ]; then
  # pre-flight mismatch on rank 1 -> every rank on c10d + staged, consistent
  TDFO_PREFLIGHT_INJECT=1 run pf_inject --rows kaggle --steps 3 --warmup 1 --batch 2048 &&
  grep -q '"comm_path": "c10d-staged"' gpurun_out/rehearse_pf_inject.log &&
  # attempt 0 diverges (exit 4, no metric line) -> the supervisors rerun once
  TDFO_INJECT_DIVERGENCE=1 TDFO_INJECT_ATTEMPT=0 run sup_fallback --rows kaggle --steps 3 \
    --warmup 1 --batch 2048 &&
  grep -q '"attempt": 1' gpurun_out/rehearse_sup_fallback.log
  exit $?
fi
run tw1tb --steps 5 --warmup 2 --batch 4096 &&
run kaggle_auto --rows kaggle --steps 5 --warmup 2 --batch 4096 &&
run dcn_rw --model dcnv2 --rows kaggle --sharding row_wise --steps 3 --warmup 1 --batch 2048 &&
run dp_tables --rows tiny --sharding data_parallel --steps 3 --warmup 1 --batch 2048 &&
run cw_kaggle --rows kaggle --sharding column_wise --steps 3 --warmup 1 --batch 2048
