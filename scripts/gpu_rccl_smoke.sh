#!/bin/bash
set -e
export PYTHONUNBUFFERED=1
O=gpurun_out/r03c; mkdir -p $O
NCCL_DEBUG=INFO timeout -k 10 120 python -X faulthandler -u scripts/rccl_smoke.py --pg > $O/rccl_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -40 $O/rccl_smoke.log; exit 1; }
tail -5 $O/rccl_smoke.log
