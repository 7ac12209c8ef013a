#!/bin/bash
# Multi-hot embedding forward: rows-in-flight builds vs the round-1 kernel.
set -u
O=gpurun_out/emb2; mkdir -p $O
L=$PWD/tdfo_amd/lib
for v in main:$L/libtdfo_hip.so rif2:$L/ab/rif2.so rif8:$L/ab/rif8.so old:$L/ab/libtdfo_hip_old.so; do
  n=${v%%:*}; p=${v#*:}
  TDFO_LIB_PATH=$p timeout -k 10 200 python -u scripts/bench_emb_fwd.py > $O/$n.jsonl 2>&1 || exit 1
done
grep -h case $O/*.jsonl
