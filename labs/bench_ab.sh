#!/bin/bash
# Interleaved A/B of an env setting on the DLRM-1TB bench (same box, same
# process image): AB_VAR=name AB_VALS="a b" [AB_ARGS=...] [AB_REPS=2].
set -u
O=gpurun_out/ab; mkdir -p $O
for r in $(seq 1 ${AB_REPS:-2}); do for v in $AB_VALS; do
  env $AB_VAR=$v timeout -k 10 200 python -u bench.py --steps ${AB_STEPS:-100} --warmup 10 ${AB_ARGS:-} > $O/b_${v}_$r.log 2>&1 || exit 1
  echo "$AB_VAR=$v rep $r: $(tail -1 $O/b_${v}_$r.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $O/summary.txt
done; done
cat $O/summary.txt
