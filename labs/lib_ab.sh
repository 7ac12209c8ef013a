#!/bin/bash
# Interleaved bench A/B of library builds: LIBS="name:path ..." [AB_ARGS] [AB_REPS].
set -u
O=gpurun_out/libab; mkdir -p $O; : > $O/summary.txt
for r in $(seq 1 ${AB_REPS:-2}); do for v in $LIBS; do
  n=${v%%:*}; p=${v#*:}
  TDFO_LIB_PATH=$p timeout -k 10 300 python -u bench.py ${AB_ARGS:-} > $O/b_${n}_$r.log 2>&1 || exit 1
  echo "$n rep $r: $(tail -1 $O/b_${n}_$r.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $O/summary.txt
done; done
cat $O/summary.txt
