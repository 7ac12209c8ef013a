# DLRM bench: session-start library (old) vs current (new), same box, alternating.
set -u
O=gpurun_out/r06/ao; rm -rf $O; mkdir -p $O
for k in 1 2 3; do
for c in old new; do
L=""; [ $c = old ] && L=$PWD/labs/ab/libtdfo_hip_old.so
TDFO_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 300 --warmup 10 > $O/b300_${c}_$k.log 2>&1 || { echo "b rc=$?"; tail -5 $O/b300_${c}_$k.log; exit 1; }
TDFO_LIB_PATH=$L timeout -k 10 300 python -u bench.py > $O/bd_${c}_$k.log 2>&1 || { echo "b rc=$?"; tail -5 $O/bd_${c}_$k.log; exit 1; }
echo "$c $k b300 $(tail -n 1 $O/b300_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*') default $(tail -n 1 $O/bd_${c}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
