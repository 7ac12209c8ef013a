set -u
O=gpurun_out/r06/i; rm -rf $O; mkdir -p $O
export TDFO_SEG_SPLIT=0
for k in 1 2; do
for v in r05 c1 cur; do
if [ $v = cur ]; then unset TDFO_LIB_PATH; else export TDFO_LIB_PATH=$PWD/ab_libs/${v}_libtdfo_hip.so; fi
timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 > $O/l_${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/l_${v}_$k.log; exit 1; }
echo "$v $k long $(tail -n 1 $O/l_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
