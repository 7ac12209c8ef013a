set -u
O=gpurun_out/r06/h; rm -rf $O; mkdir -p $O
for k in 1 2; do
for v in r05 cur; do
if [ $v = r05 ]; then export TDFO_LIB_PATH=$PWD/ab_libs/r05_libtdfo_hip.so; else unset TDFO_LIB_PATH; fi
timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 > $O/l_${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/l_${v}_$k.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/d_${v}_$k.log 2>&1 || { echo "bench rc=$?"; exit 1; }
echo "$v $k long $(tail -n 1 $O/l_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*') drv $(tail -n 1 $O/d_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
