set -u
O=gpurun_out/r06/l; rm -rf $O; mkdir -p $O
for k in 1 2; do
for v in r05 c1 cur0 CONTRACT_ON PART_PLAIN cur; do
case $v in cur|cur0) unset TDFO_LIB_PATH;; *) export TDFO_LIB_PATH=$PWD/ab_libs/${v}_libtdfo_hip.so;; esac
case $v in cur) unset TDFO_EMB_INKERNEL_COMBINE;; *) export TDFO_EMB_INKERNEL_COMBINE=0;; esac
timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 > $O/l_${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/l_${v}_$k.log; exit 1; }
echo "$v $k long $(tail -n 1 $O/l_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
