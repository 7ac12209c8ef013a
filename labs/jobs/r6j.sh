set -u
O=gpurun_out/r06/j; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "embedding or radix or dlrm" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in r05 cur cur0; do
if [ $v = r05 ]; then export TDFO_LIB_PATH=$PWD/ab_libs/${v}_libtdfo_hip.so; else unset TDFO_LIB_PATH; fi
if [ $v = cur0 ]; then export TDFO_EMB_INKERNEL_COMBINE=0; else unset TDFO_EMB_INKERNEL_COMBINE; fi
timeout -k 10 300 python -u bench.py --steps 300 --warmup 20 > $O/l_${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/l_${v}_$k.log; exit 1; }
echo "$v $k long $(tail -n 1 $O/l_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
