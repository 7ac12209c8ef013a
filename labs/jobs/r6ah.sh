# Non-temporal table-row reads/writes in the embedding update: isolated + step A/B.
set -u
O=gpurun_out/r06/ah; rm -rf $O; mkdir -p $O
NT=$PWD/labs/ab/libtdfo_hip_nt.so
TDFO_LIB_PATH=$NT timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "embedding" > $O/tests_nt.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/tests_nt.log; exit 1; }
tail -1 $O/tests_nt.log
for k in 1 2; do
for v in nt base; do
L=""; [ $v = nt ] && L=$NT
TDFO_LIB_PATH=$L timeout -k 10 300 python -u scripts/emb_iso.py > $O/iso_${v}_$k.log 2>&1 || { echo "iso rc=$?"; tail -5 $O/iso_${v}_$k.log; exit 1; }
TDFO_LIB_PATH=$L timeout -k 10 300 python -u bench.py --model dcnv2 --steps 50 --warmup 10 > $O/dcn_${v}_$k.log 2>&1 || { echo "dcn rc=$?"; tail -5 $O/dcn_${v}_$k.log; exit 1; }
TDFO_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 300 --warmup 10 > $O/dlrm_${v}_$k.log 2>&1 || { echo "dlrm rc=$?"; tail -5 $O/dlrm_${v}_$k.log; exit 1; }
echo "$v $k dcn $(tail -n 1 $O/dcn_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*') dlrm $(tail -n 1 $O/dlrm_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
grep -h "update\|chunk" $O/iso_${v}_$k.log | head -6
done; done
