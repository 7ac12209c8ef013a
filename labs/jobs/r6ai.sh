# NT row accesses on multi-hot batches only (runtime choice): tests + DCN / DLRM A/B.
set -u
O=gpurun_out/r06/${JOBTAG:-ai}; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "embedding or dcn or cross" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
for v in 1 0; do
TDFO_EMB_NT=$v timeout -k 10 300 python -u bench.py --model dcnv2 --steps 50 --warmup 10 > $O/dcn_${v}_$k.log 2>&1 || { echo "dcn rc=$?"; tail -5 $O/dcn_${v}_$k.log; exit 1; }
TDFO_EMB_NT=$v timeout -k 10 300 python -u bench.py --model dcnv2 --steps 50 --warmup 10 --dist zipf > $O/dcnz_${v}_$k.log 2>&1 || { echo "dcnz rc=$?"; tail -5 $O/dcnz_${v}_$k.log; exit 1; }
echo "nt=$v $k dcn $(tail -n 1 $O/dcn_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*') zipf $(tail -n 1 $O/dcnz_${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
timeout -k 10 300 python -u scripts/emb_iso.py > $O/iso.log 2>&1 || { echo "iso rc=$?"; exit 1; }
tail -2 $O/iso.log
