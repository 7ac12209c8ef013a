set -u
O=gpurun_out/r06/f; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "embedding or radix or dlrm" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/emb_iso.py --cases dlrm > $O/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $O/iso.log; exit 1; }
grep case $O/iso.log
for k in 1 2; do
for v in 1 0; do
TDFO_EMB_INKERNEL_COMBINE=$v timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 > $O/b${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/b${v}_$k.log; exit 1; }
echo "inkernel=$v $k $(tail -n 1 $O/b${v}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o iso -- python3 $ROOT/scripts/emb_iso.py --cases dlrm > $ROOT/$O/iso_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $ROOT
python scripts/kstats.py $O/prof/iso_kernel_stats.csv | grep tdfo
