set -u
O=gpurun_out/r06/b; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "embedding or radix" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u scripts/emb_iso.py > $O/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $O/iso.log; exit 1; }
grep case $O/iso.log
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o iso -- python3 $ROOT/scripts/emb_iso.py --cases dlrm > $ROOT/$O/iso_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $ROOT
python scripts/kstats.py $O/prof/iso_kernel_stats.csv
