set -u
O=gpurun_out/r06/a; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u scripts/emb_iso.py > $O/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $O/iso.log; exit 1; }
grep case $O/iso.log
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o iso -- python3 $ROOT/scripts/emb_iso.py > $ROOT/$O/iso_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $ROOT
f=$(ls $O/prof/*kernel_stats.csv | head -1); cut -d, -f1-8 $f | head -20
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -n 1 $O/bench.log
