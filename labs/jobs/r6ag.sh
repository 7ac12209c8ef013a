# Random-row gather rate vs table size (floor under the embedding kernels).
set -u
O=gpurun_out/r06/ag; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u labs/probes/random_rows.py > $O/random_rows.log 2>&1 || { echo "rc=$?"; tail -5 $O/random_rows.log; exit 1; }
grep '^{' $O/random_rows.log
