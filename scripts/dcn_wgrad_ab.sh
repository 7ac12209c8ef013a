set -u
O=gpurun_out/sweep; mkdir -p $O
for cs in 1 0; do for t in 256 512; do
 TDFO_WGRAD_CSUM=$cs TDFO_WGRAD_TARGET=$t timeout -k 10 300 python -u bench.py --model dcnv2 --steps 20 --warmup 3 > $O/dcn_${cs}_$t.log 2>&1 || exit 1
done; done
