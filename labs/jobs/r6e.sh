set -u
O=gpurun_out/r06/e; rm -rf $O; mkdir -p $O
for k in 1 2; do
for st in none dense_opt emb_sort emb_update emb_lookup; do
timeout -k 10 300 python -u labs/probes/step_skip.py $st --steps 100 --warmup 5 > $O/${st}_$k.log 2>&1 || { echo "$st rc=$?"; tail -5 $O/${st}_$k.log; exit 1; }
echo "$st $k $(tail -n 1 $O/${st}_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
