set -u
O=gpurun_out/r06/s; rm -rf $O; mkdir -p $O
export STEP_TIMEOUT=300
SET=guards N=2 bash scripts/rehearse_multi.sh > $O/guards.log 2>&1; rc=$?; echo "guards rc=$rc"; tail -12 $O/guards.log; [ $rc -eq 0 ] || exit 1
N=2 bash scripts/rehearse_multi.sh > $O/full.log 2>&1; rc=$?; echo "full rc=$rc"; grep "== " $O/full.log; [ $rc -eq 0 ] || { tail -20 $O/full.log; exit 1; }
cp gpurun_out/rehearse_*.log $O/
cd recipes/dlrm
TDFO_SHARE_DEVICE=1 TDFO_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 train_ps.py per_device_train_batch_size=2048 synthetic.rows=kaggle max_steps=20 log_every=10 eval_every=0 > ../../$O/recipe_ps.log 2>&1; rc=$?
cd ../..
echo "recipe rc=$rc"; grep -v "hostname\|amdgpu.ids" $O/recipe_ps.log | tail -8
