set -u
O=gpurun_out/r06/g; rm -rf $O; mkdir -p $O
timeout -k 10 120 python -u labs/dbg_meta.py > $O/dbg1.log 2>&1; echo "rc=$?"; cat $O/dbg1.log | grep -v amdgpu.ids
TDFO_EMB_INKERNEL_COMBINE=0 timeout -k 10 120 python -u labs/dbg_meta.py > $O/dbg0.log 2>&1; echo "rc=$?"; cat $O/dbg0.log | grep -v amdgpu.ids
