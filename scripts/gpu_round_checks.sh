set -u
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_data.py tests/test_gpu_two_tower.py tests/test_gpu_multirank.py > gpurun_out/t6.log 2>&1
echo "tests rc=$?"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t6.log | tail -25
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/b6a.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/b6a.log | cut -c1-260
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --host-data > gpurun_out/b6b.log 2>&1; echo "bench host rc=$?"; tail -1 gpurun_out/b6b.log | cut -c1-260
