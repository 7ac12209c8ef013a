set -u
export PYTHONUNBUFFERED=1
N=2 STEP_TIMEOUT=300 bash scripts/rehearse_multi.sh > gpurun_out/rehearse_summary.txt 2>&1
echo "rehearse rc=$?"
cat gpurun_out/rehearse_summary.txt | grep -E "==|metric" | cut -c1-300
OUT=gpurun_out/prof_dcn PROF_ARGS="--model dcnv2 --steps 10 --warmup 3" PROF_STEPS=13 timeout -k 10 400 bash scripts/profile_bench.sh > /dev/null 2>&1
echo "prof rc=$?"
head -30 gpurun_out/prof_dcn/summary.txt
