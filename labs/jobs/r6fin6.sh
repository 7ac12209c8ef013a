set -u
O=gpurun_out/r06/fin6; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
for k in 1 2; do
timeout -k 10 300 python -u bench.py --model dcnv2 --steps 50 --warmup 10 > $O/dcn_$k.log 2>&1 || { echo "dcn rc=$?"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 300 --warmup 10 > $O/b300_$k.log 2>&1 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/drv_$k.log 2>&1 || { echo "drv rc=$?"; exit 1; }
timeout -k 10 300 python -u scripts/bench_two_tower.py > $O/tt_$k.log 2>&1 || { echo "tt rc=$?"; exit 1; }
timeout -k 10 300 python -u scripts/bench_bert4rec.py > $O/b4r_$k.log 2>&1 || { echo "b4r rc=$?"; exit 1; }
echo "$k dcn $(tail -n 1 $O/dcn_$k.log | grep -o '"ms_per_step": [0-9.]*') b300 $(tail -n 1 $O/b300_$k.log | grep -o "\"ms_per_step\": [0-9.]*") drv $(tail -n 1 $O/drv_$k.log | grep -o '"ms_per_step": [0-9.]*') tt $(tail -n 1 $O/tt_$k.log | grep -o '"ms_per_step": [0-9.]*') b4r $(tail -n 1 $O/b4r_$k.log | grep -o '"ms_per_step": [0-9.]*')"
done
