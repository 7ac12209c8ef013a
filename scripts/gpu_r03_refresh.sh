#!/bin/bash
# round-3 evidence refresh: secondary-model benches + Bert4Rec / DCN-v2 kernel summaries
set -e
export PYTHONUNBUFFERED=1
R=$PWD; O=gpurun_out/r03r; mkdir -p $O
timeout -k 10 300 python -u bench.py --model dcnv2 --steps 30 --warmup 6 > $O/dcnv2.log 2>&1
echo "dcnv2 $(tail -1 $O/dcnv2.log | cut -c1-220)"
timeout -k 10 300 python -u scripts/bench_bert4rec.py --steps 50 --warmup 10 > $O/bert4rec.log 2>&1
echo "bert4rec $(tail -1 $O/bert4rec.log | cut -c1-220)"
timeout -k 10 300 python -u scripts/bench_two_tower.py --steps 50 --warmup 10 > $O/two_tower.log 2>&1
echo "two_tower $(tail -1 $O/two_tower.log | cut -c1-220)"
OUT=$O/prof_bert4rec STEPS=60 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh scripts/bench_bert4rec.py --steps 50 --warmup 10 > $O/prof_bert4rec.txt 2>&1
head -25 $O/prof_bert4rec/summary.txt
OUT=$O/prof_dcnv2 STEPS=13 PROF_TIMEOUT=300 bash scripts/profile_cmd.sh bench.py --model dcnv2 --steps 10 --warmup 3 > $O/prof_dcnv2.txt 2>&1
head -20 $O/prof_dcnv2/summary.txt
