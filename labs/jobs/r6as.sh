# Bert4Rec kernel tables (B=16 and B=256) after the round-6 Linear+CE / encoder work.
set -u
O=gpurun_out/r06/as; rm -rf $O; mkdir -p $O
ROOT=$GRAFT_REPO_ROOT
for bs in 16 256; do
timeout -k 10 300 python -u scripts/bench_bert4rec.py --batch $bs > $O/b$bs.log 2>&1 || { echo "b$bs rc=$?"; exit 1; }
echo "B=$bs $(tail -n 1 $O/b$bs.log)"
done
cd /tmp && export TMPDIR=/tmp
for bs in 16 256; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof$bs -o b4r -- python3 $ROOT/scripts/bench_bert4rec.py --steps 200 --batch $bs > $ROOT/$O/prof$bs.log 2>&1 || { echo "prof rc=$?"; tail -5 $ROOT/$O/prof$bs.log; exit 1; }
done
cd $ROOT
for bs in 16 256; do
python scripts/prof_summary.py $(ls $O/prof$bs/*kernel_trace.csv | head -1) --marker xent_pass1 --last 100 > $O/summary_b$bs.txt; cat $O/summary_b$bs.txt
done
