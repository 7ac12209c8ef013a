"""Summarise a rocprofv3 kernel-trace CSV: per-kernel totals (optionally per
step), ignoring setup kernels (data generation / table init)."""
import argparse
import csv
from collections import defaultdict

SETUP = ("distribution_elementwise", "FillFunctor", "index_elementwise", "gemvt", "arange",
         "CatArrayBatchedCopy", "fillBuffer", "BUnaryFunctor", "remainder", "AUnaryFunctor",
         "CUDAFunctor_add<", "log1p", "sigmoid", "bfloat16_copy", "direct_copy",
         "elementwise_kernel_manual_unroll")

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
args = ap.parse_args()
rows = list(csv.DictReader(open(args.csv)))
tot = defaultdict(float)
cnt = defaultdict(int)
for r in rows:
    n = r["Kernel_Name"]
    if any(s in n for s in SETUP):
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    short = n.replace("(anonymous namespace)::", "").replace("void ", "")
    short = short.split("(")[0]
    short = short[:80]
    tot[short] += d
    cnt[short] += 1
T = sum(tot.values())
div = max(1, args.steps)
print(f"{'us/step':>9} {'calls/step':>10} {'avg_us':>8} {'share':>6}  kernel")
for n, t in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"{t / div:9.1f} {cnt[n] / div:10.1f} {t / cnt[n]:8.1f} {100 * t / T:5.1f}%  {n}")
print(f"total kernel time per step: {T / div:.1f} us")
