"""Summarise a rocprofv3 kernel-trace CSV: per-kernel totals and one step."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
tot = defaultdict(float)
cnt = defaultdict(int)
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = r["Kernel_Name"]
    n = n[:90]
    tot[n] += d
    cnt[n] += 1
T = sum(tot.values())
print(f"{'total_us':>10} {'calls':>6} {'avg_us':>8}  kernel")
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:40]:
    print(f"{t:10.1f} {cnt[n]:6d} {t / cnt[n]:8.1f}  {n}")
print(f"sum {T:.1f} us")
