"""Per-queue timeline of one steady-state step from a rocprofv3 kernel-trace
CSV: for each hardware queue, the kernels of the window between the last two
dispatches of a once-per-step marker kernel, with their start offsets,
durations and the idle gaps before them (where each stream waits)."""
import argparse
import csv
from collections import defaultdict

from prof_summary import short_name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="head_bce")
    ap.add_argument("--step", type=int, default=-2, help="which marker interval (-2: last full)")
    a = ap.parse_args()
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                 short_name(r["Kernel_Name"])) for r in csv.DictReader(open(a.csv)))
    marks = [s for s, _, _, n in ev if a.marker in n]
    lo, hi = marks[a.step], marks[a.step + 1]
    lanes = defaultdict(list)
    for s, e, q, n in ev:
        if lo <= s < hi:
            lanes[q].append((s, e, n))
    print(f"step window {(hi - lo) / 1e3:.1f} us (marker {a.marker})")
    for q, ks in sorted(lanes.items()):
        busy = sum(e - s for s, e, _ in ks) / 1e3
        print(f"\n== queue {q}: {len(ks)} kernels, {busy:.1f} us busy")
        prev = lo
        for s, e, n in ks:
            gap = (s - prev) / 1e3
            print(f"  +{(s - lo) / 1e3:7.1f}  {(e - s) / 1e3:6.1f} us  gap {gap:5.1f}  {n}")
            prev = max(prev, e)


if __name__ == "__main__":
    main()
