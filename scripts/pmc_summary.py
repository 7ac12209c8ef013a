#!/usr/bin/env python
"""Summarise rocprofv3 counter_collection / kernel_trace CSVs per kernel name."""
import csv
import collections
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*?>)?)", n)
    return (m.group(1) if m else n)[:60]


def counters(path, filt=""):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if filt not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
    for k, d in acc.items():
        n = len(cnt[k])
        print(k, f"dispatches={n}")
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {v / n:16.0f}")


def trace(path, filt=""):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if filt in k:
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in d.items():
        v.sort()
        print(f"{k:60s} n={len(v)} med={v[len(v)//2]:.1f}us min={v[0]:.1f}us")


if __name__ == "__main__":
    f = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    (trace if "trace" in f else counters)(f, filt)
