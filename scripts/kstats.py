"""Compact per-kernel table from a rocprofv3 kernel_stats.csv."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(tdfo::")[0].split("(unsigned")[0].split("(int")[0].replace("(anonymous namespace)::", "")
    print(f"{int(r['Calls']):6d} avg {float(r['AverageNs']) / 1e3:8.1f} min {float(r['MinNs']) / 1e3:8.1f}  {n[:100]}")
