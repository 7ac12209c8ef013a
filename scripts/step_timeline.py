#!/usr/bin/env python
"""Print one steady-state step of a rocprofv3 kernel trace as a timeline
(us from the step's batch_load, queue, grid, kernel): which kernels of the
two streams overlap, which are starved, where the queues idle."""
import csv
import sys


def main(path, which=-3, width=60):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    bl = [i for i, r in enumerate(rows) if "batch_load" in r["Kernel_Name"]]
    i0, i1 = bl[which], bl[which + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    print(f"step span {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.1f} us")
    for r in rows[i0:i1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = r["Kernel_Name"].replace("tdfo::(anonymous namespace)::", "").replace("void ", "")
        print(f"{s:8.1f} {d:7.1f} q{r['Queue_Id']} g={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):6d} {name[:width]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -3)
