"""Summarise a rocprofv3 kernel-trace CSV: per-kernel totals per step.

Normalisation: ``--marker K --last N`` takes the steady-state window between
the (n-N)-th and the last dispatch of a once-per-step kernel K (e.g.
``head_bce`` for DLRM / DCN-v2), counts every kernel that STARTS inside it and
divides by N -- so the eager warm-up steps, the capture and the setup kernels
before the timed replays are excluded and a once-per-step kernel shows 1.0
calls/step. Without ``--marker`` totals are divided by ``--steps`` (setup
kernels filtered by name), the old, approximate mode.
"""
import argparse
import csv
from collections import defaultdict

SETUP = ("distribution_elementwise", "FillFunctor", "index_elementwise", "gemvt", "arange",
         "CatArrayBatchedCopy", "fillBuffer", "BUnaryFunctor", "remainder", "AUnaryFunctor",
         "CUDAFunctor_add<", "log1p", "sigmoid", "bfloat16_copy", "direct_copy",
         "elementwise_kernel_manual_unroll")


def short_name(n: str) -> str:
    s = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return s.split("(")[0][:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    ap.add_argument("--marker", default=None, help="once-per-step kernel name substring")
    ap.add_argument("--last", type=int, default=0, help="with --marker: steps in the window")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.csv)))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ev.sort()
    lo, hi, div = None, None, max(1, args.steps)
    if args.marker:
        marks = [s for s, _, n in ev if args.marker in n]
        if len(marks) < 2:
            raise SystemExit(f"marker {args.marker!r} found {len(marks)} times")
        n = min(args.last or len(marks) - 1, len(marks) - 1)
        lo, hi, div = marks[-1 - n], marks[-1], n
    tot = defaultdict(float)
    cnt = defaultdict(int)
    busy = []
    for s, e, n in ev:
        if lo is not None:
            if not (lo <= s < hi):
                continue
        elif any(x in n for x in SETUP):
            continue
        d = (e - s) / 1e3
        k = short_name(n)
        tot[k] += d
        cnt[k] += 1
        busy.append((s, e))
    T = sum(tot.values())
    print(f"{'us/step':>9} {'calls/step':>10} {'avg_us':>8} {'share':>6}  kernel")
    for k, t in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{t / div:9.1f} {cnt[k] / div:10.2f} {t / cnt[k]:8.1f} {100 * t / T:5.1f}%  {k}")
    print(f"total kernel time per step (sum over streams): {T / div:.1f} us")
    if lo is not None:
        # wall time of the window and the time with no kernel running at all
        busy.sort()
        covered, cur_s, cur_e = 0, None, None
        for s, e in busy:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    covered += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            covered += cur_e - cur_s
        wall = (hi - lo) / 1e3
        print(f"window: {div} steps, {wall / div:.1f} us/step wall, "
              f"{(wall - covered / 1e3) / div:.1f} us/step with no kernel running")


if __name__ == "__main__":
    main()
