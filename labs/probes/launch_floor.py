#!/usr/bin/env python
"""Per-node cost of back-to-back kernels in a replayed hipGraph (MI355X).

Captures `reps` launches of (a) a 1-element torch add, (b) our 1-k-tile GEMM
on a tiny and on a full-chip grid, into one graph each and reports the
replay time per node: the fixed cost every kernel of the graph-replayed
training step pays regardless of its work.
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402


def graph_time(fn, reps=50, iters=7):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    bf = torch.bfloat16
    t = torch.zeros(1, device="cuda")
    out = {"torch_add_1elem_us": graph_time(lambda: t.add_(1.0))}
    for M, N in [(128, 128), (8192, 512), (8192, 1024)]:
        x = torch.randn(M, 64, device="cuda").to(bf)
        w = torch.randn(N, 64, device="cuda").to(bf)
        y = torch.empty(M, N, device="cuda", dtype=bf)
        out[f"gemm_{M}x{N}x64_us"] = graph_time(lambda: ops.gemm(x, False, w, False, None, False,
                                                                 None, y, None, 1))
    print(json.dumps({k: round(v, 2) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
