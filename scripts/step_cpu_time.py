#!/usr/bin/env python
"""Host-side cost of issuing one graph-replayed DLRM step vs its GPU time.

Times the Python loop that issues N steps (load_batch + step, no sync) and
the wall time until the GPU drains. If issue time per step approaches the
GPU time, the launching thread (graph launches, event record/wait) is on
the critical path.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd.data.synthetic import SyntheticCriteo  # noqa: E402
from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer  # noqa: E402


def main():
    B, N = 8192, 100
    rows = [1000 + 37 * i for i in range(26)]
    cfg = DLRMConfig(table_rows=rows)
    tr = DLRMTrainer(cfg, B, "cuda")
    data = SyntheticCriteo(rows, B, device="cuda", seed=1)
    pool = [data.next() for _ in range(4)]
    for i in range(3):
        tr.load_batch(*pool[i % 4])
        tr.step()
    tr.capture_graph(warmup=1)
    torch.cuda.synchronize()
    out = {"graph": tr.graph if isinstance(tr.graph, str) else type(tr.graph).__name__}
    t0 = time.perf_counter()
    for i in range(N):
        tr.load_batch(*pool[i % 4])
        tr.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out.update(issue_us_per_step=round((t1 - t0) / N * 1e6, 1),
               gpu_us_per_step=round((t2 - t0) / N * 1e6, 1))
    # replay cost of one small graph in isolation
    x = torch.zeros(1, device="cuda")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x.add_(1)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        x.add_(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out.update(tiny_graph_issue_us=round((t1 - t0) / 200 * 1e6, 1),
               tiny_graph_wall_us=round((t2 - t0) / 200 * 1e6, 1))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
