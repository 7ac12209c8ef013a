#!/usr/bin/env python
"""Radix sort (embedding-backward key sort) timing vs digit width, one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402
from tdfo_amd.ops import _ext  # noqa: E402
from bench_kernels import timeit  # noqa: E402

_ext.load()
nat = torch.ops.tdfo
for n in (213_000, 1_700_000):
    keys = torch.randint(0, 188_000_000, (n,), device="cuda", dtype=torch.int32)
    vals = torch.arange(n, dtype=torch.int32, device="cuda")
    for b, sep in ((8, 0), (10, 0), (8, 1), (10, 1)):
        nat.radix_sort_max_bits(b)
        nat.radix_sort_sep_hist(sep)
        t = timeit(lambda: ops.sort_pairs(keys, vals, 28))
        # the same sort inside a hipGraph (device time, no host launch cost)
        ops.sort_pairs(keys, vals, 28)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ops.sort_pairs(keys, vals, 28)
        tg = timeit(g.replay)
        print(json.dumps({"n": n, "max_bits": b, "sep_hist": sep, "sort_us": round(t, 1),
                          "graph_sort_us": round(tg, 1)}), flush=True)
nat.radix_sort_max_bits(10)
nat.radix_sort_sep_hist(1)
