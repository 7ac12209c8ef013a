#!/usr/bin/env python
"""Pooled-embedding forward on the MLPerf DCN-v2 multi-hot bags (MI355X).

26 bags per sample with the MLPerf multi-hot pooling factors (sum 214 ids),
B = 8192, D = 128, uniform ids over one 40 M-row fp32 table that every
table aliases (row_offset 0: HBM-sized, the gathers are what is timed).
Reports us and the gathered-row bandwidth.
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402
from tdfo_amd.models.dlrm import MLPERF_MULTIHOT  # noqa: E402
from scripts.gemm_step_bench import timeit  # noqa: E402


def main():
    B, D, rows = 8192, 128, 40_000_000
    L = MLPERF_MULTIHOT
    T = len(L)
    dev = "cuda"
    W = torch.empty(rows, D, device=dev).uniform_(-0.01, 0.01)
    ro = torch.zeros(T, dtype=torch.long, device=dev)
    lens = torch.tensor(L, device=dev).repeat_interleave(B)          # table-major bags
    offs = torch.zeros(T * B + 1, dtype=torch.long, device=dev)
    offs[1:] = torch.cumsum(lens, 0)
    nnz = int(offs[-1])
    ids = torch.randint(0, rows, (nnz,), device=dev)
    oo = torch.tensor([t * D for t in range(T)], device=dev)
    out = torch.empty(B * T * D, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.embedding_bag_fwd(W, ro, ids, offs, oo, T, B, out, T * D))
    # correctness spot check vs the fp32 reference on a few bags
    from tdfo_amd.ops import reference as ref
    exp = torch.empty(B * T * D, device=dev)
    ref.embedding_bag_fwd(W, ro, ids, offs, oo, None, T, B, False, exp, T * D)
    err = float((out.float() - exp).abs().max())
    print(json.dumps({"case": "emb_fwd_multihot", "nnz": nnz, "us": round(t, 1),
                      "row_GBps": round(nnz * D * 4 / t / 1e3, 1), "max_abs_err": err}),
          flush=True)


if __name__ == "__main__":
    main()
