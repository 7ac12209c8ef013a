#!/usr/bin/env python
"""Fused bottom-MLP forward (mlp3_fwd) vs the three per-layer GEMM launches,
in isolation (graph-replayed, median of 7 x 30 launches), B = 8192."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402
from scripts.gemm_step_bench import timeit  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    dev = "cuda"
    torch.manual_seed(0)
    bf = torch.bfloat16
    ws = [(torch.randn(n, k + 64, device=dev) / k ** 0.5).to(bf)[:, :k]
          for n, k in ((512, 64), (256, 512), (128, 256))]
    bs = [None, torch.randn(256, device=dev), torch.randn(128, device=dev)]
    x = torch.randn(B, 64, device=dev).to(bf)
    ys = [torch.empty(B, n, dtype=bf, device=dev) for n in (512, 256, 128)]

    def fused():
        ops.mlp3_fwd(x, ws, bs, ys)

    def unfused():
        h = x
        for w, b, y in zip(ws, bs, ys):
            ops.gemm(h, False, w, False, b, True, None, y, None, 1)
            h = y
    out = {"B": B, "fused_us": round(timeit(fused), 2), "gemms_us": round(timeit(unfused), 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
