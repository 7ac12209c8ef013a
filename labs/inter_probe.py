#!/usr/bin/env python
"""Interaction fwd / bwd at the DLRM-1TB shape (B=8192, F=27, D=128), N calls
each, for rocprofv3 kernel-trace / PMC passes (labs/inter_pmc.sh)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B, F, D, T = 8192, 27, 128, 26
    dev, bf = "cuda", torch.bfloat16
    dense = torch.randn(B, D, device=dev).to(bf)
    emb = torch.randn(B * T * D, device=dev).to(bf)
    off = [0] + [t * D for t in range(T)]
    stride = [0] + [T * D] * T
    z = torch.empty(B, 512, device=dev, dtype=bf)
    dz = torch.randn(B, 512, device=dev).to(bf)
    dd = torch.empty(B, D, device=dev, dtype=bf)
    de = torch.empty_like(emb)
    for _ in range(n):
        ops.interaction_fwd(dense, emb, off, stride, F, D, z)
        ops.interaction_bwd(dz, dense, emb, off, stride, F, D, dd, de, off, stride, True)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
