#!/usr/bin/env python
"""Run one DLRM GEMM shape N times under a given tile policy (for rocprofv3
kernel-trace / PMC passes). Usage: gemm_probe.py fwd|dgrad|wgrad|cross M N K policy [iters]
(cross: the DCN-v2 U forward with its Hadamard / residual epilogue)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402


def main():
    kind, M, N, K, pol = sys.argv[1], *map(int, sys.argv[2:6])
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 50
    ops.gemm_policy(pol)
    bf = torch.bfloat16
    x = torch.randn(M, K, device="cuda").to(bf)
    w = torch.randn(N, K, device="cuda").to(bf)
    dy = torch.randn(M, N, device="cuda").to(bf)
    y = torch.empty(M, N, device="cuda", dtype=bf)
    dx = torch.empty(M, K, device="cuda", dtype=bf)
    gw = torch.empty(N * K, device="cuda")
    mul = torch.randn(M, N, device="cuda").to(bf) if kind == "cross" else None
    add = torch.randn(M, N, device="cuda").to(bf) if kind == "cross" else None
    y2 = torch.empty(M, N, device="cuda", dtype=bf) if kind == "cross" else None
    bias = torch.randn(N, device="cuda")
    fn = {"fwd": lambda: ops.linear_fwd(x, w, None, True, out=y),
          "cross": lambda: ops.gemm(x, False, w, False, bias, False, None, y, None, 1, mul=mul,
                                    add=add, out2=y2),
          "dgrad": lambda: ops.linear_dgrad(dy, w, mask=x, out=dx),
          "wgrad": lambda: ops.linear_wgrad(dy, x, gw)}[kind]
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
