#!/usr/bin/env python
"""GEMM kernel lab: every DLRM / DCN-v2 MLP GEMM shape (forward with bias +
ReLU, ReLU-masked dgrad, split-K weight grad with column sums) on uniform
random bf16 operands, each kernel variant (``ops.gemm_policy``) checked
against an fp32 torch oracle and timed from hipGraph replays, variants
interleaved round by round in one process (cdna_hip_programming.md §5.4
rules 24/25). Prints one JSON line per (shape, variant) plus totals.

Usage: python labs/gemm_lab.py --policies 0,31,32 [--model dlrm|dcnv2] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402

B = 8192
DLRM = [  # (name, kind, M, N, K, splits)
    ("bot1", "fwd", B, 256, 512, 1), ("bot1", "dgrad", B, 512, 256, 1),
    ("bot2", "fwd", B, 128, 256, 1),
    ("top0", "fwd", B, 1024, 512, 1), ("top0", "dgrad", B, 512, 1024, 1),
    ("top1", "fwd", B, 1024, 1024, 1), ("top1", "dgrad", B, 1024, 1024, 1),
    ("top2", "fwd", B, 512, 1024, 1), ("top2", "dgrad", B, 1024, 512, 1),
    ("top3", "fwd", B, 256, 512, 1), ("top3", "dgrad", B, 512, 256, 1),
    ("top0", "wgrad", 1024, 512, B, 4), ("top1", "wgrad", 1024, 1024, B, 4),
    ("top2", "wgrad", 512, 1024, B, 8), ("top3", "wgrad", 256, 512, B, 16),
    ("bot1", "wgrad", 256, 512, B, 16), ("bot0", "fwd", B, 512, 64, 1),
]
EDGE = [  # odd shapes: correctness of the partial-tile paths
    ("edgeA", "fwd", 1000, 200, 320, 1), ("edgeB", "dgrad", 1000, 480, 192, 1),
    ("edgeC", "wgrad", 200, 136, 1024, 2), ("edgeD", "fwd", 600, 1000, 64, 1),
]
DCN = [
    ("dcnV", "fwd", B, 512, 3456, 1), ("dcnU", "fwd", B, 3456, 512, 1),
    ("dcnU", "dgrad", B, 512, 3456, 1), ("dcnV", "dgrad", B, 3456, 512, 1),
    ("dcnU", "wgrad", 3456, 512, B, 2), ("dcnV", "wgrad", 512, 3456, B, 2),
    ("top0", "fwd", B, 1024, 3456, 1), ("top0", "dgrad", B, 3456, 1024, 1),
]


def timeit(fn, reps=20, iters=7):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
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
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


class Case:
    def __init__(self, name, kind, M, N, K, S, gen):
        self.name, self.kind, self.M, self.N, self.K, self.S = name, kind, M, N, K, S
        bf = torch.bfloat16
        dev = "cuda"
        r = lambda *s: (torch.rand(*s, generator=gen, device=dev) * 2 - 1).to(bf)  # noqa: E731
        if kind == "fwd":          # y = relu(x W^T + b)
            self.a, self.b = r(M, K), r(N, K)
            self.bias = torch.rand(N, generator=gen, device=dev) - 0.5
            self.out = torch.empty(M, N, dtype=bf, device=dev)
            ref = torch.relu(self.a.float() @ self.b.float().t() + self.bias)
        elif kind == "dgrad":      # dx = (dy W) * (x > 0)
            self.a, self.b = r(M, K), r(K, N)
            self.mask = r(M, N)
            self.out = torch.empty(M, N, dtype=bf, device=dev)
            ref = (self.a.float() @ self.b.float()) * (self.mask.float() > 0)
        else:                      # dW = dy^T x as split-K fp32 slabs, + colsum(dy) in col N
            self.a, self.b = r(K, M), r(K, N)
            self.ldc = N + 64
            self.out32 = torch.zeros(S, M, self.ldc, device=dev)
            ref = torch.cat([self.a.float().t() @ self.b.float(),
                             self.a.float().sum(0)[:, None]], 1)
        self.ref = ref
        self.flop = 2.0 * M * N * K

    def run(self):
        if self.kind == "fwd":
            ops.gemm(self.a, False, self.b, False, self.bias, True, None, self.out, None, 1)
        elif self.kind == "dgrad":
            ops.gemm(self.a, False, self.b, True, None, False, self.mask, self.out, None, 1)
        else:
            ops.gemm(self.a, True, self.b, True, None, False, None, None, self.out32, self.S,
                     ldc32=self.ldc, csum_col=self.N)

    def check(self):
        if self.kind == "wgrad":
            self.out32.zero_()
        else:
            self.out.fill_(float("nan"))
        self.run()
        torch.cuda.synchronize()
        got = (self.out32.sum(0)[:, : self.N + 1] if self.kind == "wgrad" else self.out.float())
        err = (got - self.ref).abs().max().item()
        scale = self.ref.abs().max().item() + 1e-6
        return err / scale


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--policies", default="0,31,32")
    ap.add_argument("--model", default="dlrm", choices=["dlrm", "dcnv2", "all", "edge"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    pols = [int(p) for p in args.policies.split(",")]
    shapes = {"dlrm": DLRM, "dcnv2": DCN, "all": DLRM + DCN, "edge": EDGE}[args.model]
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0)
    cases = [Case(*s, gen) for s in shapes if not args.only or args.only in f"{s[0]}.{s[1]}"]
    res = {}
    for c in cases:
        for p in pols:
            ops.gemm_policy(p)
            e = c.check()
            res[(c.name, c.kind, c.M, c.N, c.K, p)] = {"err": e, "ts": []}
            if not (e < 2e-2):
                print(json.dumps({"layer": c.name, "kind": c.kind, "policy": p, "BAD_rel_err": e}),
                      flush=True)
    for _ in range(args.rounds):
        for c in cases:
            for p in pols:
                ops.gemm_policy(p)
                res[(c.name, c.kind, c.M, c.N, c.K, p)]["ts"].append(timeit(c.run))
    tot = {p: 0.0 for p in pols}
    for c in cases:
        row = {"layer": c.name, "kind": c.kind, "MNK": [c.M, c.N, c.K], "S": c.S}
        for p in pols:
            ts = sorted(res[(c.name, c.kind, c.M, c.N, c.K, p)]["ts"])
            t = ts[len(ts) // 2]
            tot[p] += t
            row[f"p{p}_us"] = round(t, 2)
            row[f"p{p}_TF"] = round(c.flop / t / 1e6, 1)
            row[f"p{p}_err"] = float(f"{res[(c.name, c.kind, c.M, c.N, c.K, p)]['err']:.1e}")
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_us": {f"p{p}": round(v, 1) for p, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
