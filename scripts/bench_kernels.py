#!/usr/bin/env python
"""Per-kernel microbenchmarks on the DLRM-1TB shapes (MI355X).

Times each HIP kernel with HIP events (median of N launches, random data)
and, for GEMMs, the PyTorch-ROCm library GEMM (hipBLASLt) on the same
shapes as the comparison point. Prints one JSON line per case.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402


def timeit(fn, iters=7, warm=3, reps=20):
    """Median over `iters` of (time of `reps` back-to-back launches) / reps, in us."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


def gemm_cases(B, dcn=False):
    # (name, M, N, K): forward y = x W^T shapes of DLRM-1TB (+ DCN-v2's cross
    # layers V: 3456 -> 512, U: 512 -> 3456 and its 3456-wide top0)
    fwd = [("bot0", B, 512, 64), ("bot1", B, 256, 512), ("bot2", B, 128, 256),
           ("top0", B, 1024, 512), ("top1", B, 1024, 1024), ("top2", B, 512, 1024),
           ("top3", B, 256, 512)]
    if dcn:
        fwd += [("dcnV", B, 512, 3456), ("dcnU", B, 3456, 512), ("dcntop0", B, 1024, 3456)]
    return fwd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--only", default="")
    ap.add_argument("--policies", default="0", help="comma list of GEMM tile policies to A/B")
    ap.add_argument("--gemm-only", action="store_true")
    ap.add_argument("--wsplits", default="", help="comma list of wgrad split counts to time")
    ap.add_argument("--dcn", action="store_true", help="also the DCN-v2 cross-layer shapes")
    args = ap.parse_args()
    dev = "cuda"
    B = args.batch
    bf = torch.bfloat16
    out = []
    for name, M, N, K in gemm_cases(B, args.dcn):
        if args.only and args.only not in name:
            continue
        x = torch.randn(M, K, device=dev).to(bf)
        w = torch.randn(N, K, device=dev).to(bf)
        bias = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev, dtype=bf)
        dy = torch.randn(M, N, device=dev).to(bf)
        dx = torch.empty(M, K, device=dev, dtype=bf)
        gw = torch.empty(N * K, device=dev)
        fl = 2.0 * M * N * K
        for pol in [int(p) for p in args.policies.split(",")]:
            ops.gemm_policy(pol)
            t_f = timeit(lambda: ops.linear_fwd(x, w, bias, True, out=y))
            t_d = timeit(lambda: ops.linear_dgrad(dy, w, mask=x, out=dx))
            t_w = timeit(lambda: ops.linear_wgrad(dy, x, gw))
            print(json.dumps({"case": name, "policy": pol, "fwd_us": round(t_f, 1),
                              "fwd_TF": round(fl / t_f / 1e6, 1), "dgrad_us": round(t_d, 1),
                              "dgrad_TF": round(fl / t_d / 1e6, 1), "wgrad_us": round(t_w, 1),
                              "wgrad_TF": round(fl / t_w / 1e6, 1)}), flush=True)
        ops.gemm_policy(1)
        if args.wsplits:
            for sp in [int(v) for v in args.wsplits.split(",")]:
                slab = torch.empty(sp * N * K, device=dev)
                t_w = timeit(lambda: ops.linear_wgrad(dy, x, gw, slab=slab, splits=sp))
                print(json.dumps({"case": name, "wgrad_splits": sp, "wgrad_us": round(t_w, 1)}),
                      flush=True)
        if args.gemm_only:
            continue
        t_f = timeit(lambda: ops.linear_fwd(x, w, bias, True, out=y))
        t_t = timeit(lambda: torch.nn.functional.linear(x, w, bias.to(bf)))
        t_d = timeit(lambda: ops.linear_dgrad(dy, w, mask=x, out=dx))
        t_td = timeit(lambda: dy @ w)
        t_w = timeit(lambda: ops.linear_wgrad(dy, x, gw))
        t_tw = timeit(lambda: dy.t() @ x)
        t_cs = timeit(lambda: ops.colsum(dy, bias))
        rec = {"case": name, "M": M, "N": N, "K": K,
               "fwd_us": round(t_f, 1), "fwd_TF": round(fl / t_f / 1e6, 1),
               "torch_fwd_us": round(t_t, 1),
               "dgrad_us": round(t_d, 1), "dgrad_TF": round(fl / t_d / 1e6, 1),
               "torch_dgrad_us": round(t_td, 1),
               "wgrad_us": round(t_w, 1), "wgrad_TF": round(fl / t_w / 1e6, 1),
               "torch_wgrad_us": round(t_tw, 1), "colsum_us": round(t_cs, 1)}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    if args.gemm_only:
        return
    # interaction + embedding + head
    F, D, T = 27, 128, 26
    dense = torch.randn(B, D, device=dev).to(bf)
    emb = torch.randn(B * T * D, device=dev).to(bf)
    off = [0] + [t * D for t in range(T)]
    stride = [0] + [T * D] * T
    z = torch.empty(B, 512, device=dev, dtype=bf)
    t_if = timeit(lambda: ops.interaction_fwd(dense, emb, off, stride, F, D, z))
    dz = torch.randn(B, 512, device=dev).to(bf)
    dd = torch.empty(B, D, device=dev, dtype=bf)
    de = torch.empty_like(emb)
    t_ib = timeit(lambda: ops.interaction_bwd(dz, dense, emb, off, stride, F, D, dd, de, off,
                                              stride, True))
    print(json.dumps({"case": "interaction", "fwd_us": round(t_if, 1), "bwd_us": round(t_ib, 1),
                      "fwd_GBps": round((B * F * D * 2 + B * 512 * 2) / t_if / 1e3, 1),
                      "bwd_GBps": round((2 * B * F * D * 2 + B * 512 * 2) / t_ib / 1e3, 1)}),
          flush=True)
    rows = 40_000_000
    W = torch.empty(rows, D, device=dev).uniform_(-0.01, 0.01)
    ro = torch.zeros(T, dtype=torch.long, device=dev)
    ids = torch.randint(0, rows, (T * B,), device=dev)
    offs = torch.arange(T * B + 1, device=dev)
    oo = torch.tensor([t * D for t in range(T)], device=dev)
    outp = torch.empty(B * T * D, device=dev, dtype=bf)
    t_ef = timeit(lambda: ops.embedding_bag_fwd(W, ro, ids, offs, oo, T, B, outp, T * D))
    st = torch.zeros(rows, device=dev)
    hyper = torch.tensor([0.01, 1.0], device=dev)
    t_eb = timeit(lambda: ops.embedding_bwd(W, ro, ids, offs, oo, T, B, outp, T * D,
                                            ops.EMB_ROWWISE_ADAGRAD, hyper, state1=st))
    print(json.dumps({"case": "embedding", "nnz": T * B, "fwd_us": round(t_ef, 1),
                      "bwd_fused_us": round(t_eb, 1),
                      "fwd_GBps": round(T * B * (D * 4 + D * 2) / t_ef / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
