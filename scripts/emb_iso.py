#!/usr/bin/env python
"""Isolated timings of the embedding-queue kernels on the headline shapes.

DLRM-1TB (26 one-hot tables, MLPerf Criteo-TB cardinalities, B = 8192,
D = 128, row-wise Adagrad) and DCN-v2 (same tables, MLPerf multi-hot pooling,
1.75 M ids): forward lookup, backward prepare (keys + sort) and apply (segment
reduce + optimizer), each graph-replayed alone, with the bytes each one must
move and the achieved rate. Run under rocprofv3 --kernel-trace --stats for the
per-kernel split. Uniform ids, as bench.py's synthetic batches.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402
from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, MLPERF_MULTIHOT  # noqa: E402


def timeit(fn, reps=20, iters=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
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
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="dlrm,dcn")
    ap.add_argument("--batch", type=int, default=8192)
    args = ap.parse_args()
    dev = "cuda"
    B, D = args.batch, 128
    rows = CRITEO_1TB_ROWS
    T = len(rows)
    ro_h = [0]
    for r in rows[:-1]:
        ro_h.append(ro_h[-1] + r)
    total = ro_h[-1] + rows[-1]
    W = torch.empty(total, D, device=dev)
    W.uniform_(-0.01, 0.01)
    st = torch.zeros(total, device=dev)
    ro = torch.tensor(ro_h, dtype=torch.int64, device=dev)
    hyper = torch.tensor([1e-3, 1.0], device=dev)
    kb = ops.key_bits_for(total) if hasattr(ops, "key_bits_for") else 28
    out_off = torch.tensor([t * D for t in range(T)], device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    for case in args.cases.split(","):
        L = [1] * T if case == "dlrm" else list(MLPERF_MULTIHOT)
        lens = torch.tensor(L, device=dev).repeat_interleave(B)
        offs = torch.zeros(T * B + 1, dtype=torch.long, device=dev)
        offs[1:] = torch.cumsum(lens, 0)
        nnz = int(offs[-1])
        ids = torch.cat([torch.randint(0, rows[t], (B * L[t],), device=dev, generator=gen)
                         for t in range(T)])
        out = torch.empty(B * T * D, device=dev, dtype=torch.bfloat16)
        grad = (torch.randn(B * T * D, device=dev) * 1e-3).to(torch.bfloat16)
        onehot = case == "dlrm"
        seg = 1 if onehot else 0
        bag_len = None if onehot else torch.tensor(L, dtype=torch.int32, device=dev)
        ws = torch.empty(ops.embedding_bwd_workspace(nnz, D), dtype=torch.uint8, device=dev)
        fwd = lambda: ops.embedding_bag_fwd(W, ro, ids, offs, out_off, T, B, out, T * D,  # noqa
                                            onehot=onehot)
        prep = lambda: ops.embedding_bwd_prepare(W, ro, ids, offs, out_off, T, B, T * D, ws,  # noqa
                                                 key_bits=kb, segsort=seg, bag_len=bag_len)
        apply = lambda: ops.embedding_bwd_apply(W, ro, ids, offs, out_off, T, B, grad, T * D,  # noqa
                                                ops.EMB_ROWWISE_ADAGRAD, hyper, ws, state1=st,
                                                key_bits=kb, segsort=seg)
        prep()
        torch.cuda.synchronize()
        # bytes: fwd = rows read + pooled bf16 written; apply = grads read (bf16)
        # + unique rows read & written + row state read & written
        uniq = 0
        for t in range(T):
            s0, s1 = int(offs[t * B]), int(offs[(t + 1) * B])
            uniq += int(torch.unique(ids[s0:s1]).numel())
        fwd_b = nnz * D * 4 + B * T * D * 2
        app_b = nnz * D * 2 + uniq * (2 * D * 4 + 8)
        tf = timeit(fwd)
        tp = timeit(prep)
        ta = timeit(apply)

        def both():
            prep()
            apply()
        tb = timeit(both)
        print(json.dumps({"case": case, "nnz": nnz, "unique_rows": uniq,
                          "fwd_us": round(tf, 1), "fwd_TBps": round(fwd_b / tf / 1e6, 2),
                          "prep_us": round(tp, 1), "apply_us": round(ta, 1),
                          "apply_TBps": round(app_b / ta / 1e6, 2), "bwd_us": round(tb, 1)}),
              flush=True)
        del ws, out, grad, ids, offs


if __name__ == "__main__":
    main()
