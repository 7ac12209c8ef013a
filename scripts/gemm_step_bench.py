#!/usr/bin/env python
"""Time every GEMM of one DLRM / DCN-v2 training step in isolation (MI355X).

Builds a DLRMTrainer with tiny tables (the dense part, and so every GEMM, is
the same as at Criteo-1TB scale), then replays each of its GEMM calls --
forward (bias/ReLU epilogue), dgrad (ReLU-mask epilogue), split-K wgrad into
its slab -- exactly as the step issues them, each timed with HIP events over
back-to-back launches. Prints one JSON line per (policy, layer, kind) and a
per-policy total, so tile/kernel changes can be A/B'd on the real step shapes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402
from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer  # noqa: E402


def timeit(fn, iters=7, reps=30):
    """Median per-launch time of `reps` launches captured in one hipGraph (the
    step runs graph-replayed: host dispatch cost must not show up here)."""
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


def calls(tr: DLRMTrainer):
    """(name, kind, flops, fn) for every MLP GEMM of the step."""
    out = []
    B = tr.B
    layers = [(L, tr.bot_in[i], tr.bot_in[i + 1][:, :L.out] if i + 1 < len(tr.bottom_layers)
               else tr.h_out, tr.bot_grad[i], tr.bot_grad[i - 1] if i > 0 else None, i > 0)
              for i, L in enumerate(tr.bottom_layers)]
    n = len(tr.top_layers)
    for i, L in enumerate(tr.top_layers):
        o = tr.top_in[i + 1][:, :L.out] if i + 1 < n else tr.t_out
        dx = tr.top_grad[i - 1] if i > 0 else tr.dz
        layers.append((L, tr.top_in[i], o, tr.top_grad[i], dx, i > 0))
    if tr.cfg.interaction == "dcn":
        fp, Wd, r = tr.fp, tr.top_real, tr.cfg.dcn_rank
        x0 = tr.dcn_x[0]
        for i, u in enumerate(tr.dcn_u):
            V = fp.bf16(f"dcn{i}.v")
            Uw = fp.bf16(u.name + ".w")
            h, xi = tr.dcn_h[i], tr.dcn_x[i]
            fl = 2.0 * B * Wd * r
            out.append((f"dcn{i}", "V.fwd", fl, lambda xi=xi, V=V, h=h, u=u: ops.linear_fwd(
                xi[:, :Wd], V, None, relu=False, out=h[:, :u.in_real])))
            out.append((f"dcn{i}", "U.fwd", fl, lambda h=h, Uw=Uw, u=u, i=i, xi=xi: ops.gemm(
                h[:, :u.in_k], False, Uw[:, :u.in_k], False,
                None if u.bias_in_k else fp.param(u.name + ".w")[:, u.bcol], False, None,
                tr.dcn_y[i], None, 1, mul=x0, add=xi[:, :Wd], out2=tr.dcn_x[i + 1][:, :Wd])))
            dy, dh = tr._dcn_bufs(i)
            out.append((f"dcn{i}", "U.wgrad", fl, lambda u=u, h=h, dy=dy: tr._wgrad(u, h, dy)))
            out.append((f"dcn{i}", "U.dgrad", fl, lambda Uw=Uw, u=u, dy=dy, dh=dh: ops.gemm(
                dy, False, Uw[:, :u.in_k], True, None, False, None, dh, None, 1)))
            out.append((f"dcn{i}", "V.wgrad", fl, lambda i=i: tr._dcn_wgrad_v(i)))
            out.append((f"dcn{i}", "V.dgrad", fl, lambda V=V, i=i, dh=dh: ops.gemm(
                dh, False, V, True, None, False, None, None, None, 1,
                add=tr.dcn_dx[i + 1], out2=tr.dcn_dx[i])))
    for L, x, o, dy, dx, relu_in in layers:
        fl = 2.0 * B * L.out * L.in_k
        out.append((L.name, "fwd", fl, lambda L=L, x=x, o=o: tr._fwd(L, x, o)))
        if dx is not None:
            nn_ = min(dx.shape[1], L.in_k)
            out.append((L.name, "dgrad", 2.0 * B * L.out * nn_,
                        lambda L=L, x=x, dy=dy, dx=dx, r=relu_in: tr._dgrad(L, x, dy, dx, r)))
        out.append((L.name, "wgrad", 2.0 * B * L.out * L.wcols,
                    lambda L=L, x=x, dy=dy: tr._wgrad(L, x, dy)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--policies", default="0")
    ap.add_argument("--model", default="dlrm", choices=["dlrm", "dcnv2"])
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    cfg = DLRMConfig(table_rows=[1000] * 26, interaction="dot" if args.model == "dlrm" else "dcn")
    tr = DLRMTrainer(cfg, args.batch, "cuda")
    cs = calls(tr)
    for pol in [int(p) for p in args.policies.split(",")]:
        ops.gemm_policy(pol)
        tot = 0.0
        tot_fl = 0.0
        for name, kind, fl, fn in cs:
            if args.only and args.only not in f"{name}.{kind}":
                continue
            t = timeit(fn)
            tot += t
            tot_fl += fl
            print(json.dumps({"policy": pol, "layer": name, "kind": kind, "us": round(t, 2),
                              "TF": round(fl / t / 1e6, 1)}), flush=True)
        print(json.dumps({"policy": pol, "total_us": round(tot, 1),
                          "TF": round(tot_fl / max(tot, 1e-9) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
