"""Microbenchmark of the fused linear + CE kernel (Bert4Rec output layer)."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from tdfo_amd import ops  # noqa: E402

import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", type=int, default=-1, help="run only this config index")
ap.add_argument("--impls", default="1,0,1,0", help="in-process A/B order")
ap.add_argument("--no-torch", action="store_true")
args = ap.parse_args()
dev = "cuda"
CFGS = [(1_000_002, 320, 0.24), (1_000_002, 5120, 0.24), (100_002, 320, 0.24)]
for ci, (V, N, frac) in enumerate(CFGS):
    if args.cfg >= 0 and ci != args.cfg:
        continue
    H = torch.randn(N, 16, device=dev)
    W = torch.randn(V, 16, device=dev) * 0.1
    b = torch.zeros(V, device=dev)
    y = torch.randint(1, V, (N,), device=dev)
    y[torch.rand(N, device=dev) > frac] = 0
    out = [torch.empty(N, 16, device=dev), torch.empty(N, device=dev),
           torch.empty(V, 16, device=dev), torch.empty(V, device=dev)]
    us = {}
    for impl in [int(x) for x in args.impls.split(",")]:   # later rounds reported
        ops.linear_xent_impl(impl)
        for _ in range(3):
            ops.linear_xent(H, W, b, y, 0.1, 0, *out)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            ops.linear_xent(H, W, b, y, 0.1, 0, *out)
        torch.cuda.synchronize()
        us["mfma" if impl else "valu"] = (time.perf_counter() - t) / 20 * 1e6
    ops.linear_xent_impl(1)
    if args.no_torch:
        print(json.dumps({"V": V, "N": N, **{k: round(v, 1) for k, v in us.items()}}))
        continue
    # materialising reference (torch): logits + CE fwd/bwd
    Hr = H.clone().requires_grad_(True)
    Wr = W.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    def ref():
        l = torch.nn.functional.cross_entropy(Hr @ Wr.t() + br, y, ignore_index=0,
                                              label_smoothing=0.1)
        l.backward()
    for _ in range(2):
        ref()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        ref()
    torch.cuda.synchronize()
    us_ref = (time.perf_counter() - t) / 5 * 1e6
    print(json.dumps({"V": V, "N": N, "valid": int((y != 0).sum()), "fused_mfma_us": round(us.get("mfma", 0), 1),
                      "fused_valu_us": round(us.get("valu", 0), 1),
                      "torch_materialized_us": round(us_ref, 1)}))
