#!/usr/bin/env python
"""Bert4Rec training throughput on one GPU (reference config: per-device batch
16, T=20, E=16, 2 heads, 2 layers) with a Goodreads-scale vocabulary."""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from tdfo_amd.models.bert4rec import Bert4RecTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--torch-encoder", action="store_true",
                    help="torch reference attention/LayerNorm instead of the HIP kernels")
    a = ap.parse_args()
    if a.torch_encoder:
        import tdfo_amd.models.bert4rec as m
        m.USE_FUSED = False
    dev = "cuda"
    T = 20
    tr = Bert4RecTrainer(a.items, T, 16, 2, 2, a.batch, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    pool = []
    for _ in range(8):
        s = torch.randint(1, a.items + 1, (a.batch, T), device=dev, generator=g)
        m = torch.rand(a.batch, T, device=dev, generator=g) < 0.2
        m[:, -1] = True
        lab = torch.where(m, s, torch.zeros_like(s))
        s = torch.where(m, torch.full_like(s, a.items + 1), s)
        pool.append((s, lab))
    for i in range(a.warmup):
        tr.load_batch(*pool[i % 8])
        tr.step()
    if not a.no_graph:
        tr.capture_graph()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(a.steps):
        tr.load_batch(*pool[i % 8])
        tr.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(json.dumps({"model": "bert4rec", "batch": a.batch, "vocab": a.items + 2,
                      "graph": not a.no_graph, "fused_encoder": not a.torch_encoder, "ms_per_step": round(el / a.steps * 1e3, 4),
                      "sequences_per_sec": round(a.batch * a.steps / el, 1),
                      "loss": round(tr.pop_loss(), 4)}))


if __name__ == "__main__":
    main()
