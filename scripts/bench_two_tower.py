#!/usr/bin/env python
"""TwoTower (Goodreads-shaped, reference config: per-device batch 2048, E=16)
training throughput on one GPU: fused step, hipGraph replay, synthetic ids
with real Goodreads cardinalities (876k users, 2.36M books)."""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from tdfo_amd.models.two_tower import FEATURES, SIZE_KEYS, TwoTowerConfig, TwoTowerTrainer  # noqa

GOODREADS = {"user": 876145, "item": 2360650, "language": 227, "is_ebook": 2, "format": 769,
             "publisher": 126702, "pub_decade": 14}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--emb-update", default="sparse")
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    cfg = TwoTowerConfig(GOODREADS, emb_update=a.emb_update)
    tr = TwoTowerTrainer(cfg, a.batch, dev)
    # HBM-resident synthetic columns (Goodreads cardinalities and dtypes);
    # every step gathers a shuffled batch into the static buffers in one launch
    g = torch.Generator(device=dev).manual_seed(0)
    N = 8 * a.batch * 16
    cols = {f: torch.randint(0, GOODREADS[k], (N,), device=dev, generator=g).to(torch.int32)
            for f, k in zip(FEATURES, SIZE_KEYS)}
    cols["avg_rating"] = torch.rand(N, device=dev, generator=g)
    cols["num_pages"] = torch.rand(N, device=dev, generator=g)
    cols["label"] = (torch.rand(N, device=dev, generator=g) < 0.5).to(torch.int8)
    perm = torch.randperm(N, device=dev, generator=g)
    pool = [perm[i * a.batch:(i + 1) * a.batch] for i in range(N // a.batch)]
    for i in range(a.warmup):
        tr.load_columns(cols, pool[i % len(pool)], 0, a.batch)
        tr.step()
    if not a.no_graph:
        tr.capture_graph()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(a.steps):
        tr.load_columns(cols, pool[i % len(pool)], 0, a.batch)
        tr.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(json.dumps({"model": "two_tower", "batch": a.batch, "emb_update": a.emb_update,
                      "graph": not a.no_graph, "ms_per_step": round(el / a.steps * 1e3, 4),
                      "examples_per_sec": round(a.batch * a.steps / el, 1)}))


if __name__ == "__main__":
    main()
