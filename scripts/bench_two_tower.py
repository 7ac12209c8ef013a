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
    g = torch.Generator(device=dev).manual_seed(0)
    pool = []
    for i in range(8):
        d = {f: torch.randint(0, GOODREADS[k], (a.batch,), device=dev, generator=g)
             for f, k in zip(FEATURES, SIZE_KEYS)}
        d["avg_rating"] = torch.rand(a.batch, device=dev, generator=g)
        d["num_pages"] = torch.rand(a.batch, device=dev, generator=g)
        d["label"] = (torch.rand(a.batch, device=dev, generator=g) < 0.5).float()
        pool.append(d)
    for i in range(a.warmup):
        tr.load_batch(pool[i % 8])
        tr.step()
    if not a.no_graph:
        tr.capture_graph()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(a.steps):
        tr.load_batch(pool[i % 8])
        tr.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(json.dumps({"model": "two_tower", "batch": a.batch, "emb_update": a.emb_update,
                      "graph": not a.no_graph, "ms_per_step": round(el / a.steps * 1e3, 4),
                      "examples_per_sec": round(a.batch * a.steps / el, 1)}))


if __name__ == "__main__":
    main()
