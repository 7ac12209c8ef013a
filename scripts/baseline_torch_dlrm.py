#!/usr/bin/env python
"""Stock PyTorch-ROCm eager DLRM / DCN-v2 baseline (BASELINE.md protocol item (a)).

Same model/config as bench.py, built only from stock modules: one
nn.EmbeddingBag(mode="sum", sparse=True) per table, nn.Linear MLPs, bmm dot
interaction (DLRM) or the low-rank cross network x_{l+1} = x0 * (U V^T x_l +
b) + x_l (DCN-v2, 3 layers of rank 512, MLPerf multi-hot pooling),
BCEWithLogits, bf16 autocast; torch.optim.Adagrad (sparse) for the tables,
torch.optim.AdamW for the dense part. No custom kernels, no graphs, no
compiler. Prints one JSON line with examples/s.
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from tdfo_amd.data.synthetic import SyntheticCriteo  # noqa: E402
from tdfo_amd.models.dlrm import (CRITEO_1TB_ROWS, CRITEO_KAGGLE_ROWS,  # noqa: E402
                                  MLPERF_MULTIHOT)


def mlp(sizes, last_relu=True):
    layers = []
    for i in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[i], sizes[i + 1]))
        if i < len(sizes) - 2 or last_relu:
            layers.append(nn.ReLU())
    return nn.Sequential(*layers)


class TorchDLRM(nn.Module):
    def __init__(self, rows, D=128, bottom=(512, 256, 128), top=(1024, 1024, 512, 256, 1)):
        super().__init__()
        self.embs = nn.ModuleList([nn.EmbeddingBag(r, D, mode="sum", sparse=True) for r in rows])
        for e in self.embs:
            nn.init.uniform_(e.weight, -(1 / e.num_embeddings) ** 0.5, (1 / e.num_embeddings) ** 0.5)
        self.bot = mlp((13,) + tuple(bottom))
        F = len(rows) + 1
        self.li, self.lj = torch.tril_indices(F, F, offset=-1)
        self.top = mlp((D + F * (F - 1) // 2,) + tuple(top), last_relu=False)

    def forward(self, dense, ids_per_table, offsets):
        x = self.bot(dense)
        feats = [x] + [e(i, offsets) for e, i in zip(self.embs, ids_per_table)]
        X = torch.stack(feats, 1)
        Z = torch.bmm(X, X.transpose(1, 2))
        z = Z[:, self.li, self.lj]
        return self.top(torch.cat([x, z], 1)).squeeze(1)


class TorchDCN(nn.Module):
    """DCN-v2 (stacked cross network, low-rank U V^T) on stock modules."""

    def __init__(self, rows, D=128, bottom=(512, 256, 128), top=(1024, 1024, 512, 256, 1),
                 layers=3, rank=512):
        super().__init__()
        self.embs = nn.ModuleList([nn.EmbeddingBag(r, D, mode="sum", sparse=True) for r in rows])
        for e in self.embs:
            nn.init.uniform_(e.weight, -(1 / e.num_embeddings) ** 0.5, (1 / e.num_embeddings) ** 0.5)
        self.bot = mlp((13,) + tuple(bottom))
        W = (len(rows) + 1) * D
        self.V = nn.ModuleList([nn.Linear(W, rank, bias=False) for _ in range(layers)])
        self.U = nn.ModuleList([nn.Linear(rank, W) for _ in range(layers)])
        self.top = mlp((W,) + tuple(top), last_relu=False)

    def forward(self, dense, ids_per_table, offsets):
        x = self.bot(dense)
        x0 = torch.cat([x] + [e(i, o) for e, i, o in zip(self.embs, ids_per_table, offsets)], 1)
        xl = x0
        for V, U in zip(self.V, self.U):
            xl = x0 * U(V(xl)) + xl
        return self.top(xl).squeeze(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1tb", choices=["1tb", "kaggle"])
    ap.add_argument("--model", default="dlrm", choices=["dlrm", "dcnv2"])
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    rows = CRITEO_1TB_ROWS if a.rows == "1tb" else CRITEO_KAGGLE_ROWS
    L = list(MLPERF_MULTIHOT) if a.model == "dcnv2" else [1] * len(rows)
    if a.model == "dcnv2":
        model = TorchDCN(rows).to(dev)
    else:
        model = TorchDLRM(rows).to(dev)
        model.li, model.lj = model.li.to(dev), model.lj.to(dev)
    sparse = [p for e in model.embs for p in e.parameters()]
    dense = [p for n, p in model.named_parameters() if not n.startswith("embs.")]
    opt_s = torch.optim.Adagrad(sparse, lr=0.01)
    opt_d = torch.optim.AdamW(dense, lr=1e-3)
    data = SyntheticCriteo(rows, a.batch, pooling=L, device=dev, seed=1)
    pool = [data.next() for _ in range(4)]
    offs = [torch.arange(0, a.batch * l, l, device=dev) for l in L]
    lossf = nn.BCEWithLogitsLoss()

    def step(i):
        d, ids, y = pool[i % len(pool)]
        per = list(torch.split(ids, [a.batch * l for l in L]))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = (model(d, per, offs) if a.model == "dcnv2" else
                   model(d, per, offs[0]))
            loss = lossf(out.float(), y)
        opt_s.zero_grad(set_to_none=True)
        opt_d.zero_grad(set_to_none=True)
        loss.backward()
        opt_s.step()
        opt_d.step()
        return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(json.dumps({"baseline": "pytorch-rocm eager (nn.EmbeddingBag sparse + Adagrad, "
                      "nn.Linear + AdamW, bf16 autocast)", "model": a.model, "rows": a.rows,
                      "batch": a.batch,
                      "ms_per_step": round(el / a.steps * 1e3, 3),
                      "examples_per_sec": round(a.batch * a.steps / el, 1)}))


if __name__ == "__main__":
    main()
