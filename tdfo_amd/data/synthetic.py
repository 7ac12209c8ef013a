"""Synthetic Criteo-shaped batches (BASELINE.json: "synthetic Criteo-shaped
data / random-init embeddings").

Dense features are log-normal-ish like log(1 + count) Criteo integers, ids
are uniform (default) or Zipf-skewed per table, labels follow a fixed random
logistic "teacher" over the dense features and a hash of the ids so the
loss is learnable. Generation runs on-device (no host round trip); the C++
host generator in csrc/data backs the host pipeline (see loader.py).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch


class SyntheticCriteo:
    def __init__(self, table_rows: Sequence[int], batch_size: int, num_dense: int = 13,
                 pooling: Optional[Sequence[int]] = None, device="cpu", seed: int = 0,
                 dist: str = "uniform", zipf_alpha: float = 1.05, rank: int = 0):
        self.rows = [int(r) for r in table_rows]
        self.T = len(self.rows)
        self.B = int(batch_size)
        self.num_dense = num_dense
        self.L = list(pooling) if pooling is not None else [1] * self.T
        self.device = torch.device(device)
        self.dist = dist
        self.alpha = zipf_alpha
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed * 7919 + rank)
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)   # teacher shared by all ranks
        self.w_dense = (torch.randn(num_dense, generator=g) / num_dense ** 0.5).to(self.device)
        self.table_bias = (torch.randn(self.T, 64, generator=g) * 0.5).to(self.device)

    def _ids(self, t: int, n: int) -> torch.Tensor:
        r = self.rows[t]
        if self.dist == "zipf" and r > 1:
            u = torch.rand(n, generator=self.gen, device=self.device)
            # inverse-CDF approximation of a bounded power law on [1, r]
            a = self.alpha
            x = ((r ** (1 - a) - 1) * u + 1) ** (1 / (1 - a))
            return (x.long() - 1).clamp_(0, r - 1)
        return torch.randint(0, r, (n,), generator=self.gen, device=self.device)

    def next(self):
        B = self.B
        dense = torch.log1p(torch.rand(B, self.num_dense, generator=self.gen, device=self.device)
                            * 100.0)
        ids: List[torch.Tensor] = []
        score = (dense - 3.6) @ self.w_dense * 2.0 - 1.1
        for t in range(self.T):
            it = self._ids(t, B * self.L[t])
            ids.append(it)
            first = it.view(B, self.L[t])[:, 0]
            score = score + self.table_bias[t][first % 64] * (3.0 / self.T ** 0.5)
        label = (torch.rand(B, generator=self.gen, device=self.device)
                 < torch.sigmoid(score)).float()
        return dense, torch.cat(ids), label
