"""Autograd-friendly embedding modules on top of the sharded engine.

``ShardedEmbeddingModule`` exposes ``ShardedEmbeddingBags`` (table-wise /
row-wise sharded, fused optimizer in backward) as an ``nn.Module`` whose
forward returns one tensor per feature; gradients flowing back into those
tensors trigger the gradient all-to-all and the fused sort-based embedding
update inside ``backward`` — the semantics of TorchRec DMP with
``fused_params`` (torchrec/train.py:236-254), where embedding tables never
appear in the dense optimizer.

Pooled features (EmbeddingBagCollection, TwoTower/DLRM) use bag sizes from
``pooling``; sequence features (EmbeddingCollection, Bert4Rec) are bags of
size 1 over flattened positions.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .planner import ShardingPlan, plan_sharding
from .sharded import ShardedEmbeddingBags
from .tables import EmbOptimConfig, TableConfig


class _EmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, anchor, engine):
        engine.forward(ids)
        ctx.engine = engine
        return engine.recv.clone()

    @staticmethod
    def backward(ctx, grad):
        eng = ctx.engine
        eng.d_recv.copy_(grad.to(eng.d_recv.dtype))
        eng.backward_start()
        eng.backward_finish(eng._hyper)
        return None, None, None


class ShardedEmbeddingModule(torch.nn.Module):
    def __init__(self, tables: Sequence[TableConfig], batch_size: int,
                 pooling: Optional[Sequence[int]] = None, optim: Optional[EmbOptimConfig] = None,
                 device="cpu", world_size: int = 1, rank: int = 0, group=None,
                 strategy: str = "auto", plan: Optional[ShardingPlan] = None, seed: int = 0,
                 mean: bool = False, recv_dtype: str = "fp32"):
        """``recv_dtype``: "fp32" (default: the fp32 models of the reference,
        whose TBE returns fp32 rows, torchrec/models.py:158-164) or "bf16"
        (half the exchange bytes)."""
        super().__init__()
        self.tables = list(tables)
        self.pooling = list(pooling) if pooling is not None else [1] * len(self.tables)
        self.optim = optim or EmbOptimConfig("adam", lr=1e-3)
        self.plan = plan or plan_sharding(self.tables, world_size, self.optim,
                                          batch_per_rank=batch_size, pooling=self.pooling,
                                          strategy=strategy)
        self.step_bumped_by_caller = False     # the owner bumps the step counter
        self.engine = ShardedEmbeddingBags(self.tables, self.plan, rank, batch_size, self.pooling,
                                           device, self.optim, group=group, seed=seed, mean=mean,
                                           recv_dtype=recv_dtype)
        self.engine._hyper = torch.tensor([self.optim.lr, 0.0], dtype=torch.float32,
                                          device=device)
        # a differentiable anchor so autograd always calls backward
        self._anchor = torch.nn.Parameter(torch.zeros(1, device=device), requires_grad=True)
        self.B = batch_size
        self.D = self.tables[0].embedding_dim

    def set_lr(self, lr: float):
        self.engine._hyper[0:1].fill_(lr)

    def forward(self, ids: torch.Tensor) -> List[torch.Tensor]:
        """ids: flat int64, table-major, table t has B*L_t ids. Returns
        per-table pooled rows [B, D] (fp32 views over the receive buffer)."""
        if self.training and torch.is_grad_enabled():
            if not self.step_bumped_by_caller:
                self.engine._hyper[1:2].add_(1.0)
            recv = _EmbFn.apply(ids, self._anchor, self.engine)
        else:
            recv = self.engine.forward(ids).clone()
        eng = self.engine
        feats = []
        for t in range(len(self.tables)):
            feats.append(recv.as_strided((self.B, self.D), (eng.slot_stride[t], 1),
                                         eng.slot_off[t]).float())
        return feats

    def table_weight(self, t: int):
        return self.engine.get_table_weight(t)

    def set_table_weight(self, t: int, w: torch.Tensor):
        self.engine.set_table_weight(t, w)

    def extra_state(self):
        return self.engine.state_dict()
