"""Jagged sparse-feature containers and collections.

``KeyedJaggedTensor`` mirrors the torchrec container the reference feeds its
models (torchrec/train.py:33-41: ``from_lengths_sync``, ``to``, per-key
access, ``stride``; torchrec/models.py:210-212 ``to_padded_dense``): keys,
one flat ``values`` id tensor, per-(key, sample) ``lengths`` in key-major
order and the derived ``offsets``. Conversions to padded dense run on the
``tdfo::jagged_*`` HIP kernels.

``EmbeddingBagCollection`` (pooled, variable bag sizes) and
``EmbeddingCollection`` (unpooled sequences) are the single-device /
replicated collections: all tables of one width live in one
``TableBatchedEmbedding`` and one launch serves every key; the backward is
the fused sort-based optimizer (no dense table gradient). The sharded,
static-shape engine for multi-GPU training is ``ShardedEmbeddingModule``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import torch

from .. import ops
from .tables import EmbOptimConfig, TableBatchedEmbedding, TableConfig


def lengths_to_offsets(lengths: torch.Tensor) -> torch.Tensor:
    off = torch.zeros(lengths.numel() + 1, dtype=torch.int64, device=lengths.device)
    torch.cumsum(lengths.to(torch.int64), 0, out=off[1:])
    return off


@dataclass
class JaggedTensor:
    values: torch.Tensor            # [nnz] ids or [nnz, D] rows
    lengths: torch.Tensor           # [B]
    offsets: torch.Tensor           # [B + 1]

    def to_padded_dense(self, desired_length: int, padding_value=0) -> torch.Tensor:
        B = self.lengths.numel()
        if self.values.dim() == 1:
            out = torch.empty(B, desired_length, dtype=torch.int64, device=self.values.device)
            ops.jagged_ids_to_dense(self.values.to(torch.int64).contiguous(), self.offsets,
                                    int(padding_value), out)
            return out
        return JaggedToDense.apply(self.values, self.offsets, desired_length,
                                   float(padding_value))


class KeyedJaggedTensor:
    def __init__(self, keys: Sequence[str], values: torch.Tensor, lengths: torch.Tensor,
                 offsets: Optional[torch.Tensor] = None):
        self._keys = list(keys)
        self._values = values
        self._lengths = lengths.to(torch.int64)
        assert self._lengths.numel() % max(1, len(self._keys)) == 0, "lengths not key-major"
        self._offsets = offsets if offsets is not None else lengths_to_offsets(self._lengths)

    @classmethod
    def from_lengths_sync(cls, keys, values, lengths):
        return cls(keys, values, torch.as_tensor(lengths))

    @classmethod
    def from_dense(cls, keys: Sequence[str], dense: Dict[str, torch.Tensor]):
        """Fixed bag size per key: dense[k] is [B] or [B, L]."""
        vals, lens = [], []
        for k in keys:
            x = dense[k]
            x = x.view(-1, 1) if x.dim() == 1 else x
            vals.append(x.reshape(-1))
            lens.append(torch.full((x.shape[0],), x.shape[1], dtype=torch.int64,
                                   device=x.device))
        return cls(keys, torch.cat(vals), torch.cat(lens))

    def keys(self) -> List[str]:
        return list(self._keys)

    def values(self) -> torch.Tensor:
        return self._values

    def lengths(self) -> torch.Tensor:
        return self._lengths

    def offsets(self) -> torch.Tensor:
        return self._offsets

    def stride(self) -> int:
        return self._lengths.numel() // max(1, len(self._keys))

    def to(self, device, non_blocking: bool = False) -> "KeyedJaggedTensor":
        return KeyedJaggedTensor(self._keys, self._values.to(device, non_blocking=non_blocking),
                                 self._lengths.to(device, non_blocking=non_blocking),
                                 self._offsets.to(device, non_blocking=non_blocking))

    def __getitem__(self, key: str) -> JaggedTensor:
        i = self._keys.index(key)
        B = self.stride()
        o = self._offsets
        lo, hi = int(o[i * B]), int(o[(i + 1) * B])
        return JaggedTensor(self._values[lo:hi], self._lengths[i * B:(i + 1) * B],
                            o[i * B:(i + 1) * B + 1] - lo)

    def to_dict(self) -> Dict[str, JaggedTensor]:
        return {k: self[k] for k in self._keys}


class JaggedToDense(torch.autograd.Function):
    """[nnz, D] rows + offsets -> [B, T, D] (fbgemm jagged_2d_to_dense)."""

    @staticmethod
    def forward(ctx, values, offsets, T, pad):
        B = offsets.numel() - 1
        out = torch.empty(B, T, values.shape[1], dtype=torch.float32, device=values.device)
        ops.jagged_to_dense(values.float().contiguous(), offsets, T, pad, out)
        ctx.save_for_backward(offsets)
        ctx.nnz = values.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        (offsets,) = ctx.saved_tensors
        vg = torch.empty(ctx.nnz, g.shape[2], dtype=torch.float32, device=g.device)
        ops.dense_to_jagged(g.float().contiguous(), offsets, vg)
        return vg, None, None, None


class _CollectionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, owner, values, offsets, B, pooled):
        ctx.owner, ctx.args = owner, (values, offsets, B, pooled)
        return owner._lookup(values, offsets, B, pooled)

    @staticmethod
    def backward(ctx, g):
        ctx.owner._update(g.contiguous(), *ctx.args)
        return None, None, None, None, None, None


class _LocalCollection(torch.nn.Module):
    def __init__(self, tables: Sequence[TableConfig], optim: Optional[EmbOptimConfig], device,
                 seed: int = 0):
        super().__init__()
        self.tables = list(tables)
        dims = {t.embedding_dim for t in self.tables}
        assert len(dims) == 1, "one embedding width per collection"
        self.D = dims.pop()
        self.optim = optim or EmbOptimConfig("adam", lr=1e-3)
        self.store = TableBatchedEmbedding(
            [t.num_embeddings for t in self.tables], self.D, device, self.optim,
            init_ranges=[t.init_range or (1.0 / t.num_embeddings) ** 0.5 for t in self.tables],
            seed=seed)
        self.feature_to_table: Dict[str, int] = {}
        for i, t in enumerate(self.tables):
            for f in t.feature_names:
                self.feature_to_table[f] = i
        self.hyper = torch.tensor([self.optim.lr, 0.0], dtype=torch.float32, device=device)
        self._anchor = torch.nn.Parameter(torch.zeros(1, device=device))

    def _row_offsets(self, keys: Sequence[str]) -> torch.Tensor:
        ro = self.store.row_offset_host
        return torch.tensor([ro[self.feature_to_table[k]] for k in keys], dtype=torch.int64,
                            device=self.store.weight.device)

    def _lookup(self, values, offsets, B, pooled):
        nk = (offsets.numel() - 1) // B
        self._ro = self._row_offsets(self._keys)
        if pooled:
            out = torch.empty(B, nk * self.D, dtype=torch.float32, device=values.device)
            oo = torch.arange(nk, dtype=torch.int64, device=values.device) * self.D
            self.store.forward(values, offsets, self._ro, nk, B, out, oo, nk * self.D)
            return out
        # unpooled: every id is its own bag
        nnz = values.numel()
        bag_off = torch.arange(nnz + 1, dtype=torch.int64, device=values.device)
        kb = offsets[::B]                                   # key boundaries [nk + 1]
        key_of = torch.repeat_interleave(torch.arange(nk, device=values.device), kb[1:] - kb[:-1])
        keys_ro = self._ro[key_of]
        out = torch.empty(nnz, self.D, dtype=torch.float32, device=values.device)
        zero = torch.zeros(1, dtype=torch.int64, device=values.device)
        self.store.forward(values + keys_ro, bag_off, zero, 1, nnz, out, zero, self.D)
        self._flat_ids = values + keys_ro
        return out

    def _update(self, g, values, offsets, B, pooled):
        self.hyper[1:2].add_(1.0)
        if pooled:
            nk = (offsets.numel() - 1) // B
            oo = torch.arange(nk, dtype=torch.int64, device=g.device) * self.D
            self.store.backward_update(values, offsets, self._ro, nk, B, g, oo, nk * self.D,
                                       self.hyper)
        else:
            nnz = values.numel()
            bag_off = torch.arange(nnz + 1, dtype=torch.int64, device=g.device)
            zero = torch.zeros(1, dtype=torch.int64, device=g.device)
            self.store.backward_update(self._flat_ids, bag_off, zero, 1, nnz, g, zero, self.D,
                                       self.hyper)

    def _run(self, kjt: KeyedJaggedTensor, pooled: bool):
        self._keys = kjt.keys()
        B = kjt.stride()
        v = kjt.values().to(torch.int64).contiguous()
        o = kjt.offsets()
        if self.training and torch.is_grad_enabled():
            return _CollectionFn.apply(self._anchor, self, v, o, B, pooled)
        with torch.no_grad():
            return self._lookup(v, o, B, pooled)

    def table_weight(self, name: str) -> torch.Tensor:
        i = [t.name for t in self.tables].index(name)
        return self.store.table_weight(i)


class EmbeddingBagCollection(_LocalCollection):
    """Pooled (sum) lookups of variable-length bags: KJT -> {key: [B, D]}."""

    def forward(self, kjt: KeyedJaggedTensor) -> Dict[str, torch.Tensor]:
        out = self._run(kjt, pooled=True)
        D = self.D
        return {k: out[:, i * D:(i + 1) * D] for i, k in enumerate(kjt.keys())}


class EmbeddingCollection(_LocalCollection):
    """Unpooled sequence lookups: KJT -> {key: JaggedTensor([nnz_k, D])}."""

    def forward(self, kjt: KeyedJaggedTensor) -> Dict[str, JaggedTensor]:
        rows = self._run(kjt, pooled=False)
        B = kjt.stride()
        o = kjt.offsets()
        res = {}
        for i, k in enumerate(kjt.keys()):
            lo, hi = int(o[i * B]), int(o[(i + 1) * B])
            res[k] = JaggedTensor(rows[lo:hi], kjt.lengths()[i * B:(i + 1) * B],
                                  o[i * B:(i + 1) * B + 1] - lo)
        return res
