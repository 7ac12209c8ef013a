"""Sharded pooled embeddings (the north-star engine behind DLRM / DCN-v2, and
the in-node replacement of the reference's parameter-server path).

Reference capabilities this covers:
  * TorchRec DMP sharded EmbeddingCollection (torchrec/train.py:235-254):
    input-dist all-to-all of ids, local TBE lookup, output-dist all-to-all
    of embeddings, reverse in backward with a fused optimizer.
  * TF ParameterServerStrategy partitioned variables (tensorflow2/
    train_ps.py:55-61): variables partitioned over "PS" tasks, pulled and
    pushed every step -> here HBM-resident table/row shards exchanged by
    RCCL all-to-all over xGMI, synchronously.

Design (MI355X-first):
  * table-wise (TW) shards: a rank owns whole tables; ids go to the owner,
    the owner pools the *global* batch of its tables with one HIP launch,
    writing straight into the all-to-all send buffer in [src][b][tables x D]
    order, and the receiver's interaction kernel reads the pooled rows in
    place through a slot map (no permute kernel in either direction).
    Shapes are static for fixed pooling factors, so the exchange is
    hipGraph-capturable and needs no split exchange.
  * row-wise (RW) shards: rows are dealt round-robin over the ranks (owner =
    id mod W, so a hot head of low ids -- Zipf / frequency-ordered Criteo --
    is spread over every owner); ids are bucketed by owner into per-owner
    segments whose capacity is checked (all-reduced max count) before every
    exchange and grown on demand, so skewed batches never drop a lookup;
    the owner pools per (requester, bag) and one reduce-scatter returns the
    partial sums; gradients come back by all-gather and the owner's fused
    sort-based backward merges duplicates across requesters.
  * column-wise (CW) shards: block k of a table (columns [c0, c0 + Dc)) is
    looked up by its rank exactly like a table-wise shard of width Dc, its
    ids travel in a second id all-to-all, its pooled pieces ride in the same
    pooled all-to-all, and the receiver assembles each CW feature's D-wide
    row from the pieces (strided copies; the reverse for gradients).
  * bf16 on the wire for embeddings/gradients, fp32 in HBM tables.
"""
from __future__ import annotations

import os
import sys

from typing import List, Optional, Sequence

import torch

from .. import ops
from ..parallel.comm import as_comm
from .planner import ShardingPlan
from .tables import EmbOptimConfig, TableBatchedEmbedding, TableConfig


_WARNED_SKIP_RW_READ = False

class ShardedEmbeddingBags:
    """Pooled embedding features of one width D over a sharding plan.

    Input ``ids``: int64, original table order, table t occupying ``B * L_t``
    entries (bag b of table t = ids[base_t + b*L_t : base_t + (b+1)*L_t]).
    Output: ``self.recv`` (bf16) plus ``slot_off`` / ``slot_stride`` giving, per
    feature (table), the element offset and per-sample stride of its pooled
    row inside ``recv`` — the layout the interaction / concat consumers read.
    """

    def __init__(self, tables: Sequence[TableConfig], plan: ShardingPlan, rank: int,
                 batch_size: int, pooling: Sequence[int], device, optim: EmbOptimConfig,
                 group=None, seed: int = 0, mean: bool = False, rw_capacity: float = 1.25,
                 rw_comm: str = "bf16", dp_dense_max_bytes: int = 256 << 20,
                 recv_dtype: str = "bf16", rw_exchange: str = "auto"):
        """``rw_capacity``: initial per-owner segment capacity of the row-wise
        exchange as a multiple of the uniform share n/W (+256). Before every
        exchange the largest per-owner count is all-reduced and the capacity
        grows (buffers reallocated, ``layout_version`` bumped, the batch
        re-bucketized) when a segment would overflow.
        ``rw_comm``: dtype of the pooled partials' reduce-scatter ("bf16"
        halves the bytes; "fp32" sums exactly as one process would, up to
        fp32 association).
        ``rw_exchange``: "pooled" (the owner pools per requester bag, bf16
        reduce-scatter forward, all-gather of the pooled gradients backward),
        "rows" (one id per bag only: each looked-up row travels back in the
        id exchange's [W][cap + 1] layout and each gradient row to its owner,
        both by all-to-all -- ~W / 1.25 x fewer bytes, the same values) or
        "auto" (rows when every row-wise table is one-hot and the pooled rows
        are bf16).
        ``recv_dtype``: dtype of the pooled rows handed to the model and of
        their gradients, on the wire too ("bf16": the DLRM path; "fp32": fp32
        models whose embeddings must not be rounded -- the reference's TBE
        and TF PS return fp32 rows, torchrec/models.py:158-164,
        tensorflow2/train_ps.py:55-61; row-wise partials are then summed in
        fp32 as well)."""
        self.tables = list(tables)
        self.T = len(self.tables)
        dims = {t.embedding_dim for t in self.tables}
        assert len(dims) == 1, "ShardedEmbeddingBags needs one embedding width"
        self.D = D = dims.pop()
        self.plan = plan
        self.world = W = plan.world_size
        self.rank = rank
        self.B = B = int(batch_size)
        self.L = [int(x) for x in pooling]
        self.device = torch.device(device)
        self.group = group
        self.comm = as_comm(group) if plan.world_size > 1 else None
        self.dp_comm = None        # the replicated tables' reduction (default: comm)
        self.mean = mean
        self.optim = optim
        for s in plan.shards:
            if s.kind not in ("table_wise", "row_wise", "data_parallel", "column_wise"):
                raise NotImplementedError(f"sharding kind {s.kind} not supported for pooled bags")
        # ---- id layout in the input (original order)
        self.in_base = [0] * self.T
        acc = 0
        for t in range(self.T):
            self.in_base[t] = acc
            acc += B * self.L[t]
        self.nnz_local = acc
        # ---- column-wise blocks: block k of table t = columns [c0, c0 + Dc) on
        # its own rank, looked up like a table-wise shard of width Dc; the
        # consumer's D-wide rows are assembled after the pooled all-to-all
        self.cw_tables = [s.table for s in plan.shards if s.kind == "column_wise"]
        self.cw_blocks = {}
        for s in plan.shards:
            if s.kind == "column_wise":
                c0, lst = 0, []
                for r, w in zip(s.ranks, s.col_blocks):
                    lst.append((r, c0, w))
                    c0 += w
                assert c0 == D and len({r for r, _, _ in lst}) == len(lst), "bad column blocks"
                self.cw_blocks[s.table] = lst
        widths = {w for lst in self.cw_blocks.values() for (_, _, w) in lst}
        assert len(widths) <= 1, "column-wise blocks must share one width"
        self.Dc = Dc = widths.pop() if widths else 0
        self.cw_owned = [[(t, c0) for t in self.cw_tables for (r, c0, _) in self.cw_blocks[t]
                          if r == rr] for rr in range(W)]
        # ---- table-wise group
        self.tw_tables = [[s.table for s in plan.shards if s.kind == "table_wise" and s.ranks[0] == r]
                          for r in range(W)]
        mine = self.tw_tables[rank]
        self.tw_mine = mine
        self.dsum = [len(ts) * D + len(self.cw_owned[r]) * Dc for r, ts in enumerate(self.tw_tables)]
        self.tw_store = TableBatchedEmbedding([self.tables[t].num_embeddings for t in mine], D,
                                              device, optim,
                                              init_ranges=[self.tables[t].init_range or
                                                           (1.0 / self.tables[t].num_embeddings) ** 0.5
                                                           for t in mine],
                                              seed=seed * 1000 + rank)
        # send order: tables grouped by owner
        order = [t for r in range(W) for t in self.tw_tables[r]]
        self.tw_send_counts = [sum(B * self.L[t] for t in self.tw_tables[r]) for r in range(W)]
        self.tw_recv_count = sum(B * self.L[t] for t in mine)
        perm = torch.cat([torch.arange(self.in_base[t], self.in_base[t] + B * self.L[t])
                          for t in order]) if order else torch.zeros(0, dtype=torch.int64)
        self.tw_identity = bool(W == 1 and torch.equal(perm, torch.arange(perm.numel()))
                                and len(order) == self.T)
        self.tw_perm = perm.to(self.device)
        # the id permutes are static runs of the input: one native launch each
        # (ops.SegmentMap) instead of an index_select
        self.tw_map = ops.SegmentMap(self._runs(order), self.device)
        # owner-side virtual tables v = (src s, local table i)
        nv = W * len(mine)
        lens = []
        v_row_off, v_out_off = [], []
        for s in range(W):
            for i, t in enumerate(mine):
                lens += [self.L[t]] * B
                v_row_off.append(self.tw_store.row_offset_host[i])
                v_out_off.append(s * B * self.dsum[rank] + i * D)
        self.tw_nv = nv
        # one id per bag: virtual tables are W runs (one per source rank) of
        # the local tables -> per-table LDS sorts + run merge in the backward.
        # Measured (scripts/bench_segsort.py, B=8192): 110 vs 142 us at W=1,
        # 134 vs 140 at W=2, but 207 vs 135 at W=8 (few large blocks) -> only
        # up to 2 runs; beyond that the device-wide radix sort wins.
        onehot = bool(mine) and all(self.L[t] == 1 for t in mine)
        self.tw_onehot = onehot
        self.tw_segsort = W if (onehot and W <= 2) else 0
        offs = torch.zeros(len(lens) + 1, dtype=torch.int64)
        if lens:
            offs[1:] = torch.cumsum(torch.tensor(lens, dtype=torch.int64), 0)
        self.tw_v_offsets = offs.to(self.device)
        # fixed bag length per virtual table (the offsets above are regular)
        self.tw_v_len = torch.tensor([self.L[t] for s_ in range(W) for t in mine],
                                     dtype=torch.int32, device=self.device)
        self.tw_v_row_off = torch.tensor(v_row_off, dtype=torch.int64, device=self.device)
        self.tw_v_out_off = torch.tensor(v_out_off, dtype=torch.int64, device=self.device)
        self.tw_ld = self.dsum[rank]          # row pitch of the pooled TW output (alias_pooled)
        self.pooled_aliased = False
        # buffers
        if recv_dtype not in ("bf16", "fp32"):
            raise ValueError(f"recv_dtype must be bf16 or fp32, got {recv_dtype!r}")
        bf = torch.bfloat16 if recv_dtype == "bf16" else torch.float32
        self.recv_dtype = bf
        if recv_dtype == "fp32":
            rw_comm = "fp32"
        self.tw_send_ids = torch.empty(self.nnz_local_tw(), dtype=torch.int64, device=self.device)
        self.tw_recv_ids = torch.empty(W * self.tw_recv_count, dtype=torch.int64, device=self.device)
        self.tw_pooled = torch.empty(max(1, W * B * self.dsum[rank]), dtype=bf, device=self.device)
        self.tw_recv_sizes = [B * self.dsum[r] for r in range(W)]
        self.tw_recv_base = [sum(self.tw_recv_sizes[:r]) for r in range(W)]
        tw_total = sum(self.tw_recv_sizes)
        if self.cw_tables:
            cmine = self.cw_owned[rank]
            self.cw_store = TableBatchedEmbedding(
                [self.tables[t].num_embeddings for t, _ in cmine], Dc, device, optim,
                init_ranges=[self.tables[t].init_range or (1.0 / self.tables[t].num_embeddings) ** 0.5
                             for t, _ in cmine], seed=seed * 1000 + 300 + rank)
            corder = [t for r in range(W) for t, _ in self.cw_owned[r]]
            self.cw_send_counts = [sum(B * self.L[t] for t, _ in self.cw_owned[r]) for r in range(W)]
            self.cw_recv_count = sum(B * self.L[t] for t, _ in cmine)
            self.cw_perm = torch.cat([torch.arange(self.in_base[t], self.in_base[t] + B * self.L[t])
                                      for t in corder]).to(self.device)
            self.cw_map = ops.SegmentMap(self._runs(corder), self.device)
            self.cw_send_ids = torch.empty(sum(self.cw_send_counts), dtype=torch.int64,
                                           device=self.device)
            self.cw_recv_ids = torch.empty(W * self.cw_recv_count, dtype=torch.int64,
                                           device=self.device)
            lens, ro, oo = [], [], []
            for s_ in range(W):
                for k, (t, _) in enumerate(cmine):
                    lens += [self.L[t]] * B
                    ro.append(self.cw_store.row_offset_host[k])
                    oo.append(s_ * B * self.dsum[rank] + len(mine) * D + k * Dc)
            self.cw_nv = W * len(cmine)
            co = torch.zeros(len(lens) + 1, dtype=torch.int64)
            if lens:
                co[1:] = torch.cumsum(torch.tensor(lens, dtype=torch.int64), 0)
            self.cw_v_offsets = co.to(self.device)
            self.cw_v_row_off = torch.tensor(ro, dtype=torch.int64, device=self.device)
            self.cw_v_out_off = torch.tensor(oo, dtype=torch.int64, device=self.device)
        # ---- row-wise group: fixed-capacity exchange (csrc/kernels/rowwise.hip).
        # Ids are bucketed by owner block into [W][cap+1] segments, exchanged
        # with one equal-split all-to-all, pooled per (requester, bag) at the
        # owner and summed by a bf16 reduce-scatter; the backward all-gathers
        # the pooled gradients and runs the fused sort-based update on the
        # received entries. Static shapes: hipGraph-capturable, no host sync.
        self.rw_rows = False
        self.rw_tables = [s.table for s in plan.shards if s.kind == "row_wise"]
        self.rw_col = {t: j * D for j, t in enumerate(self.rw_tables)}
        self.rw_width = len(self.rw_tables) * D
        self.nrw = len(self.rw_tables)
        if self.rw_tables:
            blocks = [-(-self.tables[t].num_embeddings // W) for t in self.rw_tables]
            self.rw_block_host = blocks
            # every rank allocates a full block per table (the last block is
            # padded) so owner-local row keys agree across ranks; one scratch
            # row absorbs the padding entries of the backward
            self.rw_store = TableBatchedEmbedding(
                blocks, D, device, optim,
                init_ranges=[self.tables[t].init_range or (1.0 / self.tables[t].num_embeddings) ** 0.5
                             for t in self.rw_tables], seed=seed * 1000 + 500 + rank,
                scratch_rows=1)
            if self.rw_store.total_rows + 1 >= 1 << 32:
                raise ValueError("row-wise shard holds >= 2^32 rows on one rank (32-bit row keys)")
            self.rw_dummy = self.rw_store.total_rows
            Ls = [self.L[t] for t in self.rw_tables]
            cum = [0]
            for l_ in Ls:
                cum.append(cum[-1] + B * l_)
            self.rw_n = n = cum[-1]
            meta = ([self.in_base[t] for t in self.rw_tables] + Ls + blocks
                    + list(self.rw_store.row_offset_host) + cum)
            self.rw_meta = torch.tensor(meta, dtype=torch.int64, device=self.device)
            self.rw_cap_factor = float(rw_capacity)
            if rw_exchange not in ("auto", "pooled", "rows"):
                raise ValueError(f"rw_exchange must be auto, pooled or rows, got {rw_exchange!r}")
            onehot_rw = all(l_ == 1 for l_ in Ls)
            if rw_exchange == "rows" and not (onehot_rw and bf == torch.bfloat16):
                raise ValueError("rw_exchange='rows' needs one id per bag in every row-wise "
                                 "table and bf16 pooled rows")
            self.rw_rows = (W > 1 and onehot_rw and bf == torch.bfloat16
                            and rw_exchange != "pooled")
            from .. import ops as _ops
            self.rw_ws = torch.empty(_ops.rw_bucketize_workspace(n, W), dtype=torch.uint8,
                                     device=self.device)
            # [sticky overflow flag, largest per-owner count of the last bucketize]
            self.rw_overflow = torch.zeros(2, dtype=torch.int32, device=self.device)
            self.rw_dynamic = W > 1          # exact capacity check before every exchange
            self.rw_grows = 0
            self.rw_lag_reads = 0
            self.rw_starts = torch.zeros(W * (self.nrw * B + 1), dtype=torch.int32,
                                         device=self.device)
            bf_ = bf
            if rw_comm not in ("bf16", "fp32"):
                raise ValueError(f"rw_comm must be bf16 or fp32, got {rw_comm}")
            cdt = bf_ if rw_comm == "bf16" else torch.float32
            pooled_x = W > 1 and not self.rw_rows
            self.rw_pbuf = (torch.zeros(W * B * self.rw_width, dtype=cdt, device=self.device)
                            if pooled_x else None)
            # fp32 partials are reduced into an fp32 landing buffer, then cast
            self.rw_rs32 = (torch.zeros(B * self.rw_width, dtype=cdt, device=self.device)
                            if pooled_x and cdt == torch.float32 and bf != torch.float32 else None)
            self.rw_gbuf = (torch.zeros(W * B * self.rw_width, dtype=bf_, device=self.device)
                            if pooled_x else None)
            self._rw_scatter_pending = False
            self._rw_alloc(self.rw_capacity(n, W, rw_capacity))
            self._rw_prepared = False
        # ---- data-parallel (replicated) group: local lookup, gradient
        # all-gather, identical deterministic update on every rank
        self.dp_tables = [s.table for s in plan.shards if s.kind == "data_parallel"]
        self.dp_width = len(self.dp_tables) * D
        self.dp_base = tw_total + B * self.rw_width
        if self.dp_tables:
            dpt = self.dp_tables
            self.dp_store = TableBatchedEmbedding(
                [self.tables[t].num_embeddings for t in dpt], D, device, optim,
                init_ranges=[self.tables[t].init_range or (1.0 / self.tables[t].num_embeddings) ** 0.5
                             for t in dpt], seed=seed * 1000 + 777)        # same on all ranks
            self.dp_in_idx = torch.cat([torch.arange(self.in_base[t], self.in_base[t] + B * self.L[t])
                                        for t in dpt]).to(self.device)
            self.dp_in_map = ops.SegmentMap(self._runs(dpt), self.device)
            self.dp_nid = int(self.dp_in_idx.numel())

            def bag_offsets(nb):
                lens = torch.tensor([self.L[t] for t in dpt], dtype=torch.int64).repeat_interleave(nb)
                o = torch.zeros(lens.numel() + 1, dtype=torch.int64)
                o[1:] = torch.cumsum(lens, 0)
                return o.to(self.device)

            self.dp_offsets = bag_offsets(B)
            self.dp_out_off = torch.tensor([self.dp_base + j * D for j in range(len(dpt))],
                                           dtype=torch.int64, device=self.device)
            self.dp_ids = torch.zeros(self.dp_nid, dtype=torch.int64, device=self.device)
            # small replicated tables (the planner's default for W > 1): each
            # rank's fused backward writes a dense fp32 gradient, one
            # all-reduce sums it and every rank takes the same dense step --
            # per-rank work and bytes independent of the batch size and W
            # (only for optimizers whose zero-gradient update is a no-op: Adam's
            # moment decay or weight decay would touch rows the batch never saw)
            dp_bytes = self.dp_store.total_rows * D * 4
            zero_noop = (optim.code in (ops.EMB_SGD, ops.EMB_ADAGRAD, ops.EMB_ROWWISE_ADAGRAD)
                         and optim.weight_decay == 0.0)
            self.dp_dense = W > 1 and dp_bytes <= dp_dense_max_bytes and zero_noop
            # one id per bag: the dense-gradient backward sorts each table's
            # ids in LDS (passes for its largest id only: 2 for these small
            # tables) instead of the device-wide radix sort
            self.dp_onehot = all(self.L[t] == 1 for t in dpt)      # lookup skips offsets
            self.dp_segsort = 1 if (self.dp_onehot and B <= 8192 and not mean) else 0
            if self.dp_dense:
                self.dp_dgrad = torch.zeros(self.dp_store.total_rows, D, dtype=torch.float32,
                                            device=self.device)
                self._dp_clean = True
            elif W > 1:
                # large replicated tables: all-gather ids + pooled grads, and
                # every rank applies the identical global-batch sparse update
                self.dp_g_offsets = bag_offsets(W * B)
                self.dp_g_ids = torch.zeros(W * self.dp_nid, dtype=torch.int64, device=self.device)
                self.dp_g_grad = torch.zeros(W * B * self.dp_width, dtype=bf, device=self.device)
                self.dp_g_goff = torch.tensor([j * D for j in range(len(dpt))], dtype=torch.int64,
                                              device=self.device)
                # gathered (rank-major) ids -> table-major over W*B bags
                src, pieces = [], []
                base = dst = 0
                for t in dpt:
                    n_t = B * self.L[t]
                    for r in range(W):
                        src.append(torch.arange(r * self.dp_nid + base, r * self.dp_nid + base + n_t))
                        pieces.append((r * self.dp_nid + base, dst, n_t))
                        dst += n_t
                    base += n_t
                self.dp_g_perm = torch.cat(src).to(self.device)
                self.dp_g_map = ops.SegmentMap(pieces, self.device)
                self.dp_g_ids_t = torch.zeros_like(self.dp_g_ids)
        self.cw_base = self.dp_base + B * self.dp_width
        self.cw_width = len(self.cw_tables) * D
        self.recv = torch.zeros(self.cw_base + B * self.cw_width, dtype=bf, device=self.device)
        self.d_recv = torch.zeros_like(self.recv)
        self.d_pooled = torch.empty_like(self.tw_pooled)
        # ---- consumer slot map (per feature/table)
        self.slot_off: List[int] = [0] * self.T
        self.slot_stride: List[int] = [0] * self.T
        for r in range(W):
            for i, t in enumerate(self.tw_tables[r]):
                self.slot_off[t] = self.tw_recv_base[r] + i * D
                self.slot_stride[t] = self.dsum[r]
        for t in self.rw_tables:
            self.slot_off[t] = tw_total + self.rw_col[t]
            self.slot_stride[t] = self.rw_width
        for j, t in enumerate(self.dp_tables):
            self.slot_off[t] = self.dp_base + j * D
            self.slot_stride[t] = self.dp_width
        # CW pieces: (src offset in the pooled a2a region, stride) -> (dst in
        # the assembled CW region, stride), B x Dc elements each
        self.cw_pieces = []
        for j, t in enumerate(self.cw_tables):
            self.slot_off[t] = self.cw_base + j * D
            self.slot_stride[t] = self.cw_width
            for (r, c0, w) in self.cw_blocks[t]:
                k = self.cw_owned[r].index((t, c0))
                src = self.tw_recv_base[r] + len(self.tw_tables[r]) * D + k * Dc
                self.cw_pieces.append((src, self.dsum[r], self.cw_base + j * D + c0, self.cw_width))
        if self.cw_tables:
            # the pooled pieces -> D-wide rows (and back for the gradients):
            # one native launch each way
            self._cw_copy = ops.PieceCopy(self.cw_pieces, B, Dc, self.device)
            self._cw_copy_rev = self._cw_copy.reverse()
        self._pending = None
        self._rw_state = None
        self._rw_ids = None
        # bumped whenever a buffer captured into a hipGraph is reallocated
        # (row-wise capacity growth): the trainer re-captures its graphs
        self.layout_version = 0
        self._rw_mbox = None
        self._rw_lag_pending = False

    def _runs(self, tables):
        """(src, dst, length) pieces laying the given tables' id runs of the
        input back to back, in that order."""
        out, dst = [], 0
        for t in tables:
            n = self.B * self.L[t]
            out.append((self.in_base[t], dst, n))
            dst += n
        return out

    def alias_pooled(self, out: torch.Tensor, d_out: torch.Tensor, col0: int) -> bool:
        """One rank, table-wise tables only: pool straight into the consumer's
        row-major [B, ld] buffer ``out`` at columns col0 + t*D (e.g. DCN-v2's
        x_0 after the dense slot) and read the pooled gradients from ``d_out``
        in the same layout -- no concat / split pass through recv / d_recv.
        Returns False (nothing changed) when the layout does not allow it."""
        D, B = self.D, self.B
        if not (self.world == 1 and self.tw_identity and self.tw_nv == self.T
                and not (self.cw_tables or self.dp_tables or self.rw_tables)):
            return False
        for t_ in (out, d_out):
            if not (t_.is_contiguous() and t_.dim() == 2 and t_.shape[0] == B
                    and t_.shape[1] >= col0 + self.T * D and t_.dtype == self.recv.dtype):
                return False
        if out.shape != d_out.shape:
            return False
        ld = out.shape[1]
        self.recv = out.view(-1)
        self.d_recv = d_out.view(-1)
        self.tw_ld = ld
        self.tw_v_out_off = torch.tensor([col0 + i * D for i in range(self.T)], dtype=torch.int64,
                                         device=self.device)
        self.slot_off = [col0 + t * D for t in range(self.T)]
        self.slot_stride = [ld] * self.T
        self.pooled_aliased = True
        return True

    def nnz_local_tw(self) -> int:
        return sum(self.tw_send_counts)

    @staticmethod
    def rw_capacity(n: int, W: int, factor: float) -> int:
        """Initial per-owner capacity: factor x the uniform share n/W plus a
        slack of up to 256 ids (grown on demand before any exchange)."""
        if W == 1:
            return max(1, n)
        return max(1, min(n, -(-int(factor * n) // W) + min(256, n // (4 * W))))

    def _rw_alloc(self, cap: int):
        """(Re)allocate the [W][cap + 1] exchange buffers and the owner-side
        backward workspace for per-owner capacity ``cap``."""
        W, D = self.world, self.D
        self.rw_cap = cap
        self.rw_send = torch.zeros(W * (cap + 1), dtype=torch.int64, device=self.device)
        self.rw_recv = torch.zeros_like(self.rw_send) if W > 1 else self.rw_send
        self.rw_bwd_ws = None
        if getattr(self, "rw_rows", False):
            # "rows" exchange: owner rows out / requester rows in, requester
            # gradient rows out / owner gradient rows in, the slot map
            n = W * (cap + 1)
            mk = lambda: torch.zeros(n * D, dtype=torch.bfloat16, device=self.device)  # noqa: E731
            self.rw_rows_out, self.rw_rows_in = mk(), mk()
            self.rw_gsend, self.rw_grecv = mk(), mk()
            self.rw_smap = torch.zeros(n, dtype=torch.int32, device=self.device)
        if self.device.type == "cuda":
            from .. import ops as _ops
            self.rw_bwd_ws = torch.empty(_ops.embedding_bwd_workspace(W * cap, D),
                                         dtype=torch.uint8, device=self.device)

    def _rw_bucketize(self, ids: torch.Tensor):
        from .. import ops
        ops.rw_bucketize(ids, self.rw_meta, self.nrw, self.world, self.B, self.rw_cap,
                         self.rw_n, self.rw_send, self.rw_ws, self.rw_overflow)

    def _rw_check_capacity(self):
        """All ranks agree on the largest per-owner count of this batch (MAX
        all-reduce, one host read) and grow the capacity before the exchange
        if any segment would overflow: the batch is re-bucketized into the
        larger segments, so no lookup is dropped whatever the id skew."""
        need = self.rw_overflow[1:2].clone()
        if self.world > 1:
            self.comm.all_reduce(need, "max")
        need = int(need.item())
        if need <= self.rw_cap:
            return
        self._rw_grow(need)
        self._rw_bucketize(self._rw_ids)

    def _rw_grow(self, need: int):
        cap = min(self.rw_n, int(need * 1.25) + 256)
        self._rw_alloc(cap)
        self.rw_grows += 1
        self.layout_version += 1
        self.rw_overflow[:1].zero_()          # this batch's overflow is undone by the re-bucketize

    # -- lagged capacity check (pipelined trainers: the batch bucketized and
    # exchanged in step i's tail is consumed by step i+1). Step i publishes the
    # all-reduced per-owner need to a host mailbox (no host wait, capturable);
    # the host reads it when it issues step i+1 -- the device produced it long
    # before -- and only if a segment overflowed does it grow the capacity and
    # redo that batch's row-wise exchange (``rw_redo``) before step i+1 runs.
    # Every rank reads the same MAX, so all take the same branch.
    def _rw_mailbox(self):
        if self._rw_mbox is None:
            from ..parallel.mailbox import HostMailbox
            self._rw_mbox = HostMailbox(1, self.device)
        return self._rw_mbox

    def rw_publish_need(self, comm=None):
        """All ranks' largest per-owner count of the batch bucketized last
        (in-place MAX all-reduce on ``comm``, default the exchange comm) to the
        host mailbox. Under stream capture the replays publish; the trainer
        counts them (``rw_note_replay``)."""
        if not (self.rw_tables and self.rw_dynamic):
            return
        need = self.rw_overflow[1:2]
        if self.world > 1:
            (comm or self.comm).all_reduce(need, "max")
        self._rw_mailbox().publish(need)
        if self.device.type != "cuda" or not torch.cuda.is_current_stream_capturing():
            self._rw_lag_pending = True

    def rw_note_replay(self):
        """A graph holding one ``rw_publish_need`` was launched."""
        self._rw_mailbox().note_launch()
        self._rw_lag_pending = True

    def rw_resolve_need(self) -> bool:
        """Read the latest published need; if a segment overflowed, wait for
        the device, grow the capacity and return True -- the caller then redoes
        the row-wise exchange of that batch (``rw_redo``) before consuming it
        and re-captures its graphs (``layout_version`` changed)."""
        if not self._rw_lag_pending:
            return False
        self._rw_lag_pending = False
        if os.environ.get("TDFO_DIAG_SKIP_RW_READ") == "1":
            # diagnostics only (host never waits for the need: measures what
            # the lagged read costs; an overflow then raises at the next
            # check_overflow -- pop_loss, every log line -- instead of being
            # redone): say so once, loudly
            global _WARNED_SKIP_RW_READ
            if not _WARNED_SKIP_RW_READ:
                _WARNED_SKIP_RW_READ = True
                print("WARNING: TDFO_DIAG_SKIP_RW_READ=1 (diagnostics): row-wise capacity "
                      "overflows are not redone; a dropped lookup raises at the next "
                      "check_overflow / pop_loss", file=sys.stderr, flush=True)
            return False
        need = self._rw_mailbox().read()
        self.rw_lag_reads += 1
        if need <= self.rw_cap:
            return False
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)    # in-flight kernels hold the old buffers
        self._rw_grow(need)
        return True

    def rw_redo(self):
        """The row-wise part of the forward exchange of the batch bucketized
        last (its ids are still in the buffer ``stage_fwd_prep`` saw), into the
        grown segments: bucketize, id all-to-all, owner pooling, reduce-scatter
        into this batch's row-wise slots of ``recv``. Synchronous."""
        from .. import ops
        W = self.world
        # the first exchange's collectives may still be in flight (async
        # handles, e.g. gloo's worker threads): they must land before the
        # redo overwrites their outputs ("forward_wait" then only assembles)
        self.ids_exchange_wait()
        for w in self._pending or ():
            w.wait()
        self._pending = None
        self._rw_bucketize(self._rw_ids)
        if W > 1:
            self.comm.all_to_all(self.rw_recv, self.rw_send)
        if self.rw_rows:
            ops.rw_rows_gather(self.rw_store.weight, self.rw_recv, W, self.rw_cap, self.rw_rows_out)
            self.comm.all_to_all(self.rw_rows_in, self.rw_rows_out)
            self._rw_scatter()
            return
        out = self.rw_pbuf if W > 1 else self._rw_region(self.recv)
        ops.rw_pool(self.rw_store.weight, self.rw_recv, self.rw_meta, self.nrw, W, self.B,
                    self.rw_cap, self.mean, self.rw_starts, out, self.rw_width)
        if W > 1:
            dst = self.rw_rs32 if self.rw_rs32 is not None else self._rw_region(self.recv)
            self.comm.reduce_scatter(dst, self.rw_pbuf)
            if self.rw_rs32 is not None:
                ops.cast_bf16(self.rw_rs32, self._rw_region(self.recv))

    def _rw_scatter(self):
        """"rows" exchange: the received rows into this batch's row-wise
        slots of ``recv`` (and the slot map the backward gathers with)."""
        from .. import ops
        self._rw_scatter_pending = False
        ops.rw_rows_scatter(self.rw_send, self.world, self.rw_cap, self.B, self.D, self.rw_rows_in,
                            self._rw_region(self.recv), self.rw_width, self.rw_smap, self.nrw)

    def _rw_region(self, buf):
        base = sum(self.tw_recv_sizes)
        return buf[base: base + self.B * self.rw_width]

    def check_overflow(self):
        """Raise on every rank if any rank's row-wise segment overflowed its
        capacity (only possible with the per-exchange capacity check off):
        the flag is MAX all-reduced so no rank is left waiting in the next
        collective while another raises (host sync)."""
        if not self.rw_tables:
            return
        flag = self.rw_overflow[:1].clone()
        if self.world > 1:
            self.comm.all_reduce(flag, "max")
        if int(flag.item()):
            raise RuntimeError(
                f"row-wise exchange capacity exceeded (cap {self.rw_cap} ids per owner, "
                f"{self.rw_n} ids per rank) with the capacity check off: lookups were dropped")

    @property
    def fwd_prep_noop(self) -> bool:
        """The forward prep stage launches nothing (one table-wise rank)."""
        return self.tw_identity and not (self.cw_tables or self.dp_tables or self.rw_tables)

    def bind_ids(self, ids: torch.Tensor):
        """Alias the static id buffer where the table-wise exchange is the
        identity (one rank): the lookup reads it in place."""
        if self.tw_identity:
            self.tw_send_ids = ids
            self.tw_recv_ids = ids

    # ------------------------------------------------------------ forward
    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        self.forward_start(ids)
        self.forward_wait()
        return self.recv

    def forward_start(self, ids: torch.Tensor):
        self.stage_fwd_prep(ids)
        self.stage_fwd_ids_exchange()
        self.stage_fwd_lookup()
        self.stage_fwd_out_exchange()

    @property
    def graph_capturable(self) -> bool:
        """Every sharding kind uses static shapes (fixed-capacity RW exchange)."""
        return True

    # -- stages (compute stages are hipGraph-capturable; exchanges are RCCL)
    def _cw_assemble(self, buf):
        self._cw_copy.apply(buf)

    def _cw_disassemble(self, buf):
        self._cw_copy_rev.apply(buf)

    def stage_fwd_prep(self, ids: torch.Tensor, sharded: bool = True, dp: bool = True):
        """Bucket a batch's ids for the exchanges (``sharded``: table/column/
        row-wise send buffers) and the replicated tables' local lookup
        (``dp``); the multi-rank stream graphs run the two halves where their
        buffers' previous readers are ordered (models/dlrm_multirank.py)."""
        if self.dp_tables and dp:
            self.dp_in_map.apply(ids, self.dp_ids)
        if not sharded:
            return
        if self.cw_tables:
            self.cw_map.apply(ids, self.cw_send_ids)
            if self.world == 1:
                self.cw_recv_ids = self.cw_send_ids
        if self.tw_identity:
            self.tw_send_ids = ids
            self.tw_recv_ids = ids
        else:
            self.tw_map.apply(ids, self.tw_send_ids)
            if self.world == 1:
                self.tw_recv_ids = self.tw_send_ids
        if self.rw_tables:
            self._rw_ids = ids
            self._rw_bucketize(ids)

    def stage_fwd_ids_exchange(self, async_op: bool = False, lagged: bool = False,
                               publish: bool = True):
        """Id exchange (input dist). async_op: the collectives are left in
        flight (the pipelined trainer overlaps them with the previous step's
        dense update) until ``ids_exchange_wait``. lagged: the row-wise
        capacity is checked one step later (``rw_publish_need`` here unless
        ``publish`` is False -- the caller publishes elsewhere -- and
        ``rw_resolve_need`` before the batch is consumed) instead of by a host
        read before the exchange."""
        W = self.world
        works = []
        if self.dp_tables and W > 1 and not self.dp_dense:
            works.append(self.comm.all_gather(self.dp_g_ids, self.dp_ids, async_op=async_op))
        if W > 1 and not self.tw_identity:
            works.append(self.comm.all_to_all(self.tw_recv_ids, self.tw_send_ids,
                                              [self.tw_recv_count] * W, self.tw_send_counts,
                                              async_op=async_op))
        if W > 1 and self.cw_tables:
            works.append(self.comm.all_to_all(self.cw_recv_ids, self.cw_send_ids,
                                              [self.cw_recv_count] * W, self.cw_send_counts,
                                              async_op=async_op))
        if W > 1 and self.rw_tables:
            if self.rw_dynamic and not lagged:
                self._rw_check_capacity()
            elif self.rw_dynamic and publish:
                self.rw_publish_need()
            works.append(self.comm.all_to_all(self.rw_recv, self.rw_send, async_op=async_op))
        self._ids_works = [w for w in works if w is not None] if async_op else []

    def ids_exchange_wait(self):
        for w in getattr(self, "_ids_works", None) or ():
            w.wait()
        self._ids_works = []

    def stage_fwd_lookup(self, sharded: bool = True, dp: bool = True):
        """Pooled lookup of the exchanged ids (``sharded``) and of the
        replicated tables' local ids (``dp``)."""
        W, B = self.world, self.B
        if self.dp_tables and dp:
            self.dp_store.forward(self.dp_ids, self.dp_offsets, self.dp_store.row_offset,
                                  len(self.dp_tables), B, self.recv, self.dp_out_off,
                                  self.dp_width, mean=self.mean, onehot=self.dp_onehot)
            if W > 1 and not self.dp_dense:
                self.dp_g_map.apply(self.dp_g_ids, self.dp_g_ids_t)
        if not sharded:
            return
        if self.tw_nv:
            self.tw_store.forward(self.tw_recv_ids, self.tw_v_offsets, self.tw_v_row_off, self.tw_nv,
                                  B, self.tw_pooled if W > 1 else self.recv, self.tw_v_out_off,
                                  self.tw_ld, mean=self.mean,
                                  onehot=self.tw_onehot)
        if self.cw_tables and self.cw_nv:
            self.cw_store.forward(self.cw_recv_ids, self.cw_v_offsets, self.cw_v_row_off,
                                  self.cw_nv, B, self.tw_pooled if W > 1 else self.recv,
                                  self.cw_v_out_off, self.dsum[self.rank], mean=self.mean)
        if self.rw_tables:
            from .. import ops
            if self.rw_rows:
                ops.rw_rows_gather(self.rw_store.weight, self.rw_recv, W, self.rw_cap,
                                   self.rw_rows_out)
                return
            out = self.rw_pbuf if W > 1 else self._rw_region(self.recv)
            ops.rw_pool(self.rw_store.weight, self.rw_recv, self.rw_meta, self.nrw, W, B,
                        self.rw_cap, self.mean, self.rw_starts, out, self.rw_width)

    def stage_fwd_out_exchange(self):
        W, B = self.world, self.B
        works = []
        if W > 1:
            tw_total = sum(self.tw_recv_sizes)
            if tw_total:
                works.append(self.comm.all_to_all(self.recv[:tw_total],
                                                  self.tw_pooled[: W * B * self.dsum[self.rank]],
                                                  self.tw_recv_sizes,
                                                  [B * self.dsum[self.rank]] * W, async_op=True))
            if self.rw_tables and self.rw_rows:
                works.append(self.comm.all_to_all(self.rw_rows_in, self.rw_rows_out,
                                                  async_op=True))
                # a stream-ordered communicator (native RCCL, loopback): the
                # scatter follows on the same stream; else after the wait
                self._rw_scatter_pending = True
                if getattr(self.comm, "capturable", False):
                    self._rw_scatter()
            elif self.rw_tables:
                dst = self.rw_rs32 if self.rw_rs32 is not None else self._rw_region(self.recv)
                works.append(self.comm.reduce_scatter(dst, self.rw_pbuf, async_op=True))
        self._pending = works

    def forward_wait(self):
        for w in self._pending or ():
            w.wait()
        self._pending = None
        if self.rw_tables and self.rw_rows and self._rw_scatter_pending:
            self._rw_scatter()
        if self.cw_tables:
            self._cw_assemble(self.recv)
        if self.rw_tables and self.rw_rs32 is not None:
            from .. import ops
            ops.cast_bf16(self.rw_rs32, self._rw_region(self.recv))

    # ----------------------------------------------------------- backward
    def stage_bwd_local(self, hyper: torch.Tensor, d_recv: Optional[torch.Tensor] = None):
        """Local part of the backward that must precede the exchanges: the
        dense gradient of the small replicated tables (zeroed + written by
        the fused backward). Compute stage: the trainer runs it right after
        the interaction backward."""
        if self.dp_tables and self.world > 1 and self.dp_dense:
            from .. import ops
            d_recv = self.d_recv if d_recv is None else d_recv
            st = self.dp_store
            if not self._dp_clean:             # the dense update zeroes it as it reads
                self.dp_dgrad.zero_()
            self._dp_clean = False
            ops.embedding_bwd(st.weight, st.row_offset, self.dp_ids, self.dp_offsets,
                              self.dp_out_off, len(self.dp_tables), self.B, d_recv,
                              self.dp_width, ops.EMB_DENSE_GRAD, hyper, key_bits=st.key_bits,
                              mean=self.mean, dense_grad=self.dp_dgrad, segsort=self.dp_segsort)

    def backward(self, hyper: torch.Tensor, d_recv: Optional[torch.Tensor] = None):
        """The whole backward in one call (tests / eager use)."""
        self.stage_bwd_local(hyper, d_recv)
        self.backward_start(d_recv)
        self.backward_finish(hyper)

    def backward_start(self, d_recv: Optional[torch.Tensor] = None, exchange: bool = True,
                       dp: bool = True):
        """Start the gradient exchange (async on GPU). ``d_recv`` defaults to
        ``self.d_recv`` (same layout as ``self.recv``). ``exchange`` /
        ``dp``: only the sharded tables' exchanges (table/column-wise
        all-to-all, row-wise all-gather) / only the replicated tables'
        reduction, so the latter can wait for their dense gradient
        (``stage_bwd_local``) on another stream while the former is in
        flight; ``backward_wait`` waits for both."""
        d_recv = self.d_recv if d_recv is None else d_recv
        W, B = self.world, self.B
        if exchange:
            self._backward_exchange(d_recv)
        if dp:
            self._backward_dp(d_recv)

    def _backward_exchange(self, d_recv):
        W, B = self.world, self.B
        tw_total = sum(self.tw_recv_sizes)
        if self.cw_tables:
            self._cw_disassemble(d_recv)
        work = None
        if W > 1:
            work = self.comm.all_to_all(self.d_pooled[: W * B * self.dsum[self.rank]],
                                        d_recv[:tw_total], [B * self.dsum[self.rank]] * W,
                                        self.tw_recv_sizes, async_op=True)
        self._rw_work = None
        if W > 1 and self.rw_tables and self.rw_rows:
            from .. import ops
            ops.rw_grads_gather(self.rw_smap, W, self.rw_cap, self.D, self._rw_region(d_recv),
                                self.rw_gsend)
            self._rw_work = self.comm.all_to_all(self.rw_grecv, self.rw_gsend, async_op=True)
        elif W > 1 and self.rw_tables:
            self._rw_work = self.comm.all_gather(self.rw_gbuf, self._rw_region(d_recv),
                                                 async_op=True)
        self._bw = (work, d_recv)

    def _backward_dp(self, d_recv):
        W, B = self.world, self.B
        self._dp_work = None
        comm = self.dp_comm or self.comm
        if W > 1 and self.dp_tables and self.dp_dense:
            self._dp_work = comm.all_reduce(self.dp_dgrad, async_op=True)
        elif W > 1 and self.dp_tables:
            self._dp_work = comm.all_gather(
                self.dp_g_grad, d_recv[self.dp_base: self.dp_base + B * self.dp_width],
                async_op=True)

    def backward_wait(self):
        work, d_recv = self._bw
        if work is not None:
            work.wait()
        for name in ("_dp_work", "_rw_work"):
            w = getattr(self, name, None)
            if w is not None:
                w.wait()
                setattr(self, name, None)
        self._bw = (None, d_recv)

    def stage_bwd_prepare(self):
        """Ids-only part of the table-wise shard backward (keys + sort): needs
        no gradient, so the trainer runs it on a side stream during the dense
        forward/backward (after stage_fwd_ids_exchange)."""
        if self.tw_nv:
            self.tw_store.backward_prepare(self.tw_recv_ids, self.tw_v_offsets, self.tw_v_row_off,
                                           self.tw_nv, self.B, self.tw_v_out_off,
                                           self.tw_ld, mean=self.mean,
                                           segsort=self.tw_segsort, bag_len=self.tw_v_len)
        if self.rw_tables:
            self._rw_prepare()

    def _rw_prepare(self):
        from .. import ops
        st = self.rw_store
        ops.embedding_bwd_prepare_rw(st.weight, self.rw_recv, self.rw_meta, self.nrw, self.world,
                                     self.B, self.rw_cap, self.mean, st.key_bits,
                                     self.D if self.rw_rows else self.rw_width,
                                     self.rw_dummy, self.rw_bwd_ws, rows=self.rw_rows)
        self._rw_prepared = True

    def stage_bwd_update(self, hyper: torch.Tensor, sharded: bool = True, dp: bool = True):
        """Fused sort-based backward + optimizer on this rank's shards
        (``sharded``: table/column/row-wise; ``dp``: the replicated tables,
        whose update the multi-rank stream graphs run beside the others)."""
        d_recv = self._bw[1] if getattr(self, "_bw", None) else self.d_recv
        W, B = self.world, self.B
        grad = self.d_pooled if W > 1 else d_recv
        if self.tw_nv and sharded:
            self.tw_store.backward_apply(self.tw_recv_ids, self.tw_v_offsets, self.tw_v_row_off,
                                         self.tw_nv, B, grad, self.tw_v_out_off,
                                         self.tw_ld, hyper, mean=self.mean,
                                         segsort=self.tw_segsort)
        if self.cw_tables and self.cw_nv and sharded:
            self.cw_store.backward_update(self.cw_recv_ids, self.cw_v_offsets, self.cw_v_row_off,
                                          self.cw_nv, B, grad, self.cw_v_out_off,
                                          self.dsum[self.rank], hyper, mean=self.mean)
        if self.dp_tables and dp:
            ndp = len(self.dp_tables)
            if W > 1 and self.dp_dense:
                from .. import ops
                st, o = self.dp_store, self.optim
                ops.embedding_dense_update(st.weight, self.dp_dgrad, st.total_rows, o.code, hyper,
                                           state1=st.state1, state2=st.state2, eps=o.eps,
                                           beta1=o.beta1, beta2=o.beta2,
                                           weight_decay=o.weight_decay, clear_grad=True)
                self._dp_clean = True
            elif W > 1:
                self.dp_store.backward_update(self.dp_g_ids_t, self.dp_g_offsets,
                                              self.dp_store.row_offset, ndp, W * B, self.dp_g_grad,
                                              self.dp_g_goff, self.dp_width, hyper, mean=self.mean)
            else:
                self.dp_store.backward_update(self.dp_ids, self.dp_offsets, self.dp_store.row_offset,
                                              ndp, B, d_recv, self.dp_out_off, self.dp_width, hyper,
                                              mean=self.mean)
        if self.rw_tables and sharded:
            from .. import ops
            if not self._rw_prepared:
                self._rw_prepare()
            st, o = self.rw_store, self.optim
            if self.rw_rows:
                grad, gld = self.rw_grecv, self.D
            else:
                grad, gld = (self.rw_gbuf if W > 1 else self._rw_region(d_recv)), self.rw_width
            ops.embedding_bwd_apply_rw(st.weight, self.rw_recv, self.rw_meta, self.nrw, W, B,
                                       self.rw_cap, self.mean, st.key_bits, grad, gld,
                                       o.code, hyper, self.rw_bwd_ws, state1=st.state1,
                                       state2=st.state2, eps=o.eps, beta1=o.beta1, beta2=o.beta2,
                                       weight_decay=o.weight_decay, rows=self.rw_rows)
            self._rw_prepared = False

    def backward_finish(self, hyper: torch.Tensor):
        self.backward_wait()
        self.stage_bwd_update(hyper)
        self._bw = None

    # -------------------------------------------------------------- state
    def table_cols(self, t: int):
        """(col_start, width) of this rank's column block of table t (D-wide
        for every non-column-wise table held here), or None."""
        if t in self.cw_blocks:
            for r, c0, w in self.cw_blocks[t]:
                if r == self.rank:
                    return c0, w
            return None
        return (0, self.D) if self._local_slices(t) is not None else None

    def _local_slices(self, t: int):
        """(store, local_table_index, rows) of table t here, or None. ``rows``
        is a slice of the table's global rows: contiguous for whole tables,
        ``slice(rank, rows, W)`` for a row-wise shard (round-robin rows);
        local row k of the store holds global row rows.start + k*rows.step."""
        n = self.tables[t].num_embeddings
        if t in self.cw_blocks:
            cols = [c0 for (r, c0, _) in self.cw_blocks[t] if r == self.rank]
            if not cols:
                return None
            k = self.cw_owned[self.rank].index((t, cols[0]))
            return self.cw_store, k, slice(0, n, 1)
        if t in self.tw_mine:
            return self.tw_store, self.tw_mine.index(t), slice(0, n, 1)
        if t in self.dp_tables:
            return self.dp_store, self.dp_tables.index(t), slice(0, n, 1)
        if t in self.rw_tables:
            return self.rw_store, self.rw_tables.index(t), slice(min(self.rank, n), n, self.world)
        return None

    @staticmethod
    def slice_len(sl: slice) -> int:
        return len(range(sl.start, sl.stop, sl.step))

    def set_table_weight(self, t: int, full: torch.Tensor):
        """Copy this rank's part of table ``t`` from the full [rows, D] tensor."""
        loc = self._local_slices(t)
        if loc is not None and self.slice_len(loc[2]) > 0:
            store, i, sl = loc
            c0, w = self.table_cols(t)
            store.table_weight(i)[: self.slice_len(sl)].copy_(
                full[sl, c0:c0 + w].to(store.weight.device))

    def get_table_weight(self, t: int):
        """This rank's (global row slice, rows view) of table ``t``, or None:
        ``full[rows][:, cols] == view`` (see ``_local_slices``)."""
        loc = self._local_slices(t)
        if loc is None:
            return None
        store, i, sl = loc
        return sl, store.table_weight(i)[: self.slice_len(sl)]

    def state_dict(self):
        d = {"tw": self.tw_store.state_dict()}
        if self.cw_tables:
            d["cw"] = self.cw_store.state_dict()
        if self.rw_tables:
            d["rw"] = self.rw_store.state_dict()
        if self.dp_tables:
            d["dp"] = self.dp_store.state_dict()
        return d

    def load_state_dict(self, d):
        self.tw_store.load_state_dict(d["tw"])
        if self.cw_tables:
            self.cw_store.load_state_dict(d["cw"])
        if self.rw_tables:
            self.rw_store.load_state_dict(d["rw"])
        if self.dp_tables:
            self.dp_store.load_state_dict(d["dp"])

