"""TwoTower retrieval model (Goodreads) with a fused, hipGraph-capturable step.

Reference: jax-flax/models.py:10-102 (Flax, glorot_uniform everywhere) and
tensorflow2/models.py:4-71 (Keras, lecun_normal dense kernels). Architecture:

  user tower : e_user(16) -> Dense(16) -> swish -> Dense(16)
  item tower : [e_item e_lang e_ebook e_fmt e_pub e_decade avg_rating num_pages]
               (6*16+2 = 98) -> Dense(16) -> swish -> Dense(16)
  logit      : row-wise dot; loss = mean sigmoid BCE.

MI355X design: the seven lookups are ONE table-batched gather (all tables in
one fp32 buffer) written straight into the tower-input matrix X[B, 116]
(the concat never exists as a separate op); ``tdfo::two_tower`` then does
both towers, the dot, BCE and the complete backward in one launch; the
2,400 dense gradients are reduced in fixed order and updated by the flat
fused AdamW; embedding rows are updated by the sort-based fused optimizer.
Per step: ~8 launches, captured into one hipGraph.

Embedding update semantics:
  * ``emb_update="sparse"`` (default): decoupled-weight-decay Adam applied only
    to the rows a batch touches (the TorchRec fused-optimizer semantics).
  * ``emb_update="dense"``: exact optax.adamw parity — the embedding gradient
    is materialised densely and every row (touched or not) is decayed and
    moved by Adam's momentum each step, as jax-flax/train.py:26 does.

Data parallel (train_dp): tables are replicated; instead of the reference's
dense all-reduce of whole tables (jax-flax/train_dp.py:63), ranks all-gather
the (ids, row-gradient) pairs of the global batch and run the same
deterministic sparse update, so replicas stay bit-identical. Sharded
(train_ps, SURVEY P5 -> P7): tables live in the row/table-wise sharded engine.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..utils.capture import graph_capture
from .. import ops
from ..sparse.tables import EmbOptimConfig, TableBatchedEmbedding, TableConfig

FEATURES = ["user_id", "item_id", "language", "is_ebook", "format", "publisher", "pub_decade"]
SIZE_KEYS = ["user", "item", "language", "is_ebook", "format", "publisher", "pub_decade"]
# Flax param names (jax-flax/models.py:18-70)
EMBED_NAMES = ["user_embed", "item_embed", "language_embed", "is_ebook_embed", "format_embed",
               "publisher_embed", "pub_decade_embed"]
DENSE_LAYERS = [("user_fc1", 16), ("user_fc2", 16), ("item_fc1", 98), ("item_fc2", 16)]
E = 16
LDX = 116          # X row: 7 x 16 embeddings | avg_rating | num_pages | pad (16B rows)
NPARAM = ops.TT_NPARAM


@dataclass
class TwoTowerConfig:
    size_map: Dict[str, int]
    embed_dim: int = 16
    learning_rate: float = 3e-4
    weight_decay: float = 1e-4
    init: str = "flax"                 # "flax" (glorot_uniform) | "keras" (lecun_normal dense)
    emb_update: str = "sparse"         # "sparse" | "dense"
    seed: int = 42
    # jax-flax/train_dp.py:28-29,42,55-81 + models.py:142-151: fp16 compute
    # with Flax-style DynamicScale (loss x scale; non-finite grads skip the
    # whole update, params and optimizer state untouched, and halve the
    # scale; 2000 finite steps double it)
    mixed_precision: bool = False
    init_scale: float = 2.0 ** 15
    growth_interval: int = 2000

    def __post_init__(self):
        if self.embed_dim != E:
            raise ValueError("the fused TwoTower kernel is built for embed_dim=16 "
                             "(every reference config uses 16)")
        missing = [k for k in SIZE_KEYS if k not in self.size_map]
        if missing:
            raise ValueError(f"size_map is missing {missing}")


def _glorot(shape, gen):
    lim = math.sqrt(6.0 / (shape[0] + shape[1]))
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1).mul(lim).float()


def _lecun_normal(shape, gen):
    # truncated normal on [-2, 2] std, rescaled like jax/keras lecun_normal
    std = math.sqrt(1.0 / shape[0]) / 0.87962566103423978
    t = torch.empty(shape, dtype=torch.float32)
    torch.nn.init.trunc_normal_(t, 0.0, 1.0, -2.0, 2.0, generator=gen)
    return t * std


def init_dense_params(init: str, seed: int) -> torch.Tensor:
    """Flat 2,400 params: per layer kernel [in, out] then bias (zeros)."""
    gen = torch.Generator().manual_seed(seed)
    parts = []
    for _, fan_in in DENSE_LAYERS:
        k = _glorot((fan_in, E), gen) if init == "flax" else _lecun_normal((fan_in, E), gen)
        parts += [k.reshape(-1), torch.zeros(E)]
    return torch.cat(parts)


class TwoTowerTrainer:
    """Fused TwoTower training/eval engine (one rank)."""

    def __init__(self, cfg: TwoTowerConfig, batch_size: int, device="cpu", group=None,
                 rank: int = 0, world_size: int = 1, eval_batch_size: Optional[int] = None,
                 emb_sharding: Optional[str] = None):
        self.cfg = cfg
        self.B = int(batch_size)
        self.EB = int(eval_batch_size or batch_size)
        self.device = dev = torch.device(device)
        self.group, self.rank, self.world = group, rank, world_size
        rows = [int(cfg.size_map[k]) for k in SIZE_KEYS]
        self.rows = rows
        emb_opt = EmbOptimConfig("adam" if cfg.emb_update == "sparse" else "dense_grad",
                                 lr=cfg.learning_rate, weight_decay=cfg.weight_decay)
        # glorot_uniform on [rows, 16] tables (both reference backends)
        ranges = [math.sqrt(6.0 / (r + E)) for r in rows]
        self.emb = TableBatchedEmbedding(rows, E, dev, emb_opt, init_ranges=ranges, seed=cfg.seed)
        init_store = self.emb
        self.sharded = None
        if emb_sharding is not None:
            # parameter-server replacement (SURVEY P5 -> P7): tables sharded
            # over ranks, ids/rows exchanged with all-to-all
            if cfg.emb_update != "sparse":
                raise ValueError("sharded embeddings use the fused sparse optimizer")
            from ..sparse.planner import plan_sharding
            from ..sparse.sharded import ShardedEmbeddingBags
            tabs = [TableConfig(k, r, E, init_range=ranges[i]) for i, (k, r) in
                    enumerate(zip(SIZE_KEYS, rows))]
            plan = plan_sharding(tabs, world_size, emb_opt, batch_per_rank=self.B,
                                 pooling=[1] * len(rows), strategy=emb_sharding)
            self.plan = plan
            # fp32 pooled rows and gradients end to end: the towers are an
            # fp32 model (the reference's TF PS variables return fp32 rows)
            self.sharded = ShardedEmbeddingBags(tabs, plan, rank, self.B, [1] * len(rows), dev,
                                                emb_opt, group=group, seed=cfg.seed,
                                                recv_dtype="fp32")
            # same initial tables as the replicated path (seeded full tables)
            for t in range(len(rows)):
                self.sharded.set_table_weight(t, init_store.table_weight(t))
            del init_store
            self.emb = self.sharded.tw_store
        if cfg.emb_update == "dense":
            self.emb_grad = torch.zeros_like(self.emb.weight)
            self.emb_m = torch.zeros_like(self.emb.weight)
            self.emb_v = torch.zeros_like(self.emb.weight)
        self.T = len(rows)
        # dense params: flat fp32 + AdamW state
        self.P = torch.zeros(NPARAM + 64, dtype=torch.float32, device=dev)
        self.P[:NPARAM].copy_(init_dense_params(cfg.init, cfg.seed + 1))
        self.G = torch.zeros(ops.TT_PART_LD, dtype=torch.float32, device=dev)
        self.M = torch.zeros(NPARAM, dtype=torch.float32, device=dev)
        self.V = torch.zeros(NPARAM, dtype=torch.float32, device=dev)
        self.hyper = torch.tensor([cfg.learning_rate, 0.0, 1.0], dtype=torch.float32, device=dev)
        self.mp = bool(cfg.mixed_precision)
        # embedding hyper: [lr, step] or, with dynamic loss scaling, [lr, step,
        # 1/scale, found_inf] (the fused embedding kernels unscale the grads
        # and skip the update when found_inf > 0)
        self.emb_hyper = torch.tensor([cfg.learning_rate, 0.0] + ([1.0, 0.0] if self.mp else []),
                                      dtype=torch.float32, device=dev)
        self.dyn_scale = torch.tensor([cfg.init_scale, 0.0], dtype=torch.float32, device=dev)
        self.found_inf = torch.zeros(1, dtype=torch.float32, device=dev)
        # static step buffers (max batch = max(train, eval))
        nb = max(self.B, self.EB)
        self.X = torch.zeros(nb, LDX, dtype=torch.float32, device=dev)
        self.dX = torch.zeros(self.B, LDX, dtype=torch.float32, device=dev)
        self.ids = torch.zeros(self.T * nb, dtype=torch.int64, device=dev)
        self.offsets_full = torch.arange(self.T * nb * max(1, world_size) + 1, dtype=torch.int64,
                                         device=dev)
        self.out_off = torch.arange(self.T, dtype=torch.int64, device=dev) * E
        self.labels = torch.zeros(nb, dtype=torch.float32, device=dev)
        self.logits = torch.zeros(nb, dtype=torch.float32, device=dev)
        self.part = torch.zeros(ops.two_tower_parts(self.B), ops.TT_PART_LD, dtype=torch.float32,
                                device=dev)
        self.loss_sum = torch.zeros(1, dtype=torch.float64, device=dev)
        self.n_seen = 0
        self.nbins = 199     # tf.keras.metrics.AUC(num_thresholds=200) -> 199 buckets
        self.train_hist = torch.zeros(2 * self.nbins, dtype=torch.int64, device=dev)
        self.eval_hist = torch.zeros(2 * self.nbins, dtype=torch.int64, device=dev)
        if world_size > 1:
            self.g_ids = torch.zeros(world_size * self.T * self.B, dtype=torch.int64, device=dev)
            self.g_dX = torch.zeros(world_size * self.B, LDX, dtype=torch.float32, device=dev)
        self.graph = None
        self._cur_b = self.B
        self._bumped = False
        # one-GPU fp32 steps: the fused six-launch sequence (_step_local_fused)
        self.fused_step = os.environ.get("TDFO_TT_FUSED", "1") != "0"
        # ... with the dense step (reduce_adam) run by side blocks of the
        # embedding sort launch
        self.side_job = os.environ.get("TDFO_TT_SIDE_JOB", "1") != "0"
        # ... and the tower kernel co-launched with the per-table id sort
        # (both need only this step's inputs)
        self.colaunch = os.environ.get("TDFO_TT_COLAUNCH", "1") != "0"

    # ------------------------------------------------------------ data in
    def load_batch(self, batch: Dict[str, torch.Tensor], eval_mode: bool = False) -> int:
        """Copy one batch (dict of column tensors) into the static buffers.
        ids are laid out table-major: ids[t*b + j]. With sharded tables every
        batch is padded to the engine's static size B (id 0, ignored rows)."""
        b = int(batch["user_id"].shape[0])
        cap = self.EB if eval_mode else self.B
        assert b <= cap and (b > 0 or self.sharded is not None), (b, cap)
        if self.sharded is not None:
            assert b <= self.B, "sharded eval batches must not exceed the train batch"
            ids = self.ids[: self.T * self.B].view(self.T, self.B)
            if b < self.B:
                ids.zero_()
            ids = ids[:, :b]
        else:
            ids = self.ids[: self.T * b].view(self.T, b)
        for t, f in enumerate(FEATURES):
            ids[t].copy_(batch[f], non_blocking=True)
        self.X[:b, 112].copy_(batch["avg_rating"], non_blocking=True)
        self.X[:b, 113].copy_(batch["num_pages"], non_blocking=True)
        if "label" in batch:
            self.labels[:b].copy_(batch["label"], non_blocking=True)
        self._cur_b = b
        return b

    def load_columns(self, cols: Dict[str, torch.Tensor], idx: Optional[torch.Tensor], row0: int,
                     n: int, eval_mode: bool = False) -> int:
        """``load_batch`` straight from HBM-resident columns: rows idx[:n] (or
        [row0, row0 + n)) of every column are gathered, converted and stored
        into the static buffers by one ``gather_columns`` launch."""
        cap = self.EB if eval_mode else self.B
        assert n <= cap and (n > 0 or self.sharded is not None), (n, cap)
        stride = n
        if self.sharded is not None:
            assert n <= self.B, "sharded eval batches must not exceed the train batch"
            stride = self.B
            if n < self.B:
                self.ids[: self.T * self.B].zero_()
        src = [cols[f] for f in FEATURES] + [cols["avg_rating"], cols["num_pages"]]
        dst = [self.ids[t * stride:] for t in range(self.T)] + \
              [self.X.view(-1)[112:], self.X.view(-1)[113:]]
        st = [1] * self.T + [self.X.shape[1], self.X.shape[1]]
        if "label" in cols:
            src.append(cols["label"])
            dst.append(self.labels)
            st.append(1)
        if n:
            ops.gather_columns(src, idx, row0, n, dst, st)
        self._cur_b = n
        return n

    # ------------------------------------------------------------ step
    def _lookup(self, b: int):
        if self.sharded is not None:
            recv = self.sharded.forward(self.ids[: self.T * self.B])
            for t in range(self.T):
                src = recv.as_strided((self.B, E), (self.sharded.slot_stride[t], 1),
                                      self.sharded.slot_off[t])
                self.X[:b, t * E:(t + 1) * E].copy_(src[:b])
            return
        self.emb.forward(self.ids[: self.T * b], self.offsets_full[: self.T * b + 1],
                         self.emb.row_offset, self.T, b, self.X, self.out_off, LDX)

    def _train_compute(self, b: int):
        """Everything from the lookup to the parameter updates."""
        self._lookup(b)
        inv_n = 1.0 / (b * self.world)
        ops.two_tower(self.X[:b], self.P, self.labels[:b], inv_n, self.logits[:b], self.dX[:b],
                      self.part, loss_scale=self.dyn_scale[0:1] if self.mp else None,
                      half=self.mp)
        nparts = ops.two_tower_parts(b)
        ops.reduce_rows(self.part, nparts, NPARAM + 1, ops.TT_PART_LD, self.G)
        ops.auc_hist(self.logits[:b], self.labels[:b], self.nbins, self.train_hist)

    # ---------------------------------------------------- dynamic loss scale
    def _mp_check(self, grads):
        """Device-side finite check of every (scaled) gradient of the step, and
        the unscale factors / skip flag the fused optimizers read: no host sync."""
        if not self.mp:
            return
        self.found_inf.zero_()
        for g in grads:
            ops.check_finite(g.reshape(-1), self.found_inf)
        inv = torch.reciprocal(self.dyn_scale[0:1])
        self.hyper[2:3].copy_(inv)
        self.emb_hyper[2:3].copy_(inv)
        self.emb_hyper[3:4].copy_(self.found_inf)

    def _mp_update_scale(self):
        """Flax DynamicScale: backoff x0.5 on a non-finite step, growth x2
        after ``growth_interval`` consecutive finite steps."""
        if not self.mp:
            return
        f = self.found_inf
        good = (self.dyn_scale[1:2] + 1.0) * (1.0 - f)
        grow = (good >= float(self.cfg.growth_interval)).float()
        scale = self.dyn_scale[0:1]
        new = (1.0 - f) * scale * (1.0 + grow) + f * torch.clamp(scale * 0.5, min=1.0)
        self.dyn_scale[0:1].copy_(new)
        self.dyn_scale[1:2].copy_(good * (1.0 - grow))

    def _bump(self, hyper):
        """Advance an optimizer's step counter (not on a skipped step)."""
        if self._bumped:
            return                      # done for both optimizers in one launch
        if self.mp:
            hyper[1:2].add_(1.0 - self.found_inf)
        else:
            hyper[1:2].add_(1.0)

    def _dense_update(self):
        self.loss_sum.add_(self.G[NPARAM:NPARAM + 1].double())
        self._bump(self.hyper)
        ops.dense_optimizer(self.P[:NPARAM], self.G[:NPARAM], self.M, self.V, None,
                            ops.OPT_ADAMW, self.hyper, wd=self.cfg.weight_decay,
                            found_inf=self.found_inf if self.mp else None)

    def _emb_update(self, ids, b_total, grad):
        self._bump(self.emb_hyper)
        offs = self.offsets_full[: self.T * b_total + 1]
        if self.cfg.emb_update == "sparse":
            # one id per bag, tables contiguous: per-table LDS sorts instead of
            # the device-wide radix sort (falls back to it past 8192 ids per
            # table, embedding.hip onehot_path)
            self.emb.backward_update(ids, offs, self.emb.row_offset, self.T, b_total, grad,
                                     self.out_off, LDX, self.emb_hyper, segsort=1)
        else:
            # raw (still scaled) dense gradient; the dense AdamW unscales by
            # hyper[2] and skips on found_inf
            self.emb_grad.zero_()
            self.emb.backward_update(ids, offs, self.emb.row_offset, self.T, b_total, grad,
                                     self.out_off, LDX, self.emb_hyper[:2],
                                     dense_grad=self.emb_grad)
            ops.dense_optimizer(self.emb.weight.view(-1), self.emb_grad.view(-1),
                                self.emb_m.view(-1), self.emb_v.view(-1), None, ops.OPT_ADAMW,
                                self.hyper, wd=self.cfg.weight_decay,
                                found_inf=self.found_inf if self.mp else None)

    def _step_local_fused(self, b: int):
        """The one-GPU fp32 step in two launches: the towers + BCE + backward
        (embedding rows gathered in-kernel, both step counters bumped) beside
        the per-table id sort; then the sparse Adam update (crossing runs
        finished in-kernel for small batches) beside the partial rows'
        reduction + AdamW + loss add + AUC histogram (``reduce_adam``).
        (``side_job`` / ``colaunch`` off: those as launches of their own.) Bit-identical to the unfused
        sequence (``TDFO_TT_FUSED=0``: + the lookup, reduce_rows, auc_hist,
        bump, dense_optimizer and the loss add as launches of their own)."""
        ops.two_tower(self.X[:b], self.P, self.labels[:b], 1.0 / b, self.logits[:b], self.dX[:b],
                      self.part, bumps=[self.hyper, self.emb_hyper],
                      emb=(self.emb.weight, self.ids[: self.T * b], self.emb.row_offset),
                      defer=self.side_job and self.colaunch)
        ops.reduce_adam(self.part, ops.two_tower_parts(b), NPARAM, ops.TT_PART_LD, self.G, self.P,
                        self.M, self.V, self.hyper, wd=self.cfg.weight_decay, adamw=True,
                        loss_acc=self.loss_sum, logits=self.logits[:b], labels=self.labels[:b],
                        nb=self.nbins, hist=self.train_hist, defer=self.side_job)
        self._bumped = True
        try:
            self._emb_update(self.ids[: self.T * b], b, self.dX[:b])
        finally:
            self._bumped = False
            if self.side_job:
                ops.flush_side_job()

    def _step_local(self, b: int):
        if not self.mp and self.device.type == "cuda" and self.fused_step:
            self._step_local_fused(b)
            return
        self._train_compute(b)
        self._mp_check([self.G[:NPARAM], self.dX[:b, :112]])
        if not self.mp and self.device.type == "cuda":
            # both step counters in one native launch (no torch kernels)
            ops.bump([self.hyper[1:2], self.emb_hyper[1:2]])
            self._bumped = True
        try:
            self._dense_update()
            self._emb_update(self.ids[: self.T * b], b, self.dX[:b])
        finally:
            self._bumped = False
        self._mp_update_scale()

    def _step_dp(self, b: int):
        assert b == self.B, "data-parallel steps use full batches (drop_last)"
        self._train_compute(b)
        # dense grads + loss: one all-reduce of 2,401 floats
        dist.all_reduce(self.G[: NPARAM + 1], group=self.group)
        # sparse rows: all-gather (ids, row grads) of the global batch; every
        # rank applies the same deterministic update -> replicas stay equal
        W, T = self.world, self.T
        dist.all_gather_into_tensor(self.g_ids, self.ids[: T * b], group=self.group)
        dist.all_gather_into_tensor(self.g_dX, self.dX[:b], group=self.group)
        # the finite check sees the global gradients: every rank skips together
        self._mp_check([self.G[:NPARAM], self.g_dX[:, :112]])
        self._dense_update()
        # regroup ids rank-major [W][T][b] -> table-major [T][W*b] (bag = t*W*b + r*b + j)
        gid = self.g_ids.view(W, T, b).transpose(0, 1).reshape(-1)
        self._emb_update(gid, W * b, self.g_dX)
        self._mp_update_scale()

    def _step_sharded(self, b: int):
        assert b == self.B, "sharded training steps use full batches (drop_last)"
        if self.mp:
            raise NotImplementedError("mixed_precision is the train_dp.py path (replicated "
                                      "tables), as in the reference")
        self._train_compute(b)
        if self.world > 1:
            dist.all_reduce(self.G[: NPARAM + 1], group=self.group)
        self._dense_update()
        sh = self.sharded
        for t in range(self.T):
            dst = sh.d_recv.as_strided((b, E), (sh.slot_stride[t], 1), sh.slot_off[t])
            dst.copy_(self.dX[:b, t * E:(t + 1) * E])
        self.emb_hyper[1:2].add_(1.0)
        sh.backward_start()
        sh.backward_finish(self.emb_hyper)

    def step(self):
        b = self._cur_b
        if self.graph is not None and b == self.B:
            self.graph.replay()
        elif self.sharded is not None:
            self._step_sharded(b)
        elif self.world > 1:
            self._step_dp(b)
        else:
            self._step_local(b)
        self.n_seen += b

    def capture_graph(self, warmup: int = 2):
        """One hipGraph for the full single-process step (fixed batch B)."""
        if self.device.type != "cuda" or self.world > 1 or self.sharded is not None:
            return
        saved = [t.clone() for t in self._state_tensors()]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._step_local(self.B)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            self._step_local(self.B)
        torch.cuda.synchronize()
        for t, v in zip(self._state_tensors(), saved):   # warmup must not train
            t.copy_(v)
        self.graph = g

    def capture_execution(self, cols: Dict[str, torch.Tensor], k: int):
        """``steps_per_execution = k`` (the reference's Keras
        ``steps_per_execution``, tensorflow2/train.py:14-18): one hipGraph
        holds k consecutive (HBM gather + training step) pairs reading their
        rows from a static index buffer, so one index copy and one replay
        issue k steps. Needs the one-step graph to exist (its capture ran the
        warmup that sizes every workspace)."""
        assert self.graph is not None and k > 1
        B = self.B
        self._exec_idx = torch.zeros(k * B, dtype=torch.int64, device=self.device)
        self._exec_cols = cols
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            for j in range(k):
                self.load_columns(cols, self._exec_idx[j * B:(j + 1) * B], 0, B)
                self._step_local(B)
        torch.cuda.synchronize()
        self._exec_graph, self._exec_k = g, k

    def run_execution(self, idxs: List[torch.Tensor]):
        """Run len(idxs) == k full steps (rows idxs[j] of the columns given to
        ``capture_execution``) with one replay."""
        k, B = self._exec_k, self.B
        assert len(idxs) == k and all(int(i.numel()) == B for i in idxs)
        for j, ix in enumerate(idxs):
            self._exec_idx[j * B:(j + 1) * B].copy_(ix, non_blocking=True)
        self._exec_graph.replay()
        self._cur_b = B
        self.n_seen += k * B

    def _state_tensors(self):
        ts = [self.P, self.M, self.V, self.hyper, self.emb_hyper, self.emb.weight, self.loss_sum,
              self.train_hist, self.dyn_scale, self.found_inf]
        for x in (self.emb.state1, self.emb.state2):
            if x is not None:
                ts.append(x)
        if self.cfg.emb_update == "dense":
            ts += [self.emb_m, self.emb_v]
        return ts

    # ------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate_batch(self) -> torch.Tensor:
        """Forward the loaded eval batch; accumulates eval loss + AUC hist."""
        b = self._cur_b
        self._lookup(b)
        if b == 0:
            return self.logits[:0]
        lg = self.logits[:b]
        ops.two_tower(self.X[:b], self.P, self.labels[:b], 1.0, lg, half=self.mp)
        y = self.labels[:b]
        loss = torch.nn.functional.binary_cross_entropy_with_logits(lg, y, reduction="sum")
        self.loss_sum.add_(loss.double())
        ops.auc_hist(lg, y, self.nbins, self.eval_hist)
        self.n_seen += b
        return lg

    # ------------------------------------------------------------ metrics
    def pop_metrics(self, eval_mode: bool = False, reduce: bool = True):
        """(mean loss, bucketed ROC-AUC) since the last call; all-reduced over
        ranks (one small all-reduce per epoch, not per step: quirk Q2)."""
        hist = self.eval_hist if eval_mode else self.train_hist
        stats = torch.cat([self.loss_sum, torch.tensor([float(self.n_seen)], dtype=torch.float64,
                                                       device=self.device)])
        h = hist.clone()
        if reduce and self.world > 1:
            if eval_mode:
                dist.all_reduce(stats, group=self.group)
            else:
                # the training loss sum was already all-reduced inside each step
                stats[1] *= self.world
            dist.all_reduce(h, group=self.group)
        loss = float(stats[0] / max(1.0, float(stats[1])))
        auc = ops.reference.hist_auc(h)
        self.loss_sum.zero_()
        hist.zero_()
        self.n_seen = 0
        return loss, auc

    # ------------------------------------------------------------ params
    def flax_params(self) -> Dict[str, Dict[str, torch.Tensor]]:
        """Nested param dict with Flax names/layouts (jax-flax/models.py:18-70)."""
        out = {}
        for t, name in enumerate(EMBED_NAMES):
            out[name] = {"embedding": self.table_weight(t)}
        P = self.P[:NPARAM].detach().cpu()
        o = 0
        for name, fan_in in DENSE_LAYERS:
            out[name] = {"kernel": P[o: o + fan_in * E].view(fan_in, E).clone()}
            o += fan_in * E
            out[name]["bias"] = P[o: o + E].clone()
            o += E
        return out

    def table_weight(self, t: int) -> torch.Tensor:
        """Full table t on CPU (gathered from its shards when sharded)."""
        if self.sharded is not None:
            full = torch.zeros(self.rows[t], E, dtype=torch.float32, device=self.device)
            part = self.sharded.get_table_weight(t)
            if part is not None:
                rows, w = part
                full[rows].copy_(w)
            if self.world > 1:
                dist.all_reduce(full, group=self.group)
            return full.cpu()
        return self.emb.table_weight(t).detach().cpu().clone()

    def load_flax_params(self, params):
        for t, name in enumerate(EMBED_NAMES):
            w = torch.as_tensor(params[name]["embedding"]).float()
            if self.sharded is not None:
                self.sharded.set_table_weight(t, w.to(self.device))
            else:
                self.emb.table_weight(t).copy_(w)
        flat = []
        for name, _ in DENSE_LAYERS:
            flat += [torch.as_tensor(params[name]["kernel"]).reshape(-1),
                     torch.as_tensor(params[name]["bias"]).reshape(-1)]
        self.P[:NPARAM].copy_(torch.cat(flat).float())

    def state_dict(self):
        d = {"P": self.P, "M": self.M, "V": self.V, "hyper": self.hyper,
             "emb_hyper": self.emb_hyper, "dyn_scale": self.dyn_scale}
        if self.sharded is not None:
            for grp, sd in self.sharded.state_dict().items():
                d.update({f"emb.{grp}.{k}": v for k, v in sd.items()})
        else:
            d.update({"emb." + k: v for k, v in self.emb.state_dict().items()})
        if self.cfg.emb_update == "dense":
            d["emb_m"], d["emb_v"] = self.emb_m, self.emb_v
        return d

    def load_state_dict(self, d):
        for k, v in self.state_dict().items():
            if k in d:
                v.copy_(d[k])
