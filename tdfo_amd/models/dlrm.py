"""DLRM (and the shared dense-arch machinery for DCN-v2) with an explicit,
hipGraph-capturable training step.

This is the north-star workload of BASELINE.json (absent from the reference,
see SURVEY.md §2.7 NS2): bottom MLP -> pooled embeddings (26 tables) ->
pairwise-dot interaction -> top MLP -> BCE.

The step is written out by hand instead of going through autograd so every
buffer is preallocated, every hot op is one of our HIP kernels, the
communication is placed for overlap, and the whole thing can be captured
once into a hipGraph and replayed (no tracing compiler):

  fwd  ids a2a -> EmbeddingBag (HIP, writes a2a send layout) -> pooled a2a
       || bottom MLP (MFMA GEMM + bias + ReLU epilogue)
       -> interaction (MFMA, reads pooled rows in place) -> top MLP
       -> head_bce (last layer + BCE + dlogit + ReLU mask, one pass)
  bwd  per layer: wgrad (MFMA, split-K, transposed operands read with
       ds_read_b64_tr_b16), bias grad (colsum), dgrad (MFMA, ReLU-mask
       epilogue) -> interaction bwd (MFMA) -> grad a2a (async)
       || bottom MLP bwd || dense-grad all-reduce (one flat buffer)
       -> fused sort-based embedding backward + row-wise Adagrad
       -> fused flat AdamW (also refreshes the bf16 weight shadow).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import ops
from ..sparse.planner import ShardingPlan, plan_sharding
from ..sparse.sharded import ShardedEmbeddingBags
from ..sparse.tables import EmbOptimConfig, TableConfig
from ..utils.flat import FlatParams

# MLPerf DLRM (Criteo Terabyte, max-ind-range 40M) per-feature cardinalities.
CRITEO_1TB_ROWS = [39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 38532951, 2953546,
                   403346, 10, 2208, 11938, 155, 4, 976, 14, 39979771, 25641295, 39664984, 585935,
                   12972, 108, 36]
# Criteo Kaggle (Display Advertising Challenge) cardinalities.
CRITEO_KAGGLE_ROWS = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593,
                      3194, 27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105,
                      142572]
# MLPerf DLRM-DCNv2 synthetic multi-hot pooling factors.
MLPERF_MULTIHOT = [3, 2, 1, 2, 6, 1, 1, 1, 1, 7, 3, 8, 1, 6, 9, 5, 1, 1, 1, 12, 100, 27, 10, 3, 1,
                   1]

DENSE_OPTS = {"adamw": ops.OPT_ADAMW, "adam": ops.OPT_ADAM, "sgd": ops.OPT_SGD,
              "adagrad": ops.OPT_ADAGRAD}


def pad64(n: int) -> int:
    return -(-n // 64) * 64


@dataclass
class DLRMConfig:
    num_dense: int = 13
    embedding_dim: int = 128
    table_rows: List[int] = field(default_factory=lambda: list(CRITEO_1TB_ROWS))
    pooling: Optional[List[int]] = None            # fixed ids per bag per table (default 1)
    bottom: List[int] = field(default_factory=lambda: [512, 256, 128])
    top: List[int] = field(default_factory=lambda: [1024, 1024, 512, 256, 1])
    interaction: str = "dot"                       # "dot" (DLRM) | "dcn" (DCN-v2)
    dcn_layers: int = 3
    dcn_rank: int = 512
    dense_opt: str = "adamw"
    dense_lr: float = 1e-3
    dense_wd: float = 0.0
    emb_opt: str = "rowwise_adagrad"
    emb_lr: float = 0.01
    emb_eps: float = 1e-8
    sharding: str = "auto"                         # planner strategy
    seed: int = 0

    @property
    def num_tables(self) -> int:
        return len(self.table_rows)

    def tables(self) -> List[TableConfig]:
        return [TableConfig(f"t{i}", int(r), self.embedding_dim, [f"cat_{i}"])
                for i, r in enumerate(self.table_rows)]

    def pooling_factors(self) -> List[int]:
        return list(self.pooling) if self.pooling is not None else [1] * self.num_tables

    def dense_flops_per_example(self) -> float:
        """fwd+bwd FLOPs of the dense part (3x forward GEMM FLOPs)."""
        F = self.num_tables + 1
        D = self.embedding_dim
        dims = [pad64(self.num_dense)] + self.bottom
        f = sum(2 * a * b for a, b in zip(dims[:-1], dims[1:]))
        if self.interaction == "dot":
            f += 2 * F * F * D
            tin = pad64(D + F * (F - 1) // 2)
        else:
            w = F * D
            f += self.dcn_layers * 2 * 2 * w * self.dcn_rank
            tin = w
        tdims = [tin] + self.top
        f += sum(2 * a * b for a, b in zip(tdims[:-1], tdims[1:]))
        return 3.0 * f


class DLRMTrainer:
    """Explicit-step DLRM/DCN-v2 trainer over a sharded embedding engine.

    ``batch_size`` is per rank (weak scaling). Works on CPU (torch reference
    ops, gloo) and on MI355X (HIP kernels, RCCL); optionally captures the
    step in a hipGraph (single process).
    """

    def __init__(self, cfg: DLRMConfig, batch_size: int, device, group=None, rank: int = 0,
                 world_size: int = 1, plan: Optional[ShardingPlan] = None):
        self.cfg = cfg
        self.B = B = int(batch_size)
        self.device = dev = torch.device(device)
        self.group = group
        self.rank = rank
        self.world = world_size
        D = cfg.embedding_dim
        T = cfg.num_tables
        self.F = F = T + 1
        assert cfg.bottom[-1] == D, "bottom MLP must end at the embedding dim"
        assert cfg.top[-1] == 1
        torch.manual_seed(cfg.seed)
        # ------------------------------------------------------ embeddings
        optim = EmbOptimConfig(cfg.emb_opt, lr=cfg.emb_lr, eps=cfg.emb_eps)
        tables = cfg.tables()
        self.plan = plan or plan_sharding(tables, world_size, optim, batch_per_rank=B,
                                          pooling=cfg.pooling_factors(), strategy=cfg.sharding)
        self.emb = ShardedEmbeddingBags(tables, self.plan, rank, B, cfg.pooling_factors(), dev,
                                        optim, group=group, seed=cfg.seed)
        # ------------------------------------------------------ dense params
        self.in_pad = pad64(cfg.num_dense)
        fp = FlatParams()
        self.bottom_layers = []
        dims = [self.in_pad] + cfg.bottom
        for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
            fp.add(f"bot{i}.w", (b, a))
            fp.add(f"bot{i}.b", (b,))
            self.bottom_layers.append((f"bot{i}", a, b))
        if cfg.interaction == "dot":
            self.top_in = pad64(D + F * (F - 1) // 2)
        else:
            self.top_in = F * D
            for i in range(cfg.dcn_layers):
                fp.add(f"dcn{i}.v", (cfg.dcn_rank, self.top_in))
                fp.add(f"dcn{i}.u", (self.top_in, cfg.dcn_rank))
                fp.add(f"dcn{i}.b", (self.top_in,))
        self.top_layers = []
        tdims = [self.top_in] + cfg.top[:-1]
        for i, (a, b) in enumerate(zip(tdims[:-1], tdims[1:])):
            fp.add(f"top{i}.w", (b, a))
            fp.add(f"top{i}.b", (b,))
            self.top_layers.append((f"top{i}", a, b))
        self.head_k = tdims[-1]
        fp.add("head", (self.head_k + 1,))           # [w (K) | b]
        opt = DENSE_OPTS[cfg.dense_opt]
        self.dense_opt = opt
        fp.finalize(dev, with_adam=opt in (ops.OPT_ADAMW, ops.OPT_ADAM))
        self.fp = fp
        self._init_dense()
        # broadcast dense params from rank 0 (replicated dense arch)
        if world_size > 1:
            dist.broadcast(fp.p, src=0, group=group)
        fp.sync_bf16()
        # ------------------------------------------------------ buffers
        bf = torch.bfloat16
        z = lambda *s, dt=bf: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        self.x0 = z(B, self.in_pad)
        self.label = z(B, dt=torch.float32)
        self.ids = torch.zeros(self.emb.nnz_local, dtype=torch.int64, device=dev)
        self.bot_act = [z(B, b) for (_, _, b) in self.bottom_layers]
        self.bot_grad = [z(B, b) for (_, _, b) in self.bottom_layers]
        self.zbuf = z(B, self.top_in)
        self.dz = z(B, self.top_in)
        self.top_act = [z(B, b) for (_, _, b) in self.top_layers]
        self.top_grad = [z(B, b) for (_, _, b) in self.top_layers]
        if cfg.interaction == "dcn":
            L = cfg.dcn_layers
            self.dcn_x = [z(B, self.top_in) for _ in range(L + 1)]      # x_0 .. x_L
            self.dcn_h = [z(B, cfg.dcn_rank) for _ in range(L)]         # V^T x_l
            self.dcn_y = [z(B, self.top_in) for _ in range(L)]          # U h + b
            self.dcn_dx = [z(B, self.top_in) for _ in range(L + 1)]
            self.dcn_dx0acc = z(B, self.top_in)
            self.dcn_dh = z(B, cfg.dcn_rank)
            self.dcn_dy = z(B, self.top_in)
        self.logits = z(B, dt=torch.float32)
        self.nparts = ops.head_parts(B)
        self.head_part = z(self.nparts * (self.head_k + 2), dt=torch.float32)
        self.loss_sum = z(1, dt=torch.float32)
        max_slab = 1
        for (_, a, b) in self.bottom_layers + self.top_layers:
            s = ops.wgrad_splits(b, a, B)
            max_slab = max(max_slab, s * a * b)
        if cfg.interaction == "dcn":
            s = ops.wgrad_splits(cfg.dcn_rank, self.top_in, B)
            max_slab = max(max_slab, s * cfg.dcn_rank * self.top_in)
        self.slab = z(max_slab, dt=torch.float32)
        self.dense_hyper = torch.tensor([cfg.dense_lr, 0.0, 1.0], dtype=torch.float32, device=dev)
        self.emb_hyper = torch.tensor([cfg.emb_lr, 0.0], dtype=torch.float32, device=dev)
        self.slot_off = [0] + list(self.emb.slot_off)
        self.slot_stride = [0] + list(self.emb.slot_stride)
        self.graph = None
        self.steps = 0

    # --------------------------------------------------------------- init
    def _init_dense(self):
        g = torch.Generator(device="cpu")
        g.manual_seed(self.cfg.seed + 7)
        fp = self.fp

        def init_linear(name, out_f, in_f, real_in):
            w = torch.randn(out_f, real_in, generator=g) * math.sqrt(2.0 / (real_in + out_f))
            b = torch.randn(out_f, generator=g) * math.sqrt(1.0 / out_f)
            W = fp.param(name + ".w")
            W.zero_()
            W[:, :real_in] = w.to(W.device)
            fp.param(name + ".b").copy_(b)

        dims_real = [self.cfg.num_dense] + self.cfg.bottom
        for i, (name, a, b) in enumerate(self.bottom_layers):
            init_linear(name, b, a, dims_real[i])
        F, D = self.F, self.cfg.embedding_dim
        real_top_in = D + F * (F - 1) // 2 if self.cfg.interaction == "dot" else self.top_in
        tdims_real = [real_top_in] + self.cfg.top[:-1]
        for i, (name, a, b) in enumerate(self.top_layers):
            init_linear(name, b, a, tdims_real[i])
        if self.cfg.interaction == "dcn":
            for i in range(self.cfg.dcn_layers):
                r, w = self.cfg.dcn_rank, self.top_in
                fp.param(f"dcn{i}.v").copy_(torch.randn(r, w, generator=g) * math.sqrt(2.0 / (r + w)))
                fp.param(f"dcn{i}.u").copy_(torch.randn(w, r, generator=g) * math.sqrt(2.0 / (r + w)))
                fp.param(f"dcn{i}.b").zero_()
        K = self.head_k
        h = fp.param("head")
        h[:K] = (torch.randn(K, generator=g) * math.sqrt(2.0 / (K + 1))).to(h.device)
        h[K] = 0.0

    # ------------------------------------------------------------ batches
    def load_batch(self, dense: torch.Tensor, ids: torch.Tensor, label: torch.Tensor):
        """Copy a batch into the static input buffers (non_blocking H2D ok).

        dense [B, num_dense] (any float dtype), ids flat int64 in table order
        (table t: B*L_t ids), label [B] float.
        """
        self.x0[:, : self.cfg.num_dense].copy_(dense, non_blocking=True)
        self.ids.copy_(ids, non_blocking=True)
        self.label.copy_(label, non_blocking=True)

    # --------------------------------------------------------------- step
    def _linear_bwd(self, name, x, dy, dx, x_is_relu):
        """wgrad + bias grad (+ dgrad into dx, masked by x > 0 if x_is_relu)."""
        fp = self.fp
        gw = fp.grad(name + ".w")
        ops.linear_wgrad(dy, x, gw.view(-1), slab=self.slab)
        ops.colsum(dy, fp.grad(name + ".b"))
        if dx is not None:
            ops.linear_dgrad(dy, fp.bf16(name + ".w"), mask=x if x_is_relu else None, out=dx)

    # ---------------------------------------------------------- stages
    # The step is a fixed sequence of compute stages ("c", hipGraph-capturable)
    # and communication stages ("m", RCCL collectives issued eagerly so they
    # overlap with the next compute stage on their own stream).
    def _stages(self):
        emb = self.emb
        return [
            ("c", lambda: emb.stage_fwd_prep(self.ids)),
            ("m", emb.stage_fwd_ids_exchange),
            ("c", emb.stage_fwd_lookup),
            ("m", emb.stage_fwd_out_exchange),
            ("c", self._s_bottom_fwd),
            ("m", self._m_fwd_wait),
            ("c", self._s_top),
            ("m", emb.backward_start),
            ("c", self._s_bottom_bwd),
            ("m", self._m_allreduce_start),
            ("m", emb.backward_wait),
            ("c", self._s_emb_update),
            ("m", self._m_allreduce_wait),
            ("c", self._s_dense_update),
        ]

    def _forward_backward(self):
        for _, fn in self._stages():
            fn()

    def _s_bottom_fwd(self):
        fp = self.fp
        h = self.x0
        for i, (name, a, b) in enumerate(self.bottom_layers):
            ops.linear_fwd(h, fp.bf16(name + ".w"), fp.param(name + ".b"), relu=True,
                           out=self.bot_act[i])
            h = self.bot_act[i]

    def _m_fwd_wait(self):
        self.emb.forward_wait()
        if self.emb.rw_tables:
            self.emb._rw_forward(self.ids)

    def _s_top(self):
        cfg, fp, B = self.cfg, self.fp, self.B
        D, F = cfg.embedding_dim, self.F
        emb = self.emb
        h = self.bot_act[-1]
        if cfg.interaction == "dot":
            ops.interaction_fwd(h, emb.recv, self.slot_off, self.slot_stride, F, D, self.zbuf)
            t = self.zbuf
        else:
            t = self._dcn_forward(h)
        for i, (name, a, b) in enumerate(self.top_layers):
            ops.linear_fwd(t, fp.bf16(name + ".w"), fp.param(name + ".b"), relu=True,
                           out=self.top_act[i])
            t = self.top_act[i]
        K = self.head_k
        head = fp.param("head")
        ops.head_bce(t, head[:K], head[K:], self.label, 1.0 / (B * self.world), True, self.logits,
                     self.top_grad[-1], self.head_part)
        ops.reduce_rows(self.head_part, self.nparts, K + 1, K + 2, fp.grad("head"))
        ops.reduce_rows(self.head_part[K + 1:], self.nparts, 1, K + 2, self.loss_sum,
                        accumulate=True)
        for i in reversed(range(len(self.top_layers))):
            name = self.top_layers[i][0]
            x = self.top_act[i - 1] if i > 0 else t_in(self)
            if i > 0:
                dx = self.top_grad[i - 1]
            else:
                dx = self.dz if cfg.interaction == "dot" else self.dcn_dx[-1]
            self._linear_bwd(name, x, self.top_grad[i], dx, x_is_relu=i > 0)
        if cfg.interaction == "dot":
            ops.interaction_bwd(self.dz, h, emb.recv, self.slot_off, self.slot_stride, F, D,
                                self.bot_grad[-1], emb.d_recv, self.slot_off, self.slot_stride,
                                True)
        else:
            self._dcn_backward(h)

    def _s_bottom_bwd(self):
        for i in reversed(range(len(self.bottom_layers))):
            name = self.bottom_layers[i][0]
            x = self.bot_act[i - 1] if i > 0 else self.x0
            dx = self.bot_grad[i - 1] if i > 0 else None
            self._linear_bwd(name, x, self.bot_grad[i], dx, x_is_relu=i > 0)

    def _m_allreduce_start(self):
        self._ar_work = None
        if self.world > 1:
            self._ar_work = dist.all_reduce(self.fp.g, group=self.group, async_op=True)

    def _s_emb_update(self):
        self.emb_hyper[1:2].add_(1.0)
        self.emb.stage_bwd_update(self.emb_hyper)

    def _m_allreduce_wait(self):
        if self.emb.rw_tables:
            self.emb._rw_backward(self.emb.d_recv, self.emb_hyper)
        if self._ar_work is not None:
            self._ar_work.wait()
            self._ar_work = None

    def _s_dense_update(self):
        fp = self.fp
        self.dense_hyper[1:2].add_(1.0)
        ops.dense_optimizer(fp.p, fp.g, fp.m, fp.v, fp.p_bf16, self.dense_opt, self.dense_hyper,
                            wd=self.cfg.dense_wd)

    # DCN-v2 cross network: x_{l+1} = x0 * (U (V^T x_l) + b) + x_l. The
    # Hadamard product and the residual are fused into the U-GEMM epilogue
    # (out2 = x0 * (acc + b) + x_l), the residual of the backward into the
    # V-dgrad epilogue.
    def _dcn_forward(self, h):
        cfg, fp, D, F = self.cfg, self.fp, self.cfg.embedding_dim, self.F
        x0 = self.dcn_x[0]
        ops.concat_features(h, self.emb.recv, self.slot_off, self.slot_stride, F, D, x0)
        for i in range(cfg.dcn_layers):
            ops.linear_fwd(self.dcn_x[i], fp.bf16(f"dcn{i}.v"), None, relu=False, out=self.dcn_h[i])
            ops.gemm(self.dcn_h[i], False, fp.bf16(f"dcn{i}.u"), False, fp.param(f"dcn{i}.b"),
                     False, None, self.dcn_y[i], None, 1, mul=x0, add=self.dcn_x[i],
                     out2=self.dcn_x[i + 1])
        return self.dcn_x[-1]

    def _dcn_backward(self, h):
        cfg, fp, D, F = self.cfg, self.fp, self.cfg.embedding_dim, self.F
        L = cfg.dcn_layers
        x0 = self.dcn_x[0]
        acc = self.dcn_dx0acc
        for i in reversed(range(L)):
            dxo = self.dcn_dx[i + 1]
            # dy = dxo * x0 ; acc (+)= dxo * y (+ dxo at i == 0: x_0's residual)
            ops.cross_bwd(dxo, x0, self.dcn_y[i], self.dcn_dy, acc, i != L - 1, i == 0)
            ops.linear_wgrad(self.dcn_dy, self.dcn_h[i], fp.grad(f"dcn{i}.u").view(-1),
                             slab=self.slab)
            ops.colsum(self.dcn_dy, fp.grad(f"dcn{i}.b"))
            ops.linear_dgrad(self.dcn_dy, fp.bf16(f"dcn{i}.u"), out=self.dcn_dh)
            ops.linear_wgrad(self.dcn_dh, self.dcn_x[i], fp.grad(f"dcn{i}.v").view(-1),
                             slab=self.slab)
            # dx_i = dh V + (i > 0 ? dxo : acc)
            ops.gemm(self.dcn_dh, False, fp.bf16(f"dcn{i}.v"), True, None, False, None, None, None,
                     1, add=dxo if i > 0 else acc, out2=self.dcn_dx[i])
        ops.split_features(self.dcn_dx[0], F, D, h, self.bot_grad[-1], self.emb.d_recv,
                           self.slot_off, self.slot_stride, True)

    def step(self):
        """One training step on the batch in the static buffers."""
        if self.graph is not None:
            if isinstance(self.graph, list):
                for kind, item in self.graph:
                    item.replay() if kind == "c" else item()
            else:
                self.graph.replay()
        else:
            self._forward_backward()
        self.steps += 1

    def capture_graph(self, warmup: int = 2, staged: Optional[bool] = None):
        """Capture the step into hipGraphs. Single process: one graph for the
        whole step. Multi-process: one graph per compute stage, with the RCCL
        exchanges issued eagerly between replays (they overlap the next stage)."""
        assert self.device.type == "cuda"
        if not self.emb.graph_capturable:
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._forward_backward()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if staged is None:
            staged = self.world > 1
        if not staged:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._forward_backward()
            self.graph = g
            return
        pool = torch.cuda.graph_pool_handle()
        seq = []
        for kind, fn in self._stages():
            if kind == "c":
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    fn()
                seq.append(("c", g))
            else:
                fn()          # dry exchange keeps every rank's collective sequence aligned
                seq.append(("m", fn))
        torch.cuda.synchronize()
        self.graph = seq

    def pop_loss(self) -> float:
        """Mean training loss since the last call (one device->host read)."""
        v = float(self.loss_sum.item())
        self.loss_sum.zero_()
        return v

    # ------------------------------------------------------------ eval
    @torch.no_grad()
    def predict(self) -> torch.Tensor:
        """Forward only on the static batch; returns logits [B] (fp32)."""
        cfg, fp, D, F = self.cfg, self.fp, self.cfg.embedding_dim, self.F
        self.emb.forward(self.ids)
        h = self.x0
        for i, (name, a, b) in enumerate(self.bottom_layers):
            ops.linear_fwd(h, fp.bf16(name + ".w"), fp.param(name + ".b"), relu=True,
                           out=self.bot_act[i])
            h = self.bot_act[i]
        if cfg.interaction == "dot":
            ops.interaction_fwd(h, self.emb.recv, self.slot_off, self.slot_stride, F, D, self.zbuf)
            t = self.zbuf
        else:
            t = self._dcn_forward(h)
        for i, (name, a, b) in enumerate(self.top_layers):
            ops.linear_fwd(t, fp.bf16(name + ".w"), fp.param(name + ".b"), relu=True,
                           out=self.top_act[i])
            t = self.top_act[i]
        K = self.head_k
        head = fp.param("head")
        return t.float() @ head[:K] + head[K]

    def state_dict(self):
        return {"dense": self.fp.state_dict(), "emb": self.emb.state_dict(),
                "dense_m": self.fp.m, "dense_v": self.fp.v, "dense_hyper": self.dense_hyper,
                "emb_hyper": self.emb_hyper}


def t_in(tr: "DLRMTrainer"):
    return tr.zbuf if tr.cfg.interaction == "dot" else tr.dcn_x[-1]
