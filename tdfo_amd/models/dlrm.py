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
import os
import warnings
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from ..utils.capture import graph_capture
from .. import ops
from .dlrm_dcn import DCNMixin
from .dlrm_streams import StreamGraphsMixin
from .dlrm_multirank import MultiRankStreamsMixin
from ..parallel.comm import as_comm, dense_comm_for
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
# BASELINE config 5: a >1 TB table set for DCN-v2 row-wise sharding -- the
# MLPerf Criteo-TB cardinalities with every table above 1M rows grown 12x
# (an un-capped id space): 2.24 G rows, 1.16 TB of fp32 rows + row-wise
# Adagrad state at D=128. Five tables exceed one GPU's 245 GB budget, so
# the planner shards them row-wise; it fits 8 x 288 GB and not 4.
DCN_GT1TB_ROWS = [r * 12 if r > 1_000_000 else r for r in CRITEO_1TB_ROWS]
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
    rw_capacity: float = 1.25                      # initial row-wise segment capacity (x n/W);
    #   grown on demand before any exchange would overflow
    rw_comm: str = "bf16"                          # row-wise reduce-scatter dtype (bf16 | fp32)
    rw_exchange: str = "auto"                      # row-wise exchange: pooled | rows | auto
    dp_rule: str = "cost"                          # sharding="data_parallel": which tables to
    #   replicate (cost: where the dense all-reduce moves fewer bytes than the row-wise
    #   exchange; budget: smallest first up to 256 MB, sparse/planner.py)
    #   (rows: one-hot tables return looked-up rows by all-to-all, sparse/sharded.py)
    dense_comm: str = "fp32"                       # dense-grad all-reduce dtype (fp32 | bf16:
    #   halves the bytes on xGMI; the sum of W bf16-rounded grads, as DDP's bf16 compress hook)
    pipeline: bool = False                         # W > 1: next batch's id exchange overlaps
    #   this step's dense update (input-dist pipelining; see DLRMTrainer.prime)
    pipeline_lookup: bool = True                   # pipelined: also the next batch's lookup +
    #   pooled exchange in this step's tail (on the side stream)
    defer_wgrad: Optional[bool] = None             # top / cross weight grads after the
    #   interaction / cross backward (None: when W > 1, so the embedding-grad exchange
    #   overlaps them; on one GPU the DCN-v2 update starved them: 2.606 vs 2.52 ms/step,
    #   and DLRM-1TB runs 0.488 vs 0.440, profiles/r04/notes.md)
    opt_placement: Optional[str] = None            # one GPU: "one_pass" (dense optimizer after
    #   the bottom backward; DLRM default) | "split_main" (top part first, beside the
    #   embedding update; DCN-v2 default). (Rejected, round 4: the top part on the
    #   embedding stream behind the update, with or without deferred top weight grads:
    #   DLRM-1TB 0.458 / 0.478 vs 0.440 ms/step, profiles/r04/notes.md)
    #   (Rejected, round 4: the bottom-MLP backward before the embedding update
    #   starts, uncontended: 0.48 vs 0.44 ms/step, profiles/r04/notes.md)
    composed_graphs: Optional[bool] = None         # one GPU: chain each stream's graphs with
    #   in-graph event nodes (None: DLRM yes, DCN-v2 no)
    ids_stream: Optional[bool] = None              # one GPU, composed graphs: copy the next
    #   ids on a third stream behind the sort (None: with composed graphs)
    #   (Rejected, round 4, W > 1 stream graphs: the top weight grads before the bottom
    #   backward so the top bucket reduces beside it -- emulated W=8 0.616-0.621 vs
    #   0.590-0.594 ms/step, config 3 0.872 vs 0.849, config 5 3.035 vs 3.016)
    #   (Rejected, round 4, one GPU: the embedding stream on a CU-masked HIP stream
    #   (hipExtStreamCreateWithCUMask, 160-224 of 256 CUs) -- DLRM-1TB 2.03-2.23 vs
    #   0.444 ms/step, DCN-v2 4.57-4.87 vs 2.36: masked queues do not run beside the
    #   others here)
    #   (Rejected, round 4: the bottom MLP forward as one fused 3-layer launch with the
    #   activations in LDS -- 22.6 vs 26.8 us of kernel, but its 55-KB / 177-VGPR blocks
    #   wait ~47 us for CUs the concurrent lookup fills: DLRM-1TB 0.448-0.450 vs
    #   0.443-0.444 ms/step, W=8 0.591-0.593 vs 0.588-0.591, DCN-v2 neutral)
    stream_graphs: bool = True                     # W > 1, pipelined, capturable comm (native
    #   RCCL / loopback): the step as per-stream hipGraphs with the collectives inside
    #   (dlrm_multirank.py; 3 launches per step) instead of graphs between eagerly issued
    #   exchanges
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

    def dense_params(self) -> int:
        F, D = self.num_tables + 1, self.embedding_dim
        dims = [self.num_dense] + self.bottom
        n = sum((a + 1) * b for a, b in zip(dims[:-1], dims[1:]))
        tin = D + F * (F - 1) // 2 if self.interaction == "dot" else F * D
        tdims = [tin] + self.top
        n += sum((a + 1) * b for a, b in zip(tdims[:-1], tdims[1:]))
        if self.interaction == "dcn":
            n += self.dcn_layers * (2 * F * D * self.dcn_rank + F * D)
        return n

    def sol(self, batch: int, world: int = 1, mfma_flops: float = 1.5e15,
            hbm_bw: float = 6.3e12, link_bw: float = 153e9) -> dict:
        """Analytic speed-of-light of one training step per rank (weak scaling,
        ideal table balance), from measured-achievable MI355X rates
        (MI355X_MICROARCH.md: HBM 6.3 TB/s float4 copy; bf16 MFMA GEMMs
        ~1.5 PF under DVFS; xGMI 153 GB/s per link, 7 links).

        compute = dense FLOPs / mfma_flops + HBM bytes / hbm_bw, where the HBM
        bytes are the irreducible ones: fp32 rows gathered (fwd) and
        read+written (bwd update, + 8 B of row-wise optimizer state), bf16
        pooled rows written/read, the interaction input/outputs, and the
        fused AdamW pass (p, g, m, v read; p, m, v, bf16 shadow written).
        comm (W > 1) = the pooled-embedding all-to-all bytes per peer (both
        directions) over one xGMI link + the ring all-reduce of the dense
        grads; it can overlap compute, so sol = max(compute, comm)."""
        B, T, D = batch, self.num_tables, self.embedding_dim
        F = T + 1
        L = self.pooling_factors()
        nnz = B * sum(L)
        emb = nnz * D * 4 + B * T * D * 2                    # fwd gather + pooled out
        emb += nnz * D * 2 + nnz * (D * 8 + 8) + nnz * 16    # bwd grads, row rw + state, ids/keys
        if self.interaction == "dot":
            inter = 2 * (B * F * D * 2) + 2 * B * (D + F * (F - 1) // 2) * 2
        else:
            inter = 4 * B * F * D * 2 * self.dcn_layers
        P = self.dense_params()
        opt = P * 4 * 4 + P * (4 * 3 + 2)
        flops = self.dense_flops_per_example() * B
        t_dense = flops / mfma_flops
        t_hbm = (emb + inter + opt) / hbm_bw
        compute = t_dense + t_hbm
        comm = 0.0
        if world > 1:
            per_peer = B * T * D * 2 / world                  # pooled rows to one peer, one way
            comm = 2 * per_peer / link_bw + 2 * (world - 1) / world * P * 4 / (7 * link_bw)
        return {"sol_ms": max(compute, comm) * 1e3, "dense_ms": t_dense * 1e3,
                "hbm_ms": t_hbm * 1e3, "comm_ms": comm * 1e3, "dense_gflop": flops / 1e9,
                "hbm_mb": (emb + inter + opt) / 1e6}


@dataclass
class Lin:
    """A linear layer in the augmented layout: W is stored [out, wcols] with
    the bias in column ``bcol``; the layer's input buffer holds 1.0 in column
    ``bcol``. If ``bcol < in_k`` the bias rides inside the forward GEMM's K
    (free), otherwise it is read by the epilogue. Either way the weight-grad
    GEMM over the augmented input produces the bias gradient in column
    ``bcol`` — no separate bias-reduction kernels."""
    name: str
    in_real: int
    in_k: int
    out: int
    bcol: int
    wcols: int

    @property
    def bias_in_k(self) -> bool:
        return self.bcol < self.in_k


# Row pitch added past in_k when the bias column cannot ride in the K padding:
# 64 elements keeps every activation / weight row 128-B aligned, so each 128-B
# K chunk a GEMM stages is one cache line (an 8-element pad made 7 of 8 rows
# straddle two lines: top1 fwd 28.2 vs 23.5 us, profiles/gemm_step_ab.md).
WCOL_PAD = 64


def make_lin(name: str, in_real: int, out: int) -> Lin:
    in_k = pad64(in_real)
    if in_real < in_k:
        return Lin(name, in_real, in_k, out, in_real, in_k)
    return Lin(name, in_real, in_k, out, in_k, in_k + WCOL_PAD)




class DLRMTrainer(StreamGraphsMixin, MultiRankStreamsMixin, DCNMixin):
    """Explicit-step DLRM/DCN-v2 trainer over a sharded embedding engine.

    ``batch_size`` is per rank (weak scaling). Works on CPU (torch reference
    ops, gloo) and on MI355X (HIP kernels, RCCL). The step is a fixed list of
    compute stages and communication stages (``_stages``); it runs eagerly,
    or captured: one process as per-stream hipGraphs (dlrm_streams.py) or one
    whole-step graph, several processes as one graph per run of compute
    stages with the RCCL exchanges issued eagerly between replays.
    """

    def __init__(self, cfg: DLRMConfig, batch_size: int, device, group=None, rank: int = 0,
                 world_size: int = 1, plan: Optional[ShardingPlan] = None):
        self.cfg = cfg
        if cfg.dense_comm not in ("fp32", "bf16"):
            raise ValueError(f"dense_comm must be fp32 or bf16, got {cfg.dense_comm!r}")
        if cfg.opt_placement not in (None, "one_pass", "split_main"):
            raise ValueError(f"opt_placement must be one_pass or split_main, "
                             f"got {cfg.opt_placement!r}")
        if cfg.opt_placement is None:
            cfg.opt_placement = "split_main" if cfg.interaction == "dcn" else "one_pass"
        self.B = B = int(batch_size)
        self.device = dev = torch.device(device)
        self.group = group
        self.comm = as_comm(group) if world_size > 1 else None
        # the dense-gradient all-reduces get a communicator of their own where
        # collectives are stream-ordered (native RCCL, loopback), so they run
        # beside the embedding exchanges (dlrm_multirank.py)
        self.dcomm = dense_comm_for(self.comm) if world_size > 1 else None
        self.rank = rank
        self.world = world_size
        D = cfg.embedding_dim
        T = cfg.num_tables
        self.F = F = T + 1
        assert cfg.bottom[-1] == D, "bottom MLP must end at the embedding dim"
        assert cfg.top[-1] == 1
        assert cfg.interaction != "dcn" or cfg.dcn_rank % 64 == 0, "dcn_rank must be a multiple of 64"
        torch.manual_seed(cfg.seed)
        # ------------------------------------------------------ embeddings
        optim = EmbOptimConfig(cfg.emb_opt, lr=cfg.emb_lr, eps=cfg.emb_eps)
        tables = cfg.tables()
        self.plan = plan or plan_sharding(tables, world_size, optim, batch_per_rank=B,
                                          pooling=cfg.pooling_factors(), strategy=cfg.sharding,
                                          dp_rule=cfg.dp_rule)
        self.emb = ShardedEmbeddingBags(tables, self.plan, rank, B, cfg.pooling_factors(), dev,
                                        optim, group=self.comm, seed=cfg.seed,
                                        rw_capacity=cfg.rw_capacity, rw_comm=cfg.rw_comm,
                                        rw_exchange=cfg.rw_exchange)
        if self.dcomm is not None:
            self.emb.dp_comm = self.dcomm         # replicated tables' all-reduce beside it
        # ------------------------------------------------------ dense params
        fp = FlatParams()
        dims = [cfg.num_dense] + cfg.bottom
        self.bottom_layers = [make_lin(f"bot{i}", a, b)
                              for i, (a, b) in enumerate(zip(dims[:-1], dims[1:]))]
        if cfg.interaction == "dot":
            self.top_real = D + F * (F - 1) // 2
        else:
            self.top_real = F * D
        tdims = [self.top_real] + cfg.top[:-1]
        self.top_layers = [make_lin(f"top{i}", a, b)
                           for i, (a, b) in enumerate(zip(tdims[:-1], tdims[1:]))]
        for L in self.bottom_layers + self.top_layers:
            fp.add(L.name + ".w", (L.out, L.wcols))
        self.dcn_u = []
        if cfg.interaction == "dcn":
            Wd = self.top_real
            for i in range(cfg.dcn_layers):
                fp.add(f"dcn{i}.v", (cfg.dcn_rank, Wd))
                u = make_lin(f"dcn{i}.u", cfg.dcn_rank, Wd)
                self.dcn_u.append(u)
                fp.add(u.name + ".w", (u.out, u.wcols))
        self.head_k = tdims[-1]
        fp.add("head", (self.head_k + 1,))           # [w (K) | b]
        opt = DENSE_OPTS[cfg.dense_opt]
        self.dense_opt = opt
        fp.finalize(dev, with_adam=opt in (ops.OPT_ADAMW, ops.OPT_ADAM))
        self.fp = fp
        # gradient buckets: flat layout is [bottom MLP | top MLP, DCN, head]
        self._ar_split = fp.offset(self.top_layers[0].name + ".w")
        self._init_dense()
        if world_size > 1:                            # replicated dense arch
            self.comm.broadcast(fp.p, src=0)
        fp.sync_bf16()
        self._defer_top_wgrad = (world_size > 1 if cfg.defer_wgrad is None
                                 else bool(cfg.defer_wgrad))
        # ------------------------------------------------------ buffers
        bf = torch.bfloat16

        def z(*shape, dt=bf):
            return torch.zeros(*shape, dtype=dt, device=dev)

        def act_in(L: Lin):
            t = z(B, L.wcols)
            t[:, L.bcol] = 1.0
            return t

        # input buffer of every layer (augmented), output of the last bottom
        # layer / last top layer are plain
        self.x0 = act_in(self.bottom_layers[0])
        self.bot_in = [self.x0] + [act_in(L) for L in self.bottom_layers[1:]]
        self.h_out = z(B, D)
        # the default bottom stack forward as one fused launch (GPU; bitwise
        # the per-layer GEMMs; TDFO_FUSED_BOTTOM=0 keeps those)
        Lb = self.bottom_layers
        self._fused_bottom = (
            dev.type == "cuda" and len(Lb) == 3 and D == Lb[2].out
            and os.environ.get("TDFO_FUSED_BOTTOM", "1") != "0"
            and Lb[0].in_k == Lb[0].wcols and not Lb[1].bias_in_k and not Lb[2].bias_in_k
            and Lb[1].in_k == Lb[0].out and Lb[2].in_k == Lb[1].out
            and ops.bottom_mlp_fwd_ok(Lb[0].in_k, Lb[0].out, Lb[1].out, Lb[2].out))
        # ... which also loads a staged batch's dense features / labels (one
        # launch fewer on the MLP stream; TDFO_BOT_LOAD_FOLD=0: batch_load)
        self._bot_load_fold = os.environ.get("TDFO_BOT_LOAD_FOLD", "1") != "0"
        # the head's reduce (grad, loss, step counters) in extra blocks of the
        # first top backward GEMM pair (TDFO_HEAD_SIDE=0: its own launch)
        self._head_side = os.environ.get("TDFO_HEAD_SIDE", "1") != "0"
        self.bot_grad = [z(B, L.out) for L in self.bottom_layers]
        self.top_in = [act_in(L) for L in self.top_layers]
        self.t_out = z(B, self.head_k)
        self.top_grad = [z(B, L.out) for L in self.top_layers]
        self.dz = z(B, self.top_layers[0].in_k)
        self.label = z(B, dt=torch.float32)
        self.ids = torch.zeros(self.emb.nnz_local, dtype=torch.int64, device=dev)
        self.emb.bind_ids(self.ids)
        if cfg.interaction == "dcn":
            Lc, Wd, r = cfg.dcn_layers, self.top_real, cfg.dcn_rank
            # x_0 .. x_{L-1} plain; x_L is top0's (augmented) input buffer
            self.dcn_x = [z(B, Wd) for _ in range(Lc)] + [self.top_in[0]]
            self.dcn_h = [act_in(u) for u in self.dcn_u]      # V^T x_l (+ ones col)
            self.dcn_y = [z(B, Wd) for _ in range(Lc)]         # U h + b
            self.dcn_dx = [z(B, Wd) for _ in range(Lc + 1)]
            self.dcn_dx0acc = z(B, Wd)
            # dy = dx_{l+1} * x0 and dh = dy U of each layer: the wgrads'
            # inputs (one buffer per layer when those are deferred)
            nb = Lc if self._defer_top_wgrad else 1
            self.dcn_dhl = [z(B, r) for _ in range(nb)]
            self.dcn_dyl = [z(B, Wd) for _ in range(nb)]
        # DCN-v2, one rank: the lookup pools straight into x_0's embedding
        # columns and the bottom MLP writes its output into x_0's dense slot;
        # the embedding backward reads its gradients in place from dx_0 (no
        # concat / split of the 3456-wide rows: 46 + 20 us per step). Not with
        # deferred wgrads: layer 0's V wgrad would read x_0 while the next
        # step's early lookup rewrites it.
        self._x0_alias = False
        if (cfg.interaction == "dcn" and not self._defer_top_wgrad
                and self.emb.alias_pooled(self.dcn_x[0], self.dcn_dx[0], D)):
            self._x0_alias = True
            self.h_out = self.dcn_x[0][:, :D]
        self.logits = z(B, dt=torch.float32)
        self.nparts = ops.head_parts(B)
        self.head_part = z(self.nparts * (self.head_k + 2), dt=torch.float32)
        self.loss_sum = z(1, dt=torch.float32)
        # Weight grads: split-K over the batch into ~256 blocks (each paired
        # with its layer's dgrad in one ping-pong launch: 0.477 vs 0.504 ms/step
        # at 512 unpaired); the bias gradient comes from the same GEMM's column
        # sums of dy (N stays the 64-aligned input width). Each layer's
        # partials get their own zero-initialised slab [S][out][wcols]: one
        # process sums them inside the fused optimizer pass (no reduce launch
        # per layer); with >1 rank they are reduced first because the
        # all-reduce needs the grads.
        self._pair_bwd = dev.type == "cuda"
        dcn = cfg.interaction == "dcn"
        if dev.type == "cuda" and not os.environ.get("TDFO_GEMM_POLICY"):
            # GEMM tile policy per workload: DCN-v2's 3456-wide cross / top
            # GEMMs on 256x128 tiles, paired wgrad + dgrad on that kernel
            # (2.42 vs 2.51-2.52 ms/step on the 128x128 ping-pong dispatch,
            # same box, profiles/r03/s3/dcn_policy.md); DLRM's <= 1024-wide
            # MLPs on the ping-pong / 64-row kernels
            ops.gemm_policy(5 if dcn else 0)
        # the tile policy is process-global in the native library: each
        # trainer re-applies its own before it issues or captures GEMMs, so
        # trainers of different models can share a process
        self._gemm_pol = ops.gemm_policy(-1) if dev.type == "cuda" else None
        # DCN-v2 on 256x128 tiles: bias grads from the ones column inside the
        # wgrad's N (that kernel has no column-sum epilogue), splits sized for
        # its resident blocks (half of them beside the paired dgrad)
        self._csum = not (dcn and dev.type == "cuda" and ops.gemm_policy(-1) in (4, 5))
        self._wg_slots = (128 if self._pair_bwd else 256) if not self._csum else 0
        self.wslab = {}
        self._slab_sums = []          # (flat offset, slab, S, grad view) summed by _reduce_slabs
        self._segments = []
        self._opt_sums_slabs = dev.type == "cuda" and world_size == 1
        max_slab = 1
        if cfg.interaction == "dcn":
            max_slab = self._wg_splits(cfg.dcn_rank, self.top_real) * cfg.dcn_rank * self.top_real
        self.slab = z(max_slab, dt=torch.float32)
        for L in self.bottom_layers + self.top_layers + self.dcn_u:
            S = self._wg_splits(L.out, self._wgrad_n(L))
            if S > 1:
                sl = z(S * L.out * L.wcols, dt=torch.float32)
                self.wslab[L.name] = (sl, S)
                if self._opt_sums_slabs:
                    self._segments.append((fp.offset(L.name + ".w"), sl, S))
                else:
                    self._slab_sums.append((fp.offset(L.name + ".w"), sl, S,
                                            fp.grad(L.name + ".w").view(-1)))
        # DCN-v2 V weight grads: same treatment (per-layer slabs also with
        # more than one rank, where their sums are batched per bucket)
        if cfg.interaction == "dcn" and dev.type == "cuda":
            for i in range(cfg.dcn_layers):
                S = self._wg_splits(cfg.dcn_rank, self.top_real)
                if S > 1:
                    sl = z(S * cfg.dcn_rank * self.top_real, dt=torch.float32)
                    self.wslab[f"dcn{i}.v"] = (sl, S)
                    if self._opt_sums_slabs:
                        self._segments.append((fp.offset(f"dcn{i}.v"), sl, S))
                    else:
                        self._slab_sums.append((fp.offset(f"dcn{i}.v"), sl, S,
                                                fp.grad(f"dcn{i}.v").view(-1)))
        self.dense_hyper = torch.tensor([cfg.dense_lr, 0.0, 1.0], dtype=torch.float32, device=dev)
        self.emb_hyper = torch.tensor([cfg.emb_lr, 0.0], dtype=torch.float32, device=dev)
        self.slot_off = [0] + list(self.emb.slot_off)
        self.slot_stride = [0] + list(self.emb.slot_stride)
        self.graph = None
        self.steps = 0
        # ids-only half of the embedding backward (keys + sort) on its own
        # stream beside the top MLP: it needs no gradient, and its few
        # latency-bound blocks leave the GEMMs most of the machine
        self._ps = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        # input-dist pipelining (the role of TorchRec's TrainPipelineSparseDist
        # behind the reference's DMP, torchrec/train.py:241-247): batch i+1's
        # ids are bucketed and exchanged right after batch i's embedding
        # update -- the last reader of the exchanged-id buffers -- so the
        # exchange overlaps batch i's dense optimizer step and batch i+1
        # starts at its lookup. Numerics are identical to the unpipelined step.
        self.pipeline = bool(cfg.pipeline) and world_size > 1
        self._pipe_lookup = self.pipeline and bool(cfg.pipeline_lookup)
        # pipelined row-wise exchanges check their capacity one step late
        # (ShardedEmbeddingBags.rw_publish_need / rw_resolve_need): no host
        # read inside the step, so the row-wise plans (configs 3 and 5) run on
        # the per-stream graphs too
        self._rw_lagged = self.pipeline and bool(self.emb.rw_tables) and self.emb.rw_dynamic
        on_cuda = dev.type == "cuda"
        self._ev_loaded = torch.cuda.Event() if (on_cuda and self._pipe_lookup) else None
        self._ev_lookup = torch.cuda.Event() if (on_cuda and self._pipe_lookup) else None
        self._next = None
        self._primed = False
        self._mstream = False            # per-stream graphs (one process)
        self._bstg = None                # staged dense / labels (per-stream graphs)
        self._ms = None
        self._whole_capture = False      # capturing the multi-rank stream graphs
        self._cap_origin = None          # origin of a multi-stream capture (see _wait)
        self._stg = None                 # multi-rank graphs: next-batch staging buffers
        self._mr = None
        self._graph_layout = 0
        self._insrc = None               # in-step batch generator (attach_in_step_source)
        self._src_copy_stream = None     # the batch producer's stream (set_copy_stream)
        self._src_copy_owner = None

    # for tests / checkpoints: (weight [out, in_real], bias [out]) views
    def weight(self, name: str):
        L = next(L for L in self.bottom_layers + self.top_layers + self.dcn_u if L.name == name)
        W = self.fp.param(name + ".w")
        return W[:, :L.in_real], W[:, L.bcol]

    # --------------------------------------------------------------- init
    def _init_dense(self):
        g = torch.Generator(device="cpu")
        g.manual_seed(self.cfg.seed + 7)
        fp = self.fp
        for L in self.bottom_layers + self.top_layers + self.dcn_u:
            W = fp.param(L.name + ".w")
            W.zero_()
            w = torch.randn(L.out, L.in_real, generator=g) * math.sqrt(2.0 / (L.in_real + L.out))
            W[:, :L.in_real] = w.to(W.device)
            if not L.name.startswith("dcn"):
                W[:, L.bcol] = (torch.randn(L.out, generator=g) * math.sqrt(1.0 / L.out)).to(W.device)
        if self.cfg.interaction == "dcn":
            r, w = self.cfg.dcn_rank, self.top_real
            for i in range(self.cfg.dcn_layers):
                fp.param(f"dcn{i}.v").copy_(torch.randn(r, w, generator=g) * math.sqrt(2.0 / (r + w)))
        K = self.head_k
        h = fp.param("head")
        h[:K] = (torch.randn(K, generator=g) * math.sqrt(2.0 / (K + 1))).to(h.device)
        h[K] = 0.0

    # ------------------------------------------------------------ batches
    def load_batch(self, dense: torch.Tensor, ids: torch.Tensor, label: torch.Tensor,
                   on_device: bool = False):
        """Copy a batch into the static input buffers (non_blocking H2D ok).

        dense [B, num_dense] (any float dtype), ids flat int64 in table order
        (table t: B*L_t ids), label [B] float. on_device: the tensors are
        device-resident and ready for every stream (``input_streams()``);
        with per-stream graphs the ids are then copied on the embedding side
        right behind the previous step's embedding update, so the next lookup
        overlaps the previous step's bottom-MLP backward.
        """
        if self.graph == "streams":
            stg = self._bstg
            if self._ms_load_ids(ids, on_device, dense, label):
                if stg is None:
                    ops.batch_load(dense, self.x0, ids[:0], self.ids[:0], label, self.label)
                elif not on_device:              # (staged graphs: M1 loads from the staging)
                    stg[0].copy_(dense, non_blocking=True)
                    stg[1].copy_(label.reshape(-1), non_blocking=True)
                return
            if stg is not None:
                stg[0].copy_(dense, non_blocking=True)
                stg[1].copy_(label.reshape(-1), non_blocking=True)
                self.ids.copy_(ids)
                return
        # device-resident batch: one fused launch (ids, labels, dense -> bf16)
        ops.batch_load(dense, self.x0, ids, self.ids, label, self.label)

    def set_copy_stream(self, stream, owner=None):
        """One GPU, per-stream graphs: copy each batch's ids into the static
        buffer on ``stream`` -- the device batch producer's own stream, on a
        hardware queue the embedding stream does not share -- right behind the
        previous step's ids-only sort, instead of on the embedding stream
        between the previous step's update and the next lookup (where the
        copy and its waits idled that stream ~34 us per step). Set before
        capture_graph()."""
        if self.graph is not None:
            raise RuntimeError("set the copy stream before capture_graph()")
        self._src_copy_stream = stream
        # batches of any other producer are copied on the embedding stream
        # behind the MLP stream (which waited for them)
        self._src_copy_owner = owner

    def attach_in_step_source(self, src):
        """One GPU: every step draws its own batch inside its graphs
        (``data.synthetic.InStepSynthetic``): the ids on the embedding
        stream right before the lookup, dense features / labels on the MLP
        stream at the start of the bottom forward, the batch index read from
        the step counter on the device. Attach before capturing graphs."""
        if self.world != 1 or self.pipeline:
            raise ValueError("in-step batch generation is for the one-GPU step")
        if self.graph is not None:
            raise RuntimeError("attach the in-step source before capture_graph()")
        self._insrc = src
        src.bind(self.dense_hyper[1:2])

    def _s_gen_ids(self):
        if self._insrc is not None:
            self._insrc.gen_ids(self.ids)

    def _s_gen_dense(self):
        if self._insrc is not None:
            self._insrc.gen_dense(self.x0, self.label)

    # ------------------------------------------------- pipelined input dist
    def prime(self, dense: torch.Tensor, ids: torch.Tensor, label: torch.Tensor):
        """Pipelined mode: load the first batch and start its id exchange.
        Then per step: ``set_next_batch(next batch); step()`` -- the step
        consumes the batch loaded before it and loads / exchanges the next."""
        assert self.pipeline, "prime() needs DLRMConfig(pipeline=True) and world_size > 1"
        self.load_batch(dense, ids, label)
        self.emb._rw_lag_pending = False       # (this exchange checks its capacity itself)
        if not self.emb.fwd_prep_noop:
            self.emb.stage_fwd_prep(self.ids)
        self.emb.stage_fwd_ids_exchange(async_op=True)
        if self._pipe_lookup:                # its lookup + pooled exchange too
            self.emb.ids_exchange_wait()
            self.emb.stage_fwd_lookup()
            self._m_out_exchange_next()
        self._next = (dense, ids, label)
        self._primed = True
        self._mr_inflight = True

    def set_next_batch(self, dense: torch.Tensor, ids: torch.Tensor, label: torch.Tensor):
        """Pipelined mode: the batch the current step loads for the next one
        (device tensors that stay valid until the step has been issued).
        Whole-step graph: copied now into the static staging buffers the
        graph's tail loads from (one launch; the previous replay, the last
        reader of the staging, precedes it on this stream)."""
        if self.graph == "mstreams":
            self._mr_stage_next(dense, ids, label)
            return
        self._next = (dense, ids, label)

    def _m_load_next(self):
        if self._whole_capture:
            sx, si, sl = self._stg
            self.x0.copy_(sx)
            self.ids.copy_(si)
            self.label.copy_(sl)
            return
        dense, ids, label = self._next
        ops.batch_load(dense, self.x0, ids, self.ids, label, self.label)

    def _m_ids_exchange_next(self):
        self.emb.stage_fwd_ids_exchange(async_op=True, lagged=self._rw_lagged)

    def _rw_resolve(self):
        """Lagged row-wise capacity check of the batch the coming step
        consumes (exchanged in the previous step's tail): on growth its
        row-wise exchange is redone into the larger segments here, every
        stream idle, and the graphs are re-captured (layout_version)."""
        if self._rw_lagged and self.emb.rw_resolve_need():
            self.sync_streams()
            self.emb.rw_redo()

    # ------------------------------------------------------------- layers
    def _fwd(self, L: Lin, x, out, relu=True):
        W = self.fp.bf16(L.name + ".w")
        bias = None if L.bias_in_k else self.fp.param(L.name + ".w")[:, L.bcol]
        ops.gemm(x[:, :L.in_k], False, W[:, :L.in_k], False, bias, relu, None, out, None, 1)

    def _bwd(self, L: Lin, x, dy, dx, x_is_relu, wgrad_now: bool = True):
        """weight+bias grad (augmented wgrad) and dgrad into dx (masked by x>0).
        wgrad_now=False leaves the weight grad to a later `_wgrad` call."""
        if not wgrad_now:
            self._dgrad(L, x, dy, dx, x_is_relu)
            return
        # the weight grad and the dgrad go out as one paired launch (the slab
        # sum of more than one rank is batched per all-reduce bucket)
        with ops.gemm_batch(self._pair_bwd and dx is not None):
            self._wgrad_gemm(L, x, dy)
            self._dgrad(L, x, dy, dx, x_is_relu)

    def _wg_splits(self, M: int, N: int) -> int:
        return ops.wgrad_splits(M, N, self.B, 256, slots=self._wg_slots)

    def _wgrad_n(self, L: Lin) -> int:
        return L.in_k if self._csum else L.wcols

    def _wgrad(self, L: Lin, x, dy):
        """dW[:, :in_k] = dy^T x[:, :in_k]; db (column bcol) = colsum(dy) from
        the same GEMM when the bias is not inside K."""
        self._wgrad_gemm(L, x, dy)

    def _wgrad_gemm(self, L: Lin, x, dy):
        """The weight-grad GEMM alone. Its split-K slabs are summed by the
        fused optimizer on one GPU; with more than one rank the all-reduce
        needs the grads, so the slabs of every layer of an all-reduce bucket
        are summed in ONE launch right before that all-reduce
        (``_reduce_slabs``)."""
        csum = -1 if (L.bias_in_k or not self._csum) else L.bcol
        n = self._wgrad_n(L)
        g = self.fp.grad(L.name + ".w").view(-1)
        if L.name in self.wslab:
            sl, S = self.wslab[L.name]
            ops.gemm(dy, True, x[:, :n], True, None, False, None, None, sl, S,
                     ldc32=L.wcols, csum_col=csum)
        else:
            ops.gemm(dy, True, x[:, :n], True, None, False, None, None, g, 1,
                     ldc32=L.wcols, csum_col=csum)
        return None

    def _dgrad(self, L: Lin, x, dy, dx, x_is_relu):
        if dx is not None:
            # dgrad only over the columns dx holds (the padded K tail of the
            # augmented layout, bias column included, has no gradient consumer)
            n = min(dx.shape[1], L.in_k)
            W = self.fp.bf16(L.name + ".w")
            ops.gemm(dy, False, W[:, :n], True, None, False,
                     x[:, :n] if x_is_relu else None, dx[:, :n], None, 1)

    # ---------------------------------------------------------- stages
    # The step is a fixed sequence of compute stages ("c": main stream, "e":
    # side stream; hipGraph-capturable) and communication stages ("m" / "em":
    # RCCL collectives issued eagerly on the main / side stream, so they
    # overlap the next compute stage); "j" joins the side stream back, "jw"
    # waits only for the next batch's load on it.
    def _stages(self):
        emb = self.emb
        top_wgrad = [("c", self._s_top_wgrad)] if self._defer_top_wgrad else []
        prep = [] if emb.fwd_prep_noop else [("c", lambda: emb.stage_fwd_prep(self.ids))]
        if self.pipeline:
            # this batch's ids were exchanged during the previous step (or by
            # prime()); on the side stream the embedding update and the next
            # batch's load, bucketize and id exchange run beside the
            # dense-gradient all-reduce wait and the dense optimizer step
            eprep = [("e", k[1]) for k in prep]
            if self._pipe_lookup:
                # ... and the next batch's lookup + pooled-embedding exchange
                # follow on the side stream in this step's tail (after the
                # embedding update they must see), so the next step starts
                # at its bottom MLP with its pooled embeddings in flight or
                # landed; the main stream only waits for the next batch's
                # dense inputs ("jw")
                return [
                    ("c", self._s_bottom_fwd),
                    ("m", self._m_fwd_wait),
                    ("c", self._s_top),
                    ("m", emb.backward_start),
                ] + top_wgrad + [
                    ("m", self._m_allreduce_top_start),
                    ("c", self._s_bottom_bwd),
                    ("m", self._m_allreduce_start),
                    ("m", emb.backward_wait),
                    ("e", self._s_emb_update),
                    ("em", self._m_load_next),
                    ("em", self._m_mark_loaded),
                ] + eprep + [
                    ("em", self._m_ids_exchange_next),
                    ("em", emb.ids_exchange_wait),
                    ("e", emb.stage_fwd_lookup),
                    ("em", self._m_out_exchange_next),
                    ("m", self._m_allreduce_wait),
                    ("c", self._s_dense_update),
                    ("jw", None),
                ]
            return [
                ("m", emb.ids_exchange_wait),
                ("c", emb.stage_fwd_lookup),
                ("m", emb.stage_fwd_out_exchange),
                ("c", self._s_bottom_fwd),
                ("m", self._m_fwd_wait),
                ("c", self._s_top),
                ("m", emb.backward_start),
            ] + top_wgrad + [
                ("m", self._m_allreduce_top_start),
                ("c", self._s_bottom_bwd),
                ("m", self._m_allreduce_start),
                ("m", emb.backward_wait),
                ("e", self._s_emb_update),
                ("em", self._m_load_next),
            ] + eprep + [
                ("em", self._m_ids_exchange_next),
                ("m", self._m_allreduce_wait),
                ("c", self._s_dense_update),
                ("j", None),
            ]
        gen = [("c", lambda: (self._s_gen_ids(), self._s_gen_dense()))] if self._insrc else []
        return gen + prep + [
            ("m", emb.stage_fwd_ids_exchange),
            ("c", emb.stage_fwd_lookup),
            ("m", emb.stage_fwd_out_exchange),
            ("c", self._s_bottom_fwd),
            ("m", self._m_fwd_wait),
            ("c", self._s_top),
            ("m", emb.backward_start),
        ] + top_wgrad + [                       # (overlaps the embedding-grad exchange)
            ("m", self._m_allreduce_top_start),  # top bucket || bottom bwd + embedding update
            ("c", self._s_bottom_bwd),
            ("m", self._m_allreduce_start),      # bottom bucket
            ("m", emb.backward_wait),
            ("e", self._s_emb_update),           # beside the all-reduce wait + dense step
            ("m", self._m_allreduce_wait),
            ("c", self._s_dense_update),
            ("j", None),
        ]

    def _wait(self, dst, src):
        """``dst`` waits for the work issued on ``src``. Inside a capture
        that names its origin (``_cap_origin``), a wait between two
        non-origin streams is routed through the origin (origin waits
        ``src``, ``dst`` waits origin): hipStreamEndCapture segfaults on this
        ROCm when a stream forked into a capture is itself the source of
        another fork (labs/probes/rccl_capture_probe.py, nested_* modes)."""
        o = self._cap_origin
        if o is None or dst == o or src == o:
            dst.wait_stream(src)
        else:
            o.wait_stream(src)
            dst.wait_stream(o)

    # side stream of the multi-process stage lists ("e" / "em" / "j" stages)
    def _side(self):
        if self.device.type != "cuda" or self.world == 1:
            return None
        if getattr(self, "_sides", None) is None:
            self._sides = torch.cuda.Stream(device=self.device)
        return self._sides

    def _run_stage(self, kind, fn, graph=None):
        """Run (or replay) one stage on its stream; forks the side stream off
        the current stream at the first side stage after main-stream work."""
        se = self._side()
        if kind == "j":
            if se is not None:
                self._wait(torch.cuda.current_stream(), se)
            self._on_side = False
            return
        if kind == "jw":                     # main waits for the next batch's load only
            if se is not None and self._ev_loaded is not None:
                torch.cuda.current_stream().wait_event(self._ev_loaded)
            self._on_side = False
            return
        if kind in ("e", "em") and se is not None:
            if not getattr(self, "_on_side", False):
                self._wait(se, torch.cuda.current_stream())
                self._on_side = True
            with torch.cuda.stream(se):
                graph.replay() if graph is not None else fn()
            return
        graph.replay() if graph is not None else fn()

    def _forward_backward(self):
        self._on_side = False
        for kind, fn in self._stages():
            self._run_stage(kind, fn)

    def _s_bottom_fwd(self, staged=None):
        """``staged`` (fused stack only): the (dense fp32, label) staging of
        this step's batch, loaded by the bottom-MLP launch itself."""
        if self._fused_bottom:
            # the default 3-layer stack in one launch (csrc/kernels/mlp_fused.hip)
            Ls = self.bottom_layers
            bias = [None if L.bias_in_k else self.fp.param(L.name + ".w")[:, L.bcol] for L in Ls]
            ops.bottom_mlp_fwd(self.bot_in[0], self.fp.bf16(Ls[0].name + ".w"),
                               self.fp.bf16(Ls[1].name + ".w"), self.fp.bf16(Ls[2].name + ".w"),
                               bias[0], bias[1], bias[2], self.bot_in[1], self.bot_in[2],
                               self.h_out, dense=None if staged is None else staged[0],
                               label=None if staged is None else (staged[1], self.label))
            return
        n = len(self.bottom_layers)
        for i, L in enumerate(self.bottom_layers):
            out = self.bot_in[i + 1][:, :L.out] if i + 1 < n else self.h_out
            self._fwd(L, self.bot_in[i], out)

    def _m_fwd_wait(self):
        if self._whole_capture:
            # the previous replay completed this batch's exchanges (a graph
            # ends joined); only the post-exchange assembly runs here
            self.emb.forward_wait()
            return
        if self._pipe_lookup and self._ev_lookup is not None and self._side() is not None:
            # the lookup ran on the side stream in the previous step's tail
            # (tables it wrote straight into recv have no collective to wait on)
            torch.cuda.current_stream().wait_event(self._ev_lookup)
        self.emb.forward_wait()

    def _m_mark_loaded(self):
        if self._ev_loaded is not None and not self._whole_capture:
            self._ev_loaded.record(torch.cuda.current_stream())

    def _m_out_exchange_next(self):
        self.emb.stage_fwd_out_exchange()
        if self._ev_lookup is not None and not self._whole_capture:
            self._ev_lookup.record(torch.cuda.current_stream())

    def _s_top(self):
        self._s_top_a()
        self._s_top_b()

    def _s_top_a(self):
        """Interaction / cross forward, top MLP forward + backward (all top
        weight grads exist after it)."""
        cfg, fp, B = self.cfg, self.fp, self.B
        D, F = cfg.embedding_dim, self.F
        emb = self.emb
        if self._ps is not None and not self._mstream:
            self._wait(self._ps, torch.cuda.current_stream())
            with torch.cuda.stream(self._ps):
                emb.stage_bwd_prepare()
        h = self.h_out
        L0 = self.top_layers[0]
        if cfg.interaction == "dot":
            ops.interaction_fwd(h, emb.recv, self.slot_off, self.slot_stride, F, D, self.top_in[0],
                                L0.bcol)
        else:
            self._dcn_forward(h)
        n = len(self.top_layers)
        for i, L in enumerate(self.top_layers):
            out = self.top_in[i + 1][:, :L.out] if i + 1 < n else self.t_out
            self._fwd(L, self.top_in[i], out)
        K = self.head_k
        head = fp.param("head")
        ops.head_bce(self.t_out, head[:K], head[K:], self.label, 1.0 / (B * self.world), True,
                     self.logits, self.top_grad[-1], self.head_part)
        # head grad + loss accumulation + this step's optimizer step counters
        # (read later in the step by the embedding and dense updates): one launch
        # (deferred: the first top backward GEMM pair runs it in extra blocks)
        defer = self._head_side and self.device.type == "cuda"
        ops.head_reduce(self.head_part, self.nparts, K, fp.grad("head"), self.loss_sum,
                        (self.dense_hyper, self.emb_hyper), defer=defer)
        for i in reversed(range(n)):
            L = self.top_layers[i]
            if i > 0:
                dx = self.top_grad[i - 1]
            else:
                dx = self.dz if cfg.interaction == "dot" else self.dcn_dx[-1]
            self._bwd(L, self.top_in[i], self.top_grad[i], dx, x_is_relu=i > 0,
                      wgrad_now=not self._defer_top_wgrad)
            if defer:
                ops.flush_side_job()         # (no-op once a GEMM pair took it)

    def _s_top_b(self):
        """Interaction / cross backward: the embedding gradients."""
        cfg = self.cfg
        D, F = cfg.embedding_dim, self.F
        emb = self.emb
        h = self.h_out
        if cfg.interaction == "dot":
            ops.interaction_bwd(self.dz, h, emb.recv, self.slot_off, self.slot_stride, F, D,
                                self.bot_grad[-1], emb.d_recv, self.slot_off, self.slot_stride,
                                True)
        else:
            self._dcn_backward(h)
        if not self._whole_capture:                # (multi-rank graphs: an EC segment)
            emb.stage_bwd_local(self.emb_hyper)    # replicated tables' dense grads
        if not self._mstream and self._ps is not None:
            self._wait(torch.cuda.current_stream(), self._ps)

    def _s_top_wgrad(self):
        """Top-MLP (and DCN cross-layer) weight grads, deferred past the
        interaction / cross backward: the embedding grads exist without them
        (their all-to-all, or on one GPU the embedding update, runs meanwhile)."""
        if self._defer_top_wgrad:
            # independent GEMMs: issued in pairs
            with ops.gemm_batch(self._pair_bwd):
                for i in reversed(range(len(self.top_layers))):
                    self._wgrad_gemm(self.top_layers[i], self.top_in[i], self.top_grad[i])
                for i in reversed(range(len(self.dcn_u))):
                    dy, _ = self._dcn_bufs(i)
                    self._wgrad_gemm(self.dcn_u[i], self.dcn_h[i], dy)
            for i in reversed(range(len(self.dcn_u))):
                self._dcn_wgrad_v(i)

    def _s_bottom_bwd(self):
        for i in reversed(range(len(self.bottom_layers))):
            L = self.bottom_layers[i]
            dx = self.bot_grad[i - 1] if i > 0 else None
            self._bwd(L, self.bot_in[i], self.bot_grad[i], dx, x_is_relu=i > 0)

    # Dense gradients are all-reduced in two buckets of the flat buffer, each
    # issued as soon as its grads exist (the role of the DDP reducer,
    # torchrec/train.py:255-260 of the reference): the top MLP (+ head, DCN
    # cross layers) right after the top backward, overlapping the bottom MLP
    # backward and the embedding update; the small bottom MLP after its
    # backward.
    def _reduce_slabs(self, lo: int, hi: int):
        """Sum the split-K slabs of the weight grads in flat range [lo, hi)
        into ``fp.g`` (one launch for all of them; the layers are the same
        every step, so staged graphs and eager stages issue the same work)."""
        mine = [(sl, S, g) for off, sl, S, g in self._slab_sums if lo <= off < hi]
        if mine:
            ops.slab_reduce(mine)

    def _ar_issue(self, lo: int, hi: int):
        self._reduce_slabs(lo, hi)
        g = self.fp.g[lo:hi]
        if self.cfg.dense_comm == "bf16":
            if getattr(self, "_g16", None) is None:
                self._g16 = torch.empty(self.fp.g.numel(), dtype=torch.bfloat16,
                                        device=self.device)
            b = self._g16[lo:hi]
            ops.cast_bf16(g, b)
            return (self.dcomm.all_reduce(b, async_op=True), g, b)
        return (self.dcomm.all_reduce(g, async_op=True), None, None)

    def _m_allreduce_top_start(self):
        self._ar_top = None
        if self.world > 1:
            self._ar_top = self._ar_issue(self._ar_split, self.fp.g.numel())

    def _m_allreduce_start(self):
        self._ar_work = None
        if self.world > 1:
            self._ar_work = self._ar_issue(0, self._ar_split)

    def _s_emb_update(self):
        self.emb.stage_bwd_update(self.emb_hyper)

    def _m_allreduce_wait(self, names=("_ar_top", "_ar_work")):
        for name in names:
            w = getattr(self, name, None)
            if w is not None:
                work, g, b = w
                work.wait()
                if b is not None:                  # bf16 wire format -> fp32 grads
                    g.copy_(b)
                setattr(self, name, None)

    def _s_dense_update(self):
        if self.world == 1:
            self._reduce_slabs(0, self.fp.g.numel())
        fp = self.fp
        ops.dense_optimizer(fp.p, fp.g, fp.m, fp.v, fp.p_bf16, self.dense_opt, self.dense_hyper,
                            wd=self.cfg.dense_wd, segments=self._segments)

    def _dense_update_range(self, lo: int, hi: int):
        """The fused dense optimizer over flat elements [lo, hi) (the same
        elementwise update as _s_dense_update restricted to a range)."""
        fp = self.fp
        if self.world == 1:
            self._reduce_slabs(lo, hi)
        segs = [(st - lo, sl, S) for st, sl, S in self._segments if lo <= st < hi]
        sl = slice(lo, hi)
        ops.dense_optimizer(fp.p[sl], fp.g[sl], fp.m[sl] if fp.m is not None else None,
                            fp.v[sl] if fp.v is not None else None,
                            fp.p_bf16[sl] if fp.p_bf16 is not None else None, self.dense_opt,
                            self.dense_hyper, wd=self.cfg.dense_wd, segments=segs)

    # ------------------------------------------------------------- step
    def step(self):
        """One training step on the batch in the static buffers."""
        if self.pipeline and not self._primed:
            raise RuntimeError("pipelined trainer: call prime(first batch) before step()")
        self._rw_resolve()
        self._use_gemm_policy()
        if self.graph == "streams":
            self._ms_step()
        elif self.graph == "mstreams":
            if self.emb.layout_version != self._graph_layout:
                # a captured buffer was reallocated (row-wise capacity grown
                # here, or by an eager forward such as predict()): re-capture
                # before replaying, keeping the staged next batch
                self._mr_recapture()
            self._mr_step()
        elif isinstance(self.graph, list):
            self._staged_step()
        elif self.graph is not None:
            self.graph.replay()
        else:
            self._forward_backward()
        self.steps += 1

    def _use_gemm_policy(self):
        if self._gemm_pol is not None and ops.gemm_policy(-1) != self._gemm_pol:
            ops.gemm_policy(self._gemm_pol)

    def _staged_step(self):
        self._on_side = False
        # a captured buffer reallocated before this step (lagged row-wise
        # growth, or an eager forward such as predict() growing the capacity)
        # or inside one of its exchange stages: the compute stages run eagerly
        # until the end of the step, then the stages are re-captured
        eager = self.emb.layout_version != self._graph_layout
        for kind, item in self.graph:
            if kind in ("c", "e"):
                g, fns = item
                if eager:        # a captured buffer was reallocated this step
                    self._run_stage(kind, lambda fns=fns: [f() for f in fns])
                else:
                    self._run_stage(kind, None, graph=g)
            else:
                self._run_stage(kind, item)
                # row-wise capacity grown inside an exchange stage: the rest
                # of this step runs eagerly, then the stages are re-captured
                eager = eager or self.emb.layout_version != self._graph_layout
        if eager:
            self.sync_streams()
            torch.cuda.synchronize()
            self.capture_graph(warmup=0, staged=True)

    def capture_graph(self, warmup: int = 2, staged: Optional[bool] = None,
                      streams: bool = True):
        """Capture the step into hipGraphs. One process: per-stream graphs
        (``streams``, default) or one graph for the whole step. Several
        processes (or ``staged``): one graph per run of compute stages, with
        the RCCL exchanges issued eagerly between replays (they overlap the
        next stage). ``warmup`` eager steps run first (they train)."""
        assert self.device.type == "cuda"
        if not self.emb.graph_capturable:
            return
        self._use_gemm_policy()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._rw_resolve()
                self._forward_backward()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if staged is None:
            staged = self.world > 1
            if self._mr_ok():
                try:
                    self._mr_capture()
                    return
                except Exception as e:  # deterministic on every rank: all fall back alike
                    warnings.warn(f"multi-rank stream graphs unavailable ({e!r}); "
                                  "replaying staged graphs")
                    self._mr = None
                    self._whole_capture = False
                    torch.cuda.synchronize()
        if not staged and self.world == 1:
            if streams:
                self._capture_streams()
                return
            g = torch.cuda.CUDAGraph()
            with graph_capture(g):
                self._forward_backward()
            self.graph = g
            return
        pool = torch.cuda.graph_pool_handle()
        seq = []
        # consecutive compute stages share one graph (side-stream forks may
        # span them); each RCCL exchange sits between two graphs
        groups: list = []
        for kind, fn in self._stages():
            if kind in ("c", "e") and groups and groups[-1][0] == kind:
                groups[-1][1].append(fn)
            else:
                groups.append((kind, [fn]))
        self._on_side = False
        se = self._side()
        for kind, fns in groups:
            if kind in ("c", "e"):
                g = torch.cuda.CUDAGraph()
                # thread_local: a backend's own worker thread (gloo's async
                # device copies of a collective issued just before) must not
                # invalidate this thread's capture
                with graph_capture(g, pool=pool, stream=se if kind == "e" else None,
                                   capture_error_mode="thread_local"):
                    for fn in fns:
                        fn()
                seq.append((kind, (g, fns)))
            else:
                # dry exchange keeps every rank's collective sequence aligned
                self._run_stage(kind, fns[0])
                seq.append((kind, fns[0]))
        if se is not None:
            torch.cuda.current_stream().wait_stream(se)
        torch.cuda.synchronize()
        self.graph = seq
        self._graph_layout = self.emb.layout_version

    def pop_loss(self) -> float:
        """Mean training loss since the last call (one device->host read);
        also raises (on every rank) if a row-wise exchange dropped lookups."""
        self._rw_resolve()
        self.sync_streams()
        self.emb.check_overflow()
        v = float(self.loss_sum.item())
        self.loss_sum.zero_()
        return v

    def drain(self):
        """Pipelined trainer: wait (device-side) for the next batch's in-flight
        id / pooled-embedding exchanges and the side stream, so the static
        buffers can be reused (eval); ``prime`` restarts the pipeline."""
        if self.pipeline:
            self._rw_resolve()
            self.emb.ids_exchange_wait()
            if self.emb._pending is not None:
                self.emb.forward_wait()
        self.sync_streams()

    # ------------------------------------------------------------ eval
    @torch.no_grad()
    def predict(self) -> torch.Tensor:
        """Forward only on the static batch; returns logits [B] (fp32)."""
        self.sync_streams()
        self._use_gemm_policy()
        cfg = self.cfg
        self.emb.forward(self.ids)
        self._s_bottom_fwd()
        L0 = self.top_layers[0]
        if cfg.interaction == "dot":
            ops.interaction_fwd(self.h_out, self.emb.recv, self.slot_off, self.slot_stride, self.F,
                                cfg.embedding_dim, self.top_in[0], L0.bcol)
        else:
            self._dcn_forward(self.h_out)
        n = len(self.top_layers)
        for i, L in enumerate(self.top_layers):
            out = self.top_in[i + 1][:, :L.out] if i + 1 < n else self.t_out
            self._fwd(L, self.top_in[i], out)
        K = self.head_k
        head = self.fp.param("head")
        return self.t_out.float() @ head[:K] + head[K]

    def state_dict(self):
        # a deferred embedding update (per-stream graphs) is issued and
        # ordered before the tables are exposed
        self.sync_streams()
        return {"dense": self.fp.state_dict(), "emb": self.emb.state_dict(),
                "dense_m": self.fp.m, "dense_v": self.fp.v, "dense_hyper": self.dense_hyper,
                "emb_hyper": self.emb_hyper}

    def dense_state(self):
        """Replicated training state (dense params, moments, step counters)."""
        self.sync_streams()
        d = {"p": self.fp.p, "dense_hyper": self.dense_hyper, "emb_hyper": self.emb_hyper}
        if self.fp.m is not None:
            d["m"] = self.fp.m
        if self.fp.v is not None:
            d["v"] = self.fp.v
        return d

    def replicated_state(self):
        """name -> tensor of the training state every rank holds an identical
        copy of: dense parameters, their moments, the step counters and the
        replicated (data-parallel) embedding tables with their optimizer
        state (parallel/replicas.py checks them across ranks)."""
        d = {f"dense.{k}": v for k, v in self.dense_state().items()}
        if self.emb.dp_tables:
            for k, v in self.emb.dp_store.state_dict().items():
                if isinstance(v, torch.Tensor):
                    d[f"emb.dp.{k}"] = v
        return d

    def heartbeat_stream(self):
        """The stream whose work ends an issued step (None: the current one):
        the M stream of the multi-rank step graphs, which waits every other
        stream's previous step before it can finish the next."""
        if self.graph == "mstreams" and self._mr is not None:
            return self._mr["streams"]["M"]
        return None

    def progress(self) -> dict:
        """Host-side view of the step pipeline (hang diagnostics)."""
        r = {"rank": self.rank, "world": self.world, "steps_issued": self.steps,
             "graph": self.graph if isinstance(self.graph, (str, type(None))) else "staged",
             "pipeline": self.pipeline, "layout_version": self.emb.layout_version}
        if self.emb.rw_tables:
            r["rw_cap"] = self.emb.rw_cap
            r["rw_grows"] = self.emb.rw_grows
        if self._mr is not None:
            # each per-stream event: has the work before its latest record
            # completed (which stream is stuck)
            r["stream_events_done"] = {k: ev.query() for k, ev in self._mr["events"].items()}
        return r

    def load_dense_state(self, d):
        for k, v in self.dense_state().items():
            if k not in d:
                raise KeyError(f"checkpoint is missing dense state {k}")
            v.copy_(d[k].to(v.device))
        self.fp.sync_bf16()

    def flat_state(self):
        """Flat name -> tensor view of every piece of training state (for the
        sharded checkpoint: each rank saves its own embedding shards)."""
        out = {"dense.p": self.fp.p, "dense_hyper": self.dense_hyper, "emb_hyper": self.emb_hyper}
        if self.fp.m is not None:
            out["dense.m"] = self.fp.m
        if self.fp.v is not None:
            out["dense.v"] = self.fp.v
        for grp, sd in self.emb.state_dict().items():
            for k, v in sd.items():
                out[f"emb.{grp}.{k}"] = v
        return out

    def load_flat_state(self, d):
        for k, v in self.flat_state().items():
            if k not in d:
                raise KeyError(f"checkpoint is missing {k}")
            v.copy_(d[k].to(v.device))
        self.fp.sync_bf16()

