"""Embedding sharding planner sized for MI355X (288 GB HBM3E per GPU).

Plays the role of torchrec's default planner behind DMP
(torchrec/train.py:241-247 of the reference, which picks a sharding type per
table) and of TF's MinSizePartitioner for the parameter-server path
(tensorflow2/train_ps.py:55-58), with an explicit, deterministic cost model:

* memory per shard = rows x D x 4 B (fp32 weights) + optimizer state
  (rowwise-Adagrad 1 float/row, Adagrad D, Adam 2D floats/row);
* cost per shard, in microseconds per step on MI355X:
  - lookup + fused update: ids x ID_NS (measured: a rank's embedding time
    tracks its id count, ~1.4 ns per id fwd+bwd at D=128 --
    profiles/emb_rank_w8.jsonl) scaled by D/128;
  - xGMI: every peer link carries its share of the shard's exchange, both
    directions (fwd values, bwd gradients), at LINK_GBS:
      table-wise  the owner sends each peer that peer's B pooled rows (bf16)
      row-wise    every rank reduce-scatters [W][B][D] bf16 partials and
                  all-gathers the [B][D] gradients: B rows per link per
                  direction, on every rank (W x the table-wise bytes)
    The per-link terms assume all W-1 links run in parallel (a fully
    connected xGMI node), i.e. the all-to-all is per-link bound.

Sharding kinds:
  table_wise   whole table on one rank (pooled-embedding all-to-all)
  row_wise     rows dealt round-robin across all ranks (owner = id mod W;
               id bucketize + all-to-all of ids, owner-side pooling, bf16
               reduce-scatter of the pooled partials)
  column_wise  D split across ranks; each column block is a table-wise shard
  data_parallel  replicated (small tables; dense-gradient all-reduce)

Strategies: "data_parallel" (config 3, the reference's pmap / Mirrored /
DDP data parallelism, jax-flax/train_dp.py:63, tensorflow2/train_dp.py:71-72)
replicates the small tables -- those whose dense fp32 gradient all-reduce
moves fewer bytes per rank than their row-wise exchange would
(``dp_rule="cost"``: rows x D x 4 x 2 (W-1)/W against the ids + rows +
gradient rows of a one-hot table's "rows" exchange, or the pooled
partials / gradients of a multi-hot one), within ``dp_replicate_max_bytes``
of fp32 weights in all (256 MB); ``dp_rule="budget"``: the smallest tables
while they fit that budget -- one dense fp32 gradient all-reduce trains all
of them and their update is the same dense pass on every rank) and
owner-partitions the larger ones as row-wise shards: an exact
replica of a big table would make every rank apply the whole global batch's
update (W x the one-GPU work, plus W x B pooled gradients gathered), while
the owner-partitioned table gives the same numbers with each rank updating
only its 1/W of the rows. "replicated" keeps every table whole on every rank
(the literal pmap layout; per-rank update work grows with W).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

from .tables import EmbOptimConfig, TableConfig

HBM_BYTES = 288 * 10**9
GiB = 1 << 30
ID_NS = 1.4            # ns per looked-up id, fwd + fused bwd, D = 128 (measured)
LINK_GBS = 153.0       # xGMI GB/s per direction per point-to-point link


@dataclass
class TableShard:
    table: int
    kind: str                      # table_wise | row_wise | column_wise | data_parallel
    ranks: List[int]
    row_blocks: List[int] = field(default_factory=list)   # row_wise: rows held per rank
    #   (round-robin ownership: rank r holds rows r, r + W, r + 2W, ...)
    col_blocks: List[int] = field(default_factory=list)   # column_wise: cols per rank


@dataclass
class ShardingPlan:
    world_size: int
    shards: List[TableShard]
    mem_bytes: List[int]
    cost: List[float]

    def kind_of(self, t: int) -> str:
        return self.shards[t].kind

    def tables_on(self, rank: int, kind: str = "table_wise") -> List[int]:
        return [s.table for s in self.shards if s.kind == kind and rank in s.ranks]

    def summary(self) -> Dict:
        kinds: Dict[str, int] = {}
        for s in self.shards:
            kinds[s.kind] = kinds.get(s.kind, 0) + 1
        return {"world_size": self.world_size, "kinds": kinds,
                "mem_GiB": [round(m / GiB, 2) for m in self.mem_bytes],
                "cost": [round(c, 3) for c in self.cost]}


def _mem_per_row(dim: int, optim: EmbOptimConfig) -> int:
    return 4 * (dim + optim.state_floats_per_row(dim))


def plan_sharding(tables: Sequence[TableConfig], world_size: int, optim: EmbOptimConfig,
                  batch_per_rank: int = 8192, pooling: Optional[Sequence[float]] = None,
                  hbm_bytes: int = HBM_BYTES, reserve_frac: float = 0.15,
                  strategy: str = "auto", dp_max_bytes: int = 0,
                  row_cost: Optional[Callable[[int], float]] = None,
                  dp_max_rows: Optional[int] = None,
                  dp_replicate_max_bytes: int = 256 << 20,
                  balance: float = 1.10, dp_rule: str = "cost") -> ShardingPlan:
    """Deterministic greedy planner with a balance pass.

    strategy: "auto" (table-wise with row-wise fallback for tables that fit
    no rank), "table_wise", "row_wise", "column_wise" (tables split evenly by
    columns), "data_parallel" (replicated up to dp_replicate_max_bytes,
    owner-partitioned row-wise above), "replicated" (every table on every
    rank).

    dp_max_rows: "auto" replicates (data_parallel) every table with fewer
    rows than this (default at W > 1: batch_per_rank // 2 -- a replicated
    table's dense fp32 gradient all-reduce then moves fewer bytes than the
    table-wise pooled all-to-all it replaces, 4 B x rows vs 2 B x batch per
    column, and its lookups stay local).

    row_cost: optional per-lookup cost multiplier as a function of a table's
    row count. Default: none -- measured on MI355X at the world-8 layout
    (scripts/bench_emb_rank.py, profiles/emb_rank_w8.jsonl) a rank's
    embedding time tracks its id count far more than its table sizes (a
    4-row and a 40M-row table cost 85 vs 103 us per 65536 ids, while the
    4-table ranks of the world-8 plan, holding only small tables, are the
    slowest at 188 us vs 140-164 us for the 3-table ranks).

    balance ("auto", W > 1): a multi-hot table can cost more than a whole
    rank's fair share (DCN-v2's pooling-100 table is ~9 ms of lookups on its
    owner at W = 8, the other ranks ~1.3 ms), and greedy table-wise placement
    cannot split it. While the plan's max / min rank cost exceeds
    ``balance``, the costliest table-wise table of the costliest rank is
    re-planned row-wise (its ids spread over every rank), one table at a
    time. Along that sequence the plan with the lowest max rank cost wins
    (within 1 % of it, the most even one), and only if it beats the greedy
    plan by >= 2 %: one-hot plans whose imbalance is one table's granularity
    (DLRM-1TB) stay table-wise, since row-wise adds link traffic on every
    rank.
    """
    kw = dict(batch_per_rank=batch_per_rank, pooling=pooling, hbm_bytes=hbm_bytes,
              reserve_frac=reserve_frac, strategy=strategy, dp_max_bytes=dp_max_bytes,
              row_cost=row_cost, dp_max_rows=dp_max_rows,
              dp_replicate_max_bytes=dp_replicate_max_bytes, dp_rule=dp_rule)
    plan = _plan_once(tables, world_size, optim, frozenset(), **kw)
    if strategy != "auto" or world_size == 1 or balance is None:
        return plan
    pool = list(pooling) if pooling is not None else [1.0] * len(tables)
    if max(plan.cost) <= balance * min(plan.cost):
        return plan
    seq, cur, forced = [], plan, frozenset()
    for _ in range(len(tables)):
        hot = max(range(world_size), key=lambda r: (cur.cost[r], -r))
        tw = [s.table for s in cur.shards if s.kind == "table_wise" and s.ranks == [hot]]
        if not tw or max(cur.cost) <= 1.001 * min(cur.cost):
            break
        forced = forced | {max(tw, key=lambda t: (pool[t] * tables[t].embedding_dim, -t))}
        try:
            cur = _plan_once(tables, world_size, optim, forced, **kw)
        except MemoryError:
            break
        seq.append(cur)
    top = min([max(p.cost) for p in seq], default=max(plan.cost))
    if top > 0.98 * max(plan.cost):
        return plan
    # lowest max rank cost; within 1 % of it, the most even plan
    near = [p for p in seq if max(p.cost) <= 1.01 * top]
    return min(near, key=lambda p: max(p.cost) / min(p.cost))


def _plan_once(tables, world_size, optim, force_rw, batch_per_rank, pooling, hbm_bytes,
               reserve_frac, strategy, dp_max_bytes, row_cost, dp_max_rows,
               dp_replicate_max_bytes, dp_rule="cost") -> ShardingPlan:
    W = world_size
    cap = int(hbm_bytes * (1.0 - reserve_frac))
    T = len(tables)
    pooling = list(pooling) if pooling is not None else [1.0] * T
    gb = batch_per_rank * W
    mem = [0] * W
    cost = [0.0] * W
    shards: List[Optional[TableShard]] = [None] * T

    rc = row_cost or (lambda rows: 1.0)
    B = batch_per_rank
    if dp_max_rows is None:
        dp_max_rows = batch_per_rank // 2 if W > 1 else 0

    def link_us(rows_per_link: float, d: int) -> float:
        return 2 * rows_per_link * d * 2 / (LINK_GBS * 1e3) if W > 1 else 0.0

    def tcost(t: int) -> float:
        """table-wise cost on the owner (us/step)"""
        d = tables[t].embedding_dim
        ids = gb * pooling[t]
        return ids * ID_NS * 1e-3 * d / 128 * rc(tables[t].num_embeddings) + link_us(B, d)

    def rcost(t: int) -> float:
        """row-wise cost on every rank (us/step)"""
        d = tables[t].embedding_dim
        return gb * pooling[t] / W * ID_NS * 1e-3 * d / 128 + link_us(B, d)

    order = sorted(range(T), key=lambda t: (-tcost(t), -tables[t].num_embeddings, t))

    def row_wise(t: int):
        rows = tables[t].num_embeddings
        # rows dealt round-robin: owner(id) = id mod W, local row id div W, so
        # rank r holds ceil((rows - r) / W) rows (row_blocks, also written to
        # checkpoint manifests); every rank allocates the largest share
        blk = -(-rows // W)
        blocks = [len(range(r, rows, W)) for r in range(W)]
        per_row = _mem_per_row(tables[t].embedding_dim, optim)
        for r in range(W):
            mem[r] += (blk + 1) * per_row   # padded block + scratch row (every rank)
            cost[r] += rcost(t)
        return TableShard(t, "row_wise", list(range(W)), row_blocks=blocks)

    def column_wise(t: int):
        d = tables[t].embedding_dim
        nb = min(W, max(2, d // 32))
        while nb > 1 and (d % nb or (d // nb) % 8):      # equal blocks, 8-col aligned
            nb -= 1
        cols = [d // nb] * nb
        ranks = sorted(range(W), key=lambda r: (cost[r], mem[r], r))[:nb]
        for i, r in enumerate(ranks):
            mem[r] += tables[t].num_embeddings * 4 * (cols[i] + optim.state_floats_per_row(cols[i]))
            cost[r] += tcost(t) * cols[i] / d
        return TableShard(t, "column_wise", ranks, col_blocks=cols)

    # tables no single GPU can hold go row-wise first: their shares land on
    # every rank, and the table-wise placement below must see that memory
    if strategy == "auto" and W > 1:
        for t in order:
            if t in force_rw or (tables[t].num_embeddings *
                                 _mem_per_row(tables[t].embedding_dim, optim) > cap):
                shards[t] = row_wise(t)
    # "data_parallel": the smallest tables are replicated while their fp32
    # weights add up to at most dp_replicate_max_bytes -- the replicated set
    # then trains by ONE dense fp32 gradient all-reduce per step (the
    # reference's DP all-reduce, jax-flax/train_dp.py:63) -- and the rest are
    # owner-partitioned row-wise (an exact replica of a big table would make
    # every rank apply the whole global batch's update)
    replicate = set()
    if dp_rule not in ("cost", "budget"):
        raise ValueError(f"dp_rule must be cost or budget, got {dp_rule!r}")

    def ar_cheaper(t: int) -> bool:
        """dense fp32 gradient all-reduce (ring: 2 (W-1)/W of the table per
        rank) moves fewer bytes than the table's row-wise exchange"""
        d, L = tables[t].embedding_dim, pooling[t]
        ar = 2 * (W - 1) / W * tables[t].num_embeddings * d * 4
        if L == 1:       # "rows" exchange: ids, rows back, gradient rows out (1.25 x capacity)
            rw = B * (8 + 2 * 1.25 * d * 2) * (W - 1) / W
        else:            # pooled partials' reduce-scatter + pooled gradients' all-gather
            rw = B * L * 8 * (W - 1) / W + 2 * (W - 1) * B * d * 2
        return ar <= rw

    if strategy == "data_parallel" and W > 1:
        cum = 0
        for t in sorted(range(T), key=lambda t: (tables[t].num_embeddings *
                                                  tables[t].embedding_dim, t)):
            nb = tables[t].num_embeddings * tables[t].embedding_dim * 4
            if cum + nb > dp_replicate_max_bytes or (dp_rule == "cost" and not ar_cheaper(t)):
                break
            cum += nb
            replicate.add(t)
    for t in order:
        if shards[t] is not None:
            continue
        tb = tables[t].num_embeddings * _mem_per_row(tables[t].embedding_dim, optim)
        if strategy == "data_parallel" and W > 1 and t not in replicate:
            shards[t] = row_wise(t)                 # owner-partitioned big table
            continue
        if strategy in ("data_parallel", "replicated") or (strategy == "auto" and (
                tb <= dp_max_bytes or tables[t].num_embeddings < dp_max_rows)):
            for r in range(W):
                mem[r] += tb
                cost[r] += tcost(t) / W
            shards[t] = TableShard(t, "data_parallel", list(range(W)))
            continue
        if strategy == "row_wise" and W > 1:
            shards[t] = row_wise(t)
            continue
        if strategy == "column_wise" and W > 1:
            shards[t] = column_wise(t)
            continue
        cand = [r for r in range(W) if mem[r] + tb <= cap]
        if not cand:
            if W == 1:
                raise MemoryError(f"table {tables[t].name} ({tb / GiB:.1f} GiB) exceeds HBM budget")
            shards[t] = row_wise(t)
            continue
        r = min(cand, key=lambda r: (cost[r], mem[r], r))
        mem[r] += tb
        cost[r] += tcost(t)
        shards[t] = TableShard(t, "table_wise", [r])
    for r in range(W):
        if mem[r] > cap:
            raise MemoryError(f"rank {r} needs {mem[r] / GiB:.1f} GiB > budget {cap / GiB:.1f} GiB")
    return ShardingPlan(W, shards, mem, cost)  # type: ignore[arg-type]
