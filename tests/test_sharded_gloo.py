"""Multi-process (gloo, CPU) equivalence tests of the sharded embedding engine
and data-parallel DLRM training against single-process execution.

The same code paths run over RCCL on MI355X (backend "nccl"); here they run
with world_size 2 and 3 on CPU through the torch reference ops.
"""
import pytest
import torch

from tests.dist_harness import run_distributed

ROWS = [50, 7, 300, 1000, 3]
D = 16


def full_tables(seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(r, D, generator=g) * 0.1 for r in ROWS]


def global_ids(B, L, world, seed=1):
    """Per-rank flat id tensors (table-major, bag-major) for a global batch."""
    g = torch.Generator().manual_seed(seed)
    per_table = [torch.randint(0, r, (world * B * L[t],), generator=g) for t, r in enumerate(ROWS)]
    out = []
    for rk in range(world):
        out.append(torch.cat([per_table[t].view(world * B, L[t])[rk * B:(rk + 1) * B].reshape(-1)
                              for t in range(len(ROWS))]))
    return out, per_table


def _emb_worker(rank, world, strategy, B, L, dp_dense_max_bytes=256 << 20):
    from tdfo_amd.parallel.dist import get_info
    from tdfo_amd.sparse.planner import plan_sharding
    from tdfo_amd.sparse.sharded import ShardedEmbeddingBags
    from tdfo_amd.sparse.tables import EmbOptimConfig, TableConfig

    tables = [TableConfig(f"t{i}", r, D) for i, r in enumerate(ROWS)]
    optim = EmbOptimConfig("sgd", lr=0.5)
    plan = plan_sharding(tables, world, optim, batch_per_rank=B, pooling=L, strategy=strategy)
    emb = ShardedEmbeddingBags(tables, plan, rank, B, L, "cpu", optim, group=get_info().group,
                               dp_dense_max_bytes=dp_dense_max_bytes)
    full = full_tables()
    for t in range(len(ROWS)):
        emb.set_table_weight(t, full[t])
    ids_all, _ = global_ids(B, L, world)
    emb.forward(ids_all[rank])
    feats = []
    for t in range(len(ROWS)):
        idx = emb.slot_off[t] + torch.arange(B)[:, None] * emb.slot_stride[t] + torch.arange(D)
        feats.append(emb.recv.float()[idx])
    g = torch.Generator().manual_seed(100 + rank)
    emb.d_recv.copy_((torch.randn(emb.d_recv.numel(), generator=g) * 0.1).to(emb.d_recv.dtype))
    d_recv = emb.d_recv.float().clone()
    emb.backward(torch.tensor([0.5, 1.0]))
    shards = {}
    for t in range(len(ROWS)):
        r = emb.get_table_weight(t)
        if r is not None:
            shards[t] = ((r[0].start, r[0].stop, r[0].step), emb.table_cols(t)[0], r[1].clone())
    return feats, d_recv, shards, [list(emb.slot_off), list(emb.slot_stride)]


@pytest.mark.parametrize("strategy,world,dp_dense", [
    ("table_wise", 2, 1), ("row_wise", 2, 1), ("data_parallel", 2, 1), ("data_parallel", 2, 0),
    ("column_wise", 2, 1), ("table_wise", 3, 1), ("row_wise", 3, 1), ("column_wise", 3, 1),
    ("data_parallel", 3, 1)])
def test_sharded_embedding_fwd_bwd(strategy, world, dp_dense):
    """dp_dense=0 forces the large-replicated-table path (all-gathered ids +
    pooled grads, global sparse update) instead of the dense-grad all-reduce."""
    B, L = 6, [1, 2, 1, 3, 1]
    res = run_distributed(_emb_worker, world, strategy, B, L, (256 << 20) if dp_dense else 0)
    full = full_tables()
    ids_all, per_table = global_ids(B, L, world)
    # forward: pooled sums of bf16-rounded output
    for rank in range(world):
        feats = res[rank][0]
        for t in range(len(ROWS)):
            ids = per_table[t].view(world * B, L[t])[rank * B:(rank + 1) * B]
            exp = full[t][ids].sum(1)
            assert torch.allclose(feats[t], exp, atol=2e-2), (rank, t)
    # backward: SGD with summed grads from all ranks
    new = [w.clone() for w in full]
    for rank in range(world):
        d_recv = res[rank][1]
        off, stride = res[rank][3]
        for t in range(len(ROWS)):
            ids = per_table[t].view(world * B, L[t])[rank * B:(rank + 1) * B]
            idx = off[t] + torch.arange(B)[:, None] * stride[t] + torch.arange(D)
            gb = d_recv.view(-1)[idx]
            for b in range(B):
                for i in ids[b]:
                    new[t][i] -= 0.5 * gb[b]
    for rank in range(world):
        for t, (lo, c0, w) in res[rank][2].items():
            exp = new[t][slice(*lo)][:, c0:c0 + w.shape[1]]
            assert torch.allclose(w, exp, atol=1e-2), (rank, t)


def _dlrm_worker(rank, world, B, steps, strategy, emb_opt="rowwise_adagrad", rw_comm="fp32",
                 pipeline=False, dense_comm="fp32", dist="uniform", alpha=1.05, rw_capacity=1.25,
                 pipe_lookup=True, skew_from=None, pooling=(1, 2, 1, 1, 1), rw_exchange="auto"):
    """skew_from: batches from this index on carry only even ids (every
    row-wise id of a 2-rank job then goes to owner 0)."""
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    from tdfo_amd.parallel.dist import get_info

    cfg = DLRMConfig(embedding_dim=32, table_rows=ROWS, bottom=[64, 32], top=[64, 32, 1],
                     dense_lr=1e-2, emb_lr=0.05, sharding=strategy, pooling=list(pooling),
                     emb_opt=emb_opt, rw_comm=rw_comm, pipeline=pipeline, dense_comm=dense_comm,
                     rw_capacity=rw_capacity, pipeline_lookup=pipe_lookup, rw_exchange=rw_exchange)
    tr = DLRMTrainer(cfg, B, "cpu", group=get_info().group, rank=rank, world_size=world)
    assert tr.pipeline == (pipeline and world > 1)
    if tr.emb.rw_tables and rw_exchange != "auto":
        assert tr.emb.rw_rows == (rw_exchange == "rows" and world > 1)
    g = torch.Generator().manual_seed(5)
    for t, r in enumerate(ROWS):
        tr.emb.set_table_weight(t, torch.randn(r, 32, generator=g) * 0.1)
    data = SyntheticCriteo(ROWS, B * world, pooling=cfg.pooling, device="cpu", seed=9, dist=dist,
                           zipf_alpha=alpha)

    def local(batch):
        dense, ids, label = batch
        # slice this rank's part of the global batch
        parts, off = [], 0
        for t, Lt in enumerate(cfg.pooling):
            n = B * world * Lt
            parts.append(ids[off:off + n].view(B * world, Lt)[rank * B:(rank + 1) * B].reshape(-1))
            off += n
        return (dense[rank * B:(rank + 1) * B].clone(), torch.cat(parts),
                label[rank * B:(rank + 1) * B].clone())

    batches = [local(data.next()) for _ in range(steps + 1)]
    if skew_from is not None:
        batches = [(d, i - i % 2 if k >= skew_from else i, y) for k, (d, i, y) in enumerate(batches)]
    if tr.pipeline:
        tr.prime(*batches[0])
    for i in range(steps):
        if tr.pipeline:
            tr.set_next_batch(*batches[i + 1])
        else:
            tr.load_batch(*batches[i])
        tr.step()
    tabs = {}
    for t in range(len(ROWS)):
        r = tr.emb.get_table_weight(t)
        if r is not None:
            tabs[t] = ((r[0].start, r[0].stop, r[0].step), tr.emb.table_cols(t)[0], r[1].clone())
    grows = tr.emb.rw_grows if tr.emb.rw_tables else 0
    tr.pop_loss()                               # raises on every rank if a lookup was dropped
    if skew_from is not None:
        return tr.fp.p.clone(), tabs, grows, tr.emb.rw_lag_reads if tr.emb.rw_tables else 0
    return tr.fp.p.clone(), tabs, grows


@pytest.mark.parametrize("strategy,opt", [
    ("table_wise", "rowwise_adagrad"), ("row_wise", "rowwise_adagrad"),
    ("data_parallel", "rowwise_adagrad"), ("data_parallel", "adam"),
    ("column_wise", "adagrad"), ("auto", "rowwise_adagrad")])
def test_dlrm_data_parallel_matches_single_process(strategy, opt):
    """Every sharding kind at W=2 equals one process on the global batch.
    Row-wise Adagrad keeps one state per row *per column block* under CW (as
    TorchRec CW shards do), so CW is checked with elementwise Adagrad; Adam on
    replicated tables must not decay the moments of rows the batch never
    touched (the dense-gradient path is off for it)."""
    B, steps = 8, 3
    multi = run_distributed(_dlrm_worker, 2, B, steps, strategy, opt)
    single = run_distributed(_dlrm_worker, 1, 2 * B, steps, "table_wise", opt)[0]
    p1, tabs1, _ = single
    for rank in range(2):
        p, tabs, _ = multi[rank]
        assert torch.allclose(p, p1, atol=2e-4), (rank, (p - p1).abs().max())
        for t, (lo, c0, w) in tabs.items():
            ref = tabs1[t][2][slice(*lo)][:, c0:c0 + w.shape[1]]
            assert torch.allclose(w, ref, atol=2e-4), (rank, t, (w - ref).abs().max())


@pytest.mark.parametrize("strategy", ["table_wise", "row_wise", "auto"])
@pytest.mark.parametrize("pipe_lookup", ["1", "0"])
def test_dlrm_pipelined_input_dist_is_exact(strategy, pipe_lookup):
    """Input-dist pipelining (next batch's ids exchanged during this step's
    dense update; with pipeline_lookup also its lookup and pooled-embedding
    exchange, after this step's embedding update) changes only when the
    exchanges run: parameters and tables after 4 steps equal the unpipelined
    run bit for bit."""
    B, steps = 8, 4
    plain = run_distributed(_dlrm_worker, 2, B, steps, strategy, "rowwise_adagrad", "fp32", False)
    piped = run_distributed(_dlrm_worker, 2, B, steps, strategy, "rowwise_adagrad", "fp32", True,
                            "fp32", "uniform", 1.05, 1.25, pipe_lookup == "1")
    for rank in range(2):
        p0, tabs0, _ = plain[rank]
        p1, tabs1, _ = piped[rank]
        assert torch.equal(p0, p1), (rank, (p0 - p1).abs().max())
        assert tabs0.keys() == tabs1.keys()
        for t in tabs0:
            assert torch.equal(tabs0[t][2], tabs1[t][2]), (rank, t)


def test_dlrm_bf16_dense_allreduce_close_to_fp32():
    """dense_comm="bf16" (bf16 wire format for the dense-grad all-reduce)
    tracks the fp32 all-reduce run closely; tables are unaffected by design
    only through the dense path, so both are compared."""
    B, steps = 8, 3
    f32 = run_distributed(_dlrm_worker, 2, B, steps, "table_wise", "rowwise_adagrad", "fp32",
                          False, "fp32")
    b16 = run_distributed(_dlrm_worker, 2, B, steps, "table_wise", "rowwise_adagrad", "fp32",
                          False, "bf16")
    for rank in range(2):
        p0 = f32[rank][0]
        p1 = b16[rank][0]
        assert not torch.equal(p0, p1)                     # the wire format is really bf16
        d = (p0 - p1).abs()
        # AdamW (lr 1e-2) normalises each update, so elements whose gradient
        # is ~0 can move by up to lr per step either way: bound the worst case
        # by 3 steps x lr and require the bulk to agree closely
        assert float(d.max()) <= 3e-2 and float(d.mean()) < 1e-3, (float(d.max()), float(d.mean()))
    assert torch.equal(b16[0][0], b16[1][0])               # replicas stay identical


@pytest.mark.parametrize("strategy,world", [("row_wise", 2), ("row_wise", 3), ("auto", 2)])
@pytest.mark.parametrize("alpha", [1.05, 1.2])
def test_dlrm_zipf_ids_match_single_process(strategy, world, alpha):
    """Power-law ids (the hot head at the low ids, as in frequency-ordered
    Criteo): the row-wise exchange deals rows round-robin and grows its
    per-owner capacity before any segment would overflow (started here at a
    deliberately small 0.3 x n/W), so training equals one process exactly
    and no lookup is dropped (pop_loss raises on every rank otherwise)."""
    B, steps = 8, 3
    multi = run_distributed(_dlrm_worker, world, B, steps, strategy, "rowwise_adagrad", "fp32",
                            False, "fp32", "zipf", alpha, 0.3)
    single = run_distributed(_dlrm_worker, 1, world * B, steps, "table_wise", "rowwise_adagrad",
                             "fp32", False, "fp32", "zipf", alpha)[0]
    p1, tabs1, _ = single
    if strategy == "row_wise":
        assert all(m[2] > 0 for m in multi)      # the capacity really had to grow
    for rank in range(world):
        p, tabs, _ = multi[rank]
        assert torch.allclose(p, p1, atol=2e-4), (rank, (p - p1).abs().max())
        for t, (lo, c0, w) in tabs.items():
            ref = tabs1[t][2][slice(*lo)][:, c0:c0 + w.shape[1]]
            assert torch.allclose(w, ref, atol=2e-4), (rank, t, (w - ref).abs().max())


def test_dlrm_lagged_rw_growth_is_exact():
    """Pipelined row-wise exchanges check their capacity one step late (the
    need is published in step i's tail and read when step i+1 is issued):
    when the ids turn skewed after the prime (every id even -> one owner), the
    lagged check grows the capacity and redoes that batch's exchange before it
    is consumed -- parameters and tables equal the unpipelined run (capacity
    checked by a host read before every exchange) bit for bit, and one
    process up to fp32 association."""
    B, steps = 64, 5
    plain = run_distributed(_dlrm_worker, 2, B, steps, "row_wise", "rowwise_adagrad", "fp32", False,
                            "fp32", "uniform", 1.05, 1.25, True, 2)
    lag = run_distributed(_dlrm_worker, 2, B, steps, "row_wise", "rowwise_adagrad", "fp32", True,
                          "fp32", "uniform", 1.05, 1.25, True, 2)
    single = run_distributed(_dlrm_worker, 1, 2 * B, steps, "table_wise", "rowwise_adagrad", "fp32",
                             False, "fp32", "uniform", 1.05, 1.25, True, 2)[0]
    for rank in range(2):
        p0, tabs0, g0, _ = plain[rank]
        p1, tabs1, g1, reads = lag[rank]
        assert g0 > 0 and g1 > 0 and reads >= steps - 1, (g0, g1, reads)
        assert torch.equal(p0, p1), (rank, (p0 - p1).abs().max())
        for t in tabs0:
            assert torch.equal(tabs0[t][2], tabs1[t][2]), (rank, t)
        assert torch.allclose(p1, single[0], atol=2e-4)
        for t, (lo, c0, w) in tabs1.items():
            ref = single[1][t][2][slice(*lo)][:, c0:c0 + w.shape[1]]
            assert torch.allclose(w, ref, atol=2e-4), (rank, t)


@pytest.mark.parametrize("world,pipeline,skew", [(2, False, None), (3, False, None),
                                                 (2, True, None), (2, True, 2)])
def test_dlrm_rw_rows_exchange_matches_pooled(world, pipeline, skew):
    """One-hot row-wise tables: returning the looked-up rows (and sending
    each gradient row to its owner) by all-to-all moves ~W/1.25 x fewer
    bytes than the pooled reduce-scatter / gradient all-gather and gives the
    same values -- parameters and tables equal the pooled exchange bit for
    bit, also across a lagged capacity growth (skew: redo of the batch)."""
    B, steps = 64, 4
    args = (world, B, steps, "row_wise", "rowwise_adagrad", "fp32", pipeline, "fp32", "uniform",
            1.05, 1.25, True, skew, (1, 1, 1, 1, 1))
    pooled = run_distributed(_dlrm_worker, *args, "pooled")
    rows = run_distributed(_dlrm_worker, *args, "rows")
    for rank in range(world):
        p0, tabs0 = pooled[rank][0], pooled[rank][1]
        p1, tabs1 = rows[rank][0], rows[rank][1]
        if skew is not None:
            assert pooled[rank][2] > 0 and rows[rank][2] > 0      # the capacity grew
        assert torch.equal(p0, p1), (rank, (p0 - p1).abs().max())
        assert tabs0.keys() == tabs1.keys()
        for t in tabs0:
            assert torch.equal(tabs0[t][2], tabs1[t][2]), (rank, t)
