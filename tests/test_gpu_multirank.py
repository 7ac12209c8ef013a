"""Multi-rank DLRM step on the real HIP kernels: 2 ranks share cuda:0 and talk
over gloo (RCCL refuses two ranks on one GPU), each replaying the staged
hipGraphs the driver's N-GPU bench runs (compute stages captured, the
exchanges issued eagerly between them), compared with one process stepping
the 2x batch. Table-wise, row-wise (fixed-capacity exchange), column-wise and
data-parallel tables are all covered; the same stage code runs over RCCL on
an 8-GPU node. Mirrors tests/test_sharded_gloo.py (CPU references) on GPU.
"""
import pytest
import torch

from tests.dist_harness import run_distributed

pytestmark = pytest.mark.gpu

ROWS = [5000, 7, 30000, 1000, 3, 800]
POOL = [1, 2, 1, 3, 1, 1]
B = 256
STEPS = 3


def _worker(rank, world, Bk, strategy, graph, rw_comm, emb_opt="rowwise_adagrad", pipeline=False,
            dist="uniform", alpha=1.05, rw_capacity=1.25, pipe_lookup=True, predict_skew=False,
            pool=POOL, rw_exchange="auto"):
    """dist="zipf": the two eager steps see uniform ids, the graph-replayed
    ones power-law ids -- the row-wise capacity then has to grow after the
    capture (eager rest of that step, re-capture). predict_skew: between two
    replayed steps a predict() on a batch whose ids all map to one owner grows
    the row-wise capacity outside any step."""
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    from tdfo_amd.parallel.dist import get_info

    dev = get_info().device if world > 1 else torch.device("cuda", 0)
    cfg = DLRMConfig(embedding_dim=64, table_rows=ROWS, bottom=[128, 64], top=[128, 64, 1],
                     dense_opt="sgd", dense_lr=0.05, emb_lr=0.05, sharding=strategy,
                     pooling=list(pool), rw_comm=rw_comm, emb_opt=emb_opt, pipeline=pipeline,
                     rw_capacity=rw_capacity, pipeline_lookup=pipe_lookup, rw_exchange=rw_exchange)
    tr = DLRMTrainer(cfg, Bk, dev, group=get_info().group, rank=rank, world_size=world)
    g = torch.Generator().manual_seed(5)
    for t, r in enumerate(ROWS):
        tr.emb.set_table_weight(t, torch.randn(r, 64, generator=g) * 0.1)
    data = SyntheticCriteo(ROWS, B * 2, pooling=list(pool), device="cpu", seed=9)
    skew = SyntheticCriteo(ROWS, B * 2, pooling=list(pool), device="cpu", seed=9, stream=1,
                           dist=dist, zipf_alpha=alpha)
    batches = []
    for i in range(STEPS + 3):
        dense, ids, label = (data if i < 2 else skew).next()
        parts, off = [], 0
        for t, Lt in enumerate(pool):
            n = B * 2 * Lt
            v = ids[off:off + n].view(B * 2, Lt)
            parts.append(v[rank * Bk:(rank + 1) * Bk].reshape(-1))
            off += n
        sl = slice(rank * Bk, (rank + 1) * Bk)
        batches.append((dense[sl].to(dev), torch.cat(parts).to(dev), label[sl].to(dev)))
    # two eager steps, then (graph) capture -- capture's warm-up replays the
    # last loaded batch, so the step sequence is the same in both modes
    # pipelined input dist: step i runs on the batch loaded by step i - 1 (or
    # prime()) and loads / exchanges batch i + 1 -- the same batch sequence
    def feed(i):
        if tr.pipeline:
            tr.set_next_batch(*batches[i + 1])
        else:
            tr.load_batch(*batches[i])

    if tr.pipeline:
        tr.prime(*batches[0])
    for i in range(2):
        feed(i)
        tr.step()
    if graph:
        tr.capture_graph(warmup=0)
        assert tr.graph is not None
    for i in range(2, 2 + STEPS):
        if predict_skew and i == 3:
            d, ids_, y = batches[i]
            tr.load_batch(d, ids_ - ids_ % world, y)
            tr.predict()
        feed(i)
        tr.step()
    torch.cuda.synchronize()
    loss = tr.pop_loss()
    tabs = {}
    for t in range(len(ROWS)):
        r = tr.emb.get_table_weight(t)
        if r is not None:
            tabs[t] = ((r[0].start, r[0].stop, r[0].step), tr.emb.table_cols(t)[0],
                       r[1].detach().cpu().clone())
    grows = tr.emb.rw_grows if tr.emb.rw_tables else 0
    if rw_exchange != "auto" and tr.emb.rw_tables:
        assert tr.emb.rw_rows == (rw_exchange == "rows")
    return tr.fp.p.detach().cpu().clone(), tabs, loss, grows


@pytest.fixture(scope="module")
def single():
    """One process stepping the 2x batch (table-wise at world 1)."""
    cache = {}

    def get(emb_opt: str, dist: str = "uniform", alpha: float = 1.05):
        key = (emb_opt, dist, alpha)
        if key not in cache:
            cache[key] = run_distributed(_worker, 1, 2 * B, "table_wise", True, "fp32", emb_opt,
                                         False, dist, alpha, device="cuda")[0][:3]
        return cache[key]
    return get


def _check(multi, ref, tol):
    p1, tabs1, loss1 = ref
    loss = sum(m[2] for m in multi)
    assert abs(loss - loss1) / abs(loss1) < tol, (loss, loss1)
    for rank, m in enumerate(multi):
        p, tabs = m[0], m[1]
        assert torch.allclose(p, p1, atol=tol, rtol=tol), (rank, float((p - p1).abs().max()))
        for t, (lo, c0, w) in tabs.items():
            ref_w = tabs1[t][2][slice(*lo)][:, c0:c0 + w.shape[1]]
            assert torch.allclose(w, ref_w, atol=tol, rtol=tol), (rank, t,
                                                                   float((w - ref_w).abs().max()))


@pytest.mark.parametrize("strategy,pipeline", [("table_wise", True), ("row_wise", True),
                                               ("auto", True), ("auto", False)])
def test_four_ranks_match_one_process(strategy, pipeline, single):
    """The W >= 3 paths together on the real kernels: 4 ranks sharing cuda:0
    (uneven table-wise plans, the radix-sorted owner backward, W-run
    layouts, row-wise at W = 4), staged hipGraphs, pipelined input dist."""
    multi = run_distributed(_worker, 4, B // 2, strategy, True, "fp32", "rowwise_adagrad", pipeline,
                            device="cuda", timeout=600)
    _check(multi, single("rowwise_adagrad"), 3e-3)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("alpha", [1.05, 1.2])
def test_zipf_row_wise_grows_capacity_after_capture(world, alpha, single):
    """Power-law ids after the capture (initial capacity 0.3 x n/W): the
    capacity check grows the row-wise segments inside the exchange stage, the
    rest of that step runs eagerly and the stages are re-captured; the result
    equals one process and no lookup is dropped (pop_loss raises otherwise)."""
    multi = run_distributed(_worker, world, 2 * B // world, "row_wise", True, "fp32",
                            "rowwise_adagrad", False, "zipf", alpha, 0.3, device="cuda",
                            timeout=600)
    assert all(m[3] > 0 for m in multi)
    _check(multi, single("rowwise_adagrad", "zipf", alpha), 3e-3)


# Column-wise keeps one row-wise Adagrad state per column block (as TorchRec CW
# shards do), so it is compared with elementwise Adagrad on both sides. The
# bf16 row-wise reduce-scatter rounds pooled partials differently from one
# process; row-wise Adagrad (lr / sqrt(mean g^2), zero initial state) turns
# that into O(lr) differences on rows whose gradient is ~0, so that case is
# compared under SGD (exactness of the exchange itself: the fp32 case). The
# data-parallel strategy owner-partitions most of these tables row-wise too
# (replicated only where the dense all-reduce is cheaper), so it runs the
# exact fp32 exchange here.
@pytest.mark.parametrize("strategy,graph,rw_comm,emb_opt", [
    ("table_wise", True, "bf16", "rowwise_adagrad"), ("table_wise", False, "bf16", "rowwise_adagrad"),
    ("row_wise", True, "fp32", "rowwise_adagrad"), ("row_wise", True, "bf16", "sgd"),
    ("column_wise", True, "bf16", "adagrad"), ("data_parallel", True, "fp32", "rowwise_adagrad"),
    ("auto", True, "bf16", "rowwise_adagrad")])
def test_two_ranks_match_one_process(strategy, graph, rw_comm, emb_opt, single):
    multi = run_distributed(_worker, 2, B, strategy, graph, rw_comm, emb_opt, device="cuda",
                            timeout=600)
    p1, tabs1, loss1 = single(emb_opt)
    tol = 1e-2 if (strategy == "row_wise" and rw_comm == "bf16") else 3e-3
    loss = multi[0][2] + multi[1][2]
    assert abs(loss - loss1) / abs(loss1) < tol, (loss, loss1)
    for rank in range(2):
        p, tabs = multi[rank][0], multi[rank][1]
        assert torch.allclose(p, p1, atol=tol, rtol=tol), (rank, float((p - p1).abs().max()))
        for t, (lo, c0, w) in tabs.items():
            ref_w = tabs1[t][2][slice(*lo)][:, c0:c0 + w.shape[1]]
            assert torch.allclose(w, ref_w, atol=tol, rtol=tol), (rank, t,
                                                                   float((w - ref_w).abs().max()))


@pytest.mark.parametrize("strategy,rw_comm,pipe_lookup", [
    ("table_wise", "bf16", "1"), ("auto", "bf16", "1"), ("row_wise", "fp32", "1"),
    ("data_parallel", "fp32", "1"), ("auto", "bf16", "0")])
def test_two_ranks_pipelined_input_dist(strategy, rw_comm, pipe_lookup, single):
    """Input-dist pipelining (next batch's ids exchanged during the dense
    update; pipeline_lookup: also its lookup and pooled-embedding exchange
    on the side stream in the step's tail) on the staged hipGraphs: same
    result as one process."""
    multi = run_distributed(_worker, 2, B, strategy, True, rw_comm, "rowwise_adagrad", True,
                            "uniform", 1.05, 1.25, pipe_lookup == "1", device="cuda",
                            timeout=600)
    p1, tabs1, loss1 = single("rowwise_adagrad")
    tol = 3e-3
    loss = multi[0][2] + multi[1][2]
    assert abs(loss - loss1) / abs(loss1) < tol, (loss, loss1)
    for rank in range(2):
        p, tabs = multi[rank][0], multi[rank][1]
        assert torch.allclose(p, p1, atol=tol, rtol=tol), (rank, float((p - p1).abs().max()))
        for t, (lo, c0, w) in tabs.items():
            ref_w = tabs1[t][2][slice(*lo)][:, c0:c0 + w.shape[1]]
            assert torch.allclose(w, ref_w, atol=tol, rtol=tol), (rank, t)


def test_row_wise_growth_in_predict_between_replays(single):
    """Row-wise capacity grown by a predict() between two replayed steps
    (outside any step): the next step runs its stages eagerly against the
    reallocated exchange buffers and re-captures, instead of replaying graphs
    that still hold the freed ones -- the result equals one process."""
    multi = run_distributed(_worker, 2, B, "row_wise", True, "fp32", "rowwise_adagrad", False,
                            "uniform", 1.05, 1.25, True, True, device="cuda", timeout=600)
    assert all(m[3] > 0 for m in multi)
    _check(multi, single("rowwise_adagrad"), 3e-3)


@pytest.mark.parametrize("world,pipeline,dist", [(2, False, "uniform"), (4, True, "uniform"),
                                                 (2, False, "zipf")])
def test_row_wise_rows_exchange_matches_pooled(world, pipeline, dist):
    """One-hot row-wise tables on the real kernels: the "rows" exchange (the
    owner's bf16 rows back by all-to-all, gradient rows to the owner) equals
    the pooled reduce-scatter / all-gather exchange bit for bit -- staged
    hipGraphs, pipelined input dist, and (zipf) capacity growth after the
    capture with the eager redo of that step."""
    pool = [1] * len(ROWS)
    args = (world, 2 * B // world, "row_wise", True, "fp32", "rowwise_adagrad", pipeline, dist,
            1.2, 0.3 if dist == "zipf" else 1.25, True, False, pool)
    pooled = run_distributed(_worker, *args, "pooled", device="cuda", timeout=600)
    rows = run_distributed(_worker, *args, "rows", device="cuda", timeout=600)
    for rank in range(world):
        assert torch.equal(pooled[rank][0], rows[rank][0]), rank
        assert pooled[rank][2] == rows[rank][2], rank
        for t in pooled[rank][1]:
            assert torch.equal(pooled[rank][1][t][2], rows[rank][1][t][2]), (rank, t)
