"""Native collective layer (csrc/comm/rccl_comm.cpp, ``RcclComm``) and the
whole-step multi-rank hipGraph it enables.

* RcclComm on a one-rank RCCL communicator (the box has one GPU; RCCL
  refuses two ranks on one device): every op against its definition, eager
  and captured into a hipGraph, sync and async (comm-stream fork / join).
* The W > 1 DLRM step as per-stream graphs with the collectives inside
  (``DLRMConfig.stream_graphs``, models/dlrm_multirank.py) with loopback
  collectives (rank 0 of a W-rank job, ``LoopbackComm``) is bit-identical to
  the staged replay (graphs between eagerly issued exchanges) over the same
  batches.
"""
import os

import pytest
import torch

from tests.dist_harness import run_distributed

pytestmark = pytest.mark.gpu


def _rccl_ops(rank, world):
    from tdfo_amd.parallel.comm import RcclComm, as_comm
    from tdfo_amd.utils.capture import graph_capture

    c = as_comm(None)
    assert isinstance(c, RcclComm) and c.world == world == 1
    dev = torch.device("cuda", 0)
    x = torch.randn(1000, device=dev)
    # all-to-all: equal and explicit splits (one rank: out = inp)
    out = torch.empty_like(x)
    c.all_to_all(out, x)
    torch.testing.assert_close(out, x, rtol=0, atol=0)
    o2 = torch.zeros(1000, dtype=torch.bfloat16, device=dev)
    w = c.all_to_all(o2, x.bfloat16(), [1000], [1000], async_op=True)
    w.wait()
    torch.testing.assert_close(o2, x.bfloat16(), rtol=0, atol=0)
    # all-reduce sum / max, int64 ids, reduce-scatter, all-gather, broadcast
    t = x.clone()
    c.all_reduce(t)
    torch.testing.assert_close(t, x, rtol=0, atol=0)
    t.fill_(3.0)
    c.all_reduce(t, "max", async_op=True).wait()
    assert float(t.max()) == 3.0
    ids = torch.arange(64, dtype=torch.int64, device=dev)
    oi = torch.empty_like(ids)
    c.all_to_all(oi, ids)
    assert torch.equal(oi, ids)
    rs = torch.empty(1000, device=dev)
    c.reduce_scatter(rs, x, async_op=True).wait()
    torch.testing.assert_close(rs, x, rtol=0, atol=0)
    ag = torch.empty(1000, device=dev)
    c.all_gather(ag, x)
    torch.testing.assert_close(ag, x, rtol=0, atol=0)
    c.broadcast(t, 0)
    # captured: a graph holding compute -> async all-to-all -> join -> compute
    a = torch.randn(4096, device=dev)
    b = torch.empty_like(a)
    y = torch.empty_like(a)
    for _ in range(2):      # eager warm-up
        w = c.all_to_all(b, a * 2.0, async_op=True)
        w.wait()
        y.copy_(b + 1.0)
    # captured with the comm stream as the capture origin (RCCL under capture
    # must run there) and the compute on a stream forked from it
    g = torch.cuda.CUDAGraph()
    origin, ms = torch.cuda.Stream(), torch.cuda.Stream()
    with graph_capture(g, stream=origin, capture_error_mode="thread_local"):
        ms.wait_stream(origin)
        with torch.cuda.stream(ms), c.capture_origin(origin):
            tmp = a * 2.0
            w = c.all_to_all(b, tmp, async_op=True)
            c.all_reduce(a, async_op=False)
            w.wait()
            y.copy_(b + 1.0)
        origin.wait_stream(ms)
    for k in range(3):
        a.copy_(torch.full_like(a, float(k)))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, torch.full_like(a, 2.0 * k + 1.0)), k
    # a collective captured without naming the origin is refused (it would
    # crash hipStreamEndCapture)
    g2 = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="capture_origin"):
        with graph_capture(g2, capture_error_mode="thread_local"):
            c.all_reduce(a, async_op=True)
    info = torch.ops.tdfo.rccl_info(c.h)
    assert info[0] == 1 and info[3] > 0
    return True


def test_rccl_comm_one_rank_ops_eager_and_captured():
    """One-rank RCCL group through the real launcher path (nccl backend)."""
    res = run_distributed(_rccl_ops, 1, device="cuda_rccl")
    assert res == [True]


def _trainer(whole: bool, W: int, strategy: str):
    """strategy "row_wise_onehot": row-wise with one id per bag (the "rows"
    exchange: rows back by all-to-all, scatter on the exchange stream)."""
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    from tdfo_amd.parallel.comm import LoopbackComm

    rows = [5000, 7, 30000, 1000, 3, 800, 64, 129]
    onehot = strategy == "row_wise_onehot"
    cfg = DLRMConfig(embedding_dim=64, table_rows=rows, bottom=[128, 64], top=[128, 64, 1],
                     sharding="row_wise" if onehot else strategy, pipeline=True,
                     pooling=[1] * 8 if onehot else [1, 2, 1, 3, 1, 1, 1, 1],
                     stream_graphs=whole, seed=3)
    dev = torch.device("cuda", 0)
    comm = LoopbackComm(W, 0, dev)
    tr = DLRMTrainer(cfg, 256, dev, group=comm, rank=0, world_size=W)
    return tr, rows, cfg


@pytest.mark.parametrize("strategy,skew", [("table_wise", False), ("auto", False),
                                           ("column_wise", False), ("data_parallel", False),
                                           ("row_wise", False), ("row_wise", True),
                                           ("row_wise_onehot", False), ("row_wise_onehot", True)])
def test_stream_graphs_match_staged(strategy, skew):
    """Row-wise tables run on the stream graphs with the lagged capacity
    check; ``skew``: the batches after the capture carry only ids that are
    multiples of W (one owner gets every row-wise id), so the capacity grows
    between two replays (redo of that batch's exchange, re-capture)."""
    from tdfo_amd.data.synthetic import SyntheticCriteo

    W = 4
    out = []
    for whole in (False, True):
        tr, rows, cfg = _trainer(whole, W, strategy)
        data = SyntheticCriteo(rows, 256, pooling=cfg.pooling_factors(), device="cuda:0", seed=9)
        batches = [data.next() for _ in range(9)]
        if skew:
            batches = batches[:3] + [(d, i - i % W, y) for d, i, y in batches[3:]]
        tr.prime(*batches[0])
        for i in range(2):
            tr.set_next_batch(*batches[i + 1])
            tr.step()
        tr.capture_graph(warmup=0)
        assert (tr.graph == "mstreams") == whole, tr.graph
        for i in range(2, 8):
            tr.set_next_batch(*batches[i + 1])
            tr.step()
        torch.cuda.synchronize()
        assert (tr.graph == "mstreams") == whole, tr.graph      # (still, after any growth)
        if strategy.startswith("row_wise"):
            assert tr.emb.rw_lag_reads >= 6
            assert (tr.emb.rw_grows > 0) == skew, tr.emb.rw_grows
            assert tr.emb.rw_rows == (strategy == "row_wise_onehot")
        loss = tr.pop_loss()
        tr.drain()
        torch.cuda.synchronize()
        tabs = []
        for t in range(len(rows)):
            r = tr.emb.get_table_weight(t)
            tabs.append(None if r is None else r[1].clone())
        out.append((loss, tr.fp.p.clone(), tabs))
    (l0, p0, t0), (l1, p1, t1) = out
    assert l0 == l1
    assert torch.equal(p0, p1)
    for a, b in zip(t0, t1):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)


def test_stream_graphs_host_cost():
    """Three graph launches per step: the host issues a step of the emulated
    W=8 job in a small fraction of the staged path's time."""
    import time

    from tdfo_amd.data.synthetic import SyntheticCriteo

    res = {}
    for whole in (False, True):
        tr, rows, cfg = _trainer(whole, 8, "table_wise")
        data = SyntheticCriteo(rows, 256, pooling=cfg.pooling_factors(), device="cuda:0", seed=9)
        batches = [data.next() for _ in range(4)]
        tr.prime(*batches[0])
        tr.set_next_batch(*batches[1])
        tr.step()
        tr.capture_graph(warmup=0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(30):
            tr.set_next_batch(*batches[2 + i % 2])
            tr.step()
        res[whole] = (time.perf_counter() - t) / 30
        torch.cuda.synchronize()
    assert res[True] < 0.5 * res[False], res
