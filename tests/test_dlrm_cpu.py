"""DLRM engine on CPU (BASELINE config 1: DLRM-tiny through train.py's engine)
plus reference-op self-checks."""
import pytest
import torch

from tdfo_amd import ops
from tdfo_amd.data.synthetic import SyntheticCriteo
from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
from tdfo_amd.ops import reference as ref


def tiny_cfg(**kw):
    base = dict(embedding_dim=32, table_rows=[1000, 50, 300, 20000, 7], bottom=[64, 32],
                top=[64, 32, 1], dense_lr=1e-2, emb_lr=0.05)
    base.update(kw)
    return DLRMConfig(**base)


def test_dlrm_tiny_cpu_learns():
    cfg = tiny_cfg()
    tr = DLRMTrainer(cfg, 128, "cpu")
    data = SyntheticCriteo(cfg.table_rows, 128, device="cpu", seed=1)
    losses = []
    for i in range(240):
        tr.load_batch(*data.next())
        tr.step()
        if i % 60 == 59:
            losses.append(tr.pop_loss() / (60 * 128))
    assert losses[-1] < losses[0] - 0.03, losses


def test_dlrm_multihot_and_optimizers_cpu():
    for eo, do in [("sgd", "sgd"), ("adam", "adam"), ("adagrad", "adagrad")]:
        cfg = tiny_cfg(pooling=[2, 1, 3, 1, 4], emb_opt=eo, dense_opt=do)
        tr = DLRMTrainer(cfg, 64, "cpu")
        data = SyntheticCriteo(cfg.table_rows, 64, pooling=cfg.pooling, device="cpu", seed=2)
        for _ in range(5):
            tr.load_batch(*data.next())
            tr.step()
        assert torch.isfinite(tr.fp.p).all()


def test_reference_interaction_matches_naive():
    torch.manual_seed(0)
    B, F, D = 5, 4, 32
    T = F - 1
    dense = torch.randn(B, D).bfloat16()
    emb = torch.randn(B * T * D).bfloat16()
    off = [0] + [t * D for t in range(T)]
    stride = [0] + [T * D] * T
    out = torch.empty(B, 64 * 3, dtype=torch.bfloat16)
    ref.interaction_fwd(dense, emb, off, stride, F, D, out)
    X = torch.cat([dense.float()[:, None], emb.float().view(B, T, D)], 1)
    k = D
    for i in range(F):
        for j in range(i):
            exp = (X[:, i] * X[:, j]).sum(1)
            assert torch.allclose(out[:, k].float(), exp, rtol=2e-2, atol=2e-2)
            k += 1


def test_reference_gemm_layouts():
    torch.manual_seed(0)
    A = torch.randn(64, 128).bfloat16()
    W = torch.randn(32, 128).bfloat16()
    o = torch.empty(64, 32, dtype=torch.bfloat16)
    ops.linear_fwd(A, W, None, False, out=o)
    assert torch.allclose(o.float(), A.float() @ W.float().t(), rtol=1e-2, atol=1e-1)
    dy = torch.randn(64, 32).bfloat16()
    dx = ops.linear_dgrad(dy, W)
    assert torch.allclose(dx.float(), dy.float() @ W.float(), rtol=1e-2, atol=1e-1)
    gw = torch.empty(32 * 128)
    ops.linear_wgrad(dy, A, gw)
    assert torch.allclose(gw.view(32, 128), dy.float().t() @ A.float(), rtol=1e-4, atol=1e-3)


def test_auc_helpers():
    s = torch.tensor([0.1, 0.4, 0.35, 0.8])
    y = torch.tensor([0., 0., 1., 1.])
    assert abs(ref.exact_auc(s, y) - 0.75) < 1e-9
    h = torch.zeros(2000, dtype=torch.long)
    logits = torch.randn(5000)
    yy = (torch.rand(5000) < torch.sigmoid(2 * logits)).float()
    ref.auc_hist(logits, yy, 1000, h)
    assert abs(ref.hist_auc(h) - ref.exact_auc(logits, yy)) < 2e-3


def test_debug_id_bounds_check_raises():
    """§5.2: with debug checks on, an out-of-range id raises before the lookup."""
    import pytest

    from tdfo_amd.sparse import tables as T
    from tdfo_amd.sparse.tables import EmbOptimConfig, TableBatchedEmbedding

    st = TableBatchedEmbedding([10, 20], 8, "cpu", EmbOptimConfig("sgd"))
    B = 2
    ids = torch.tensor([3, 9, 19, 0])             # table0: 3, 9 ; table1: 19, 0
    offs = torch.arange(5)
    out = torch.zeros(B, 16)
    oo = torch.tensor([0, 8])
    T.set_debug_checks(True)
    try:
        st.forward(ids, offs, st.row_offset, 2, B, out, oo, 16)       # in range: fine
        bad = torch.tensor([3, 10, 19, 0])        # 10 >= 10 rows of table 0
        with pytest.raises(IndexError):
            st.forward(bad, offs, st.row_offset, 2, B, out, oo, 16)
    finally:
        T.set_debug_checks(False)


def test_profiling_helpers_cpu():
    from tdfo_amd.utils.profiling import ProfileWindow, StepTimer, parse_window, trace_range

    assert parse_window("5:3") == (5, 3) and parse_window("") is None
    with trace_range("x"):
        pass
    t = StepTimer(enabled=False)
    t.start(); t.stop()
    assert t.mean_ms() is None
    w = ProfileWindow("1:2")
    for s in range(4):
        w.before_step(s); w.after_step(s + 1)


@pytest.mark.parametrize("interaction", ["dot", "dcn"])
def test_deferred_wgrads_bitwise_equal(interaction):
    """Weight grads deferred past the cross / interaction backward
    (DLRMConfig.defer_wgrad, default on with more than one rank) change only
    the issue order: parameters after a few steps are bit-identical."""
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    res = []
    for flag in (False, True):
        cfg = DLRMConfig(embedding_dim=32, table_rows=[100, 20, 300], bottom=[64, 32],
                         top=[64, 32, 1], interaction=interaction, dcn_layers=2, dcn_rank=64,
                         pooling=[2, 1, 3], dense_lr=1e-2, emb_lr=0.05, defer_wgrad=flag)
        tr = DLRMTrainer(cfg, 64, "cpu")
        assert tr._defer_top_wgrad == flag
        data = SyntheticCriteo(cfg.table_rows, 64, pooling=cfg.pooling, device="cpu", seed=5)
        for _ in range(3):
            tr.load_batch(*data.next())
            tr.step()
        res.append((tr.fp.p.clone(), tr.emb.tw_store.weight.clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


def test_bump_counters_cpu():
    """ops.bump adds one to the first element of each float / int64 counter."""
    h = torch.tensor([0.5, 3.0, 1.0])
    r = torch.zeros(1, dtype=torch.int64)
    ops.bump([h[1:2], r])
    ops.bump([h[1:2], r])
    assert h.tolist() == [0.5, 5.0, 1.0] and int(r) == 2


def test_wgrad_splits_slot_sizing():
    """128x128-tile target: ~target blocks, >= 8 K tiles per split. Slot
    sizing (256x128 kernel, DCN-v2): the split count that minimises block
    rounds x K tiles plus the slab-traffic penalty, never more K splits than
    the K tiles allow."""
    assert ops.wgrad_splits(1024, 1024, 8192, 256) == 4
    assert ops.wgrad_splits(256, 512, 8192, 256) == 16
    assert ops.wgrad_splits(64, 64, 512, 256) == 1          # K = 8 tiles: no split
    for M, N in [(512, 3456), (3456, 576), (1024, 3520)]:
        s = ops.wgrad_splits(M, N, 8192, 256, slots=128)
        assert 1 <= s <= 8192 // 64 // 8
        tiles = -(-M // 256) * -(-N // 128)
        assert tiles * s <= 4 * 128 or s == 1               # a few rounds of the resident blocks
