"""Fused linear + label-smoothed CE kernel and the Bert4Rec trainer on MI355X."""
import pytest
import torch

from tdfo_amd import ops
from tdfo_amd.models.bert4rec import Bert4RecTrainer
from tests.test_bert4rec import _batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from tdfo_amd.ops import _ext

    assert _ext.load(), "native library must load on the GPU box"


@pytest.fixture(params=[2, 1, 0], ids=["mfma_x3", "mfma", "valu"])
def xent_impl(request):
    old = ops.linear_xent_impl(request.param)
    yield request.param
    ops.linear_xent_impl(old)


@pytest.mark.parametrize("V,N,hs", [(10, 7, 1.0), (1000, 320, 1.0), (4099, 1030, 1.0),
                                    (600_001, 320, 1.0), (5003, 200, 12.0)])
def test_linear_xent_kernel_matches_reference(V, N, hs, xent_impl):
    """hs scales H: large logits exercise the running-max rescale; N=1030
    (~410 valid tokens) takes the multi-block token paths."""
    torch.manual_seed(N)
    H = torch.randn(N, 16, device=DEV) * hs
    W = torch.randn(V, 16, device=DEV) * 0.2
    b = torch.randn(V, device=DEV) * 0.1
    y = torch.randint(1, V, (N,), device=DEV)
    y[torch.rand(N, device=DEV) < 0.6] = 0
    out = [torch.zeros(N, 16, device=DEV), torch.zeros(N, device=DEV),
           torch.zeros(V, 16, device=DEV), torch.zeros(V, device=DEV)]
    ops.linear_xent(H, W, b, y, 0.1, 0, *out)
    ref = [torch.zeros(N, 16), torch.zeros(N), torch.zeros(V, 16), torch.zeros(V)]
    ops.reference.linear_xent(H.cpu(), W.cpu(), b.cpu(), y.cpu(), 0.1, 0, *ref)
    torch.cuda.synchronize()
    for name, a, r in zip(("dH", "loss", "dW", "db"), out, ref):
        err = float((a.cpu() - r).abs().max() / (r.abs().max() + 1e-12))
        assert err < 2e-4, (name, err)


@pytest.mark.parametrize("opt", [ops.OPT_ADAM, ops.OPT_ADAMW])
@pytest.mark.parametrize("V,N", [(4099, 320), (5003, 1030), (600_001, 320), (100, 64)])
def test_linear_xent_fused_step_matches_separate_optimizer(V, N, opt, xent_impl):
    """The output layer's Adam step inside the kernels (one token block: the
    wgrad epilogue; several: the slab sum; VALU impl: a trailing optimizer
    launch) equals linear_xent + the flat dense optimizer, bit for bit; N=64
    with every label ignored checks the zero-gradient step."""
    torch.manual_seed(V + N)
    H = torch.randn(N, 16, device=DEV)
    W = torch.randn(V, 16, device=DEV) * 0.2
    b = torch.randn(V, device=DEV) * 0.1
    y = torch.randint(1, V, (N,), device=DEV)
    y[torch.rand(N, device=DEV) < 0.6] = 0
    if V == 100:
        y.zero_()
    pad = -(-V // 64) * 64                    # flat-buffer padding (optim/flat.py ALIGN)
    mom = [torch.rand(V * 16, device=DEV), torch.rand(V * 16, device=DEV),
           torch.rand(pad, device=DEV), torch.rand(pad, device=DEV)]
    hyper = torch.tensor([1e-3, 7.0, 1.0], device=DEV)
    prm = (0.9, 0.999, 1e-8, 1e-2)
    # separate: gradient, then the flat optimizer on W and bias
    Wa, ba = W.clone(), torch.zeros(pad, device=DEV)
    ba[:V] = b
    ma = [m.clone() for m in mom]
    dH, lv, dW, db = (torch.zeros(N, 16, device=DEV), torch.zeros(N, device=DEV),
                      torch.zeros(V, 16, device=DEV), torch.zeros(pad, device=DEV))
    ops.linear_xent(H, Wa, ba[:V], y, 0.1, 0, dH, lv, dW, db[:V])
    ops.dense_optimizer(Wa.view(-1), dW.view(-1), ma[0], ma[1], None, opt, hyper, *prm)
    ops.dense_optimizer(ba, db, ma[2], ma[3], None, opt, hyper, *prm)
    # fused
    Wb, bb = W.clone(), torch.zeros(pad, device=DEV)
    bb[:V] = b
    mb = [m.clone() for m in mom]
    dH2, lv2 = torch.zeros(N, 16, device=DEV), torch.zeros(N, device=DEV)
    ops.linear_xent(H, Wb, bb[:V], y, 0.1, 0, dH2, lv2, torch.zeros(V, 16, device=DEV),
                    torch.zeros(V, device=DEV),
                    step=(opt, [mb[0], mb[1], mb[2][:V], mb[3][:V]], hyper, *prm))
    torch.cuda.synchronize()
    assert torch.equal(dH, dH2) and torch.equal(lv, lv2)
    assert torch.equal(Wa, Wb)
    assert torch.equal(ba[:V], bb[:V])
    for x, z in zip(ma, mb):
        assert torch.equal(x[:V * 16 if x.numel() == V * 16 else V],
                           z[:V * 16 if z.numel() == V * 16 else V])


def test_linear_xent_all_ignored(xent_impl):
    N, V = 64, 100
    H = torch.randn(N, 16, device=DEV)
    W = torch.randn(V, 16, device=DEV)
    b = torch.zeros(V, device=DEV)
    y = torch.zeros(N, dtype=torch.int64, device=DEV)
    dH, lv = torch.ones(N, 16, device=DEV), torch.ones(N, device=DEV)
    dW, db = torch.ones(V, 16, device=DEV), torch.ones(V, device=DEV)
    ops.linear_xent(H, W, b, y, 0.1, 0, dH, lv, dW, db)
    torch.cuda.synchronize()
    assert float(dH.abs().sum()) == 0 and float(lv.abs().sum()) == 0
    assert float(dW.abs().sum()) == 0 and float(db.abs().sum()) == 0


def test_bert4rec_gpu_matches_cpu():
    n, T, B = 300, 20, 16
    kw = dict(lr=3e-3, dropout=0.0, seed=3)
    gpu = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    cpu = Bert4RecTrainer(n, T, 16, 2, 2, B, device="cpu", **kw)
    cpu.item.store.weight.copy_(gpu.item.store.weight.cpu())
    cpu.opt.flat.copy_(gpu.opt.flat.cpu())
    g = torch.Generator().manual_seed(0)
    for _ in range(10):
        s, l = _batch(g, B, T, n)
        gpu.load_batch(s.to(DEV), l.to(DEV))
        cpu.load_batch(s, l)
        gpu.step()
        cpu.step()
    torch.cuda.synchronize()
    assert abs(gpu.pop_loss() - cpu.pop_loss()) < 1e-3
    torch.testing.assert_close(gpu.opt.flat.cpu(), cpu.opt.flat, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(gpu.item.weight.cpu(), cpu.item.weight, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("fused_xent", ["1", "0"])
def test_bert4rec_direct_grads_bit_identical(monkeypatch, fused_xent):
    """Encoder / prologue gradients written by the kernels' reductions
    straight into the flat buffer (and no zero fill of what they cover) vs
    the returned-gradient path: same bits after several steps with dropout."""
    n, T, B = 3000, 20, 16
    kw = dict(lr=3e-3, dropout=0.1, seed=5)
    monkeypatch.setenv("TDFO_XENT_FUSED_STEP", fused_xent)
    monkeypatch.setenv("TDFO_B4R_DIRECT_GRADS", "1")
    a = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    monkeypatch.setenv("TDFO_B4R_DIRECT_GRADS", "0")
    b = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    assert a._zero_ranges is not None and b._zero_ranges is None
    if fused_xent == "1":
        assert a._zero_ranges == []          # every flat gradient written directly
    g = torch.Generator().manual_seed(0)
    for _ in range(6):
        s, l = _batch(g, B, T, n)
        for t in (a, b):
            t.load_batch(s.to(DEV), l.to(DEV))
            t.step()
    torch.cuda.synchronize()
    assert torch.equal(a.opt.flat, b.opt.flat)
    assert torch.equal(a.item.weight, b.item.weight)
    assert a.pop_loss() == b.pop_loss()


def test_bert4rec_bump_in_lookup_bit_identical(monkeypatch):
    """The step counters advanced by the item lookup launch instead of a bump
    launch of their own: same counters, same bits."""
    import tdfo_amd.models.bert4rec as m

    n, T, B = 3000, 20, 16
    kw = dict(lr=3e-3, dropout=0.1, seed=7)
    a = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    b = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    g = torch.Generator().manual_seed(1)
    for _ in range(4):
        s, l = _batch(g, B, T, n)
        for t, fold in ((a, True), (b, False)):
            monkeypatch.setattr(m, "_FOLD_BUMP", fold)
            t.load_batch(s.to(DEV), l.to(DEV))
            t.step()
    torch.cuda.synchronize()
    assert torch.equal(a.opt.hyper, b.opt.hyper)
    assert torch.equal(a.model.rng_step, b.model.rng_step)
    assert torch.equal(a.opt.flat, b.opt.flat)
    assert torch.equal(a.item.weight, b.item.weight)


def test_bert4rec_graph_replay_matches_eager():
    n, T, B = 5000, 20, 16
    kw = dict(lr=3e-3, dropout=0.0, seed=3)
    a = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    b = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    g = torch.Generator().manual_seed(0)
    s, l = _batch(g, B, T, n)
    for t in (a, b):
        t.load_batch(s.to(DEV), l.to(DEV))
    b.capture_graph(warmup=2)
    for _ in range(2):           # capture warmup trained b for 2 steps (capture itself does not run)
        a.step()
    for _ in range(5):
        s, l = _batch(g, B, T, n)
        for t in (a, b):
            t.load_batch(s.to(DEV), l.to(DEV))
            t.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(a.opt.flat, b.opt.flat, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a.item.weight, b.item.weight, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("E,C", [(16, 101), (32, 64), (64, 200)])
def test_rank_metrics_kernel(E, C):
    """Fused eval scoring + ranking kernel vs the fp32 reference (ties with the
    positive rank it behind, as recall_ndcg_sums)."""
    from tdfo_amd import ops
    from tdfo_amd.ops import reference as ref

    torch.manual_seed(1)
    B, V = 1000, 5000
    h = torch.randn(B, E, device="cuda")
    W = torch.randn(V, E, device="cuda")
    b = torch.randn(V, device="cuda")
    cand = torch.randint(0, V, (B, C), device="cuda")
    cand[:50, 3] = cand[:50, 0]
    out = torch.empty(7, device="cuda")
    ops.rank_metrics(h, W, b, cand, (10, 20, 50), out)
    exp = torch.empty(7, device="cuda")
    ref.rank_metrics(h, W, b, cand, (10, 20, 50), exp)
    assert torch.allclose(out, exp, atol=1e-2), (out, exp)


def test_bert4rec_parked_encoder_reduce_bit_identical(monkeypatch):
    """Each encoder layer's parameter-gradient reduction run by extra blocks
    of the next backward launch (layer below / sequence prologue) instead of
    a launch of its own: same bits, eager and graph-replayed."""
    import tdfo_amd.models.bert4rec as m

    n, T, B = 3000, 20, 16
    kw = dict(lr=3e-3, dropout=0.1, seed=9)
    a = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    b = Bert4RecTrainer(n, T, 16, 2, 2, B, device=DEV, **kw)
    g = torch.Generator().manual_seed(2)
    for _ in range(4):
        s, l = _batch(g, B, T, n)
        for t, park in ((a, True), (b, False)):
            monkeypatch.setattr(m, "_DEFER_ENC_RED", park)
            t.load_batch(s.to(DEV), l.to(DEV))
            t.step()
    torch.cuda.synchronize()
    assert torch.equal(a.opt.flat, b.opt.flat)
    assert torch.equal(a.item.weight, b.item.weight)
    monkeypatch.setattr(m, "_DEFER_ENC_RED", True)
    a.capture_graph(warmup=1)
    monkeypatch.setattr(m, "_DEFER_ENC_RED", False)
    b.capture_graph(warmup=1)
    for _ in range(3):
        s, l = _batch(g, B, T, n)
        for t in (a, b):
            t.load_batch(s.to(DEV), l.to(DEV))
            t.step()
    torch.cuda.synchronize()
    assert torch.equal(a.opt.flat, b.opt.flat)
    assert torch.equal(a.item.weight, b.item.weight)
