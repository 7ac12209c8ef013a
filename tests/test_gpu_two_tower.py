"""Fused TwoTower HIP kernel and trainer on MI355X vs the fp32 autograd oracle."""
import pytest
import torch

from tdfo_amd import ops
from tdfo_amd.models.two_tower import TwoTowerConfig, TwoTowerTrainer, init_dense_params
from tdfo_amd.ops import reference as ref
from tests.test_two_tower import SM, make_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from tdfo_amd.ops import _ext

    assert _ext.load(), "native library must load on the GPU box"


@pytest.mark.parametrize("B", [1, 100, 128, 2048, 3001])
def test_two_tower_kernel_matches_autograd(B):
    torch.manual_seed(B)
    X = torch.randn(B, 116, device=DEV) * 0.5
    P = torch.zeros(ops.TT_NPARAM + 64, device=DEV)
    P[:ops.TT_NPARAM] = init_dense_params("flax", 1).to(DEV) * 2
    y = (torch.rand(B, device=DEV) < 0.4).float()
    inv = 1.0 / B
    nparts = ops.two_tower_parts(B)
    lg = torch.zeros(B, device=DEV)
    dX = torch.zeros(B, 116, device=DEV)
    part = torch.zeros(nparts, ops.TT_PART_LD, device=DEV)
    ops.two_tower(X, P, y, inv, lg, dX, part)
    lr_, dXr = torch.zeros(B), torch.zeros(B, 116)
    partr = torch.zeros(nparts, ops.TT_PART_LD)
    ref.two_tower(X.cpu(), P.cpu(), y.cpu(), inv, lr_, dXr, partr)
    torch.cuda.synchronize()
    torch.testing.assert_close(lg.cpu(), lr_, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dX[:, :112].cpu(), dXr[:, :112], rtol=1e-3, atol=1e-6)
    g = part.sum(0).cpu()
    gr = partr.sum(0)
    torch.testing.assert_close(g[:ops.TT_NPARAM], gr[:ops.TT_NPARAM], rtol=1e-3, atol=1e-5)
    assert abs(float(g[ops.TT_NPARAM] - gr[ops.TT_NPARAM])) < 1e-3 * B
    # eval (forward only) path
    lg2 = torch.zeros(B, device=DEV)
    ops.two_tower(X, P, y, 1.0, lg2)
    torch.testing.assert_close(lg2, lg, rtol=0, atol=0)


@pytest.mark.parametrize("emb_update", ["sparse", "dense"])
def test_two_tower_trainer_gpu_matches_cpu(emb_update):
    cfg = TwoTowerConfig(SM, learning_rate=3e-3, emb_update=emb_update)
    B = 512
    g = TwoTowerTrainer(cfg, B, DEV)
    c = TwoTowerTrainer(cfg, B, "cpu")
    c.emb.weight.copy_(g.emb.weight.cpu())
    c.P.copy_(g.P.cpu())
    for i in range(15):
        b = make_batch(B, i)
        g.load_batch({k: v.to(DEV) for k, v in b.items()})
        c.load_batch(b)
        g.step()
        c.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(g.P.cpu(), c.P, rtol=2e-3, atol=2e-4)
    torch.testing.assert_close(g.emb.weight.cpu(), c.emb.weight, rtol=2e-3, atol=2e-4)
    lg, lc = g.pop_metrics(), c.pop_metrics()
    assert abs(lg[0] - lc[0]) < 1e-3 and abs(lg[1] - lc[1]) < 1e-3


@pytest.mark.parametrize("emb_update,B,mode", [
    ("sparse", 2048, "colaunch"), ("sparse", 1000, "colaunch"), ("sparse", 320, "colaunch"),
    ("sparse", 4096, "colaunch"), ("dense", 512, "colaunch"), ("sparse", 2048, "radix"),
    ("sparse", 2048, "side"), ("sparse", 1000, "side"), ("sparse", 2048, "plain")])
def test_two_tower_fused_step_bit_identical(emb_update, B, mode):
    """The fused step against the separate launches: same bits everywhere.
    colaunch: towers beside the per-table sort, reduce_adam beside the update
    (B = 1000: no in-kernel-combine update, so on its own; 4096: the larger
    sort, towers first); side: towers on their own, reduce_adam beside the
    sort; plain: neither; radix: the device-wide sort (nothing co-launched)."""
    cfg = TwoTowerConfig(SM, learning_rate=3e-3, emb_update=emb_update, weight_decay=1e-2)
    a = TwoTowerTrainer(cfg, B, DEV)
    b = TwoTowerTrainer(cfg, B, DEV)
    a.fused_step, b.fused_step = True, False
    a.side_job = mode in ("colaunch", "side", "radix")
    a.colaunch = mode in ("colaunch", "radix")
    prev = ops.embedding_segsort(0 if mode == "radix" else -1)
    try:
        _run_pair(a, b, B)
    finally:
        ops.embedding_segsort(prev)


def _run_pair(a, b, B):
    for i in range(10):
        x = {k: v.to(DEV) for k, v in make_batch(B, i).items()}
        a.load_batch(x)
        b.load_batch(x)
        a.step()
        b.step()
    torch.cuda.synchronize()
    for name in ("P", "M", "V", "hyper", "emb_hyper", "loss_sum", "train_hist"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    assert torch.equal(a.G[:ops.TT_NPARAM + 1], b.G[:ops.TT_NPARAM + 1])
    assert torch.equal(a.emb.weight, b.emb.weight)
    assert a.pop_metrics() == b.pop_metrics()


def test_reduce_adam_matches_reference():
    torch.manual_seed(3)
    n, ld, rows = 2400, 2432, 77
    part = torch.randn(rows * ld, device=DEV)
    p, m, v = (torch.randn(n, device=DEV) for _ in range(3))
    v = v.abs()
    hyper = torch.tensor([1e-2, 3.0, 0.5], device=DEV)
    grad = torch.zeros(n + 1, device=DEV)
    acc = torch.zeros(1, dtype=torch.float64, device=DEV)
    lg = torch.randn(1000, device=DEV) * 3
    y = (torch.rand(1000, device=DEV) < 0.3).float()
    h = torch.zeros(2 * 199, dtype=torch.int64, device=DEV)
    pc, mc, vc, gc, accc, hc = (t.cpu().clone() for t in (p, m, v, grad, acc, h))
    ops.reduce_adam(part, rows, n, ld, grad, p, m, v, hyper, wd=0.1, adamw=True, loss_acc=acc,
                    logits=lg, labels=y, nb=199, hist=h)
    ops.reduce_adam(part.cpu(), rows, n, ld, gc, pc, mc, vc, hyper.cpu(), wd=0.1, adamw=True,
                    loss_acc=accc, logits=lg.cpu(), labels=y.cpu(), nb=199, hist=hc)
    assert torch.equal(h.cpu(), hc)
    torch.testing.assert_close(grad.cpu(), gc, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(p.cpu(), pc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m.cpu(), mc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(v.cpu(), vc, rtol=1e-5, atol=1e-6)
    assert abs(float(acc.cpu() - accc)) < 1e-3


def test_two_tower_graph_replay_matches_eager():
    cfg = TwoTowerConfig(SM, learning_rate=3e-3)
    B = 1024
    a = TwoTowerTrainer(cfg, B, DEV)
    b = TwoTowerTrainer(cfg, B, DEV)
    b.load_batch({k: v.to(DEV) for k, v in make_batch(B, 0).items()})
    b.capture_graph(warmup=2)            # restores the state after warmup
    for i in range(8):
        x = {k: v.to(DEV) for k, v in make_batch(B, i + 1).items()}
        a.load_batch(x)
        b.load_batch(x)
        a.step()
        b.step()
    torch.cuda.synchronize()
    assert b.graph is not None
    torch.testing.assert_close(a.P, b.P, rtol=0, atol=0)
    torch.testing.assert_close(a.emb.weight, b.emb.weight, rtol=0, atol=0)
    assert a.pop_metrics() == b.pop_metrics()


@pytest.mark.parametrize("B", [100, 2048])
def test_two_tower_kernel_fp16_with_loss_scale(B):
    """fp16-compute variant (mixed_precision) with a device loss scale vs the
    float16 autograd oracle (same scale)."""
    torch.manual_seed(B)
    X = torch.randn(B, 116, device=DEV) * 0.5
    P = torch.zeros(ops.TT_NPARAM + 64, device=DEV)
    P[:ops.TT_NPARAM] = init_dense_params("flax", 1).to(DEV) * 2
    y = (torch.rand(B, device=DEV) < 0.4).float()
    inv, scale = 1.0 / B, torch.tensor([1024.0], device=DEV)
    nparts = ops.two_tower_parts(B)
    lg, dX = torch.zeros(B, device=DEV), torch.zeros(B, 116, device=DEV)
    part = torch.zeros(nparts, ops.TT_PART_LD, device=DEV)
    ops.two_tower(X, P, y, inv, lg, dX, part, loss_scale=scale, half=True)
    lr_, dXr = torch.zeros(B), torch.zeros(B, 116)
    partr = torch.zeros(nparts, ops.TT_PART_LD)
    ref.two_tower(X.cpu(), P.cpu(), y.cpu(), inv, lr_, dXr, partr, scale.cpu(), True)
    torch.cuda.synchronize()
    torch.testing.assert_close(lg.cpu(), lr_, rtol=2e-2, atol=2e-2)
    g, gr = part.sum(0).cpu()[:ops.TT_NPARAM], partr.sum(0)[:ops.TT_NPARAM]
    assert float((g - gr).norm() / gr.norm()) < 2e-2
    assert float((dX[:, :112].cpu() - dXr[:, :112]).norm() / dXr[:, :112].norm()) < 2e-2


def test_mixed_precision_skip_on_gpu():
    """The fused embedding kernels honour the skip flag / unscale on device."""
    from tests.test_two_tower import test_mixed_precision_dynamic_scale_skips_non_finite as t
    import tdfo_amd.models.two_tower as tt

    orig = tt.TwoTowerTrainer.__init__

    def on_gpu(self, cfg, B, device="cpu", **kw):
        orig(self, cfg, B, DEV, **kw)
    tt.TwoTowerTrainer.__init__ = on_gpu
    try:
        t("sparse")
        t("dense")
    finally:
        tt.TwoTowerTrainer.__init__ = orig
