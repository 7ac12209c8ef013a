"""TwoTower: fused-step semantics on CPU, data-parallel
and sharded (parameter-server replacement) equivalence over gloo, Flax
checkpoint layout."""
import math

import numpy as np
import pytest
import torch

from tdfo_amd import ops
from tdfo_amd.models.two_tower import (DENSE_LAYERS, EMBED_NAMES, FEATURES, SIZE_KEYS,
                                       TwoTowerConfig, TwoTowerTrainer, init_dense_params)
from tdfo_amd.utils import checkpoint as ckpt
from tests.dist_harness import run_distributed

SM = {"user": 300, "item": 400, "language": 7, "is_ebook": 2, "format": 9, "publisher": 50,
      "pub_decade": 14}


def make_batch(B, seed, sm=SM):
    g = torch.Generator().manual_seed(seed)
    d = {f: torch.randint(0, sm[k], (B,), generator=g) for f, k in zip(FEATURES, SIZE_KEYS)}
    d["avg_rating"] = torch.rand(B, generator=g)
    d["num_pages"] = torch.rand(B, generator=g)
    d["label"] = ((d["user_id"] % 3 == 0) ^ (d["item_id"] % 2 == 0)).float()
    return d


def test_reference_two_tower_matches_manual_forward():
    torch.manual_seed(0)
    B = 37
    X = torch.randn(B, 116)
    P = init_dense_params("flax", 3)
    p = ops.reference.two_tower_unpack(P)
    sw = lambda z: z * torch.sigmoid(z)   # noqa: E731
    u = sw(X[:, :16] @ p["user_fc1.kernel"] + p["user_fc1.bias"]) @ p["user_fc2.kernel"]
    i = sw(X[:, 16:114] @ p["item_fc1.kernel"] + p["item_fc1.bias"]) @ p["item_fc2.kernel"]
    want = ((u + p["user_fc2.bias"]) * (i + p["item_fc2.bias"])).sum(1)
    lg = torch.zeros(B)
    ops.two_tower(X, P, torch.zeros(B), 1.0, lg)
    torch.testing.assert_close(lg, want, rtol=1e-5, atol=1e-5)


def test_init_schemes():
    f = init_dense_params("flax", 0)
    k = init_dense_params("keras", 0)
    assert f.numel() == k.numel() == ops.TT_NPARAM
    # glorot_uniform bound for the 98x16 item kernel; lecun_normal is truncated at 2 std
    o = 2 * (16 * 16 + 16)
    kf = f[o: o + 98 * 16]
    assert kf.abs().max() <= math.sqrt(6 / (98 + 16)) + 1e-6
    kk = k[o: o + 98 * 16]
    assert kk.abs().max() <= 2 * math.sqrt(1 / 98) / 0.87962566103423978 + 1e-5
    assert float(f[16 * 16: 16 * 17].abs().sum()) == 0.0      # zero bias


@pytest.mark.parametrize("emb_update", ["sparse", "dense"])
def test_two_tower_cpu_learns(emb_update):
    cfg = TwoTowerConfig(SM, learning_rate=5e-3, emb_update=emb_update)
    tr = TwoTowerTrainer(cfg, 256, "cpu")
    losses = []
    for i in range(120):
        tr.load_batch(make_batch(256, i))
        tr.step()
        if i % 40 == 39:
            losses.append(tr.pop_metrics())
    assert losses[-1][0] < 0.5 * losses[0][0], losses
    assert losses[-1][1] > 0.9


def test_dense_mode_decays_untouched_rows():
    """emb_update="dense" reproduces optax.adamw: rows never looked up still
    move (weight decay) — the sparse mode leaves them untouched."""
    out = {}
    for mode in ("sparse", "dense"):
        cfg = TwoTowerConfig(SM, learning_rate=1e-2, weight_decay=0.5, emb_update=mode)
        tr = TwoTowerTrainer(cfg, 64, "cpu")
        w0 = tr.emb.table_weight(0).clone()
        b = make_batch(64, 0)
        b["user_id"] = torch.zeros(64, dtype=torch.int64)          # only user row 0
        tr.load_batch(b)
        tr.step()
        out[mode] = (w0, tr.emb.table_weight(0).clone())
    w0, w1 = out["sparse"]
    assert torch.equal(w0[1:], w1[1:]) and not torch.equal(w0[0], w1[0])
    w0, w1 = out["dense"]
    assert not torch.equal(w0[1:], w1[1:])
    torch.testing.assert_close(w1[5], w0[5] * (1 - 1e-2 * 0.5))


def test_partial_last_batch_and_eval():
    cfg = TwoTowerConfig(SM)
    tr = TwoTowerTrainer(cfg, 128, "cpu", eval_batch_size=200)
    tr.load_batch(make_batch(50, 1))
    tr.step()
    loss, _ = tr.pop_metrics()
    assert 0.5 < loss < 0.9
    tr.load_batch(make_batch(200, 2), eval_mode=True)
    lg = tr.evaluate_batch()
    assert lg.shape == (200,)
    el, auc = tr.pop_metrics(eval_mode=True)
    assert 0.5 < el < 0.9 and 0.0 <= auc <= 1.0


def test_flax_params_roundtrip(tmp_path):
    cfg = TwoTowerConfig(SM)
    tr = TwoTowerTrainer(cfg, 32, "cpu")
    params = tr.flax_params()
    assert set(params) == set(EMBED_NAMES) | {n for n, _ in DENSE_LAYERS}
    assert params["item_fc1"]["kernel"].shape == (98, 16)      # Flax [in, out]
    assert params["user_embed"]["embedding"].shape == (SM["user"], 16)
    path = tmp_path / "model_params.pt"
    ckpt.save_flax_params(params, str(path))
    back = ckpt.load_flax_params(str(path))
    for k in params:
        for kk in params[k]:
            assert isinstance(back[k][kk], np.ndarray) and back[k][kk].dtype == np.float32
            np.testing.assert_array_equal(back[k][kk], params[k][kk].numpy())
    tr2 = TwoTowerTrainer(TwoTowerConfig(SM, seed=7), 32, "cpu")
    tr2.load_flax_params(back)
    torch.testing.assert_close(tr2.P, tr.P)
    torch.testing.assert_close(tr2.emb.weight, tr.emb.weight)


def test_flax_msgpack_bytes_layout():
    """Byte layout of flax.serialization.to_bytes for a known tree: a map of
    ExtType(1, msgpack([shape, dtype, raw bytes]))."""
    import msgpack
    arr = np.arange(6, dtype=np.float32).reshape(2, 3)
    b = ckpt.to_flax_bytes({"layer": {"kernel": arr}})
    tree = msgpack.unpackb(b, raw=False)
    ext = tree["layer"]["kernel"]
    assert isinstance(ext, msgpack.ExtType) and ext.code == 1
    shape, dtype, raw = msgpack.unpackb(ext.data, raw=False)
    assert shape == [2, 3] and dtype == "float32" and raw == arr.tobytes()


# ------------------------------------------------------------------ gloo
def _dp_worker(rank, world, B, steps, mode):
    from tdfo_amd.parallel.dist import get_info
    info = get_info()
    cfg = TwoTowerConfig(SM, learning_rate=1e-2)
    strategy = "row_wise" if mode == "ps" else None
    tr = TwoTowerTrainer(cfg, B, "cpu", group=info.group, rank=rank, world_size=world,
                         emb_sharding=strategy)
    for s in range(steps):
        full = make_batch(B * world, 100 + s)
        tr.load_batch({k: v[rank * B:(rank + 1) * B] for k, v in full.items()})
        tr.step()
    loss, auc = tr.pop_metrics()
    tabs = [tr.table_weight(t) for t in range(len(SIZE_KEYS))]
    return {"P": tr.P[:ops.TT_NPARAM].clone(), "tabs": tabs, "loss": loss}


def _single(B, steps):
    cfg = TwoTowerConfig(SM, learning_rate=1e-2)
    tr = TwoTowerTrainer(cfg, B, "cpu")
    for s in range(steps):
        tr.load_batch(make_batch(B, 100 + s))
        tr.step()
    loss, _ = tr.pop_metrics()
    return {"P": tr.P[:ops.TT_NPARAM].clone(),
            "tabs": [tr.emb.table_weight(t).clone() for t in range(len(SIZE_KEYS))], "loss": loss}


@pytest.mark.parametrize("mode", ["dp", "ps"])
def test_two_tower_distributed_matches_single(mode):
    B, steps, world = 32, 4, 2
    ref = _single(B * world, steps)
    outs = run_distributed(_dp_worker, world, B, steps, mode)
    tol = 1e-5    # ps: fp32 pooled rows and gradients end to end (recv_dtype="fp32")
    for o in outs:
        torch.testing.assert_close(o["P"], ref["P"], rtol=tol, atol=tol)
        for a, b in zip(o["tabs"], ref["tabs"]):
            torch.testing.assert_close(a, b, rtol=tol, atol=tol)
        assert abs(o["loss"] - ref["loss"]) < 10 * tol
    if mode == "dp":      # replicas stay identical
        torch.testing.assert_close(outs[0]["P"], outs[1]["P"], rtol=0, atol=0)


@pytest.mark.parametrize("emb_update", ["sparse", "dense"])
def test_mixed_precision_dynamic_scale_skips_non_finite(emb_update):
    """jax-flax/train_dp.py:55-81: a step with non-finite (scaled) gradients
    leaves params AND optimizer state untouched, does not advance Adam's step,
    halves the loss scale; finite steps train and count towards growth."""
    cfg = TwoTowerConfig(SM, learning_rate=5e-3, emb_update=emb_update, mixed_precision=True,
                         growth_interval=3)
    tr = TwoTowerTrainer(cfg, 64, "cpu")
    tr.load_batch(make_batch(64, 1))
    tr.step()
    assert float(tr.dyn_scale[0]) == cfg.init_scale and float(tr.dyn_scale[1]) == 1
    snap = [t.clone() for t in tr._state_tensors()[:6]] + \
        [x.clone() for x in (tr.emb.state1, tr.emb.state2) if x is not None]
    bad = make_batch(64, 2)
    bad["avg_rating"][5] = float("inf")                   # poisons every dense grad
    tr.load_batch(bad)
    tr.step()
    assert float(tr.found_inf[0]) == 1.0
    assert float(tr.dyn_scale[0]) == cfg.init_scale / 2 and float(tr.dyn_scale[1]) == 0
    now = [t for t in tr._state_tensors()[:6]] + \
        [x for x in (tr.emb.state1, tr.emb.state2) if x is not None]
    names = ["P", "M", "V", "hyper", "emb_hyper", "emb.weight", "state1", "state2"]
    for n, a, b in zip(names, snap, now):
        if n in ("hyper", "emb_hyper"):
            assert torch.equal(a[:2], b[:2]), n            # lr + step counter unchanged
        else:
            assert torch.equal(a, b), n
    for i in range(4):                                    # finite again: trains, grows at 3
        tr.load_batch(make_batch(64, 10 + i))
        tr.step()
    assert float(tr.found_inf[0]) == 0.0
    assert float(tr.dyn_scale[0]) == cfg.init_scale       # halved once, doubled once
    assert not torch.equal(tr.P, snap[0])
    assert float(tr.hyper[1]) == 5.0                      # 6 steps, 1 skipped


def test_mixed_precision_matches_fp32_closely():
    """fp16 compute with loss scaling trains like fp32 (same data, 20 steps)."""
    losses = {}
    for mp in (False, True):
        cfg = TwoTowerConfig(SM, learning_rate=5e-3, mixed_precision=mp)
        tr = TwoTowerTrainer(cfg, 128, "cpu")
        for i in range(20):
            tr.load_batch(make_batch(128, 100 + i))
            tr.step()
        losses[mp] = tr.pop_metrics(reduce=False)[0]
    assert abs(losses[True] - losses[False]) < 2e-2 * abs(losses[False])
