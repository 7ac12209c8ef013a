"""Failure detection + checkpoint/resume: a rank is killed
mid-training (fault injection), the job is detected as failed, and a resumed
run from the last sharded checkpoint ends bit-identical to an uninterrupted
run. Also: the non-finite-loss guard and the manifest/world-size checks."""
import math

import pytest
import torch

from tdfo_amd.config import from_dict
from tdfo_amd.utils import checkpoint as ckpt
from tests.dist_harness import run_distributed

BASE = {"model": "dlrm", "embed_dim": 16, "per_device_train_batch_size": 32,
        "bottom_mlp": [32, 16], "top_mlp": [32, 1], "table_rows": [300, 40, 500, 70],
        "learning_rate": 1e-2, "emb_learning_rate": 0.05, "log_every": 5, "max_steps": 10,
        "synthetic": {"enabled": True}}


def _worker(rank, world, overrides, strategy_mode):
    from tdfo_amd.train.dlrm import run
    cfg = from_dict({**BASE, **overrides})
    out = run(cfg, mode=strategy_mode, device="cpu")
    st = out["trainer"].flat_state()
    return {k: v.detach().clone() for k, v in st.items()}


@pytest.mark.parametrize("mode", ["ps", "dp"])
def test_kill_rank_then_resume_matches_uninterrupted(tmp_path, monkeypatch, mode):
    world = 2
    ref = run_distributed(_worker, world, {}, mode)
    ck = str(tmp_path / "ck")
    monkeypatch.setenv("TDFO_FAULT_AT_STEP", "7")
    monkeypatch.setenv("TDFO_FAULT_RANK", "1")
    with pytest.raises((RuntimeError, TimeoutError)):
        run_distributed(_worker, world, {"ckpt_dir": ck, "ckpt_every": 4}, mode, timeout=120)
    monkeypatch.delenv("TDFO_FAULT_AT_STEP")
    man = ckpt.load_manifest(ck + "/step_4")
    assert man is not None and man["step"] == 4 and man["world_size"] == world
    res = run_distributed(_worker, world, {"ckpt_dir": ck, "ckpt_every": 4, "resume": True},
                          mode)
    for r in range(world):
        for k, v in ref[r].items():
            assert torch.equal(res[r][k], v), (r, k)


def test_resume_rejects_other_world_size(tmp_path):
    d = str(tmp_path / "c")
    ckpt.save_sharded(d, 0, 1, 3, {"x": torch.ones(2)}, {"model": "dlrm"})
    with pytest.raises(ValueError):
        ckpt.load_sharded(d, 0, 2)
    with pytest.raises(ValueError):
        ckpt.load_sharded(d, 0, 1, expect_meta={"model": "dcnv2"})
    assert ckpt.load_sharded(d, 0, 1)["step"] == 3


def test_non_finite_loss_halts():
    from tdfo_amd.train.dlrm import run
    cfg = from_dict({**BASE, "learning_rate": 1e30, "emb_learning_rate": 1e30, "max_steps": 10})
    with pytest.raises(FloatingPointError):
        run(cfg, mode="single", device="cpu")


def _ckpt_worker(rank, world, path, strategy, action, chunk_bytes):
    """Train a few steps and save (action "save"), or build a fresh trainer
    under a different world size / plan and load (action "load"); return the
    full tables (assembled from this rank's pieces) + dense state."""
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    from tdfo_amd.parallel.dist import get_info
    from tdfo_amd.utils import sharded_ckpt

    rows = [300, 40, 500, 70, 9]
    cfg = DLRMConfig(embedding_dim=16, table_rows=rows, bottom=[32, 16], top=[32, 1],
                     pooling=[1, 2, 1, 1, 1], sharding=strategy,
                     emb_opt="adagrad" if strategy == "column_wise" else "rowwise_adagrad")
    g = get_info()
    tr = DLRMTrainer(cfg, 8, "cpu", group=g.group, rank=rank, world_size=world)
    bar = (lambda: torch.distributed.barrier()) if world > 1 else None
    if action == "save":
        data = SyntheticCriteo(rows, 8, pooling=cfg.pooling, seed=3, rank=rank)
        for _ in range(3):
            tr.load_batch(*data.next())
            tr.step()
        sharded_ckpt.save(tr, path, 3, rank, world, {"model": "dlrm"}, barrier=bar,
                          chunk_bytes=chunk_bytes)
    else:
        assert sharded_ckpt.load(tr, path, rank, world, expect_meta={"model": "dlrm"},
                                 chunk_bytes=chunk_bytes) == 3
    out = {"dense": {k: v.clone() for k, v in tr.dense_state().items()}, "pieces": []}
    for p in sharded_ckpt.local_pieces(tr.emb):
        out["pieces"].append((p["table"], p["lo"], p["step"], p["c0"], p["weight"].clone(),
                              p["states"]["state1"].clone()))
    return out


def _assemble(res, rows, D=16):
    full = {t: torch.full((r, D), float("nan")) for t, r in enumerate(rows)}
    st = {t: torch.full((r, D), float("nan")) for t, r in enumerate(rows)}
    for r in res:
        for t, lo, step, c0, w, s1 in r["pieces"]:
            # (round-robin row-wise shards: rows lo, lo + step, ...)
            full[t][lo::step][: w.shape[0], c0:c0 + w.shape[1]] = w
            st[t][lo::step][: w.shape[0], c0:c0 + w.shape[1]] = (s1[:, None] if s1.dim() == 1
                                                                 else s1)
    return full, st


@pytest.mark.parametrize("save_w,save_s,load_w,load_s", [
    (2, "table_wise", 3, "table_wise"), (2, "row_wise", 3, "row_wise"),
    (2, "row_wise", 1, "table_wise"), (3, "auto", 2, "row_wise"),
    (2, "column_wise", 3, "column_wise")])
def test_sharded_checkpoint_reshards(tmp_path, save_w, save_s, load_w, load_s):
    """Save at world W (one plan), load at world W' (another plan): every table
    row, every optimizer state and the dense state survive; pieces are
    streamed in tiny chunks (64 B) to exercise the bounded-memory path."""
    rows = [300, 40, 500, 70, 9]
    path = str(tmp_path / "ck")
    a = run_distributed(_ckpt_worker, save_w, path, save_s, "save", 64)
    b = run_distributed(_ckpt_worker, load_w, path, load_s, "load", 64)
    (fa, sa), (fb, sb) = _assemble(a, rows), _assemble(b, rows)
    for t in range(len(rows)):
        assert not torch.isnan(fb[t]).any(), t
        assert torch.equal(fa[t], fb[t]), t
        assert torch.equal(sa[t], sb[t]), t            # optimizer state too
    for k, v in a[0]["dense"].items():
        assert torch.equal(v, b[0]["dense"][k]), k
    man = ckpt.load_manifest(path)
    assert man["format"] == "tdfo-sharded-v2" and man["world_size"] == save_w
