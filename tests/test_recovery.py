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
