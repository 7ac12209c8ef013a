"""The DLRM recipe loop (train/dlrm.py on train/loop.py) runs the step that
bench.py measures: input-dist pipelining at W > 1, steps_per_execution
rounds, eval in the middle of a pipelined run, and the same batch stream as
the unpipelined single-process loop."""
import math

import pytest
import torch

from tdfo_amd.config import from_dict
from tests.dist_harness import run_distributed

BASE = {"model": "dlrm", "embed_dim": 16, "per_device_train_batch_size": 16,
        "bottom_mlp": [32, 16], "top_mlp": [32, 1], "table_rows": [300, 40, 500, 70, 9],
        "learning_rate": 1e-2, "emb_learning_rate": 0.05, "log_every": 4, "max_steps": 12,
        "synthetic": {"enabled": True}}


def _worker(rank, world, overrides, mode):
    from tdfo_amd.train.dlrm import run
    cfg = from_dict({**BASE, **overrides})
    out = run(cfg, mode=mode, device="cpu")
    tr = out["trainer"]
    st = {k: v.detach().clone() for k, v in tr.flat_state().items()}
    return tr.pipeline, [h["train_loss"] for h in out["history"]], \
        [h.get("eval_auc") for h in out["history"]], st


@pytest.mark.parametrize("mode", ["ps", "dp"])
def test_recipe_is_pipelined_at_two_ranks(mode):
    """train_ps.py / train_dp.py at W=2 run the pipelined step (prime +
    set_next_batch), with an eval in the middle that must not disturb the
    batch in flight: same parameters as the run without eval."""
    res = run_distributed(_worker, 2, {"eval_every": 4}, mode)
    ref = run_distributed(_worker, 2, {}, mode)
    for r in range(2):
        piped, losses, aucs, st = res[r]
        assert piped and len(losses) == 3 and all(math.isfinite(x) for x in losses)
        assert all(a is not None for a in aucs)
        for k, v in ref[r][3].items():
            assert torch.equal(st[k], v), (r, k)


@pytest.mark.parametrize("k", [3, 5])
def test_steps_per_execution_is_exact(k):
    """steps_per_execution=k issues k steps per host round (log and
    checkpoint boundaries still honoured): same parameters and logged losses
    as k=1, one process and two."""
    for world, mode in ((1, "single"), (2, "ps")):
        a = run_distributed(_worker, world, {"steps_per_execution": k}, mode)
        b = run_distributed(_worker, world, {}, mode)
        for r in range(world):
            assert a[r][1] == b[r][1]
            for key, v in b[r][3].items():
                assert torch.equal(a[r][3][key], v), (world, r, key)


def test_jit_xla_false_means_eager(monkeypatch):
    """jit_xla = false (tensorflow2 config key) turns hipGraph capture off;
    on CPU nothing is captured either way and training proceeds."""
    res = run_distributed(_worker, 1, {"jit_xla": False, "max_steps": 4}, "single")
    assert len(res[0][1]) == 1 and math.isfinite(res[0][1][0])
