"""Pre-flight collective self-test (parallel/preflight.py) and the bench
supervisor's fallback (utils/supervise.py), on CPU over gloo."""
import os

import pytest

from tests.dist_harness import run_distributed


def _pf(rank, world, inject):
    from tdfo_amd.parallel.preflight import preflight
    if inject is not None:
        os.environ["TDFO_PREFLIGHT_INJECT"] = str(inject)
    else:
        os.environ.pop("TDFO_PREFLIGHT_INJECT", None)
    os.environ.pop("TDFO_COMM", None)
    r = preflight(None, "cpu", timeout_s=60)
    r["comm_env"] = os.environ.get("TDFO_COMM")
    return r


@pytest.mark.parametrize("world", [2, 3])
def test_preflight_passes_on_gloo(world):
    res = run_distributed(_pf, world, None)
    for r in range(world):
        assert res[r]["ok"], res[r]
        assert res[r]["failed"] == []
        assert res[r]["comm_env"] is None


def test_preflight_injected_mismatch_sends_every_rank_to_fallback():
    res = run_distributed(_pf, 2, 1)
    assert res[1]["failed"], res[1]
    for r in range(2):
        assert not res[r]["ok"]
        assert res[r]["comm_env"] == "torch"


def test_case_expectations_are_consistent_single_rank():
    # W = 1: every collective is the identity / own chunk
    import torch

    from tdfo_amd.parallel.preflight import CASES, make_case
    for kind, dtype, n in CASES:
        out, exp, _ = make_case(kind, dtype, n, 1, 0, torch.device("cpu"), 0)
        if kind in ("ar", "armax"):
            assert torch.equal(out, exp)
        assert exp.dtype == dtype
