import pytest

from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, DLRMConfig
from tdfo_amd.sparse.planner import GiB, plan_sharding
from tdfo_amd.sparse.tables import EmbOptimConfig


def test_plan_1tb_fits_one_gpu():
    cfg = DLRMConfig()
    p = plan_sharding(cfg.tables(), 1, EmbOptimConfig("rowwise_adagrad"))
    assert all(s.kind == "table_wise" for s in p.shards)
    assert 90 < p.mem_bytes[0] / GiB < 100


@pytest.mark.parametrize("world", [2, 4, 8])
def test_plan_1tb_tw_balanced(world):
    cfg = DLRMConfig()
    p = plan_sharding(cfg.tables(), world, EmbOptimConfig("rowwise_adagrad"))
    counts = [len(p.tables_on(r)) for r in range(world)]
    assert sum(counts) == 26
    assert max(counts) - min(counts) <= 1
    assert p == plan_sharding(cfg.tables(), world, EmbOptimConfig("rowwise_adagrad"))


def test_plan_row_wise_fallback_when_too_big():
    rows = [x * 12 for x in CRITEO_1TB_ROWS]   # ~1.15 TB fp32
    cfg = DLRMConfig(table_rows=rows)
    p = plan_sharding(cfg.tables(), 8, EmbOptimConfig("rowwise_adagrad"))
    assert "row_wise" in p.summary()["kinds"]
    assert max(p.mem_bytes) <= 288e9 * 0.85
    with pytest.raises(MemoryError):
        plan_sharding(cfg.tables(), 1, EmbOptimConfig("rowwise_adagrad"))


def test_plan_adam_state_counts():
    cfg = DLRMConfig()
    p = plan_sharding(cfg.tables(), 8, EmbOptimConfig("adam"))
    tot = sum(p.mem_bytes)
    assert tot > 2.9 * sum(t.bytes_fp32 for t in cfg.tables())
