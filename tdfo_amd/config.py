"""Typed superset configuration (reference: jax-flax/utils.py:10-33,
tensorflow2/utils.py:10-38, torchrec/utils.py:8-34 and their config.toml).

Every key of the three reference ``config.toml`` files is accepted verbatim
(same names, same meaning), plus optional keys for the new workloads
(``model``, DLRM/DCN arch keys, ``[sharding]``, ``[synthetic]``...). Like the
reference's ``Config(**config)``, unknown keys are rejected (typos fail
loudly). ``size_map.json`` / ``size_map_bert4rec.json`` written by the ETL are
merged in as ``size_map`` (jax-flax/utils.py:31-32, torchrec/train.py:221-222).
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence

try:
    import tomllib as _toml  # py3.11+
except ModuleNotFoundError:  # pragma: no cover - py3.10
    import tomli as _toml


@dataclass
class ShardingConfig:
    strategy: str = "auto"            # auto | table_wise | row_wise | column_wise | data_parallel
    #                                   | replicated
    hbm_gb: float = 288.0
    reserve_frac: float = 0.15
    dp_max_mb: float = 0.0


@dataclass
class SyntheticConfig:
    enabled: bool = False
    rows: str = "tiny"                # tiny | kaggle | 1tb | gt1tb | list given in table_rows
    dist: str = "uniform"             # uniform | zipf
    zipf_alpha: float = 1.05
    num_batches: int = 100
    host_data: bool = False           # GPU: C++ host generator -> pinned -> copy-stream H2D


@dataclass
class Config:
    # ---- common reference keys
    data_dir: Path = Path("data/goodreads")
    train_data: str = "train_part_*.parquet"
    eval_data: str = "eval_part_*.parquet"
    n_epochs: int = 10
    learning_rate: float = 3e-4
    weight_decay: float = 1e-4
    embed_dim: int = 16
    per_device_train_batch_size: int = 2048
    per_device_eval_batch_size: int = 2048
    seed: int = 42
    # jax-flax
    streaming: bool = True
    mixed_precision: bool = False
    # tensorflow2
    write_format: str = "parquet"
    num_workers: int = 2
    steps_per_execution: int = 1
    jit_xla: Optional[bool] = None
    use_tpu: bool = False
    # torchrec (Bert4Rec)
    n_heads: int = 2
    n_layers: int = 2
    max_len: int = 20
    sliding_step: int = 10
    mask_prob: float = 0.2
    model_parallel: bool = False
    # derived
    size_map: Dict[str, int] = field(default_factory=dict)
    # ---- new (optional) keys
    model: str = "two_tower"          # two_tower | bert4rec | dlrm | dcnv2
    dtype: str = "bf16"               # compute dtype on GPU
    num_dense: int = 13
    table_rows: List[int] = field(default_factory=list)
    pooling: List[int] = field(default_factory=list)
    bottom_mlp: List[int] = field(default_factory=lambda: [512, 256, 128])
    top_mlp: List[int] = field(default_factory=lambda: [1024, 1024, 512, 256, 1])
    dcn_layers: int = 3
    dcn_rank: int = 512
    emb_optimizer: str = "rowwise_adagrad"
    emb_learning_rate: float = 0.01
    dense_optimizer: str = "adamw"
    hip_graph: bool = True
    emb_update: str = "sparse"        # two_tower: sparse (fused row Adam) | dense (optax parity)
    tower_init: str = ""              # two_tower: flax | keras ("" = by entrypoint flavor)
    data_on_device: bool = True       # keep processed splits resident in HBM
    log_every: int = 100
    eval_every: int = 0
    ckpt_dir: str = ""
    ckpt_every: int = 0
    resume: bool = False
    metrics_file: str = ""
    max_steps: int = 0
    profile_steps: str = ""           # "START:COUNT" -> roctx profile_window (§5.1)
    debug_checks: bool = False        # embedding id bounds checks on every lookup (§5.2)
    sharding: ShardingConfig = field(default_factory=ShardingConfig)
    synthetic: SyntheticConfig = field(default_factory=SyntheticConfig)

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        d["data_dir"] = str(self.data_dir)
        return d


_NESTED = {"sharding": ShardingConfig, "synthetic": SyntheticConfig}


def _coerce(name: str, value: Any, cur: Any) -> Any:
    """Coerce a CLI override string to the type of the current value."""
    if not isinstance(value, str):
        return value
    if isinstance(cur, bool) or cur is None and value.lower() in ("true", "false"):
        return value.lower() in ("1", "true", "yes", "on")
    if isinstance(cur, int):
        return int(value)
    if isinstance(cur, float):
        return float(value)
    if isinstance(cur, list):
        return [int(x) for x in value.split(",") if x]
    if isinstance(cur, Path):
        return Path(value)
    return value


def from_dict(raw: Dict[str, Any]) -> Config:
    raw = dict(raw)
    known = {f.name for f in dataclasses.fields(Config)}
    unknown = sorted(set(raw) - known)
    if unknown:
        raise TypeError(f"unknown config keys: {unknown}")
    for key, cls in _NESTED.items():
        if key in raw and isinstance(raw[key], dict):
            sub_known = {f.name for f in dataclasses.fields(cls)}
            bad = sorted(set(raw[key]) - sub_known)
            if bad:
                raise TypeError(f"unknown [{key}] keys: {bad}")
            raw[key] = cls(**raw[key])
    if "data_dir" in raw:
        raw["data_dir"] = Path(raw["data_dir"])
    cfg = Config(**raw)
    validate(cfg)
    return cfg


def validate(cfg: Config) -> None:
    if cfg.write_format not in ("tfrecord", "parquet"):       # tensorflow2/utils.py:37
        raise ValueError(f"write_format must be tfrecord|parquet, got {cfg.write_format!r}")
    if cfg.max_len < cfg.sliding_step:                          # torchrec/utils.py:33
        raise ValueError("max_len must be >= sliding_step")
    if cfg.embed_dim <= 0 or cfg.per_device_train_batch_size <= 0:
        raise ValueError("embed_dim and batch sizes must be positive")
    if cfg.model not in ("two_tower", "bert4rec", "dlrm", "dcnv2"):
        raise ValueError(f"unknown model {cfg.model!r}")
    if cfg.n_heads <= 0 or cfg.embed_dim % cfg.n_heads:          # torchrec/models.py:40
        raise ValueError("embed_dim must be divisible by n_heads")


def read_configs(path: Optional[Path | str] = None, overrides: Sequence[str] = (),
                 size_map: bool = True) -> Config:
    """Load ``config.toml`` (default: next to the calling script's cwd)."""
    path = Path(path) if path is not None else Path("config.toml")
    raw = _toml.loads(path.read_text())
    cfg = from_dict(raw)
    cfg = apply_overrides(cfg, overrides)
    if not cfg.data_dir.is_absolute():
        base = path.resolve().parent
        cand = (base / cfg.data_dir)
        cfg.data_dir = cand if cand.exists() or not cfg.data_dir.exists() else cfg.data_dir.absolute()
    if size_map:
        for name in ("size_map.json", "size_map_bert4rec.json"):
            fname = "size_map_bert4rec.json" if cfg.model == "bert4rec" else "size_map.json"
            if name != fname:
                continue
            p = cfg.data_dir / name
            if p.exists():
                cfg.size_map = json.loads(p.read_text())
    return cfg


def apply_overrides(cfg: Config, overrides: Sequence[str]) -> Config:
    """``key=value`` / ``section.key=value`` overrides (benchmarking CLI)."""
    for ov in overrides:
        if "=" not in ov:
            raise ValueError(f"override must be key=value: {ov!r}")
        key, value = ov.split("=", 1)
        if "." in key:
            sec, sub = key.split(".", 1)
            obj = getattr(cfg, sec)
            if not hasattr(obj, sub):
                raise TypeError(f"unknown config key {key!r}")
            setattr(obj, sub, _coerce(sub, value, getattr(obj, sub)))
        else:
            if not hasattr(cfg, key):
                raise TypeError(f"unknown config key {key!r}")
            setattr(cfg, key, _coerce(key, value, getattr(cfg, key)))
    validate(cfg)
    return cfg


def read_cluster(path: Path | str) -> Dict[str, Any]:
    """tensorflow2/cluster.json: only the topology size is used (the PS path
    runs as in-node sharded embeddings, tensorflow2/train_ps.py:44-53)."""
    d = json.loads(Path(path).read_text())
    cl = d.get("cluster", {})
    return {"num_workers": len(cl.get("worker", [])), "num_ps": len(cl.get("ps", [])),
            "task": d.get("task", {})}
