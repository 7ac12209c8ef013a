"""TwoTower training driver behind the reference-compatible entrypoints.

  mode "single": jax-flax/train.py:95-164, tensorflow2/train.py:22-57
  mode "dp"    : jax-flax/train_dp.py:144-247, tensorflow2/train_dp.py:107-188
                 (one process per GPU, RCCL; per-device batch x world = global)
  mode "ps"    : tensorflow2/train_ps.py:125-165 — parameter servers become
                 sharded embedding tables in HBM (all-to-all over xGMI); the
                 ckpt/ backup/ log/ directories are kept (ModelCheckpoint,
                 BackupAndRestore and TensorBoard equivalents).

Log lines follow the reference formats; every epoch also
appends a JSON line to ``metrics_file`` (or ``log/metrics.jsonl`` for ps).
"""
from __future__ import annotations

import json
import math
import os
import time
from pathlib import Path
from typing import Dict, List, Optional

import torch

from ..config import Config
from ..data.columnar import DeviceColumns
from ..data import goodreads as G
from ..models.two_tower import TwoTowerConfig, TwoTowerTrainer
from ..parallel.dist import init_distributed
from ..utils import checkpoint as ckpt
from ..utils import guarded

TRAIN_DTYPES = {"label": torch.float32, "avg_rating": torch.float32, "num_pages": torch.float32}
ID_COLS = ["user_id", "item_id", "language", "is_ebook", "format", "publisher", "pub_decade"]


def _load_split(cfg: Config, which: str) -> Dict:
    pattern = cfg.train_data if which == "train" else cfg.eval_data
    if cfg.write_format == "tfrecord" or pattern.endswith(".tfrecord"):
        cols = G.read_tfrecord_columns(str(cfg.data_dir / "tfrecord" / pattern))
    else:
        cols = G.read_parquet_columns(str(cfg.data_dir / "parquet" / pattern))
    keep = ID_COLS + ["avg_rating", "num_pages", "label"]
    return {k: cols[k] for k in keep}


def _columns(cfg: Config, which: str, data_dev) -> DeviceColumns:
    """A split's columns on ``data_dev``. ``streaming`` (parquet): read in
    bounded chunks straight into the preallocated columns; otherwise the
    split is read whole on the host first (the reference's in-memory
    loader)."""
    pattern = cfg.train_data if which == "train" else cfg.eval_data
    if cfg.streaming and not (cfg.write_format == "tfrecord" or pattern.endswith(".tfrecord")):
        keep = ID_COLS + ["avg_rating", "num_pages", "label"]
        return DeviceColumns.from_parquet_stream(str(cfg.data_dir / "parquet" / pattern),
                                                 data_dev, keep, _dtypes())
    return DeviceColumns(_load_split(cfg, which), data_dev, _dtypes())


def _dtypes():
    d = dict(TRAIN_DTYPES)
    d.update({k: torch.int64 for k in ID_COLS})
    return d


def _log(line: str, rank: int):
    if rank == 0:
        print(line, flush=True)


def run(cfg: Config, mode: str = "single", flavor: str = "flax", out_dir: str = ".",
        device: Optional[str] = None) -> List[Dict]:
    if cfg.use_tpu:
        raise ValueError("use_tpu: TPUs are not a target of this framework (MI355X only)")
    if not cfg.size_map:
        raise FileNotFoundError(f"{cfg.data_dir}/size_map.json missing: run preprocessing first")
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    info = init_distributed(device) if mode in ("dp", "ps") else None
    if info is not None:
        guarded.rank_preflight(info)     # W > 1: collective self-test, c10d on mismatch
    rank = info.rank if info else 0
    world = info.world_size if info else 1
    dev = info.device if info else torch.device(device if device != "cuda" else "cuda:0")
    group = info.group if info else None
    out = Path(out_dir)

    data_dev = dev if cfg.data_on_device else torch.device("cpu")
    train, evald = _columns(cfg, "train", data_dev), _columns(cfg, "eval", data_dev)
    n_train, n_eval = len(train), len(evald)
    _log(f"===== train size: {n_train:,}, eval size: {n_eval:,} =====", rank)
    if mode != "single":
        _log(f"===== num devices: {world} =====\n", rank)

    B, EB = cfg.per_device_train_batch_size, cfg.per_device_eval_batch_size
    init = cfg.tower_init or ("keras" if flavor == "keras" else "flax")
    # mixed_precision is a train_dp.py key in the reference (jax-flax/config.toml:12,
    # jax-flax/train_dp.py:170-177); the other entrypoints train in fp32
    tcfg = TwoTowerConfig(dict(cfg.size_map), cfg.embed_dim, cfg.learning_rate, cfg.weight_decay,
                          init=init, emb_update=cfg.emb_update, seed=cfg.seed,
                          mixed_precision=bool(cfg.mixed_precision) and mode == "dp")
    strategy = None
    if mode == "ps":
        strategy = cfg.sharding.strategy if cfg.sharding.strategy != "auto" else "row_wise"
    tr = TwoTowerTrainer(tcfg, B, dev, group=group, rank=rank, world_size=world,
                         eval_batch_size=EB if mode != "ps" else B, emb_sharding=strategy)
    if mode == "ps":
        EB = B       # the sharded engine has one static batch shape
    drop_last = mode != "single"
    start_epoch = 1
    backup = out / "backup"
    # ps: BackupAndRestore semantics (restored whenever present); dp at W > 1
    # keeps the same per-epoch backup/, restored when resume is requested
    # (the supervisor's fallback attempt, utils/guarded.py)
    keep_backup = mode == "ps" or (mode == "dp" and world > 1)
    if mode == "ps":
        for d in ("ckpt", "backup", "log"):
            (out / d).mkdir(parents=True, exist_ok=True)
    if keep_backup and (mode == "ps" or guarded.resume_requested(cfg.resume)):
        man = ckpt.load_manifest(str(backup))
        if man is not None and man["world_size"] == world:
            st = ckpt.load_sharded(str(backup), rank, world)
            tr.load_state_dict({k: v.to(dev) for k, v in st["tensors"].items()})
            start_epoch = int(st["meta"]["epoch"]) + 1
            _log(f"===== restored from backup: resuming at epoch {start_epoch} =====", rank)
    metrics_path = cfg.metrics_file or (str(out / "log" / "metrics.jsonl") if mode == "ps" else "")
    history: List[Dict] = []
    # jit_xla (tensorflow2/train.py:16, train_dp.py:76): false = eager kernel
    # launches, no hipGraph (the XLA-compiled step's counterpart)
    use_graph = (cfg.hip_graph and cfg.jit_xla is not False and dev.type == "cuda"
                 and mode == "single")
    k_exec = max(1, int(cfg.steps_per_execution))
    for epoch in range(start_epoch, cfg.n_epochs + 1):
        t0 = time.perf_counter()
        steps = 0
        pend: List[torch.Tensor] = []          # full batches waiting for a k-step execution
        # HBM-resident columns: one gather launch per batch straight into the
        # trainer's static buffers; host-resident columns: per-column H2D
        for idx, s, n in train.batch_slices(B, shuffle=True, seed=cfg.seed, epoch=epoch,
                                            drop_last=drop_last, rank=rank, world_size=world):
            if (k_exec > 1 and use_graph and tr.graph is not None and train.device == dev
                    and idx is not None and n == B
                    and not (cfg.max_steps and steps + len(pend) + 1 > cfg.max_steps)):
                if getattr(tr, "_exec_graph", None) is None:
                    tr.capture_execution(train.cols, k_exec)
                pend.append(idx)
                if len(pend) == k_exec:
                    tr.run_execution(pend)
                    steps += k_exec
                    pend = []
                continue
            for ix in pend:                    # a partial execution: one step at a time
                tr.load_columns(train.cols, ix, 0, B)
                tr.step()
                steps += 1
            pend = []
            if train.device == dev:
                b = tr.load_columns(train.cols, idx, s, n)
            else:
                cols = {k: (v[s: s + n] if idx is None else v.index_select(0, idx.cpu()))
                        for k, v in train.cols.items()}
                b = tr.load_batch({k: v.to(dev, non_blocking=True) for k, v in cols.items()})
            if b == 0:
                continue
            tr.step()
            steps += 1
            if use_graph and tr.graph is None and b == B and steps >= 2:
                tr.capture_graph()
            if cfg.max_steps and steps >= cfg.max_steps:
                break
        for ix in pend:
            tr.load_columns(train.cols, ix, 0, B)
            tr.step()
            steps += 1
        if dev.type == "cuda":
            torch.cuda.synchronize()
        el = time.perf_counter() - t0
        tr_loss, tr_auc = tr.pop_metrics()
        ex_s = steps * B * world / max(el, 1e-9)
        if flavor == "keras":
            _log(f"Epoch {epoch} train loss: {tr_loss:.4f}, train auc: {tr_auc:.4f}", rank)
        elif mode == "single":
            _log(f"\nEpoch {epoch} train loss: {tr_loss:.4f}", rank)
        else:
            _log(f"\nEpoch {epoch} train loss: {tr_loss:.4f}, roc_auc: {tr_auc:.4f}", rank)
        for idx, s, n in evald.batch_slices(EB, shuffle=False, drop_last=False, rank=rank,
                                            world_size=world):
            if n == 0 and tr.sharded is None:
                continue
            if evald.device == dev:
                tr.load_columns(evald.cols, idx, s, n, eval_mode=True)
            else:
                tr.load_batch({k: v[s: s + n].to(dev, non_blocking=True)
                               for k, v in evald.cols.items()}, eval_mode=True)
            tr.evaluate_batch()
        ev_loss, ev_auc = tr.pop_metrics(eval_mode=True)
        if flavor == "keras":
            _log(f"Epoch {epoch} eval loss: {ev_loss:.4f}, eval auc: {ev_auc:.4f}", rank)
        elif mode == "single":
            _log(f"\nEpoch {epoch} eval loss: {ev_loss:.4f}", rank)
        else:
            _log(f"\nEpoch {epoch} eval loss: {ev_loss:.4f}, roc_auc: {ev_auc:.4f}", rank)
        rec = {"epoch": epoch, "train_loss": tr_loss, "train_auc": tr_auc, "eval_loss": ev_loss,
               "eval_auc": ev_auc, "steps": steps, "examples_per_sec": ex_s, "world_size": world}
        history.append(rec)
        _log(f"[throughput] epoch {epoch}: {ex_s:,.0f} examples/s over {world} device(s)", rank)
        if metrics_path and rank == 0:
            Path(metrics_path).parent.mkdir(parents=True, exist_ok=True)
            with open(metrics_path, "a") as f:
                f.write(json.dumps(rec) + "\n")
        if keep_backup:
            state = {k: v for k, v in tr.state_dict().items()}
            bar = (lambda: torch.distributed.barrier()) if world > 1 else None
            if mode == "ps":
                ckpt.save_sharded(str(out / "ckpt" / f"epoch_{epoch}"), rank, world, epoch,
                                  state, {"epoch": epoch}, barrier=bar)
            ckpt.save_sharded(str(backup), rank, world, epoch, state, {"epoch": epoch},
                              barrier=bar)
    params = tr.flax_params()
    if rank == 0 and flavor == "flax":
        ckpt.save_flax_params(params, str(out / "model_params.pt"))
    if keep_backup and rank == 0:
        # training finished: BackupAndRestore deletes its backup on success
        for f in backup.glob("*"):
            f.unlink()
    if info is not None and world > 1:
        torch.distributed.barrier()
    return history
