"""DLRM / DCN-v2 training driver (north-star workloads, BASELINE.json configs 1-5).

Entry points (recipes/dlrm):
  train.py     single process (CPU: DLRM-tiny, config 1; one GPU: config 2)
  train_dp.py  one process per GPU, replicated tables (``data_parallel``
               sharding: local lookups, row-gradient all-gather) + dense
               all-reduce over RCCL (config 3)
  train_ps.py  the parameter-server entry point of the reference collapsed
               into the sharded engine: table-wise / row-wise shards with
               all-to-all over xGMI (configs 4-5)

Training loop services: JSONL metrics + stdout log lines,
examples/s throughput, held-out synthetic eval (loss + bucketed ROC-AUC),
non-finite loss detection (halt with a clear error), sharded checkpoints
(one file per rank + manifest, atomically completed) and resume, and a
fault-injection hook (``TDFO_FAULT_AT_STEP``) used by the recovery tests.
"""
from __future__ import annotations

import json
import math
import os
import time
from pathlib import Path
from typing import Dict, List, Optional

import torch

from .. import ops
from ..config import Config
from ..data.synthetic import HostSyntheticCriteo, SyntheticCriteo
from ..models.dlrm import (CRITEO_1TB_ROWS, CRITEO_KAGGLE_ROWS, DCN_GT1TB_ROWS, MLPERF_MULTIHOT,
                           DLRMConfig, DLRMTrainer)
from ..parallel.dist import init_distributed
from ..sparse import tables as _tables
from ..utils import checkpoint as ckpt
from ..utils import sharded_ckpt
from ..utils.profiling import ProfileWindow, StepTimer, trace_range

TINY_ROWS = [40_000] * 26          # DLRM-tiny: ~1M embedding rows (BASELINE config 1)


def table_rows(cfg: Config) -> List[int]:
    if cfg.table_rows:
        return list(cfg.table_rows)
    return {"tiny": TINY_ROWS, "kaggle": CRITEO_KAGGLE_ROWS, "1tb": CRITEO_1TB_ROWS,
            "gt1tb": DCN_GT1TB_ROWS}[cfg.synthetic.rows]


def dlrm_config(cfg: Config, strategy: str) -> DLRMConfig:
    dcn = cfg.model == "dcnv2"
    pooling = list(cfg.pooling) if cfg.pooling else (list(MLPERF_MULTIHOT) if dcn else None)
    return DLRMConfig(num_dense=cfg.num_dense, embedding_dim=cfg.embed_dim,
                      table_rows=table_rows(cfg), pooling=pooling, bottom=list(cfg.bottom_mlp),
                      top=list(cfg.top_mlp), interaction="dcn" if dcn else "dot",
                      dcn_layers=cfg.dcn_layers, dcn_rank=cfg.dcn_rank,
                      dense_opt=cfg.dense_optimizer, dense_lr=cfg.learning_rate,
                      dense_wd=cfg.weight_decay, emb_opt=cfg.emb_optimizer,
                      emb_lr=cfg.emb_learning_rate, sharding=strategy, seed=cfg.seed)


class _Data:
    """Per-rank synthetic batch stream; batch i is reproducible after resume.

    CPU: the C++ host generator. GPU: the device generator, or with
    ``synthetic.host_data`` the C++ generator behind the pinned, copy-stream
    prefetcher (data/prefetch.py) -- the host data plane a real input
    pipeline would use."""

    def __init__(self, cfg: Config, dcfg: DLRMConfig, B: int, device, rank: int, seed_off: int,
                 prefetch: bool = True):
        self.host = device.type == "cpu"
        self.pf = None
        kw = dict(pooling=dcfg.pooling_factors(), seed=cfg.seed, rank=rank,
                  dist=cfg.synthetic.dist, stream=seed_off)
        self._args = (cfg, dcfg, B, device, kw)
        if self.host:
            self.gen = HostSyntheticCriteo(dcfg.table_rows, B, dcfg.num_dense,
                                           zipf_alpha=cfg.synthetic.zipf_alpha, threads=4, **kw)
        elif cfg.synthetic.host_data and prefetch:
            self.pf = self._prefetcher(0)
        else:
            self.gen = SyntheticCriteo(dcfg.table_rows, B, dcfg.num_dense, device=device,
                                       zipf_alpha=cfg.synthetic.zipf_alpha, **kw)
        self.device = device
        self.i = 0
        self._slot = None

    def _prefetcher(self, start: int):
        from ..data.prefetch import host_prefetcher
        cfg, dcfg, B, device, kw = self._args
        return host_prefetcher(dcfg.table_rows, B, device, num_dense=dcfg.num_dense,
                               zipf_alpha=cfg.synthetic.zipf_alpha, start=start, **kw)

    def seek(self, i: int):
        if self.pf is not None:
            self.pf.close()
            self.pf = self._prefetcher(i)
        elif self.host:
            self.gen.index = i
        else:                  # device generator: replay the stream
            for _ in range(i - self.i):
                self.gen.next()
        self.i = i

    def next(self):
        self.i += 1
        if self.pf is not None:
            if self._slot is not None:
                self.pf.release(self._slot)       # previous batch was consumed
            batch, self._slot = self.pf.next()
            return batch
        return self.gen.next()


def _log(rank, msg):
    if rank == 0:
        print(msg, flush=True)


def run(cfg: Config, mode: str = "single", out_dir: str = ".",
        device: Optional[str] = None) -> Dict:
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    info = init_distributed(device)
    rank, world, dev, group = info.rank, info.world_size, info.device, info.group
    if cfg.debug_checks:
        _tables.set_debug_checks(True)
    if mode == "single" and world > 1:
        raise ValueError("train.py is single-process; use train_dp.py / train_ps.py for >1 rank")
    if mode == "dp":
        strategy = "data_parallel"
    elif mode == "ps":
        strategy = cfg.sharding.strategy if cfg.sharding.strategy != "data_parallel" else "auto"
    else:
        strategy = cfg.sharding.strategy
    dcfg = dlrm_config(cfg, strategy)
    B = cfg.per_device_train_batch_size
    tr = DLRMTrainer(dcfg, B, dev, group=group, rank=rank, world_size=world)
    _log(rank, f"===== model: {cfg.model}, tables: {dcfg.num_tables} "
               f"({sum(dcfg.table_rows):,} rows x {dcfg.embedding_dim}), "
               f"per-device batch {B}, num devices: {world} =====")
    _log(rank, f"===== sharding plan: {json.dumps(tr.plan.summary())} =====")
    data = _Data(cfg, dcfg, B, dev, rank, 0)
    total_steps = cfg.max_steps or cfg.synthetic.num_batches * cfg.n_epochs
    start = 0
    meta = {"model": cfg.model, "world_size": world, "strategy": strategy,
            "tables": len(dcfg.table_rows), "dim": dcfg.embedding_dim}
    if cfg.resume and cfg.ckpt_dir:
        latest = _latest(cfg.ckpt_dir)
        if latest is not None:
            if sharded_ckpt.is_v2(str(latest)):        # streamed, reshardable
                start = sharded_ckpt.load(tr, str(latest), rank, world, expect_meta=meta)
            else:                                       # legacy per-rank files (same plan)
                st = ckpt.load_sharded(str(latest), rank, world, expect_meta=meta)
                tr.load_flat_state(st["tensors"])
                start = int(st["step"])
            data.seek(start)
            _log(rank, f"===== resumed from {latest} at step {start} =====")
    metrics_path = cfg.metrics_file
    fault_at = int(os.environ.get("TDFO_FAULT_AT_STEP", "0") or 0)
    fault_rank = int(os.environ.get("TDFO_FAULT_RANK", "0") or 0)
    use_graph = cfg.hip_graph and dev.type == "cuda" and tr.emb.graph_capturable
    history: List[Dict] = []
    t0 = time.perf_counter()
    last_t, last_step = t0, start
    step = start
    prof = ProfileWindow(cfg.profile_steps or None)
    timer = StepTimer(enabled=dev.type == "cuda")
    while step < total_steps:
        prof.before_step(step)
        with trace_range("load_batch"):
            dense, ids, label = data.next()
            tr.load_batch(dense.to(dev, non_blocking=True), ids.to(dev, non_blocking=True),
                          label.to(dev, non_blocking=True))
        timer.start()
        with trace_range("train_step"):
            tr.step()
        timer.stop()
        step += 1
        prof.after_step(step)
        if use_graph and tr.graph is None and step - start == 2:
            tr.capture_graph(warmup=0)
        if fault_at and step == fault_at and rank == fault_rank:
            os._exit(17)                               # simulated rank failure
        if step % cfg.log_every == 0 or step == total_steps:
            if dev.type == "cuda":
                torch.cuda.synchronize()
            n = step - last_step
            loss = tr.pop_loss() / max(1, n * B)
            if world > 1:
                lt = torch.tensor([loss], dtype=torch.float64, device=dev)
                torch.distributed.all_reduce(lt, group=group)
                loss = float(lt) / world
            if not math.isfinite(loss):
                raise FloatingPointError(f"non-finite training loss at step {step}")
            now = time.perf_counter()
            ex_s = n * B * world / max(now - last_t, 1e-9)
            rec = {"step": step, "train_loss": loss, "examples_per_sec": ex_s}
            dev_ms = timer.mean_ms()
            if dev_ms is not None:
                rec["device_ms_per_step"] = dev_ms
            if cfg.eval_every and (step % cfg.eval_every == 0 or step == total_steps):
                with trace_range("eval"):
                    rec.update(evaluate(tr, cfg, dcfg, B, dev, rank, world, group))
            _log(rank, "step {step} train loss: {train_loss:.4f}, {examples_per_sec:,.0f} ex/s"
                 .format(**rec) + (f", eval loss: {rec['eval_loss']:.4f}, "
                                   f"eval auc: {rec['eval_auc']:.4f}" if "eval_auc" in rec else ""))
            history.append(rec)
            if metrics_path and rank == 0:
                with open(metrics_path, "a") as f:
                    f.write(json.dumps(rec) + "\n")
            last_t, last_step = time.perf_counter(), step
        if cfg.ckpt_dir and cfg.ckpt_every and step % cfg.ckpt_every == 0:
            with trace_range("checkpoint"):
                save(tr, cfg.ckpt_dir, step, rank, world, meta)
    if cfg.ckpt_dir:
        save(tr, cfg.ckpt_dir, step, rank, world, meta)
    return {"history": history, "steps": step, "trainer": tr}


def _latest(ckpt_dir: str) -> Optional[Path]:
    d = Path(ckpt_dir)
    if not d.exists():
        return None
    cands = [p for p in d.glob("step_*") if (p / "manifest.json").exists()]
    if not cands:
        return None
    return max(cands, key=lambda p: int(p.name.split("_")[1]))


def save(tr: DLRMTrainer, ckpt_dir: str, step: int, rank: int, world: int, meta: Dict):
    """Streamed per-piece checkpoint (bounded host memory at TB scale), loadable
    at any world size / sharding plan (utils/sharded_ckpt.py)."""
    barrier = (lambda: torch.distributed.barrier()) if world > 1 else None
    if tr.device.type == "cuda":
        torch.cuda.synchronize()
    sharded_ckpt.save(tr, str(Path(ckpt_dir) / f"step_{step}"), step, rank, world, meta,
                      barrier=barrier)


@torch.no_grad()
def evaluate(tr: DLRMTrainer, cfg: Config, dcfg: DLRMConfig, B: int, dev, rank: int,
             world: int, group, batches: int = 4) -> Dict[str, float]:
    """Held-out synthetic batches (a different seed): loss + bucketed AUC,
    reduced over ranks. Uses the trainer's static buffers, so the current
    training batch is restored afterwards."""
    saved = (tr.x0[:, :dcfg.num_dense].clone(), tr.ids.clone(), tr.label.clone())
    gen = _Data(cfg, dcfg, B, dev, rank, 7, prefetch=False)
    hist = torch.zeros(2 * 199, dtype=torch.int64, device=dev)
    loss = torch.zeros(2, dtype=torch.float64, device=dev)
    for _ in range(batches):
        d, i, y = gen.next()
        tr.load_batch(d.to(dev), i.to(dev), y.to(dev))
        lg = tr.predict().float()
        yy = tr.label.float()
        loss[0] += torch.nn.functional.binary_cross_entropy_with_logits(lg, yy, reduction="sum")
        loss[1] += lg.numel()
        ops.auc_hist(lg, yy, 199, hist)
    if world > 1:
        torch.distributed.all_reduce(hist, group=group)
        torch.distributed.all_reduce(loss, group=group)
    tr.load_batch(*saved)
    return {"eval_loss": float(loss[0] / loss[1]), "eval_auc": ops.reference.hist_auc(hist)}
