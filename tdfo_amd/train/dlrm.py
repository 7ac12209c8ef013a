"""DLRM / DCN-v2 training driver (north-star workloads, BASELINE.json configs 1-5).

Entry points (recipes/dlrm):
  train.py     single process (CPU: DLRM-tiny, config 1; one GPU: config 2)
  train_dp.py  one process per GPU, ``data_parallel`` sharding (the small
               tables replicated and trained by one dense-gradient
               all-reduce, the large ones owner-partitioned row-wise) + dense
               all-reduce over RCCL (config 3)
  train_ps.py  the parameter-server entry point of the reference collapsed
               into the sharded engine: table-wise / row-wise shards with
               all-to-all over xGMI (configs 4-5)

Training loop services: JSONL metrics + stdout log lines,
examples/s throughput, held-out synthetic eval (loss + bucketed ROC-AUC),
non-finite loss detection (halt with a clear error), sharded checkpoints
(one file per rank + manifest, atomically completed) and resume, and a
fault-injection hook (``TDFO_FAULT_AT_STEP``) used by the recovery tests;
on a GPU a step watchdog (utils/watchdog.py, ``TDFO_WATCHDOG_S``, default
600 s) ends a hung rank with a diagnostic, and a multi-rank run checks at
the end that every rank's replicated state is bit-identical
(parallel/replicas.py) and raises otherwise.
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
from ..models.dlrm import (CRITEO_1TB_ROWS, CRITEO_KAGGLE_ROWS, DCN_GT1TB_ROWS, MLPERF_MULTIHOT,
                           DLRMConfig, DLRMTrainer)
from ..parallel.dist import init_distributed
from ..sparse import tables as _tables
from ..utils import checkpoint as ckpt
from ..utils import guarded, sharded_ckpt
from ..utils.profiling import ProfileWindow, StepTimer, trace_range
from .loop import StepLoop, make_source

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


def _source(cfg: Config, dcfg: DLRMConfig, B: int, device, rank: int, stream: int,
            start: int, eval_: bool = False):
    """Batch source positioned at batch ``start`` (train/loop.py): the C++ host
    generator on CPU; on a GPU the one-launch device generator (a fresh batch
    per step on a side stream), or with ``synthetic.host_data`` the C++
    generator behind the pinned copy-stream prefetcher -- the host data plane
    a real input pipeline would use. Batch i is reproducible after resume."""
    kind = "cpu" if device.type == "cpu" else (
        "host" if cfg.synthetic.host_data and not eval_ else "fresh")
    return make_source(dcfg.table_rows, B, device, dcfg.pooling_factors(), cfg.seed, rank,
                       dist=cfg.synthetic.dist, zipf_alpha=cfg.synthetic.zipf_alpha, start=start,
                       stream=stream, kind=kind, num_dense=dcfg.num_dense)


def _log(rank, msg):
    if rank == 0:
        print(msg, flush=True)


def run(cfg: Config, mode: str = "single", out_dir: str = ".",
        device: Optional[str] = None) -> Dict:
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    info = init_distributed(device)
    rank, world, dev, group = info.rank, info.world_size, info.device, info.group
    # W > 1: collective self-test before the trainer exists; a mismatch puts
    # every rank on c10d collectives + staged replay (utils/guarded.py)
    pf = guarded.rank_preflight(info)
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
    # more than one rank: input-dist pipelining, the step bench.py measures
    dcfg.pipeline = world > 1
    dcfg.stream_graphs = dcfg.stream_graphs and guarded.stream_graphs_allowed()
    B = cfg.per_device_train_batch_size
    tr = DLRMTrainer(dcfg, B, dev, group=group, rank=rank, world_size=world)
    _log(rank, f"===== model: {cfg.model}, tables: {dcfg.num_tables} "
               f"({sum(dcfg.table_rows):,} rows x {dcfg.embedding_dim}), "
               f"per-device batch {B}, num devices: {world} =====")
    _log(rank, f"===== sharding plan: {json.dumps(tr.plan.summary())} =====")
    if world > 1:
        from ..parallel.comm import RcclComm
        _log(rank, f"===== attempt {os.environ.get('TDFO_ATTEMPT', '0')}, collectives: "
                   f"{'native' if isinstance(tr.comm, RcclComm) else 'c10d'}, "
                   f"stream graphs: {dcfg.stream_graphs}, preflight: "
                   f"{'ok' if pf is None or pf['ok'] else 'FAILED ' + str(pf['failed'])} =====")
    total_steps = cfg.max_steps or cfg.synthetic.num_batches * cfg.n_epochs
    start = 0
    meta = {"model": cfg.model, "world_size": world, "strategy": strategy,
            "tables": len(dcfg.table_rows), "dim": dcfg.embedding_dim}
    if guarded.resume_requested(cfg.resume) and cfg.ckpt_dir:
        latest = _latest(cfg.ckpt_dir)
        if latest is not None:
            if sharded_ckpt.is_v2(str(latest)):        # streamed, reshardable
                start = sharded_ckpt.load(tr, str(latest), rank, world, expect_meta=meta)
            else:                                       # legacy per-rank files (same plan)
                st = ckpt.load_sharded(str(latest), rank, world, expect_meta=meta)
                tr.load_flat_state(st["tensors"])
                start = int(st["step"])
            _log(rank, f"===== resumed from {latest} at step {start} =====")
    wd = None
    wd_s = float(os.environ.get("TDFO_WATCHDOG_S", "600") or 0)
    if dev.type == "cuda" and wd_s > 0:
        from ..utils.watchdog import StepWatchdog
        wd = StepWatchdog(dev, wd_s, rank=rank, describe=tr.progress)
    loop = StepLoop(tr, _source(cfg, dcfg, B, dev, rank, 0, start), start, watchdog=wd)
    metrics_path = cfg.metrics_file
    fault_at = int(os.environ.get("TDFO_FAULT_AT_STEP", "0") or 0)
    fault_rank = int(os.environ.get("TDFO_FAULT_RANK", "0") or 0)
    fa = os.environ.get("TDFO_FAULT_ATTEMPT")       # only in this supervisor attempt
    if fa is not None and fa != os.environ.get("TDFO_ATTEMPT", "0"):
        fault_at = 0
    # jit_xla = false (tensorflow2/train.py:16): eager launches, no hipGraph
    use_graph = (cfg.hip_graph and cfg.jit_xla is not False and dev.type == "cuda"
                 and tr.emb.graph_capturable)
    # steps_per_execution (tensorflow2/train.py:17): steps issued per host
    # round; logging, checkpoints and the fault hook run between rounds
    k_exec = max(1, int(cfg.steps_per_execution))
    history: List[Dict] = []
    t0 = time.perf_counter()
    last_t, last_step = t0, start
    step = start
    prof = ProfileWindow(cfg.profile_steps or None)
    timer = StepTimer(enabled=dev.type == "cuda")

    def boundary(s: int) -> int:
        """Next step count at which the host must look (log / ckpt / fault /
        graph capture / end), so executions never straddle one."""
        cands = [total_steps, (s // cfg.log_every + 1) * cfg.log_every]
        if cfg.ckpt_dir and cfg.ckpt_every:
            cands.append((s // cfg.ckpt_every + 1) * cfg.ckpt_every)
        if fault_at and s < fault_at:
            cands.append(fault_at)
        if use_graph and tr.graph is None:
            cands.append(max(s + 1, start + 2))
        w = prof.win
        if w is not None:
            cands += [x for x in (w[0], w[0] + w[1]) if x > s]
        return min(cands)

    while step < total_steps:
        n = max(1, min(k_exec, boundary(step) - step))
        prof.before_step(step)
        timer.start()
        with trace_range("train_step"):
            loop.run(n)
        timer.stop(n)
        step += n
        prof.after_step(step)
        if use_graph and tr.graph is None and step - start >= 2:
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
    loop.close()
    if wd is not None:
        wd.close()
    if world > 1:
        from ..parallel.replicas import check_replicas
        ok, per = check_replicas(tr.replicated_state(), group)
        _log(rank, f"===== replicated state consistent across ranks: {ok} =====")
        if not ok:
            raise RuntimeError(f"rank {rank}: replicated state differs across ranks: {per}")
    if cfg.ckpt_dir:
        save(tr, cfg.ckpt_dir, step, rank, world, meta)
    return {"history": history, "steps": step, "trainer": tr, "start": start, "preflight": pf,
            "comm_path": _comm_path(tr, world)}


def _comm_path(tr: DLRMTrainer, world: int) -> Optional[str]:
    if world <= 1:
        return None
    from ..parallel.comm import RcclComm
    return (("native" if isinstance(tr.comm, RcclComm) else "c10d")
            + ("-graphs" if tr.graph == "mstreams" else "-staged"))


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
    tr.drain()
    saved = (tr.x0[:, :dcfg.num_dense].float(), tr.ids.clone(), tr.label.clone())
    src = _source(cfg, dcfg, B, dev, rank, 7, 0, eval_=True)
    hist = torch.zeros(2 * 199, dtype=torch.int64, device=dev)
    loss = torch.zeros(2, dtype=torch.float64, device=dev)
    for _ in range(batches):
        (d, i, y), slot = src.next()
        tr.load_batch(d, i, y)
        if slot is not None:
            src.release(slot)
        lg = tr.predict().float()
        yy = tr.label.float()
        loss[0] += torch.nn.functional.binary_cross_entropy_with_logits(lg, yy, reduction="sum")
        loss[1] += lg.numel()
        ops.auc_hist(lg, yy, 199, hist)
    if world > 1:
        torch.distributed.all_reduce(hist, group=group)
        torch.distributed.all_reduce(loss, group=group)
    if tr.pipeline:              # the next step's batch: reload and re-exchange it
        tr.drain()
        tr.prime(*saved)
    else:
        tr.load_batch(*saved)
    return {"eval_loss": float(loss[0] / loss[1]), "eval_auc": ops.reference.hist_auc(hist)}
