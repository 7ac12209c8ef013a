"""Process topology: one process per GPU, torch.distributed over RCCL (the
"nccl" backend on ROCm) or gloo on CPU.

Replaces the reference's launch plumbing (torchrec/train.py:186-198 env +
init_process_group; tensorflow2/train_ps.py:43-62 TF_CONFIG/cluster.json;
jax-flax/train_dp.py:149 single-process pmap). Collective timeouts are always
set (failure detection: a hung peer raises instead of stalling forever).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    group: Optional[object] = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_INFO: Optional[DistInfo] = None


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", 0))))


def init_distributed(device: Optional[str] = None, backend: Optional[str] = None,
                     timeout_s: float = 600.0) -> DistInfo:
    """Initialise (idempotently) from RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* env.

    ``device``: "cuda" | "cpu" | None (auto: cuda if available).
    """
    global _INFO
    if _INFO is not None:
        return _INFO
    rank, world, local = env_world()
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    # Rehearsal knobs for a 1-GPU box: TDFO_SHARE_DEVICE=1 puts every rank on
    # cuda:0 and TDFO_DIST_BACKEND=gloo swaps RCCL (which refuses two ranks on
    # one GPU) for gloo, so the multi-rank step logic runs on real kernels.
    if os.environ.get("TDFO_SHARE_DEVICE") == "1":
        local = 0
    backend = backend or os.environ.get("TDFO_DIST_BACKEND") or None
    if device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if backend is None:
        backend = "nccl" if dev.type == "cuda" else "gloo"
    info = DistInfo(rank=rank, world_size=world, local_rank=local, device=dev, backend=None)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if not dist.is_initialized():
            kw = {}
            if dev.type == "cuda" and backend == "nccl":
                kw["device_id"] = dev
            prefix = os.environ.get("TDFO_STORE_PREFIX")
            if prefix:
                # a supervised attempt (utils/supervise.py): a client of the
                # launcher's (or the supervisor's) store under this attempt's
                # key prefix, so no key of an earlier attempt is read
                tcp = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]),
                                    world_size=world, is_master=False,
                                    timeout=datetime.timedelta(seconds=timeout_s))
                kw["store"] = dist.PrefixStore(prefix, tcp)
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        info.backend = backend
        info.group = dist.group.WORLD
    _INFO = info
    return info


def get_info() -> DistInfo:
    return _INFO if _INFO is not None else DistInfo()


def reset():
    """Tear down (tests / end of training)."""
    global _INFO
    from .comm import release_native
    release_native()
    if dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def all_reduce_max(x: float, device) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum_(t: torch.Tensor):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return t
