"""Cross-rank consistency of the replicated training state.

Data parallelism keeps every rank's copy of the dense parameters, their
optimizer moments, the step counters and the replicated (data-parallel)
embedding tables identical -- the all-reduced gradients are bitwise equal on
every rank and the updates are deterministic. DDP guarantees that by
construction (the reference's torchrec/train.py:255-260); here a multi-rank
run checks it: ``fingerprint`` hashes the bits of each replicated tensor on
the device (position-weighted int64 sums, exact), and ``check_replicas``
MIN- and MAX-all-reduces the fingerprints -- equal on every rank iff the
replicas agree bit for bit (up to hash collisions). ``bench.py`` runs it
after the timed steps at N > 1 and fails the run on a mismatch, so a
throughput is never reported for diverged replicas.
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

import torch
import torch.distributed as dist

_CHUNK = 1 << 24


def _bits(t: torch.Tensor) -> torch.Tensor:
    t = t.detach().contiguous().view(-1)
    if t.dtype in (torch.float32, torch.int32):
        return t.view(torch.int32)
    if t.dtype in (torch.bfloat16, torch.float16, torch.int16):
        return t.view(torch.int16)
    if t.dtype in (torch.float64, torch.int64):
        return t.view(torch.int64)
    return t.to(torch.int64)


def fingerprint(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """int64 [2 * len(tensors)]: per tensor (sum of its bit patterns,
    position-weighted sum) -- computed on the tensors' device, chunked so a
    large replicated table needs no full-size temporary."""
    out = []
    for t in tensors:
        b = _bits(t)
        dev = b.device
        s0 = torch.zeros((), dtype=torch.int64, device=dev)
        s1 = torch.zeros((), dtype=torch.int64, device=dev)
        for lo in range(0, b.numel(), _CHUNK):
            c = b[lo:lo + _CHUNK].to(torch.int64)
            w = (torch.arange(lo, lo + c.numel(), dtype=torch.int64, device=dev) % 1000003) + 1
            s0 += c.sum()
            s1 += (c * w).sum()
        out += [s0, s1]
    if not out:
        return torch.zeros(0, dtype=torch.int64)
    return torch.stack(out)


def check_replicas(named: Dict[str, torch.Tensor], group=None) -> Tuple[bool, Dict]:
    """All ranks agree on every tensor in ``named`` (collective: every rank
    calls it with the same names). Returns (consistent, {name: agrees})."""
    names = sorted(named)
    fp = fingerprint([named[k] for k in names])
    if not (dist.is_initialized() and dist.get_world_size(group) > 1) or fp.numel() == 0:
        return True, {k: True for k in names}
    if dist.get_backend(group) == "gloo":
        fp = fp.cpu()
    lo, hi = fp.clone(), fp.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    same = (lo == hi).view(-1, 2).all(1).cpu().tolist()
    per = {k: bool(v) for k, v in zip(names, same)}
    return all(per.values()), per
