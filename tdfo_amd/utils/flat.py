"""Flat parameter storage for dense (MLP) parameters.

All dense parameters of a model live in ONE fp32 buffer (plus a bf16 shadow
the MFMA kernels read, one fp32 gradient buffer and the optimizer moments).
Consequences on MI355X:
  * the fused optimizer is a single launch over the whole model;
  * data-parallel gradient reduction is one (or a few bucketed) RCCL
    all-reduce(s) over a contiguous buffer — no per-tensor collectives;
  * every tensor view starts 256-B aligned (16-B vector loads, glds staging).
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import torch

ALIGN = 64  # elements (256 B fp32 / 128 B bf16)


class FlatParams:
    def __init__(self):
        self.specs: List[Tuple[str, Tuple[int, ...], int]] = []
        self.numel = 0
        self.finalized = False

    def add(self, name: str, shape) -> None:
        assert not self.finalized
        n = int(math.prod(shape))
        self.specs.append((name, tuple(shape), self.numel))
        self.numel += -(-n // ALIGN) * ALIGN

    def finalize(self, device, with_adam: bool = True, with_m: bool = True):
        self.finalized = True
        n = max(ALIGN, self.numel)
        self.p = torch.zeros(n, dtype=torch.float32, device=device)
        self.g = torch.zeros(n, dtype=torch.float32, device=device)
        self.p_bf16 = torch.zeros(n, dtype=torch.bfloat16, device=device)
        self.m = torch.zeros(n, dtype=torch.float32, device=device) if (with_adam or with_m) else None
        self.v = torch.zeros(n, dtype=torch.float32, device=device) if with_adam else None
        self._views: Dict[str, Tuple[int, Tuple[int, ...]]] = {}
        for name, shape, off in self.specs:
            self._views[name] = (off, shape)
        return self

    def _view(self, buf, name):
        off, shape = self._views[name]
        return buf[off: off + int(math.prod(shape))].view(shape)

    def offset(self, name) -> int:
        return self._views[name][0]

    def param(self, name):
        return self._view(self.p, name)

    def grad(self, name):
        return self._view(self.g, name)

    def bf16(self, name):
        return self._view(self.p_bf16, name)

    def names(self):
        return [s[0] for s in self.specs]

    def sync_bf16(self):
        self.p_bf16.copy_(self.p.to(torch.bfloat16))

    def state_dict(self):
        d = {name: self.param(name).detach().clone().cpu() for name in self.names()}
        return d

    def load_state_dict(self, d):
        for name in self.names():
            self.param(name).copy_(d[name])
        self.sync_bf16()
