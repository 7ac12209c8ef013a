"""Flat fused optimizer for torch ``nn.Module`` dense parameters.

Reference optimizers this replaces: optax.adamw (jax-flax/train.py:26),
keras AdamW (tensorflow2/train.py:11), torch Adam (torchrec/train.py:250-260).

All parameters are re-homed into ONE contiguous fp32 buffer (``p.data`` becomes
a view) and their ``.grad`` into ONE contiguous gradient buffer, so:
  * the update is a single HIP launch (``tdfo::dense_optimizer``) for the
    whole model, which also refreshes a bf16 shadow copy when requested;
  * data-parallel gradient averaging is one RCCL all-reduce over the flat
    buffer (bucketed for overlap when ``bucket_mb`` is set);
  * fp16-style dynamic loss scaling (Flax DynamicScale, jax-flax/train_dp.py:
    56-81) is a device-side finite check that skips the update — no host
    sync, no state rollback needed.
"""
from __future__ import annotations

import math
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist

from .. import ops

_OPT = {"adamw": ops.OPT_ADAMW, "adam": ops.OPT_ADAM, "sgd": ops.OPT_SGD,
        "adagrad": ops.OPT_ADAGRAD}
ALIGN = 64


class FlatOptimizer:
    def __init__(self, params: Iterable[torch.nn.Parameter], name: str = "adamw",
                 lr: float = 1e-3, weight_decay: float = 0.0, betas=(0.9, 0.999),
                 eps: float = 1e-8, momentum: float = 0.0, group=None,
                 bf16_shadow: bool = False, dynamic_scale: bool = False):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        assert self.params, "no parameters"
        self.opt = _OPT[name]
        self.name = name
        self.wd = weight_decay
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.momentum = momentum
        self.group = group
        dev = self.params[0].device
        self.device = dev
        sizes = [p.numel() for p in self.params]
        offs, o = [], 0
        for n in sizes:
            offs.append(o)
            o += -(-n // ALIGN) * ALIGN
        self.numel = max(o, ALIGN)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        for p, off, n in zip(self.params, offs, sizes):
            self.flat[off: off + n].copy_(p.data.reshape(-1).float())
            p.data = self.flat[off: off + n].view_as(p)
            p.grad = self.grad[off: off + n].view_as(p)
        self._views = list(zip(self.params, offs, sizes))
        need_m = self.opt in (ops.OPT_ADAMW, ops.OPT_ADAM, ops.OPT_ADAGRAD) or momentum != 0
        self.m = torch.zeros_like(self.flat) if need_m else None
        self.v = torch.zeros_like(self.flat) if self.opt in (ops.OPT_ADAMW, ops.OPT_ADAM) else None
        self.shadow = torch.zeros(self.numel, dtype=torch.bfloat16, device=dev) if bf16_shadow else None
        self.hyper = torch.tensor([lr, 0.0, 1.0], dtype=torch.float32, device=dev)
        self._inv_set = 1.0                  # hyper[2] as last written
        self.step_bumped_by_caller = False   # the caller bumps hyper[1] (ops.bump)
        self.dynamic_scale = dynamic_scale
        self.found_inf = torch.zeros(1, dtype=torch.float32, device=dev) if dynamic_scale else None
        self.scale = 2.0 ** 15 if dynamic_scale else 1.0
        self._good_steps = 0
        self._ranges = [(0, self.numel)]     # flat ranges step() / zero_grads() cover

    def exclude(self, params) -> None:
        """Leave ``params`` out of step() and zero_grads(): a kernel that
        holds their complete gradient applies the same element update in its
        epilogue (e.g. linear_xent's fused output-layer step)."""
        ids = {id(p) for p in params}
        cut = sorted((off, off + -(-n // ALIGN) * ALIGN) for p, off, n in self._views
                     if id(p) in ids)
        ranges, lo = [], 0
        for a, b in cut:
            if a > lo:
                ranges.append((lo, a))
            lo = max(lo, b)
        if lo < self.numel:
            ranges.append((lo, self.numel))
        self._ranges = ranges

    def moments(self, p):
        """(m, v) views of parameter ``p``'s optimizer state."""
        for q, off, n in self._views:
            if q is p:
                return (self.m[off: off + n].view_as(p) if self.m is not None else None,
                        self.v[off: off + n].view_as(p) if self.v is not None else None)
        raise KeyError("not a parameter of this optimizer")

    def zero_grads(self):
        """Zero the gradients step() will read (excluded ranges untouched)."""
        if self._ranges == [(0, self.numel)]:
            self.grad.zero_()
        else:
            for lo, hi in self._ranges:
                self.grad[lo:hi].zero_()

    # ------------------------------------------------------------------
    def zero_grad(self):
        self.grad.zero_()
        for p, off, n in self._views:       # re-attach views if autograd replaced them
            if p.grad is None or p.grad.data_ptr() != self.grad[off:].data_ptr():
                p.grad = self.grad[off: off + n].view_as(p)

    def _gather_stray_grads(self):
        for p, off, n in self._views:
            g = p.grad
            if g is not None and g.data_ptr() != self.grad[off:].data_ptr():
                self.grad[off: off + n].copy_(g.reshape(-1))
                p.grad = self.grad[off: off + n].view_as(p)

    def all_reduce_grads(self, average: bool = True):
        if self.group is None or not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        dist.all_reduce(self.grad, group=self.group)
        if average:
            self.grad.mul_(1.0 / dist.get_world_size(self.group))

    def set_lr(self, lr: float):
        self.hyper[0:1].fill_(lr)

    @property
    def lr(self) -> float:
        return float(self.hyper[0])

    def step(self, grad_scale: Optional[float] = None):
        self._gather_stray_grads()
        inv = 1.0 / self.scale if self.dynamic_scale else (grad_scale or 1.0)
        if inv != self._inv_set:        # (a constant unscale factor is written once)
            self.hyper[2:3].fill_(inv)
            self._inv_set = None if self.dynamic_scale else inv
        if self.dynamic_scale:
            self.found_inf.zero_()
            ops.check_finite(self.grad, self.found_inf)
        if not self.step_bumped_by_caller:  # (else: the caller's one-launch ops.bump)
            self.hyper[1:2].add_(1.0)
        for lo, hi in self._ranges:
            sl = slice(lo, hi)
            ops.dense_optimizer(self.flat[sl], self.grad[sl],
                                self.m[sl] if self.m is not None else None,
                                self.v[sl] if self.v is not None else None,
                                self.shadow[sl] if self.shadow is not None else None, self.opt,
                                self.hyper, self.beta1, self.beta2, self.eps, self.wd,
                                self.momentum, self.found_inf)
        if self.dynamic_scale:
            self._update_scale()

    def _update_scale(self):
        # Flax DynamicScale defaults: growth 2x every 2000 finite steps, backoff 0.5
        if float(self.found_inf.item()) > 0:
            self.scale = max(1.0, self.scale * 0.5)
            self.hyper[1:2].sub_(1.0)          # skipped step does not advance Adam's t
            self._good_steps = 0
        else:
            self._good_steps += 1
            if self._good_steps >= 2000:
                self.scale *= 2.0
                self._good_steps = 0

    def state_dict(self):
        d = {"flat": self.flat.detach().cpu(), "hyper": self.hyper.detach().cpu(),
             "scale": self.scale}
        if self.m is not None:
            d["m"] = self.m.detach().cpu()
        if self.v is not None:
            d["v"] = self.v.detach().cpu()
        return d

    def load_state_dict(self, d):
        self.flat.copy_(d["flat"])
        self.hyper.copy_(d["hyper"])
        self.scale = d.get("scale", self.scale)
        if self.m is not None and "m" in d:
            self.m.copy_(d["m"])
        if self.v is not None and "v" in d:
            self.v.copy_(d["v"])


def lr_at(step: int, base: float, warmup: int = 0, decay_start: int = 0, decay_steps: int = 0,
          end_lr: float = 0.0) -> float:
    """Linear warmup + polynomial(1) decay schedule (MLPerf DLRM style)."""
    if warmup and step < warmup:
        return base * (step + 1) / warmup
    if decay_steps and step >= decay_start:
        frac = min(1.0, (step - decay_start) / decay_steps)
        return end_lr + (base - end_lr) * (1 - frac)
    return base


def cosine(step: int, base: float, total: int) -> float:
    return 0.5 * base * (1 + math.cos(math.pi * min(step, total) / max(1, total)))
