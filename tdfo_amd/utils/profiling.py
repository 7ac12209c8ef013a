"""Tracing / profiling helpers (the reference has none beyond
tqdm and perf_counter around ETL phases).

* ``trace_range(name)``: a roctx range (``torch.cuda.nvtx`` maps to roctx on
  ROCm) around a host phase, visible in ``rocprofv3 --marker-trace``; no-op on
  CPU.
* ``StepTimer``: device-event step timing (no host sync per step): record a
  start/end event pair per step and read the mean ms/step when logging.
* ``ProfileWindow``: ``TDFO_PROFILE=START:COUNT`` (or config ``profile_steps``)
  brackets steps [START, START+COUNT) with a ``profile_window`` roctx range
  and hipProfilerStart/Stop, so a run under
  ``rocprofv3 --kernel-trace --marker-trace`` can be narrowed to steady-state
  steps.
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional, Tuple

import torch


def _gpu() -> bool:
    return torch.cuda.is_available()


@contextlib.contextmanager
def trace_range(name: str):
    if _gpu():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


class StepTimer:
    """Mean device time per step over the steps recorded since the last read."""

    def __init__(self, enabled: Optional[bool] = None):
        self.enabled = _gpu() if enabled is None else enabled
        self._pairs: List[Tuple[object, object]] = []
        self._open = None

    def start(self):
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._open = e

    def stop(self, steps: int = 1):
        """Close the interval opened by ``start``; it covered ``steps`` steps."""
        if self.enabled and self._open is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._pairs.append((self._open, e, int(steps)))
            self._open = None

    def mean_ms(self) -> Optional[float]:
        """Synchronises on the last event; None if nothing was recorded."""
        if not self._pairs:
            return None
        self._pairs[-1][1].synchronize()
        ms = sum(a.elapsed_time(b) for a, b, _ in self._pairs)
        n = sum(k for _, _, k in self._pairs)
        self._pairs.clear()
        return ms / max(1, n)


def parse_window(spec: str) -> Optional[Tuple[int, int]]:
    if not spec:
        return None
    a, _, b = spec.partition(":")
    return int(a), int(b or 1)


class ProfileWindow:
    def __init__(self, spec: Optional[str] = None):
        self.win = parse_window(spec if spec is not None else os.environ.get("TDFO_PROFILE", ""))
        self.active = False

    def before_step(self, step: int):
        if self.win and _gpu() and step == self.win[0] and not self.active:
            torch.cuda.synchronize()
            torch.cuda.nvtx.range_push("profile_window")
            try:
                torch.cuda.profiler.start()
            except Exception:      # profiler API absent: the roctx range still marks it
                pass
            self.active = True

    def after_step(self, step: int):
        if self.active and step >= self.win[0] + self.win[1]:
            torch.cuda.synchronize()
            try:
                torch.cuda.profiler.stop()
            except Exception:
                pass
            torch.cuda.nvtx.range_pop()
            self.active = False
