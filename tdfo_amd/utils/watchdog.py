"""Hang guard for training steps whose collectives run inside hipGraphs.

c10d collectives carry a timeout (parallel/dist.py), but the RCCL
collectives replayed inside the multi-rank step graphs (models/
dlrm_multirank.py, ``RcclComm``) have none: a cross-rank mismatch there would
spin every rank's GPU until an outside kill, with no diagnostic. The
reference makes such failures surface instead (``GRPC_FAIL_FAST``,
tensorflow2/train_ps.py:39).

``StepWatchdog``: after each issued step the loop enqueues a heartbeat --
one host-mailbox publish (parallel/mailbox.py) on the stream that ends the
step -- and a thread checks that every heartbeat lands within ``timeout_s``
of its issue, and that the host, while inside a step loop, issues a step at
least that often. Otherwise it prints what it knows (rank, steps issued and
completed, the trainer's per-stream progress) to stderr and ends the process
with ``os._exit(exit_code)`` -- no exec, no Python unwinding through a hung
runtime. The launcher (torch.distributed.run) then tears down the other
ranks, whose own watchdogs fire as well.
"""
from __future__ import annotations

import collections
import json
import os
import sys
import threading
import time
from contextlib import contextmanager
from typing import Callable, Optional

import torch

from ..parallel.mailbox import HostMailbox


class StepWatchdog:
    def __init__(self, device, timeout_s: Optional[float] = None, rank: int = 0,
                 describe: Optional[Callable[[], dict]] = None, exit_code: int = 3,
                 poll_s: Optional[float] = None):
        env = os.environ.get("TDFO_WATCHDOG_S")
        self.timeout = float(env) if env else float(timeout_s if timeout_s is not None else 300.0)
        self.device = torch.device(device)
        self.rank = int(rank)
        self.describe = describe
        self.exit_code = int(exit_code)
        self.mbox = HostMailbox(1, self.device)
        self._one = torch.ones(1, dtype=torch.int32, device=self.device)
        self._pending = collections.deque()       # (sequence number, issue time, step)
        self.issued = 0
        self.completed = 0
        self._busy = 0
        self._last_issue = time.monotonic()
        self._stop = threading.Event()
        self.fired = None
        self._poll = poll_s if poll_s is not None else max(0.05, min(1.0, self.timeout / 20))
        self._thread = threading.Thread(target=self._run, name="tdfo-watchdog", daemon=True)
        if self.timeout > 0:
            self._thread.start()

    # ------------------------------------------------------------ main thread
    def beat(self, stream=None, step: Optional[int] = None):
        """Enqueue the heartbeat of the step just issued on ``stream`` (the
        stream whose work ends the step; default the current one)."""
        if stream is not None and self.device.type == "cuda":
            with torch.cuda.stream(stream):
                self.mbox.publish(self._one)
        else:
            self.mbox.publish(self._one)
        self.issued += 1
        now = time.monotonic()
        self._pending.append((self.mbox.expect[0] & 0xFFFFFFFF, now, step))
        self._last_issue = now

    @contextmanager
    def active(self):
        """The host is inside a step loop: it must issue a step (``beat``)
        at least every ``timeout_s``."""
        self._busy += 1
        self._last_issue = time.monotonic()
        try:
            yield self
        finally:
            self._busy -= 1

    def close(self):
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(timeout=2 * self._poll + 1)

    # ------------------------------------------------------------- the thread
    def _landed(self) -> int:
        if self.device.type != "cuda":
            return self.mbox.expect[0] & 0xFFFFFFFF
        return self.mbox._word(0)[0]

    def check(self, now: Optional[float] = None) -> Optional[str]:
        """One poll: the reason to fire, or None."""
        now = time.monotonic() if now is None else now
        done = self._landed()
        while self._pending and ((done - self._pending[0][0]) & 0xFFFFFFFF) < (1 << 31):
            self._pending.popleft()
            self.completed += 1
        if self._pending and now - self._pending[0][1] > self.timeout:
            return (f"device: the heartbeat of step {self._pending[0][2]} has not landed "
                    f"{now - self._pending[0][1]:.1f} s after it was issued")
        if self._busy and now - self._last_issue > self.timeout:
            return f"host: no step issued for {now - self._last_issue:.1f} s inside the step loop"
        return None

    def _run(self):
        while not self._stop.wait(self._poll):
            why = self.check()
            if why is not None:
                self._fire(why)
                return

    def _fire(self, why: str):
        rep = {"watchdog": "hang", "rank": self.rank, "why": why, "timeout_s": self.timeout,
               "steps_issued": self.issued, "steps_completed": self.completed}
        if self.describe is not None:
            try:
                rep["trainer"] = self.describe()
            except Exception as e:          # diagnostics must not mask the hang
                rep["trainer"] = f"describe() failed: {e!r}"
        self.fired = rep
        try:
            print(json.dumps(rep, default=str), file=sys.stderr, flush=True)
        finally:
            if self.exit_code >= 0:
                os._exit(self.exit_code)
