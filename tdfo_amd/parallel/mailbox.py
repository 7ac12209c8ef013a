"""Device -> host values without stalling the stream that produces them.

A ``HostMailbox`` slot is one 64-bit word of host-mapped coherent memory
(``hipHostMalloc(Coherent | Mapped)``). ``publish`` enqueues one tiny kernel
(csrc/kernels/elementwise.hip ``host_publish_kernel``) that bumps the slot's
device-side sequence number and stores ``seq << 32 | value`` into the word
with a single system-scope vector store -- no event, no fence, so nothing
on any queue waits for it, and it can be captured into a hipGraph like any
kernel. The host keeps its own count of the publishes it launched (eager
calls, plus ``note_launch`` for every replay of a graph that holds one) and
``read`` polls the word until that sequence number appears: a late store can
only delay the read, never hand it a stale value.

Used by the lagged row-wise capacity check (sparse/sharded.py
``rw_publish_need`` / ``rw_resolve_need``): the all-reduced per-owner need of
the batch bucketized in step i is read when step i+1 is issued, by which
time the device has long produced it, so the host never drains the stream
(the reference's input dist never stalls its training loop either:
torchrec/train.py:241-247). Also the step heartbeat of the watchdog
(utils/watchdog.py).
"""
from __future__ import annotations

import time
from typing import List

import torch


class HostMailbox:
    def __init__(self, slots: int, device):
        self.device = torch.device(device)
        self.slots = int(slots)
        self.cuda = self.device.type == "cuda"
        self.expect: List[int] = [0] * self.slots
        self.wait_s = 0.0           # host time spent polling in read()
        if self.cuda:
            from ..ops._ext import load, ops
            if not load():
                raise RuntimeError("HostMailbox needs the native HIP library")
            self._native = ops()
            self.host = self._native.host_mailbox_alloc(self.slots)
            self.seq = torch.zeros(self.slots, dtype=torch.int32, device=self.device)
        else:                       # CPU runs: the value is known at once
            self._native = None
            self.host = None
            self.seq = None
            self._cpu = [0] * self.slots

    def publish(self, value: torch.Tensor, slot: int = 0):
        """Enqueue (or, under stream capture, record) the publish of the
        int32 ``value[0]``. Eager calls count themselves; a captured publish
        is counted by ``note_launch`` at each replay of its graph."""
        if self.cuda:
            self._native.host_publish(value, self.seq[slot:slot + 1], self.host, slot)
            if not torch.cuda.is_current_stream_capturing():
                self.expect[slot] += 1
        else:
            self.expect[slot] += 1
            self._cpu[slot] = int(value.reshape(-1)[0].item())

    def note_launch(self, slot: int = 0, n: int = 1):
        """A graph holding ``n`` publishes of ``slot`` was launched."""
        self.expect[slot] += n

    def _word(self, slot: int):
        w = int(self.host[slot]) & 0xFFFFFFFFFFFFFFFF
        return w >> 32, w & 0xFFFFFFFF

    def ready(self, slot: int = 0) -> bool:
        if not self.cuda:
            return True
        return self._word(slot)[0] == self.expect[slot] & 0xFFFFFFFF

    def read(self, slot: int = 0, timeout_s: float = 60.0) -> int:
        """The value of the latest publish launched into ``slot`` (signed
        int32), polling until it has landed. After ``timeout_s`` the device is
        synchronised once and the word read again; a sequence number that
        still disagrees is a bookkeeping error and raises."""
        if not self.cuda:
            return self._cpu[slot]
        want = self.expect[slot] & 0xFFFFFFFF
        s, v = self._word(slot)
        if s == want:
            return v - (1 << 32) if v & 0x80000000 else v
        t0 = time.monotonic()
        spins = 0
        while True:
            s, v = self._word(slot)
            if s == want:
                self.wait_s += time.monotonic() - t0
                return v - (1 << 32) if v & 0x80000000 else v
            spins += 1
            if spins & 1023 == 0:
                if time.monotonic() - t0 > timeout_s:
                    break
                time.sleep(0)          # let a watchdog thread run
        torch.cuda.synchronize(self.device)
        self.wait_s += time.monotonic() - t0
        s, v = self._word(slot)
        if s != want:
            raise RuntimeError(f"HostMailbox slot {slot}: sequence {s} after a device sync, "
                               f"expected {want} (publish launches miscounted)")
        return v - (1 << 32) if v & 0x80000000 else v
