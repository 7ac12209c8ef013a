"""The DLRM / DCN-v2 step loop shared by ``bench.py`` and the recipes
(``recipes/dlrm/train*.py`` via ``train/dlrm.py``), so the training loop is
exactly the step that is benchmarked (the reference benchmarks its own
training loop, torchrec/train.py:81-111).

A batch source hands out batch ``i`` of a reproducible stream:

* ``DeviceSyntheticStream`` (GPU default): one-launch HIP generator on a
  side stream, a fresh batch per step;
* ``HostPrefetcher`` (``synthetic.host_data``): C++ host generator, pinned
  slots, copy-stream H2D;
* ``HostBatches`` (CPU runs): the C++ host generator, synchronously;
* ``PoolBatches`` (``bench.py --data pool``): a fixed pool cycled.

``StepLoop`` feeds the trainer: one process uses ``load_batch`` before each
step; with input-dist pipelining (W > 1) ``prime`` loads the first batch and
every step is handed the *next* one (``set_next_batch``), which it loads and
starts exchanging in its tail. Slots of streamed sources are released once
the step has enqueued its reads of them.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence


class PoolBatches:
    """Cycle a list of device batches (no generation in the step)."""

    def __init__(self, pool: Sequence, start: int = 0):
        self.pool = list(pool)
        self.i = int(start)

    def next(self, streams=None):
        b = self.pool[self.i % len(self.pool)]
        self.i += 1
        return b, None

    def release(self, slot, streams=None):
        return None


class HostBatches:
    """A host batch generator (``batch(i)`` / ``next()``) as a source."""

    def __init__(self, gen, start: int = 0):
        self.gen = gen
        if hasattr(gen, "index"):
            gen.index = int(start)

    def next(self, streams=None):
        return self.gen.next(), None

    def release(self, slot, streams=None):
        return None


def make_source(table_rows: Sequence[int], batch: int, device, pooling: Optional[List[int]],
                seed: int, rank: int, dist: str = "uniform", zipf_alpha: float = 1.05,
                start: int = 0, stream: int = 0, kind: str = "auto", num_dense: int = 13,
                threads: int = 8):
    """The batch source for ``kind``: "fresh" (device generator), "instep"
    (the same generator inside the trainer's step; one GPU), "host" (host
    generator + prefetcher), "cpu" (host generator, synchronous) or "auto"
    (fresh on a GPU, cpu otherwise). Batch ``i`` is the same pure function of
    (seed, stream, rank, i) for every kind (uniform ids)."""
    import torch
    dev = torch.device(device)
    if kind == "auto":
        kind = "fresh" if dev.type == "cuda" else "cpu"
    if kind == "instep":
        from ..data.synthetic import InStepSynthetic
        return InStepSynthetic(table_rows, batch, dev, num_dense=num_dense, pooling=pooling,
                               seed=seed, dist=dist, zipf_alpha=zipf_alpha, rank=rank,
                               stream=stream, start=start)
    if kind == "fresh":
        from ..data.synthetic import DeviceSyntheticStream
        return DeviceSyntheticStream(table_rows, batch, dev, num_dense=num_dense, pooling=pooling,
                                     seed=seed, dist=dist, zipf_alpha=zipf_alpha, rank=rank,
                                     stream=stream, start=start)
    if kind == "host":
        from ..data.prefetch import host_prefetcher
        return host_prefetcher(table_rows, batch, dev, pooling=pooling, seed=seed, rank=rank,
                               dist=dist, zipf_alpha=zipf_alpha, threads=threads, start=start,
                               stream=stream, num_dense=num_dense)
    if kind == "cpu":
        from ..data.synthetic import HostSyntheticCriteo
        return HostBatches(HostSyntheticCriteo(table_rows, batch, num_dense, pooling=pooling,
                                               seed=seed, rank=rank, dist=dist,
                                               zipf_alpha=zipf_alpha, stream=stream,
                                               threads=min(threads, 4)), start)
    raise ValueError(f"unknown batch source {kind!r}")


class StepLoop:
    """Drive ``trainer`` (a ``DLRMTrainer``) from ``source``, which must be
    positioned at batch ``start`` (the step about to run)."""

    def __init__(self, trainer, source, start: int = 0, watchdog=None, beat_every: int = 8):
        """``watchdog``: a ``utils.watchdog.StepWatchdog`` -- every
        ``beat_every`` steps (and at the end of each ``run``) a heartbeat is
        enqueued behind the step, and the host must keep issuing steps."""
        self.tr = trainer
        self.src = source
        self.step_index = int(start)
        self._primed = False
        self.wd = watchdog
        self.beat_every = max(1, int(beat_every))
        self.in_step = bool(getattr(source, "in_step", False))
        if self.in_step:
            trainer.attach_in_step_source(source)
        elif (os.environ.get("TDFO_SRC_COPY", "1") != "0"
              and getattr(source, "copy_stream", None) is not None
              and hasattr(trainer, "set_copy_stream") and getattr(trainer, "graph", 1) is None
              and getattr(trainer, "world", 1) == 1 and not getattr(trainer, "pipeline", False)):
            trainer.set_copy_stream(source.copy_stream, owner=source)

    def _streams(self):
        return None if self.tr.pipeline else self.tr.input_streams()

    def _next(self):
        on_gpu = self.tr.device.type == "cuda"
        return self.src.next(streams=self._streams() if on_gpu else None)

    def _release(self, slot):
        if slot is not None:
            self.src.release(slot, streams=self._streams())

    def prime(self):
        """Pipelined trainer: load batch ``start`` and start its exchange."""
        if self.tr.pipeline and not self._primed:
            b, slot = self.src.next()
            self.tr.prime(*b)
            self.src.release(slot) if slot is not None else None
            self._primed = True

    def run(self, n: int):
        """Issue n training steps (no host synchronisation)."""
        tr = self.tr
        if tr.pipeline and not self._primed:
            self.prime()
        on_dev = tr.device.type == "cuda"
        wd = self.wd
        flush = getattr(tr, "flush_pending", None)   # every issued step complete
        if wd is None:
            self._run(n, on_dev)
            if flush is not None:
                flush()
            return
        with wd.active():
            self._run(n, on_dev)
            if flush is not None:
                flush()
            if n:
                wd.beat(tr.heartbeat_stream(), self.step_index)

    def _run(self, n: int, on_dev: bool):
        tr, wd = self.tr, self.wd
        if self.in_step and hasattr(self.src, "check_steps"):
            self.src.check_steps(self.step_index, n)
        for k in range(n):
            if self.in_step:                   # the step draws its own batch
                tr.step()
                self.step_index += 1
                if wd is not None and (self.step_index % self.beat_every == 0) and k + 1 < n:
                    wd.beat(tr.heartbeat_stream(), self.step_index)
                continue
            batch, slot = self._next()
            if tr.pipeline:
                tr.set_next_batch(*batch)
            else:
                # device sources order each batch on every input stream
                tr.load_batch(*batch, on_device=on_dev)
            tr.step()
            self._release(slot)
            self.step_index += 1
            if wd is not None and (self.step_index % self.beat_every == 0) and k + 1 < n:
                wd.beat(tr.heartbeat_stream(), self.step_index)

    def close(self):
        if hasattr(self.src, "close"):
            self.src.close()
