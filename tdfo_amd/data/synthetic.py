"""Synthetic Criteo-shaped batches (BASELINE.json: "synthetic Criteo-shaped
data / random-init embeddings").

Dense features are log-normal-ish like log(1 + count) Criteo integers, ids
are uniform (default) or Zipf-skewed per table, labels follow a fixed random
logistic "teacher" over the dense features and a hash of the ids so the
loss is learnable. ``SyntheticCriteo`` generates with torch ops (any device);
``HostSyntheticCriteo`` is the multi-threaded C++ generator
(csrc/data/synthetic.cpp, counter-based so every batch is reproducible
independently) used for CPU runs and host-pipeline benchmarks;
``DeviceSyntheticStream`` is its one-launch HIP twin
(csrc/kernels/synthetic.hip) that draws a fresh batch per training step on a
side stream (the benchmark's default data source).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch


class SyntheticCriteo:
    def __init__(self, table_rows: Sequence[int], batch_size: int, num_dense: int = 13,
                 pooling: Optional[Sequence[int]] = None, device="cpu", seed: int = 0,
                 dist: str = "uniform", zipf_alpha: float = 1.05, rank: int = 0, stream: int = 0):
        """``seed`` fixes the teacher (labels' ground truth); ``stream`` picks an
        independent sample stream of the same task (e.g. held-out eval)."""
        self.rows = [int(r) for r in table_rows]
        self.T = len(self.rows)
        self.B = int(batch_size)
        self.num_dense = num_dense
        self.L = list(pooling) if pooling is not None else [1] * self.T
        self.device = torch.device(device)
        self.dist = dist
        self.alpha = zipf_alpha
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed * 7919 + rank + stream * 1_000_003)
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)   # teacher shared by all ranks
        self.w_dense = (torch.randn(num_dense, generator=g) / num_dense ** 0.5).to(self.device)
        self.table_bias = (torch.randn(self.T, 64, generator=g) * 0.5).to(self.device)

    def _ids(self, t: int, n: int) -> torch.Tensor:
        r = self.rows[t]
        if self.dist == "zipf" and r > 1:
            u = torch.rand(n, generator=self.gen, device=self.device)
            # inverse-CDF approximation of a bounded power law on [1, r]
            a = self.alpha
            x = ((r ** (1 - a) - 1) * u + 1) ** (1 / (1 - a))
            return (x.long() - 1).clamp_(0, r - 1)
        return torch.randint(0, r, (n,), generator=self.gen, device=self.device)

    def next(self):
        B = self.B
        dense = torch.log1p(torch.rand(B, self.num_dense, generator=self.gen, device=self.device)
                            * 100.0)
        ids: List[torch.Tensor] = []
        score = (dense - 3.6) @ self.w_dense * 2.0 - 1.1
        for t in range(self.T):
            it = self._ids(t, B * self.L[t])
            ids.append(it)
            first = it.view(B, self.L[t])[:, 0]
            score = score + self.table_bias[t][first % 64] * (3.0 / self.T ** 0.5)
        label = (torch.rand(B, generator=self.gen, device=self.device)
                 < torch.sigmoid(score)).float()
        return dense, torch.cat(ids), label


class HostSyntheticCriteo:
    """Same teacher as ``SyntheticCriteo``, generated on the host by the C++
    library (pinned output when ``pin``); batch ``i`` is a pure function of
    (seed, rank, i), so a resumed run regenerates exactly the same stream."""

    def __init__(self, table_rows: Sequence[int], batch_size: int, num_dense: int = 13,
                 pooling: Optional[Sequence[int]] = None, seed: int = 0, dist: str = "uniform",
                 zipf_alpha: float = 1.05, rank: int = 0, threads: int = 4, pin: bool = False,
                 stream: int = 0, nbuf: int = 2):
        """``nbuf`` output buffer sets; batch ``i`` is written into set
        ``i % nbuf`` (a prefetcher keeps ``nbuf - 1`` batches in flight)."""
        import numpy as np
        self.rows = np.asarray([int(r) for r in table_rows], dtype=np.int64)
        self.T = len(self.rows)
        self.B = int(batch_size)
        self.num_dense = num_dense
        self.L = np.asarray(list(pooling) if pooling is not None else [1] * self.T,
                            dtype=np.int32)
        self.seed, self.rank, self.threads, self.stream = seed, rank, threads, stream
        self.dist = 1 if dist == "zipf" else 0
        self.alpha = zipf_alpha
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        self.w_dense = (torch.randn(num_dense, generator=g) / num_dense ** 0.5).contiguous()
        self.table_bias = (torch.randn(self.T, 64, generator=g) * 0.5).contiguous()
        self.index = 0
        nnz = int((self.L.astype(np.int64) * self.B).sum())
        mk = (lambda t: t.pin_memory()) if pin else (lambda t: t)
        self.nbuf = max(1, int(nbuf))
        self._bufs = [(mk(torch.empty(self.B, num_dense)), mk(torch.empty(nnz, dtype=torch.int64)),
                       mk(torch.empty(self.B))) for _ in range(self.nbuf)]

    def batch(self, index: int):
        from .native import lib
        dense, ids, label = self._bufs[index % self.nbuf]
        lib().tdfo_synth_criteo(self.seed + self.stream * 1_000_003, self.rank, index, self.B, self.num_dense, self.T,
                                self.rows.ctypes.data, self.L.ctypes.data, self.dist, self.alpha,
                                self.w_dense.data_ptr(), self.table_bias.data_ptr(),
                                dense.data_ptr(), ids.data_ptr(), label.data_ptr(), self.threads)
        return dense, ids, label

    def next(self):
        out = self.batch(self.index)
        self.index += 1
        return out


class DeviceSyntheticStream:
    """Fresh synthetic batches generated on the GPU, one launch per batch, on
    a side stream, into ``slots`` rotating device buffer sets; batch ``i`` is
    the same pure function of (seed, rank, i) as ``HostSyntheticCriteo``'s
    (bit-identical ids for uniform draws). Same contract as
    ``prefetch.HostPrefetcher``: ``next(streams)`` -> ((dense, ids, label),
    slot), ordered on every consumer stream; ``release(slot, streams)`` once
    the consumer has enqueued its reads -- the slot is regenerated only after
    they ran (device-side event waits on the generator stream)."""

    def __init__(self, table_rows: Sequence[int], batch_size: int, device, num_dense: int = 13,
                 pooling: Optional[Sequence[int]] = None, seed: int = 0, dist: str = "uniform",
                 zipf_alpha: float = 1.05, rank: int = 0, stream: int = 0, slots: int = 3,
                 start: int = 0):
        from .. import ops
        self.ops = ops
        self.dev = torch.device(device)
        assert self.dev.type == "cuda", "DeviceSyntheticStream runs on the GPU"
        T = len(table_rows)
        L = list(pooling) if pooling is not None else [1] * T
        self.B, self.T = int(batch_size), T
        self.rows = torch.tensor([int(r) for r in table_rows], dtype=torch.int64, device=self.dev)
        self.pool_ = torch.tensor(L, dtype=torch.int32, device=self.dev)
        base, acc = [], 0
        for x in L:
            base.append(acc)
            acc += self.B * int(x)
        self.base = torch.tensor(base, dtype=torch.int64, device=self.dev)
        self.nnz = acc
        self.seed = int(seed) + int(stream) * 1_000_003
        self.rank, self.dist, self.alpha = int(rank), (1 if dist == "zipf" else 0), zipf_alpha
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)   # the teacher of SyntheticCriteo / HostSyntheticCriteo
        self.w_dense = (torch.randn(num_dense, generator=g) / num_dense ** 0.5).to(self.dev)
        self.table_bias = (torch.randn(T, 64, generator=g) * 0.5).contiguous().to(self.dev)
        self.S = int(slots)
        self.bufs = [(torch.empty(self.B, num_dense, device=self.dev),
                      torch.empty(self.nnz, dtype=torch.int64, device=self.dev),
                      torch.empty(self.B, device=self.dev)) for _ in range(self.S)]
        self.gs = torch.cuda.Stream(device=self.dev)
        # Events without the system-scope release fence (producer and
        # consumers are kernels on this device; no host reads these buffers):
        # a default event record writes back L2 at every record, which left
        # every consumer queue idle ~24 us per step (0.465 vs 0.444 ms/step
        # against a pre-generated pool). One generation event per slot and
        # one release event per (slot, consumer stream): a wait binds to the
        # latest record enqueued before it, so reusing them is safe.
        self.gen_ev = [ops.SyncEvent(2) for _ in range(self.S)]
        self.rel_ev = [[] for _ in range(self.S)]
        self.use_ev = [None] * self.S
        self.i = int(start)

    def generate(self, index: int, out):
        dense, ids, label = out
        self.ops.synth_criteo(self.seed, self.rank, index, self.B, self.rows, self.pool_,
                              self.base, self.dist, self.alpha, self.w_dense, self.table_bias,
                              dense, ids, label)

    def next(self, streams=None):
        j = self.i
        self.i += 1
        s = j % self.S
        with torch.cuda.stream(self.gs):
            for ue in (self.use_ev[s] or ()):
                self.gs.wait_event(ue)          # the slot's previous batch has been consumed
            self.generate(j, self.bufs[s])
            ev = self.gen_ev[s]
            ev.record(self.gs)
        for st in (streams or [torch.cuda.current_stream(self.dev)]):
            st.wait_event(ev)
        return self.bufs[s], s

    @property
    def copy_stream(self):
        """The generator's stream: a consumer may copy a batch out of its
        slot there (in order behind the generation, and before the slot is
        regenerated)."""
        return self.gs

    def owns(self, t: torch.Tensor) -> bool:
        """``t`` is one of this stream's slot buffers (ids, dense or labels)."""
        p = t.data_ptr()
        return any(p == b.data_ptr() for bs in self.bufs for b in bs)

    def release(self, slot: int, streams=None):
        sts = streams or [torch.cuda.current_stream(self.dev)]
        pool = self.rel_ev[slot]
        while len(pool) < len(sts):
            pool.append(self.ops.SyncEvent(2))
        for e, st in zip(pool, sts):
            e.record(st)
        self.use_ev[slot] = pool[:len(sts)]


class InStepSynthetic:
    """``DeviceSyntheticStream``'s batch sequence generated INSIDE the
    trainer's step (one-GPU DLRM / DCN-v2, ``DLRMTrainer.attach_in_step_source``):
    the ids kernel runs on the embedding stream right before the lookup and
    writes the trainer's id buffer, the dense/label kernel runs on the MLP
    stream at the start of the bottom forward and writes x0 (bf16) and the
    labels -- no side-stream generation, no copies and no cross-stream event
    waits per step (each costs ~10-23 us of queue idle on this ROCm,
    profiles/r04/prof_dlrm/step_lanes.txt). The batch index is read on the
    device from the trainer's step counter, so every graph replay draws the
    next batch; batch i equals ``DeviceSyntheticStream``'s batch i bit for bit."""

    in_step = True

    def __init__(self, table_rows: Sequence[int], batch_size: int, device, num_dense: int = 13,
                 pooling: Optional[Sequence[int]] = None, seed: int = 0, dist: str = "uniform",
                 zipf_alpha: float = 1.05, rank: int = 0, stream: int = 0, start: int = 0):
        self.g = DeviceSyntheticStream(table_rows, batch_size, device, num_dense=num_dense,
                                       pooling=pooling, seed=seed, dist=dist,
                                       zipf_alpha=zipf_alpha, rank=rank, stream=stream, slots=1,
                                       start=start)
        self.start = int(start)
        self.counter = None
        self.counter0 = None
        self.base = None

    # the batch index comes from the trainer's fp32 step counter, which
    # counts integers exactly only up to 2^24 (StepLoop refuses to run past)
    COUNTER_LIMIT = 1 << 24

    def bind(self, counter: torch.Tensor):
        """``counter``: the trainer's float step counter (bumped once per
        step, after both generators of the step have read it)."""
        self.counter = counter
        self.counter0 = int(round(float(counter.reshape(-1)[0].item())))
        self.base = self.start - self.counter0

    def check_steps(self, step_index: int, n: int):
        """Raise if steps [step_index, step_index + n) would read the fp32
        counter past its exact-integer range."""
        if self.counter0 is not None and \
                self.counter0 + (step_index - self.start) + n > self.COUNTER_LIMIT:
            raise RuntimeError("InStepSynthetic: the fp32 step counter indexes batches exactly "
                               f"only up to 2^24 steps; use --data fresh for longer runs")

    def gen_ids(self, ids: torch.Tensor):
        g = self.g
        g.ops._native().synth_ids(g.seed, g.rank, self.base, g.B, g.rows, g.pool_, g.base,
                                  g.dist, float(g.alpha), self.counter, g.nnz, ids)

    def gen_dense(self, x0: torch.Tensor, label: torch.Tensor):
        g = self.g
        g.ops._native().synth_dense(g.seed, g.rank, self.base, g.B, g.rows, g.pool_, g.base,
                                    g.dist, float(g.alpha), self.counter, g.w_dense,
                                    g.table_bias, x0, label)

    def next(self, streams=None):
        raise RuntimeError("InStepSynthetic batches are generated inside the trainer's step")

    def release(self, slot, streams=None):
        return None
