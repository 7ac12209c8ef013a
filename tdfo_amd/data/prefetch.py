"""Host -> device input pipeline for the DLRM / DCN-v2 trainers.

The role of the reference's ``prefetch_to_device(size=2)``
(jax-flax/train_dp.py:210-211) and tf.data's AUTOTUNE prefetch
(tensorflow2/data.py:171-210): the multi-threaded C++ generator
(csrc/data/synthetic.cpp, or any host batch source with the same
``batch(i)`` contract) fills pinned host slots on a background thread,
``lookahead`` batches ahead; each batch is copied host -> device on a
dedicated copy stream into one of ``stages`` rotating device staging slots
(default 6: deep enough that the host polling loop never has to block), and
the compute stream only waits on that copy's event. The trainer's ``load_batch`` then
moves staging -> its static (graph-captured) inputs with one fused kernel,
so the H2D of batch i+1 overlaps step i.

Slot reuse is event-ordered both ways, checked on the launching thread by
polling (never by blocking waits that would hold the GIL, never by
device-side waits that make ROCm's async copy block the host): a host slot
is rewritten only after the H2D that read it completed, a device staging
slot is overwritten only after the consumer's kernels that read it ran.
"""
from __future__ import annotations

import time
from concurrent.futures import ThreadPoolExecutor
from typing import Optional, Tuple

import torch


class HostPrefetcher:
    def __init__(self, gen, device, start: int = 0, lookahead: int = 2, stages: int = 6):
        """``gen``: host batch source with ``batch(i) -> (dense, ids, label)``
        writing into pinned buffer set ``i % gen.nbuf`` (needs nbuf >=
        lookahead + 2). ``stages`` device staging slots."""
        if gen.nbuf < lookahead + 2:
            raise ValueError("host generator needs >= lookahead + 2 buffer sets")
        self.gen = gen
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.L = int(lookahead)
        self.H = gen.nbuf
        self.S = int(stages)
        self.copy = torch.cuda.Stream(self.dev) if self.cuda else None
        from .. import ops
        self.ops = ops
        d0, i0, l0 = gen._bufs[0]
        self.stage = [(torch.empty(d0.shape, dtype=d0.dtype, device=self.dev),
                       torch.empty(i0.shape, dtype=i0.dtype, device=self.dev),
                       torch.empty(l0.shape, dtype=l0.dtype, device=self.dev))
                      for _ in range(self.S)]
        self.h2d_ev = [None] * self.H
        self.use_ev = [None] * self.S
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="tdfo-prefetch")
        self.futs = {}
        self.t_wait_gen = self.t_submit = 0.0      # host seconds blocked (diagnostics)
        self.i = int(start)
        for j in range(self.i, self.i + self.L):
            self._submit(j)

    def _submit(self, j: int):
        # host slot j % H was last read by the H2D of batch j - H; with H >=
        # L + 2 that copy was issued >= 2 steps ago, so this wait (on the
        # launching thread, never inside the worker: a worker blocking in
        # Event.synchronize() holds the GIL the launching thread needs) is
        # back-pressure only when the GPU falls that far behind
        ev = self.h2d_ev[j % self.H]
        while ev is not None and not ev.query():
            time.sleep(20e-6)       # poll: a spinning hipEventSynchronize steals a core
        self.futs[j] = self.pool.submit(self.gen.batch, j)   # ctypes: GIL released

    def next(self, streams=None) -> Tuple[Tuple[torch.Tensor, torch.Tensor, torch.Tensor], int]:
        """Device tensors (dense, ids, label) of the next batch (ordered on the
        current stream, or on every stream of ``streams``) and their staging
        slot; call ``release(slot)`` once the consumer has enqueued its reads
        of them."""
        j = self.i
        self.i += 1
        t0 = time.perf_counter()
        host = self.futs.pop(j).result()
        self.t_wait_gen += time.perf_counter() - t0
        s = j % self.S
        dst = self.stage[s]
        if self.cuda:
            # staging slot s was last read by batch j - S's load; check that on
            # the host (a device-side wait on the copy stream makes ROCm's
            # hipMemcpyAsync block the launching thread until the GPU gets
            # there: measured 0.5 ms per step). With S above the depth the
            # launching thread runs ahead, this poll only bites as back-pressure.
            for ue in (self.use_ev[s] or ()):
                while not ue.query():
                    time.sleep(20e-6)
            with torch.cuda.stream(self.copy):
                for d, h in zip(dst, host):
                    d.copy_(h, non_blocking=True)
                # (events without the system-scope fence: see
                # DeviceSyntheticStream; the host only polls their completion)
                ev = self.ops.SyncEvent(2)
                ev.record(self.copy)
            self.h2d_ev[j % self.H] = ev
            for st in (streams or [torch.cuda.current_stream(self.dev)]):
                st.wait_event(ev)
        else:
            for d, h in zip(dst, host):
                d.copy_(h)
        t1 = time.perf_counter()
        self._submit(j + self.L)
        self.t_submit += time.perf_counter() - t1
        return dst, s

    def release(self, slot: int, streams=None):
        """``streams``: every stream that reads the slot (default: current);
        the slot is refilled once each of them has passed this point."""
        if self.cuda:
            evs = []
            for st in (streams or [torch.cuda.current_stream(self.dev)]):
                e = self.ops.SyncEvent(2)
                e.record(st)
                evs.append(e)
            self.use_ev[slot] = evs

    def close(self):
        self.pool.shutdown(wait=True)


def host_prefetcher(table_rows, batch: int, device, pooling=None, seed: int = 0, rank: int = 0,
                    dist: str = "uniform", zipf_alpha: float = 1.05, threads: int = 4,
                    start: int = 0, lookahead: int = 2, stream: int = 0,
                    num_dense: int = 13) -> Optional[HostPrefetcher]:
    """Prefetcher over the C++ synthetic Criteo generator (pinned host slots)."""
    from .synthetic import HostSyntheticCriteo
    cuda = torch.device(device).type == "cuda"
    gen = HostSyntheticCriteo(table_rows, batch, num_dense, pooling=pooling, seed=seed, dist=dist,
                              zipf_alpha=zipf_alpha, rank=rank, threads=threads, pin=cuda,
                              stream=stream, nbuf=lookahead + 4)
    return HostPrefetcher(gen, device, start=start, lookahead=lookahead)
