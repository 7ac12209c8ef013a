"""Collective layer of the sharded engine and the DLRM trainer.

Every exchange the north-star step makes goes through a ``Comm``: the
pooled-embedding / id all-to-alls, the row-wise reduce-scatter and
all-gathers, the bucketed dense-gradient all-reduce and the capacity MAX
all-reduce (the reference's equivalents: TorchRec DMP's input/output dists
and the DDP reducer, torchrec/train.py:241-260; TF PS pulls/pushes,
tensorflow2/train_ps.py:55-61).

Three implementations:

* ``RcclComm`` (default for an RCCL group): the native layer
  ``csrc/comm/rccl_comm.cpp`` -- a communicator of its own, every collective
  enqueued from C++ (no c10d work objects), so the whole multi-rank step
  captures into one hipGraph (``capturable``);
* ``ProcessGroupComm``: a torch.distributed group -- gloo on CPU and in the
  shared-GPU rehearsal, or RCCL through c10d with ``TDFO_COMM=torch``.
  Collectives run on the process group's own stream; ``async_op`` handles
  make the caller's current stream wait device-side (never the host).
* ``LoopbackComm``: rank ``rank`` of a ``world``-rank job emulated in one
  process (``bench.py --emulate-world 8``): the real W-rank plan, layouts and
  kernels run, and each collective becomes device copies of the same byte
  count on a dedicated comm stream, with the data of this rank's own
  segment replicated into every peer's slot (so exchanged ids stay valid row
  ids of the tables this rank owns). Device time per step then shows every
  W-dependent kernel cost and the host time per step the full issue cost of
  the multi-rank step, without needing W GPUs.

All count calls and bytes per kind (``stats``), so a step's collective
volume is reported next to its time.
"""
from __future__ import annotations

import os
from collections import defaultdict
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


class _Done:
    def wait(self):
        return None


class _EventWork:
    """Handle of a collective enqueued on a comm stream: ``wait`` orders the
    caller's current stream after it (device-side)."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


def _splits(n: int, W: int, splits: Optional[Sequence[int]]) -> List[int]:
    if splits is None:
        assert n % W == 0, f"equal-split exchange of {n} elements over {W} ranks"
        return [n // W] * W
    s = [int(x) for x in splits]
    assert len(s) == W and sum(s) == n, (s, n, W)
    return s


class Comm:
    """Collective interface (subclasses implement the ``_``-prefixed ops)."""

    world: int = 1
    rank: int = 0
    # every op only enqueues device work (no host wait, no host-side
    # transport): a step issuing them can be captured into one hipGraph
    capturable: bool = False

    def __init__(self):
        self.stats = defaultdict(lambda: [0, 0])     # kind -> [calls, bytes moved by this rank]

    def _count(self, kind: str, t: torch.Tensor):
        s = self.stats[kind]
        s[0] += 1
        s[1] += t.numel() * t.element_size()

    def reset_stats(self):
        self.stats.clear()

    # -- public API (counting wrappers)
    def all_to_all(self, out, inp, out_splits=None, in_splits=None, async_op=False):
        """out[slot r] = what rank r sends here; inp[slot r] goes to rank r."""
        self._count("all_to_all", inp)
        return self._all_to_all(out, inp, out_splits, in_splits, async_op)

    def all_gather(self, out, inp, async_op=False):
        """out = concat over ranks of inp (rank-major)."""
        self._count("all_gather", out)
        return self._all_gather(out, inp, async_op)

    def reduce_scatter(self, out, inp, async_op=False):
        """out = sum over ranks of their inp chunk [rank] (equal chunks)."""
        self._count("reduce_scatter", inp)
        return self._reduce_scatter(out, inp, async_op)

    def all_reduce(self, t, op: str = "sum", async_op=False):
        self._count("all_reduce_" + op, t)
        return self._all_reduce(t, op, async_op)

    def broadcast(self, t, src: int = 0):
        self._count("broadcast", t)
        return self._broadcast(t, src)

    def barrier(self):
        return None


class ProcessGroupComm(Comm):
    """torch.distributed group (RCCL on MI355X, gloo on CPU)."""

    def __init__(self, group=None):
        super().__init__()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.backend = dist.get_backend(group) if dist.is_initialized() else None

    def _all_to_all(self, out, inp, out_splits, in_splits, async_op):
        if out_splits is None and in_splits is None and not (inp.is_cuda and self.backend == "gloo"):
            return dist.all_to_all_single(out, inp, group=self.group, async_op=async_op)
        # explicit splits: gloo's equal-split device all-to-all mangles bf16
        # (measured on the shared-GPU rehearsal); the split-size form is exact
        os_ = _splits(out.numel(), self.world, out_splits)
        is_ = _splits(inp.numel(), self.world, in_splits)
        return dist.all_to_all_single(out, inp, output_split_sizes=os_, input_split_sizes=is_,
                                      group=self.group, async_op=async_op)

    def _all_gather(self, out, inp, async_op):
        return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)

    def _reduce_scatter(self, out, inp, async_op):
        if inp.is_cuda and self.backend == "gloo":
            # gloo has no device reduce-scatter (shared-GPU rehearsal backend):
            # an all-to-all of the chunks + an in-order sum
            W = self.world
            tmp = torch.empty_like(inp)
            n = inp.numel() // W
            self._all_to_all(tmp, inp, [n] * W, [n] * W, False)
            out.copy_(tmp.view(W, -1).float().sum(0))
            return _Done()
        return dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=async_op)

    def _all_reduce(self, t, op, async_op):
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        return dist.all_reduce(t, op=rop, group=self.group, async_op=async_op)

    def _broadcast(self, t, src):
        return dist.broadcast(t, src=src, group=self.group)

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)


class _RcclWork:
    __slots__ = ("h", "tok")

    def __init__(self, h: int, tok: int):
        self.h, self.tok = h, tok

    def wait(self):
        torch.ops.tdfo.rccl_wait(self.h, self.tok)


class RcclComm(Comm):
    """The native collective layer (``csrc/comm/rccl_comm.cpp``): an RCCL
    communicator of its own over the ranks of ``group``, every op issued from
    C++ on the caller's stream (sync) or forked onto the communicator's stream
    (async, joined by ``wait``) -- nothing blocks the host, so a whole
    multi-rank step, collectives included, captures into one hipGraph
    (``capturable``). The torch process group only carries the unique id."""

    capturable = True

    def __init__(self, group=None, device=None):
        super().__init__()
        from .. import ops  # noqa: F401  (loads the native library)
        from ..ops import _ext
        if not _ext.load():
            raise RuntimeError("RcclComm needs the native HIP library (tdfo_amd/lib/libtdfo_hip.so)")
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        dev = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.device = dev
        self._origin = None
        uid = torch.ops.tdfo.rccl_unique_id() if self.rank == 0 else torch.zeros(128, dtype=torch.uint8)
        if self.world > 1:
            backend = dist.get_backend(group)
            t = uid.to(dev) if backend == "nccl" else uid
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(t, src=src, group=group)
            uid = t.cpu()
        with torch.cuda.device(dev):
            self.h = int(torch.ops.tdfo.rccl_init(uid, self.world, self.rank))

    # Under stream capture RCCL must be enqueued on the capture's ORIGIN
    # stream: a collective on any stream joined into the capture by an event
    # wait (torch's own async c10d collectives included) crashes
    # hipStreamEndCapture on this ROCm (labs/probes/rccl_capture_probe.py). So a
    # capturing caller names its origin (``capture_origin``) and every
    # collective goes there -- origin waits on the caller's stream, the
    # collective runs, the caller's stream waits on it (async: when the handle
    # is waited). Eagerly, async ops fork onto the communicator's own stream
    # in C++ (event record + wait, no Python stream objects).
    def capture_origin(self, stream):
        """Context: route collectives through ``stream`` (the origin of the
        capture in progress)."""
        comm = self

        class _Ctx:
            def __enter__(self_):
                comm._origin = stream

            def __exit__(self_, *a):
                comm._origin = None
                return False

        return _Ctx()

    def _run(self, fn, async_op: bool):
        o = self._origin
        if o is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("RcclComm: collective inside a stream capture without "
                                   "capture_origin(stream) (RCCL must run on the origin stream)")
            tok = fn(async_op)
            return _RcclWork(self.h, int(tok)) if async_op else None
        cur = torch.cuda.current_stream(self.device)
        if cur == o:
            fn(False)
            return None if not async_op else _Done()
        o.wait_stream(cur)
        with torch.cuda.stream(o):
            fn(False)
        if not async_op:
            cur.wait_stream(o)
            return None
        ev = torch.cuda.Event()
        ev.record(o)
        return _EventWork(ev)

    def _all_to_all(self, out, inp, out_splits, in_splits, async_op):
        os_ = [] if out_splits is None else [int(x) for x in out_splits]
        is_ = [] if in_splits is None else [int(x) for x in in_splits]
        o, i = out.view(-1), inp.reshape(-1)
        return self._run(lambda a: torch.ops.tdfo.rccl_all_to_all(self.h, o, i, os_, is_, a),
                         async_op)

    def _all_gather(self, out, inp, async_op):
        o, i = out.view(-1), inp.reshape(-1)
        return self._run(lambda a: torch.ops.tdfo.rccl_all_gather(self.h, o, i, a), async_op)

    def _reduce_scatter(self, out, inp, async_op):
        o, i = out.view(-1), inp.reshape(-1)
        return self._run(lambda a: torch.ops.tdfo.rccl_reduce_scatter(self.h, o, i, a), async_op)

    def _all_reduce(self, t, op, async_op):
        code = {"sum": 0, "max": 1, "min": 2}[op]
        v = t.view(-1)
        return self._run(lambda a: torch.ops.tdfo.rccl_all_reduce(self.h, v, code, a), async_op)

    def _broadcast(self, t, src):
        torch.ops.tdfo.rccl_broadcast(self.h, t.view(-1), int(src))

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    def close(self):
        if getattr(self, "h", None) is not None:
            torch.ops.tdfo.rccl_destroy(self.h)
            self.h = None


class LoopbackComm(Comm):
    """Rank ``rank`` of a ``world``-rank job in one process (see module doc).

    Data semantics: every peer is taken to send what this rank sends to
    itself (all-to-all), to hold this rank's tensor (all-gather), and to
    contribute nothing to a reduction (all-reduce / reduce-scatter keep this
    rank's values) -- so the numbers stay finite and exchanged ids stay in
    range. Byte counts per call equal the real collective's."""

    def __init__(self, world: int, rank: int = 0, device=None, link_gbps: float = 0.0,
                 latency_us: float = 0.0):
        super().__init__()
        assert 0 <= rank < world
        self.capturable = device is not None and torch.device(device).type == "cuda"
        self.world, self.rank = int(world), int(rank)
        self.device = torch.device(device) if device is not None else None
        self._stream = None
        self._scratch = None
        # modelled xGMI time (GPU only): after its local copies each collective
        # holds the comm stream for latency_us + (bytes over the links) /
        # link_gbps -- this rank's injection bandwidth into the other W-1 --
        # so the emulated step also shows where the exchanges would sit on
        # the critical path (0: copies only)
        self.link_gbps = float(link_gbps)
        self.latency_us = float(latency_us)
        self.modelled_us = 0.0
        self._origin = None
        self._idx = {}
        self._maps = {}
        self._rs_tmp = None

    def _copy_pieces(self, src, dst, pieces) -> bool:
        """dst[b:b+n] = src[a:a+n] for (a, b, n) in pieces (flat elements of
        one dtype) in one native seg_copy launch over an int64 view, cached per
        piece list, so the emulated exchanges run no torch kernels. False when
        not applicable (CPU, misaligned, too many pieces)."""
        if not src.is_cuda or not pieces or len(pieces) > 4096:
            return False
        from .. import ops
        if not ops.native_available():
            return False
        es = src.element_size()
        if dst.element_size() != es or not (src.is_contiguous() and dst.is_contiguous()):
            return False
        if (src.numel() * es) % 8 or (dst.numel() * es) % 8 \
                or (src.storage_offset() * es) % 8 or (dst.storage_offset() * es) % 8:
            return False
        if any((v * es) % 8 for p in pieces for v in p):
            return False
        key = (tuple(pieces), es, str(src.device))
        m = self._maps.get(key)
        if m is None:
            if len(self._maps) >= 256:
                self._maps.clear()
            m = self._maps[key] = ops.SegmentMap([(a * es // 8, b * es // 8, n * es // 8)
                                                  for a, b, n in pieces], src.device)
        m.apply(src.reshape(-1).view(torch.int64), dst.reshape(-1).view(torch.int64))
        return True

    def _model(self, link_bytes: float):
        if self._stream is None or (self.link_gbps <= 0 and self.latency_us <= 0):
            return
        us = self.latency_us + (link_bytes / (self.link_gbps * 1e3) if self.link_gbps > 0 else 0.0)
        self.modelled_us += us
        from .. import ops
        ops.spin_us(us)

    def capture_origin(self, stream):
        """Context: during a whole-step capture the emulated collectives run
        on the capture's origin stream (as RcclComm's must), so no forked
        stream is the source of another fork (see DLRMTrainer._wait)."""
        comm = self

        class _Ctx:
            def __enter__(self_):
                comm._origin = stream

            def __exit__(self_, *a):
                comm._origin = None
                return False

        return _Ctx()

    def _begin(self, t):
        if not t.is_cuda:
            return None
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=t.device)
        s = self._origin if self._origin is not None else self._stream
        cur = torch.cuda.current_stream(t.device)
        if cur != s:
            s.wait_stream(cur)
        return s

    def _end(self, s, async_op):
        if s is None:
            return _Done()
        if s == torch.cuda.current_stream(s.device):     # ran on the caller's stream
            return _Done() if async_op else None
        ev = torch.cuda.Event()
        ev.record(s)
        w = _EventWork(ev)
        if not async_op:
            w.wait()
            return None
        return w

    def _all_to_all(self, out, inp, out_splits, in_splits, async_op):
        W, r = self.world, self.rank
        os_ = _splits(out.numel(), W, out_splits)
        is_ = _splits(inp.numel(), W, in_splits)
        src0 = sum(is_[:r])
        own = inp.view(-1)[src0: src0 + is_[r]]
        o = out.view(-1)
        s = self._begin(inp)
        es = inp.element_size()
        with torch.cuda.stream(s) if s is not None else _nullctx():
            if all(n == own.numel() for n in os_):          # one broadcast copy
                n = own.numel()
                if not self._copy_pieces(inp, o, [(src0, k * n, n) for k in range(W)]):
                    o.view(W, -1).copy_(own.view(1, -1).expand(W, -1))
            elif inp.is_floating_point():
                # values (pooled rows / gradients): only their finiteness
                # matters downstream -- one contiguous copy of as many bytes as
                # fit (the exact tiling below ran ~100 us at W = 8, an
                # emulation cost a real exchange does not have)
                k = min(o.numel(), inp.numel())
                o[:k].copy_(inp.reshape(-1)[:k])
            elif own.numel():
                # out[slot r] = this rank's own segment tiled to slot r's
                # length: one gather launch through a cached index map (a copy
                # per slot cost ~4 us of device time each at W = 8)
                # gathered in units of u elements (<= 64 B) that divide every
                # segment, so the index map is u x shorter
                u = 1
                for c in (64 // es, 32 // es, 16 // es, 8 // es, 4 // es, 2 // es):
                    if c > 1 and all(x % c == 0 for x in list(os_) + list(is_) + [src0]):
                        u = c
                        break
                n_own, pieces, b = own.numel(), [], 0
                for n in os_:
                    for k in range(0, n, n_own):
                        pieces.append((src0, b + k, min(n_own, n - k)))
                    b += n
                if not self._copy_pieces(inp, o, pieces):
                    key = (tuple(os_), src0, own.numel(), u, str(o.device))
                    idx = self._idx.get(key)
                    if idx is None:
                        n_own = own.numel() // u
                        parts = [torch.arange(n // u, dtype=torch.int64) % n_own for n in os_]
                        idx = self._idx[key] = (torch.cat(parts) + src0 // u).to(o.device)
                    torch.index_select(inp.reshape(-1, u), 0, idx, out=o.view(-1, u))
            self._model(max(sum(is_) - is_[r], sum(os_) - os_[r]) * es)
        return self._end(s, async_op)

    def _all_gather(self, out, inp, async_op):
        s = self._begin(inp)
        with torch.cuda.stream(s) if s is not None else _nullctx():
            n = inp.numel()
            if not self._copy_pieces(inp, out, [(0, k * n, n) for k in range(self.world)]):
                out.view(self.world, -1).copy_(inp.view(1, -1).expand(self.world, -1))
            self._model(out.numel() * out.element_size() * (self.world - 1) / self.world)
        return self._end(s, async_op)

    def _reduce_scatter(self, out, inp, async_op):
        n = out.numel()
        s = self._begin(inp)
        with torch.cuda.stream(s) if s is not None else _nullctx():
            # reads all W chunks like the real reduction (their sum would
            # scale the values W-fold; this rank's own chunk is kept)
            from .. import ops
            if inp.is_cuda and inp.dtype == torch.float32 and ops.native_available() \
                    and inp.numel() == self.world * n:
                if self._rs_tmp is None or self._rs_tmp.numel() < n:
                    self._rs_tmp = torch.empty(n, dtype=torch.float32, device=inp.device)
                ops.slab_reduce([(inp, self.world, self._rs_tmp[:n])])
            else:
                tmp = inp.view(self.world, -1)[:, :n].sum(0, dtype=torch.float32)
                del tmp
            if not self._copy_pieces(inp, out, [(self.rank * n, 0, n)]):
                out.view(-1).copy_(inp.view(-1)[self.rank * n: (self.rank + 1) * n])
            self._model(inp.numel() * inp.element_size() * (self.world - 1) / self.world)
        return self._end(s, async_op)

    def _all_reduce(self, t, op, async_op):
        s = self._begin(t)
        with torch.cuda.stream(s) if s is not None else _nullctx():
            if t.numel() > 64:
                # a ring all-reduce reads and writes the buffer ~2x
                if self._scratch is None or self._scratch.numel() < t.numel() * t.element_size():
                    self._scratch = torch.empty(t.numel() * t.element_size(), dtype=torch.uint8,
                                                device=t.device)
                sc = self._scratch[: t.numel() * t.element_size()].view(t.dtype).view(t.shape)
                sc.copy_(t)
                t.copy_(sc)
            self._model(2 * t.numel() * t.element_size() * (self.world - 1) / self.world)
        return self._end(s, async_op)

    def _broadcast(self, t, src):
        return None


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_NATIVE: dict = {}
_TWINS: dict = {}


def dense_comm_for(comm: Comm) -> Comm:
    """A second communicator over the same ranks for the dense-gradient
    all-reduces, where collectives are stream-ordered enqueues (native RCCL:
    a new communicator, created collectively here the first time and cached
    per communicator, so trainers built one after another share it; loopback:
    a twin), so they run concurrently with the embedding exchanges on their
    own stream. Other layers (c10d / gloo) share ``comm``.

    Two communicators are deadlock-free here because their collectives are
    issued in one fixed order on every rank: each communicator's collectives
    sit on one stream (embedding exchanges on EC, dense all-reduces on D),
    inside graphs every rank captured from the same code and launches in the
    same order (models/dlrm_multirank.py); the staged / eager paths issue both
    from one host thread in the same stage order on every rank."""
    if isinstance(comm, RcclComm):
        twin = _TWINS.get(id(comm))
        if twin is None or twin.h is None:
            twin = _TWINS[id(comm)] = RcclComm(comm.group, comm.device)
        return twin
    if isinstance(comm, LoopbackComm):
        return LoopbackComm(comm.world, comm.rank, comm.device, comm.link_gbps, comm.latency_us)
    return comm


def as_comm(group=None) -> Comm:
    """A ``Comm`` for ``group``: itself if it is one; for an RCCL ("nccl")
    group the native ``RcclComm`` (one communicator per group, cached;
    ``TDFO_COMM=torch`` keeps the c10d path); else the torch process group
    wrapped (gloo, or None outside torch.distributed: a one-rank no-op)."""
    if isinstance(group, Comm):
        return group
    if (dist.is_initialized() and dist.get_backend(group) == "nccl"
            and os.environ.get("TDFO_COMM", "native") != "torch"):
        key = id(group) if group is not None else None
        c = _NATIVE.get(key)
        if c is None:
            c = _NATIVE[key] = RcclComm(group)
        return c
    return ProcessGroupComm(group)


def release_native():
    """Destroy the cached native communicators and their ``dense_comm_for``
    twins (before the process group)."""
    for c in list(_TWINS.values()) + list(_NATIVE.values()):
        c.close()
    _TWINS.clear()
    _NATIVE.clear()
