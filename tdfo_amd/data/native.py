"""ctypes bindings of the C++ host data library (``csrc/data``):
TFRecord/Example codec (tfrecord.cpp) and the threaded batch loader
(loader.cpp). The library is built by ``python -m tdfo_amd._build``; if it is
missing these functions raise (no silent Python fallback)."""
from __future__ import annotations

import ctypes as C
import threading
from pathlib import Path
from typing import Dict, Iterator, List, Optional, Sequence

import numpy as np
import torch

_LIB = Path(__file__).resolve().parent.parent / "lib" / "libtdfo_data.so"
_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    with _lock:
        if _lib is None:
            if not _LIB.exists():
                from tdfo_amd._build import build_data
                build_data()
            L = C.CDLL(str(_LIB))
            L.tdfo_crc32c.restype = C.c_uint32
            L.tdfo_crc32c.argtypes = [C.c_void_p, C.c_size_t]
            L.tdfo_masked_crc32c.restype = C.c_uint32
            L.tdfo_masked_crc32c.argtypes = [C.c_void_p, C.c_size_t]
            L.tdfo_tfrecord_write.restype = C.c_int
            L.tdfo_tfrecord_write.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_char_p),
                                              C.POINTER(C.c_int), C.POINTER(C.c_void_p),
                                              C.c_int64]
            L.tdfo_tfrecord_count.restype = C.c_int64
            L.tdfo_tfrecord_count.argtypes = [C.c_char_p, C.c_int, C.c_int]
            L.tdfo_tfrecord_read.restype = C.c_int64
            L.tdfo_tfrecord_read.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_char_p),
                                             C.POINTER(C.c_int), C.POINTER(C.c_void_p), C.c_int64,
                                             C.c_int]
            L.tdfo_loader_create.restype = C.c_void_p
            L.tdfo_loader_create.argtypes = [C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int),
                                             C.c_int64, C.c_int64, C.c_uint64, C.c_int, C.c_int,
                                             C.c_int, C.c_int, C.c_int, C.c_int,
                                             C.POINTER(C.c_void_p)]
            L.tdfo_loader_start_epoch.restype = C.c_int64
            L.tdfo_loader_start_epoch.argtypes = [C.c_void_p, C.c_int64]
            L.tdfo_loader_next.restype = C.c_int
            L.tdfo_loader_next.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
            L.tdfo_loader_release.restype = None
            L.tdfo_loader_release.argtypes = [C.c_void_p, C.c_int]
            L.tdfo_loader_destroy.restype = None
            L.tdfo_loader_destroy.argtypes = [C.c_void_p]
            L.tdfo_synth_criteo.restype = None
            L.tdfo_synth_criteo.argtypes = [C.c_uint64, C.c_int, C.c_int64, C.c_int, C.c_int,
                                            C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_double,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_int]
            _lib = L
    return _lib


def crc32c(data: bytes) -> int:
    return lib().tdfo_crc32c(data, len(data))


# ------------------------------------------------------------ TFRecord
def _schema(columns: Dict[str, np.ndarray]):
    names = list(columns)
    types = []
    arrs = []
    for n in names:
        a = np.asarray(columns[n])
        if a.dtype.kind in "iub":
            arrs.append(np.ascontiguousarray(a, dtype=np.int64))
            types.append(0)
        elif a.dtype.kind == "f":
            arrs.append(np.ascontiguousarray(a, dtype=np.float32))
            types.append(1)
        else:
            raise TypeError(f"column {n}: unsupported dtype {a.dtype}")
    return names, types, arrs


def tfrecord_write(path: str, columns: Dict[str, np.ndarray], gzip: bool = True):
    """One tf.train.Example per row; int columns -> Int64List, floats -> FloatList
    (the layout of tensorflow2/data.py:108-131)."""
    names, types, arrs = _schema(columns)
    n = len(arrs[0])
    assert all(len(a) == n for a in arrs)
    cn = (C.c_char_p * len(names))(*[s.encode() for s in names])
    ct = (C.c_int * len(types))(*types)
    cp = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    rc = lib().tdfo_tfrecord_write(str(path).encode(), int(gzip), len(names), cn, ct, cp, n)
    if rc != 0:
        raise IOError(f"tfrecord write failed ({rc}): {path}")


def tfrecord_count(path: str, gzip: bool = True, check_crc: bool = True) -> int:
    n = lib().tdfo_tfrecord_count(str(path).encode(), int(gzip), int(check_crc))
    if n < 0:
        raise IOError(f"corrupt tfrecord file: {path}")
    return n


def tfrecord_read(path: str, schema: Dict[str, str], gzip: bool = True,
                  check_crc: bool = True) -> Dict[str, np.ndarray]:
    """schema: name -> "int64" | "float32". Returns numpy columns."""
    n = tfrecord_count(path, gzip, check_crc)
    names = list(schema)
    types = [0 if schema[k] == "int64" else 1 for k in names]
    outs = [np.zeros(n, dtype=np.int64 if t == 0 else np.float32) for t in types]
    cn = (C.c_char_p * len(names))(*[s.encode() for s in names])
    ct = (C.c_int * len(types))(*types)
    cp = (C.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
    r = lib().tdfo_tfrecord_read(str(path).encode(), int(gzip), len(names), cn, ct, cp, n,
                                 int(check_crc))
    if r != n:
        raise IOError(f"tfrecord read failed ({r}) in {path}")
    return dict(zip(names, outs))


# ------------------------------------------------------------ loader
class HostLoader:
    """Threaded, deterministic, rank-sharded batch loader over host columns.

    ``columns`` are numpy arrays of equal length (kept alive by this object);
    batches are collated by C++ worker threads into ``nslots`` pinned slots
    and handed out in order. Iterating yields dicts of torch tensors: device
    tensors if ``device`` is given (async H2D, slot released once the copy has
    completed), else CPU views that are valid until the next iteration.
    """

    def __init__(self, columns: Dict[str, np.ndarray], batch_size: int, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False, rank: int = 0, world_size: int = 1,
                 num_workers: int = 2, prefetch: int = 4, device=None, pin: Optional[bool] = None):
        self.names = list(columns)
        self.cols = [np.ascontiguousarray(columns[k]) for k in self.names]
        n = len(self.cols[0])
        assert all(len(c) == n for c in self.cols), "ragged columns"
        self.nrows, self.B = n, int(batch_size)
        self.device = torch.device(device) if device is not None else None
        pin = (self.device is not None and self.device.type == "cuda") if pin is None else pin
        self.nslots = max(2, int(prefetch))
        self.slots: List[List[torch.Tensor]] = []
        for _ in range(self.nslots):
            row = []
            for c in self.cols:
                t = torch.from_numpy(np.zeros(self.B, dtype=c.dtype))
                row.append(t.pin_memory() if pin else t)
            self.slots.append(row)
        ptrs = [self.slots[s][c].data_ptr() for s in range(self.nslots) for c in range(len(self.cols))]
        cp = (C.c_void_p * len(self.cols))(*[c.ctypes.data for c in self.cols])
        es = (C.c_int * len(self.cols))(*[c.dtype.itemsize for c in self.cols])
        sp = (C.c_void_p * len(ptrs))(*ptrs)
        self._h = lib().tdfo_loader_create(len(self.cols), cp, es, n, self.B, seed, int(shuffle),
                                           int(drop_last), rank, world_size, max(1, num_workers),
                                           self.nslots, sp)
        if not self._h:
            raise ValueError("invalid loader arguments")
        self.epoch = 0
        self.world, self.drop_last = world_size, drop_last
        # H2D runs on its own stream (the compute stream only waits on an
        # event), so copies of the next batch overlap the current step
        self._copy_stream = (torch.cuda.Stream(self.device)
                             if self.device is not None and self.device.type == "cuda" else None)

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def __len__(self):
        gb = self.B * self.world
        return self.nrows // gb if self.drop_last else -(-self.nrows // gb)

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        L = lib()
        nb = L.tdfo_loader_start_epoch(self._h, self.epoch)
        rows = C.c_int64(0)
        pending = None          # (slot, event)
        for _ in range(nb):
            slot = L.tdfo_loader_next(self._h, C.byref(rows))
            if slot < 0:
                break
            r = int(rows.value)
            if self.device is None:
                if pending is not None:
                    L.tdfo_loader_release(self._h, pending[0])
                pending = (slot, None)
                yield {k: self.slots[slot][i][:r] for i, k in enumerate(self.names)}
            else:
                ev = None
                if self._copy_stream is not None:
                    cur = torch.cuda.current_stream(self.device)
                    with torch.cuda.stream(self._copy_stream):
                        out = {k: self.slots[slot][i][:r].to(self.device, non_blocking=True)
                               for i, k in enumerate(self.names)}
                        ev = torch.cuda.Event()
                        ev.record(self._copy_stream)
                    cur.wait_event(ev)
                    for t in out.values():        # allocated on the copy stream, used on cur
                        t.record_stream(cur)
                else:
                    out = {k: self.slots[slot][i][:r].to(self.device, non_blocking=True)
                           for i, k in enumerate(self.names)}
                if pending is not None:
                    if pending[1] is not None:
                        pending[1].synchronize()
                    L.tdfo_loader_release(self._h, pending[0])
                pending = (slot, ev)
                yield out
        if pending is not None:
            if pending[1] is not None:
                pending[1].synchronize()
            L.tdfo_loader_release(self._h, pending[0])

    def close(self):
        if getattr(self, "_h", None):
            lib().tdfo_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
