"""hipGraph capture with Python's cyclic garbage collector paused.

A collection that runs while a stream is being captured can finalize objects
of an earlier trainer (torch CUDAGraphs, HIP events) sitting in a reference
cycle; their HIP destroy calls are illegal during a capture, and torch's graph
destructor then terminates the process. Collect first, then capture with the
collector off.
"""
from __future__ import annotations

import contextlib
import gc

import torch


@contextlib.contextmanager
def graph_capture(g: "torch.cuda.CUDAGraph", **kw):
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(g, **kw):
            yield
    finally:
        if was:
            gc.enable()
