"""Loader for the native HIP library (``tdfo_amd/lib/libtdfo_hip.so``).

Policy: GPU tensors always run the hand-written HIP kernels. If the library
is missing or fails to load while a GPU is present, every op raises — there
is no silent eager fallback on the GPU. CPU tensors run the fp32 torch
reference implementations in ``tdfo_amd.ops.reference`` (these are also the
oracles the GPU tests compare against).
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

# TDFO_LIB_PATH: load another build of the library (same-box A/B runs)
_LIB_PATH = Path(os.environ.get("TDFO_LIB_PATH") or
                 Path(__file__).resolve().parent.parent / "lib" / "libtdfo_hip.so")
_lock = threading.Lock()
_loaded = False
_error: Exception | None = None


def lib_path() -> Path:
    return _LIB_PATH


def load(build_if_missing: bool = True) -> bool:
    """Load the native op library once; returns True on success."""
    global _loaded, _error
    with _lock:
        if _loaded:
            return True
        try:
            if not _LIB_PATH.exists() and build_if_missing and os.environ.get("TDFO_NO_BUILD") != "1":
                from tdfo_amd._build import build_hip

                build_hip()
            torch.ops.load_library(str(_LIB_PATH))
            _loaded = True
            _error = None
        except Exception as e:  # pragma: no cover - reported by ops()
            _error = e
        return _loaded


def ops():
    """Return ``torch.ops.tdfo``; raise loudly if the native library is absent."""
    if not _loaded and not load():
        raise RuntimeError(
            f"tdfo_amd native HIP library unavailable ({_LIB_PATH}): {_error!r}. "
            "Run `python -m tdfo_amd._build` (hipcc --offload-arch=gfx950).")
    return torch.ops.tdfo


def available() -> bool:
    return load()
