"""Multi-rank guards for the contract entrypoints (``recipes/*/train*.py``).

``bench.py`` is not the only multi-rank entry: ``torchrun ... train_dp.py`` /
``train_ps.py`` (DLRM configs 3-5, TwoTower) and ``recipes/bert4rec/train.py``
go onto the same native RCCL-in-graphs path. They get the same two guards:

* ``supervised(main)`` wraps a recipe's ``__main__``: at world size > 1 every
  rank process becomes a GPU-free supervisor (utils/supervise.py) that runs
  the rank code as a child. If any rank's child fails (watchdog exit 3, a
  replica mismatch, a pre-flight hang, a crash), every rank starts one
  fallback child with ``FALLBACK_ENV``: c10d collectives, staged replay (no
  collectives inside graphs) and ``TDFO_RESUME=1``, so the second attempt
  restores the latest complete checkpoint (DLRM ``ckpt_dir`` step_N,
  TwoTower ``backup/``) instead of starting at step 0.
* ``rank_preflight(info)`` runs inside each rank before the trainer is built:
  the collective self-test of parallel/preflight.py on both communicators;
  on a mismatch every rank switches to the c10d path (``TDFO_COMM=torch``,
  ``TDFO_STREAM_GRAPHS=0``) in-process.

The reference pairs fail-fast with automatic restore on its multi-process
path (``GRPC_FAIL_FAST``, tensorflow2/train_ps.py:39; ``BackupAndRestore``,
tensorflow2/train_ps.py:148-157) and keeps c10d DDP as its known-good path
(torchrec/train.py:197-198,255-260).
"""
from __future__ import annotations

import json
import os
import sys
from typing import Callable, Dict, Optional

from . import supervise

FALLBACK_ENV = {"TDFO_COMM": "torch", "TDFO_STREAM_GRAPHS": "0", "TDFO_RESUME": "1"}

# HIP runtime mode of one-GPU, one-process runs (bench.py and the one-GPU
# recipes): graph nodes dispatched at launch instead of from AQL packets
# captured at instantiation. DLRM-1TB 0.405-0.409 vs 0.422-0.425 ms/step;
# DCN-v2 / TwoTower neutral. Not for rank processes: it raises host issue
# per step (emulated W=8 340 -> 477 us) that a rank cannot afford
# (profiles/r05/notes.md). A DEBUG_ CLR knob: the JSON line of bench.py
# reports its value and who set it. Read by the runtime at its first call,
# so this must run before any GPU work. An explicit setting wins.
PACKET_CAPTURE = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"


def one_gpu_runtime_mode(one_gpu: bool) -> Dict[str, str]:
    """Set the one-GPU HIP runtime mode (if ``one_gpu`` and not set by the
    caller); returns {"value", "source"} for reporting."""
    if PACKET_CAPTURE in os.environ:
        return {"value": os.environ[PACKET_CAPTURE], "source": "environment"}
    if one_gpu:
        os.environ[PACKET_CAPTURE] = "0"
        return {"value": "0", "source": "tdfo default (one GPU)"}
    return {"value": "1", "source": "runtime default"}


def _world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def supervised(main: Callable[[], object], argv=None) -> None:
    """Run ``main`` directly (one rank, a supervised child, or
    ``TDFO_SUPERVISE=0``), or supervise this very command at world size > 1
    and exit with the supervisor's code. Call before any GPU work."""
    if _world() > 1 and not supervise.is_child() and \
            os.environ.get("TDFO_SUPERVISE", "1") == "1":
        cmd = [sys.executable, os.path.abspath(sys.argv[0]),
               *(sys.argv[1:] if argv is None else argv)]
        sys.exit(supervise.supervise(cmd, attempts=[{}, dict(FALLBACK_ENV)]))
    main()


def resume_requested(cfg_resume: bool = False) -> bool:
    """Config ``resume = true`` or the supervisor's fallback attempt."""
    return bool(cfg_resume) or os.environ.get("TDFO_RESUME") == "1"


def stream_graphs_allowed() -> bool:
    """False on the fallback path (collectives stay outside graphs)."""
    return os.environ.get("TDFO_STREAM_GRAPHS", "1") != "0"


def rank_preflight(info) -> Optional[Dict]:
    """Collective self-test at world size > 1 (every rank calls it, before
    the trainer is built). Skipped when already on the c10d path or with
    ``TDFO_PREFLIGHT=0``. On failure: ``TDFO_COMM=torch`` (set by preflight)
    and ``TDFO_STREAM_GRAPHS=0``."""
    if info.world_size <= 1 or os.environ.get("TDFO_PREFLIGHT", "1") == "0":
        return None
    if os.environ.get("TDFO_COMM") == "torch":
        return {"ok": True, "skipped": "c10d path"}
    from ..parallel.preflight import preflight
    timeout = float(os.environ.get("TDFO_PREFLIGHT_TIMEOUT_S", "120"))
    pf = preflight(info.group, info.device, timeout_s=timeout)
    if not pf["ok"]:
        os.environ["TDFO_STREAM_GRAPHS"] = "0"
    path = ("native" if pf.get("comm") == "RcclComm" else "c10d") if pf["ok"] else "c10d-staged"
    print(json.dumps({"preflight": pf, "rank": info.rank, "comm_path": path}),
          file=sys.stderr, flush=True)
    return pf
