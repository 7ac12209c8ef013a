"""Per-rank supervisor of a multi-rank run: a known-good fallback for the
first real N > 1 run.

Every rank process that ``torch.distributed.run`` starts (the driver's own
launch, or ``bench.py``'s self-launch) becomes a supervisor that never
touches the GPU: it runs the real rank code as a child process and waits.
The supervisors of all ranks then exchange their child's exit code through
the launcher's TCP store. If every child succeeded, the job is done. If any
failed -- the step watchdog's exit 3 (a hang), the replica check's exit 4
(diverged replicas), a pre-flight hang, a crash -- every supervisor starts
ONE fresh child on the known-good path (c10d collectives, staged replay:
``TDFO_COMM=torch`` and the caller's fallback arguments) and reports that
attempt's outcome. No exec is involved: the supervisor only ever starts
children.

Children rendezvous through a per-attempt key prefix of the same store
(``TDFO_STORE_PREFIX``, read by ``parallel/dist.init_distributed``), so an
attempt never reads a stale key of the one before it.

The reference's counterparts: fail-fast RPCs (tensorflow2/train_ps.py:39)
and c10d DDP as the always-available path (torchrec/train.py:197-198,
255-260).
"""
from __future__ import annotations

import ctypes
import datetime
import json
import os
import signal
import subprocess
import sys
import tempfile
from typing import Dict, List, Optional, Sequence

CHILD_ENV = "TDFO_SUPERVISED_CHILD"
METRIC_ENV = "TDFO_METRIC_OUT"


def emit_result(line: str) -> None:
    """A supervised child's result line: into the supervisor's per-attempt
    file (printed only if every rank's attempt succeeded), else stdout."""
    path = os.environ.get(METRIC_ENV)
    if not path:
        print(line, flush=True)
        return
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(line + "\n")
    os.replace(tmp, path)


def is_child() -> bool:
    return os.environ.get(CHILD_ENV) == "1"


def _die_with_parent():
    # the child gets SIGTERM if its supervisor dies (e.g. the launcher tears
    # the job down): no orphan keeps the GPU
    try:
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)   # PR_SET_PDEATHSIG
    except OSError:
        pass


def _store(rank: int, world: int, timeout_s: float):
    from torch.distributed import TCPStore
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    to = datetime.timedelta(seconds=timeout_s)
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
        return TCPStore(addr, port, world_size=world, is_master=False, timeout=to)
    # no launcher store: rank 0's supervisor hosts one (its children connect
    # as clients, never host)
    return TCPStore(addr, port, world_size=world, is_master=rank == 0, timeout=to,
                    wait_for_workers=False)


def _exchange(store, tag: str, rank: int, world: int, rc: int) -> List[int]:
    store.set(f"tdfo_sup/{tag}/rc/{rank}", str(rc))
    out = []
    for r in range(world):
        k = f"tdfo_sup/{tag}/rc/{r}"
        try:
            store.wait([k])
            out.append(int(store.get(k)))
        except Exception:  # noqa: BLE001 -- a peer supervisor that never reports
            out.append(-1000)
    return out


def _wait_or_peer_failed(child, store, tag: str, rank: int, world: int, poll_s: float) -> int:
    """Wait for the child; if another rank's child already failed this
    attempt (its supervisor posted a non-zero code), end ours instead of
    leaving it blocked in a collective until its watchdog fires (fail fast,
    the role of GRPC_FAIL_FAST in tensorflow2/train_ps.py:39)."""
    import time
    peers = [r for r in range(world) if r != rank]
    while True:
        try:
            return child.wait(timeout=poll_s)
        except subprocess.TimeoutExpired:
            pass
        for r in peers:
            key = f"tdfo_sup/{tag}/rc/{r}"
            try:
                if store.check([key]) and int(store.get(key)) != 0:
                    child.terminate()
                    try:
                        child.wait(timeout=10)
                    except subprocess.TimeoutExpired:
                        child.kill()
                        child.wait()
                    print(json.dumps({"supervisor": "peer failed, child ended", "rank": rank,
                                      "peer": r}), file=sys.stderr, flush=True)
                    return 128 + signal.SIGTERM
            except Exception:  # noqa: BLE001 -- a store hiccup: keep waiting
                time.sleep(poll_s)


def supervise(child_argv: Sequence[str], attempts: Sequence[Dict[str, str]],
              fallback_argv: Sequence[Sequence[str]] = (), rank: Optional[int] = None,
              world: Optional[int] = None, timeout_s: float = 1800.0,
              poll_s: float = 0.5) -> int:
    """Run ``child_argv`` once per attempt until every rank's child exits 0.

    attempts[k]: extra environment of attempt k; fallback_argv[k] (k >= 1):
    extra arguments appended on attempt k. Returns the exit code to report
    (0, or the last attempt's first non-zero code)."""
    rank = int(os.environ.get("RANK", 0)) if rank is None else rank
    world = int(os.environ.get("WORLD_SIZE", 1)) if world is None else world
    store = _store(rank, world, timeout_s)
    child = None

    def _fwd(sig, _frame):
        if child is not None and child.poll() is None:
            child.send_signal(sig)
        sys.exit(128 + sig)
    for s in (signal.SIGTERM, signal.SIGINT):
        signal.signal(s, _fwd)
    run_id = os.environ.get("TORCHELASTIC_RUN_ID", "") + os.environ.get(
        "TORCHELASTIC_RESTART_COUNT", "")
    rc_final = 1
    metric_files: Dict[int, str] = {}
    ok_attempt = None
    for k, extra in enumerate(attempts):
        env = dict(os.environ)
        env.update(extra)
        env[CHILD_ENV] = "1"
        env["TDFO_ATTEMPT"] = str(k)
        env["TDFO_STORE_PREFIX"] = f"tdfo/{run_id}/attempt{k}/"
        # a child's result line (bench.py's metric JSON) goes to this file;
        # only the attempt every rank completed gets it printed on stdout
        env[METRIC_ENV] = metric_files[k] = os.path.join(
            tempfile.gettempdir(), f"tdfo_metric_{os.getpid()}_{k}.json")
        argv = list(child_argv) + (list(fallback_argv[k - 1]) if k >= 1 and
                                   k - 1 < len(fallback_argv) else [])
        child = subprocess.Popen(argv, env=env, preexec_fn=_die_with_parent)
        rc = _wait_or_peer_failed(child, store, f"{run_id}/{k}", rank, world, poll_s)
        child = None
        rcs = _exchange(store, f"{run_id}/{k}", rank, world, rc)
        if all(x == 0 for x in rcs):
            rc_final = 0
            ok_attempt = k
            break
        rc_final = next(x for x in rcs if x != 0)
        if rc_final == -1000:
            rc_final = 1
        if rank == 0:
            print(json.dumps({"supervisor": "attempt failed", "attempt": k, "exit_codes": rcs,
                              "next": ("fallback: " + json.dumps(attempts[k + 1]))
                              if k + 1 < len(attempts) else None}),
                  file=sys.stderr, flush=True)
    for k, path in metric_files.items():
        if not os.path.exists(path):
            continue
        with open(path) as f:
            line = f.read().strip()
        os.unlink(path)
        if k == ok_attempt:
            print(line, flush=True)
        elif line:
            print(json.dumps({"supervisor": "metric line of a failed attempt discarded",
                              "attempt": k}), file=sys.stderr, flush=True)
    # keep the store (hosted by rank 0's supervisor when there is no launcher
    # store) alive until every supervisor has read the verdict
    try:
        store.add(f"tdfo_sup/{run_id}/done", 1)
        if rank == 0:
            import time
            t0 = time.monotonic()
            while int(store.add(f"tdfo_sup/{run_id}/done", 0)) < world and \
                    time.monotonic() - t0 < 60:
                time.sleep(0.05)
    except Exception:  # noqa: BLE001
        pass
    return rc_final
