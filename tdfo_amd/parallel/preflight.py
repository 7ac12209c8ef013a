"""Pre-flight self-test of the collective layer before a multi-rank run.

At N > 1 the training step replays RCCL collectives from a communicator of
our own (``RcclComm``, plus its dense-gradient twin) inside per-stream
hipGraphs. ``preflight`` exercises exactly those entry points for a few
milliseconds before the trainer is built -- every collective kind and dtype
the step uses, on both communicators, issued eagerly (sync and async) and
replayed from a captured graph -- and checks the results bit for bit
against values every rank computes locally (each rank's inputs are a known
function of its rank; integer-valued data, so any reduction order gives the
exact sum). The ranks then agree on the verdict through a MIN all-reduce on
the process group.

On a mismatch (or an exception) the native communicators are released and
``TDFO_COMM=torch`` is set, so the trainer built next takes the known-good
path: c10d collectives and staged replay (no collectives inside graphs; the
caller turns ``stream_graphs`` off). A hang inside the pre-flight ends the
rank with exit code 3 after ``timeout_s`` -- ``bench.py``'s supervisor then
restarts the ranks on the c10d path.

The reference keeps a known-good path in the same spirit: c10d DDP beside
DMP (torchrec/train.py:197-198,255-260) and fail-fast RPCs
(tensorflow2/train_ps.py:39).

Test hook: ``TDFO_PREFLIGHT_INJECT=<rank>`` corrupts that rank's first
result, which must drive every rank to the fallback.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, Dict, List, Tuple

import torch
import torch.distributed as dist

from .comm import Comm, RcclComm, as_comm, dense_comm_for, release_native

# (kind, dtype, elements per rank chunk): the step's collectives -- id
# all-to-alls (int64 / int32), pooled rows and their gradients (bf16), uneven
# all-to-all, row-wise reduce-scatter / all-gather (fp32, bf16), the dense
# gradient all-reduce (fp32 or bf16) and the capacity / metric MAX all-reduce
CASES = [("a2a", torch.int64, 96), ("a2a", torch.int32, 40), ("a2a", torch.bfloat16, 256),
         ("a2av", torch.float32, 0), ("ag", torch.float32, 64), ("ag", torch.bfloat16, 48),
         ("rs", torch.float32, 128), ("rs", torch.bfloat16, 64), ("ar", torch.float32, 1000),
         ("ar", torch.bfloat16, 512), ("armax", torch.float32, 33)]


def _data(r: int, n: int, dtype, device, salt: int) -> torch.Tensor:
    """Rank r's input: small integers (exact in bf16 and in any sum of up to
    64 of them), distinct per rank, position and salt; ids rank-tagged."""
    i = torch.arange(n, device=device, dtype=torch.int64)
    v = (i * 7 + r * 13 + salt * 5) % 61 - 30
    if dtype in (torch.int32, torch.int64):
        v = v + 1000 * r
    return v.to(dtype)


def _uneven(W: int, r: int) -> List[int]:
    """Elements rank r sends to each peer in the uneven all-to-all."""
    return [1 + ((r * 3 + p * 5) % 7) * 4 for p in range(W)]


def make_case(kind: str, dtype, n: int, W: int, r: int, device, salt: int
              ) -> Tuple[torch.Tensor, torch.Tensor, Callable[[Comm, bool], object]]:
    """(output buffer, expected output, issue(comm, async_op)) of one
    collective; the output of an all-reduce starts as this rank's input and
    ``issue`` resets it first (so a captured graph replays correctly)."""
    if kind == "a2a":
        inp = _data(r, n * W, dtype, device, salt)
        out = torch.empty_like(inp)
        exp = torch.cat([_data(p, n * W, dtype, device, salt)[r * n:(r + 1) * n]
                         for p in range(W)])
        return out, exp, lambda c, a: c.all_to_all(out, inp, async_op=a)
    if kind == "a2av":
        ins = _uneven(W, r)
        outs = [_uneven(W, p)[r] for p in range(W)]
        inp = _data(r, sum(ins), dtype, device, salt)
        out = torch.empty(sum(outs), dtype=dtype, device=device)
        parts = []
        for p in range(W):
            sp = _uneven(W, p)
            off = sum(sp[:r])
            parts.append(_data(p, sum(sp), dtype, device, salt)[off:off + sp[r]])
        return out, torch.cat(parts), lambda c, a: c.all_to_all(out, inp, outs, ins, async_op=a)
    if kind == "ag":
        inp = _data(r, n, dtype, device, salt)
        out = torch.empty(n * W, dtype=dtype, device=device)
        exp = torch.cat([_data(p, n, dtype, device, salt) for p in range(W)])
        return out, exp, lambda c, a: c.all_gather(out, inp, async_op=a)
    if kind == "rs":
        inp = _data(r, n * W, dtype, device, salt)
        out = torch.empty(n, dtype=dtype, device=device)
        exp = sum(_data(p, n * W, dtype, device, salt)[r * n:(r + 1) * n].double()
                  for p in range(W)).to(dtype)
        return out, exp, lambda c, a: c.reduce_scatter(out, inp, async_op=a)
    inp = _data(r, n, dtype, device, salt)
    out = inp.clone()
    if kind == "ar":
        exp = sum(_data(p, n, dtype, device, salt).double() for p in range(W)).to(dtype)
        op = "sum"
    else:
        exp = torch.stack([_data(p, n, dtype, device, salt) for p in range(W)]).amax(0)
        op = "max"

    def issue(c, a):
        out.copy_(inp)
        return c.all_reduce(out, op, async_op=a)
    return out, exp, issue


def _eager(comm: Comm, W: int, r: int, device, salt: int, mode: str, bad: List[str],
           inject: bool) -> None:
    for kind, dtype, n in CASES:
        out, exp, issue = make_case(kind, dtype, n, W, r, device, salt)
        h = issue(comm, mode == "async")
        if mode == "async" and h is not None:
            h.wait()
        if inject and not bad:
            out.view(-1)[0] += 1
        if not torch.equal(out.cpu(), exp.cpu()):
            bad.append(f"{type(comm).__name__}:{mode}:{kind}:{str(dtype)[6:]}")


def _captured(comm: Comm, W: int, r: int, device, salt: int, bad: List[str]) -> None:
    """Every collective captured into one graph on a side stream (the
    capture's origin, as the step graphs route them), replayed twice."""
    cases = [make_case(kind, dtype, n, W, r, device, salt) for kind, dtype, n in CASES]
    torch.cuda.synchronize(device)
    s = torch.cuda.Stream(device)
    g = torch.cuda.CUDAGraph()
    ctx = comm.capture_origin(s) if isinstance(comm, RcclComm) else None
    with torch.cuda.stream(s):
        if ctx is not None:
            ctx.__enter__()
        try:
            with torch.cuda.graph(g, stream=s):
                for out, exp, issue in cases:
                    issue(comm, False)
        finally:
            if ctx is not None:
                ctx.__exit__(None, None, None)
    for _ in range(2):
        for out, _, _ in cases:
            out.fill_(0)
        g.replay()
        torch.cuda.synchronize(device)
        for (kind, dtype, _), (out, exp, _) in zip(CASES, cases):
            if not torch.equal(out.cpu(), exp.cpu()):
                bad.append(f"{type(comm).__name__}:graph:{kind}:{str(dtype)[6:]}")
                return


def preflight(group=None, device=None, capture: bool = True, timeout_s: float = 120.0) -> Dict:
    """Self-test the collectives the multi-rank step will use (collective:
    every rank calls it). Returns {"ok", "failed", "comm", "ms"}; on failure
    the native communicators are released and ``TDFO_COMM=torch`` is set."""
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    device = torch.device(device) if device is not None else torch.device("cpu")
    t0 = time.perf_counter()
    done = threading.Event()

    def _guard():
        if not done.wait(timeout_s):
            print(f'{{"preflight": "hang", "rank": {r}, "timeout_s": {timeout_s}}}',
                  file=sys.stderr, flush=True)
            os._exit(3)
    if timeout_s > 0:
        threading.Thread(target=_guard, name="tdfo-preflight-guard", daemon=True).start()
    inj = os.environ.get("TDFO_PREFLIGHT_INJECT")
    inject = inj is not None and int(inj) == r
    bad: List[str] = []
    name = "?"
    try:
        c = as_comm(group)
        name = type(c).__name__
        comms = [c]
        d = dense_comm_for(c)
        if d is not c:
            comms.append(d)
        for k, cm in enumerate(comms):
            for mode in ("sync", "async"):
                _eager(cm, W, r, device, k, mode, bad, inject)
            if capture and device.type == "cuda" and cm.capturable:
                _captured(cm, W, r, device, 7 + k, bad)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
    except Exception as e:  # noqa: BLE001 -- any failure selects the fallback
        bad.append(f"exception: {type(e).__name__}: {e}")
    # every rank must take the same path: agree through the process group
    pg_dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    flag = torch.tensor([0 if bad else 1], dtype=torch.int32, device=pg_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    ok = bool(flag.item())
    done.set()
    if not ok:
        release_native()
        os.environ["TDFO_COMM"] = "torch"
    return {"ok": ok, "failed": bad[:8], "comm": name,
            "ms": round((time.perf_counter() - t0) * 1e3, 1)}
