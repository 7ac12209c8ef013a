"""Multi-process CPU (gloo) test harness: run ``fn(rank, world, *args)`` in
``world`` spawned processes and collect their return values."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _to_bytes(obj):
    import io

    import torch
    buf = io.BytesIO()
    torch.save(obj, buf)        # by value: no shared-memory fds outlive the worker
    return buf.getvalue()


def _from_bytes(b):
    import io

    import torch
    return torch.load(io.BytesIO(b), weights_only=True)


def _worker(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        import torch
        torch.set_num_threads(1)
        from tdfo_amd.parallel import dist as tdist
        tdist.init_distributed("cpu", "gloo", timeout_s=120)
        out = fn(rank, world, *args)
        q.put((rank, "ok", _to_bytes(out)))
        tdist.reset()
    except Exception:  # pragma: no cover
        q.put((rank, "err", traceback.format_exc()))


def run_distributed(fn, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{out}")
            res[rank] = _from_bytes(out)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [res[r] for r in range(world)]
