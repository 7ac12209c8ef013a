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


def _worker(rank, world, port, fn, args, q, device="cpu"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    if device == "cuda":
        # every rank on cuda:0, gloo between them (RCCL refuses two ranks on
        # one GPU): the multi-rank step runs on the real HIP kernels
        os.environ.update(TDFO_SHARE_DEVICE="1", TDFO_DIST_BACKEND="gloo")
    try:
        import torch
        torch.set_num_threads(1)
        from tdfo_amd.parallel import dist as tdist
        if device == "cuda_rccl":
            # one rank per GPU over RCCL (a one-rank group on a one-GPU box)
            import datetime

            import torch.distributed as dist
            torch.cuda.set_device(rank)
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=120),
                                    device_id=torch.device("cuda", rank))
            out = fn(rank, world, *args)
            q.put((rank, "ok", _to_bytes(out)))
            tdist.reset()
            return
        tdist.init_distributed(device, "gloo", timeout_s=120)
        out = fn(rank, world, *args)
        q.put((rank, "ok", _to_bytes(out)))
        tdist.reset()
    except Exception:  # pragma: no cover
        q.put((rank, "err", traceback.format_exc()))


def run_distributed(fn, world, *args, timeout=300, device="cpu"):
    """``device="cuda"``: ranks share cuda:0 over gloo (fresh spawned processes);
    ``"cuda_rccl"``: rank r on cuda:r over RCCL (world <= visible GPUs)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q, device))
             for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    res = {}
    failed = False
    try:
        deadline = time.time() + timeout
        while len(res) < world:
            try:
                rank, status, out = q.get(timeout=0.5)
            except queue.Empty:
                dead = [i for i, p in enumerate(procs) if p.exitcode not in (None, 0)
                        and i not in res]
                if dead:
                    failed = True
                    raise RuntimeError(f"rank(s) {dead} died with exit codes "
                                       f"{[procs[i].exitcode for i in dead]}")
                if time.time() > deadline:
                    failed = True
                    raise TimeoutError("distributed test timed out")
                continue
            if status != "ok":
                failed = True
                raise RuntimeError(f"rank {rank} failed:\n{out}")
            res[rank] = _from_bytes(out)
    finally:
        for p in procs:
            p.join(timeout=1 if failed else 30)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return [res[r] for r in range(world)]
