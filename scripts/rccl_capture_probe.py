#!/usr/bin/env python
"""Which RCCL collectives survive hipGraph stream capture on this image?
Each mode runs in a child process (a crash ends only that child)."""
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MODES = ["pg_a2a_async", "pg_a2a_async_prio2", "pg_a2a_async_prio0", "pg_a2a_torchstream",
         "raw_a2a_torchstream", "pg_torch_a2a_async", "pg_cls_async"]


def child(mode):
    import datetime

    import torch.distributed as dist
    from tdfo_amd.ops import _ext
    assert _ext.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if mode.startswith("pg"):
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29541", RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", rank=0, world_size=1,
                                timeout=datetime.timedelta(seconds=60), device_id=dev)
    h = int(torch.ops.tdfo.rccl_init(torch.ops.tdfo.rccl_unique_id(), 1, 0))
    side = torch.cuda.Stream()
    cls = None
    if mode == "pg_cls_async":
        from tdfo_amd.parallel.comm import as_comm
        cls = as_comm(None)
    a = torch.randn(4096, device=dev)
    b = torch.empty_like(a)

    def body():
        if mode.endswith("ar_sync") or mode.endswith("ar_sync_nomix"):
            torch.ops.tdfo.rccl_all_reduce(h, a, 0, False)
        elif mode.endswith("a2a_sync") or mode.endswith("a2a_sync_n2"):
            torch.ops.tdfo.rccl_all_to_all(h, b, a, [], [], False)
        elif "a2a_async" in mode and "torch" not in mode:
            t = torch.ops.tdfo.rccl_all_to_all(h, b, a, [], [], True)
            torch.ops.tdfo.rccl_wait(h, t)
        elif mode.endswith("torchstream"):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                torch.ops.tdfo.rccl_all_to_all(h, b, a, [], [], False)
            torch.cuda.current_stream().wait_stream(side)
        elif mode == "pg_cls_async":
            w = cls.all_to_all(b, a, async_op=True)
            cls.all_reduce(a, async_op=True).wait()
            w.wait()
        elif mode == "pg_torch_a2a_async":
            dist.all_to_all_single(b, a, async_op=True).wait()
        elif mode == "pg_torch_ar":
            dist.all_reduce(a)
        b.add_(1.0)

    body()
    torch.cuda.synchronize()
    print(mode, "eager ok", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        body()
    print(mode, "captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(mode, "replay ok", flush=True)


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    for m in MODES:
        env = dict(os.environ)
        if m.endswith("nomix"):
            env["NCCL_GRAPH_MIXING_SUPPORT"] = "0"
        if "prio" in m:
            env["TDFO_RCCL_PRIO"] = m[-1]
        r = subprocess.run([sys.executable, "-X", "faulthandler", "-u", __file__, m], env=env,
                           capture_output=True, text=True, timeout=120)
        last = [l for l in r.stdout.splitlines() if l.startswith(m)]
        print(f"{m}: rc={r.returncode} last={last[-1] if last else None}", flush=True)
        if r.returncode != 0:
            err = [l for l in r.stderr.splitlines() if "File" in l or "error" in l.lower()][:6]
            print("   ", "\n    ".join(err), flush=True)


if __name__ == "__main__":
    main()
