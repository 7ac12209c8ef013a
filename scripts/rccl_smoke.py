#!/usr/bin/env python
"""Step-by-step smoke of the native RCCL layer on a one-rank communicator
(prints before every call; run with -X faulthandler to see a crash site)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def p(*a):
    print(*a, flush=True)


def main():
    from tdfo_amd.ops import _ext
    assert _ext.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    p("maps:", sorted({l.split()[-1] for l in open("/proc/self/maps") if "rccl" in l}))
    uid = torch.ops.tdfo.rccl_unique_id()
    p("uid", uid[:8].tolist())
    h = int(torch.ops.tdfo.rccl_init(uid, 1, 0))
    p("init ok", h, torch.ops.tdfo.rccl_info(h))
    x = torch.randn(1000, device=dev)
    t = x.clone()
    p("all_reduce sync")
    torch.ops.tdfo.rccl_all_reduce(h, t, 0, False)
    torch.cuda.synchronize()
    p("ok", bool(torch.equal(t, x)))
    out = torch.empty_like(x)
    p("all_to_all sync")
    torch.ops.tdfo.rccl_all_to_all(h, out, x, [], [], False)
    torch.cuda.synchronize()
    p("ok", bool(torch.equal(out, x)))
    p("all_to_all async")
    tok = torch.ops.tdfo.rccl_all_to_all(h, out, x, [1000], [1000], True)
    torch.ops.tdfo.rccl_wait(h, tok)
    torch.cuda.synchronize()
    p("ok", tok)
    p("destroy")
    torch.ops.tdfo.rccl_destroy(h)
    p("done raw")
    if "--pg" in sys.argv:
        import datetime

        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", rank=0, world_size=1,
                                timeout=datetime.timedelta(seconds=60), device_id=dev)
        p("pg ok")
        from tdfo_amd.parallel.comm import as_comm
        c = as_comm(None)
        p("comm", type(c).__name__, c.h)
        c.all_to_all(out, x)
        torch.cuda.synchronize()
        p("a2a ok")
        w = c.all_to_all(out, x.bfloat16().float(), [1000], [1000], async_op=True)
        w.wait()
        torch.cuda.synchronize()
        p("a2a async ok")
        from tdfo_amd.utils.capture import graph_capture
        a = torch.randn(4096, device=dev)
        b = torch.empty_like(a)
        y = torch.empty_like(a)
        g = torch.cuda.CUDAGraph()
        p("capture")
        with graph_capture(g, capture_error_mode="thread_local"):
            tmp = a * 2.0
            w = c.all_to_all(b, tmp, async_op=True)
            p(" in capture: a2a issued")
            c.all_reduce(a, async_op=False)
            p(" in capture: ar issued")
            w.wait()
            y.copy_(b + 1.0)
        p("captured")
        g.replay()
        torch.cuda.synchronize()
        p("replay ok", bool(torch.equal(y, a * 2 + 1)))
        from tdfo_amd.parallel.dist import reset
        reset()
        p("reset ok")


if __name__ == "__main__":
    main()
