#!/usr/bin/env python
"""Which RCCL collectives survive hipGraph stream capture on this image?
Each mode runs in a child process (a crash ends only that child)."""
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MODES = ["nested_fresh", "single_used", "nested_used", "nested_fresh_origin_arg"]


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

    if mode in ("pg_origin_side", "pg_compose"):
        # capture on a non-default origin stream (the comm stream) and, for
        # compose, chain it into one executable graph with event nodes
        from tdfo_amd import ops
        cs = torch.cuda.Stream()
        ev0, ev1 = ops.SyncEvent(2), ops.SyncEvent(2)
        gs = []
        for k in range(2):
            g = torch.cuda.CUDAGraph(keep_graph=mode == "pg_compose")
            with torch.cuda.graph(g, stream=cs, capture_error_mode="thread_local"):
                if k == 0:
                    torch.ops.tdfo.rccl_all_to_all(h, b, a, [], [], False)
                else:
                    torch.ops.tdfo.rccl_all_reduce(h, b, 0, False)
                    b.add_(1.0)
            gs.append(g)
        print(mode, "captured", flush=True)
        a.fill_(2.0)
        if mode == "pg_compose":
            cg = ops.ComposedGraph([("graph", gs[0]), ("record", ev0), ("wait", ev0),
                                    ("graph", gs[1])])
            print(mode, "composed", flush=True)
            with torch.cuda.stream(cs):
                cg.replay()
        else:
            with torch.cuda.stream(cs):
                gs[0].replay()
                gs[1].replay()
        torch.cuda.synchronize()
        print(mode, "replay ok", bool((b == 3.0).all()), flush=True)
        return
    if mode.startswith("nested_") or mode == "single_used":
        x = torch.randn(1 << 20, device=dev)
        M, P = torch.cuda.Stream(), torch.cuda.Stream()
        if "used" in mode:
            with torch.cuda.stream(P):
                x.mul_(1.0)
            torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        kw = {"stream": torch.cuda.Stream()} if mode.endswith("origin_arg") else {}
        with torch.cuda.graph(g, capture_error_mode="thread_local", **kw):
            o = torch.cuda.current_stream()
            if mode.startswith("nested"):
                M.wait_stream(o)
                with torch.cuda.stream(M):
                    x.mul_(1.0)
                    P.wait_stream(M)
                    with torch.cuda.stream(P):
                        x.add_(1.0)
                    M.wait_stream(P)
                o.wait_stream(M)
            else:
                P.wait_stream(o)
                with torch.cuda.stream(P):
                    x.add_(1.0)
                o.wait_stream(P)
        print(mode, "captured", flush=True)
        g.replay()
        torch.cuda.synchronize()
        print(mode, "replay ok", flush=True)
        return
    if mode.startswith("fork_") or mode == "origin_memcpy":
        S = torch.cuda.Stream()
        x = torch.randn(1 << 20, device=dev)
        y = torch.empty_like(x)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            x.mul_(1.0)
            cur = torch.cuda.current_stream()
            if mode == "origin_memcpy":
                y.copy_(x)
            else:
                S.wait_stream(cur)
                with torch.cuda.stream(S):
                    if mode == "fork_memcpy":
                        y.copy_(x)
                    elif mode == "fork_memset":
                        y.zero_()
                    elif mode == "fork_kernel":
                        y.copy_(x * 1.0)
                    elif mode == "fork_memcpy_native_ev":
                        y.copy_(x)
                cur.wait_stream(S)
        print(mode, "captured", flush=True)
        g.replay()
        torch.cuda.synchronize()
        print(mode, "replay ok", flush=True)
        return
    if mode.startswith("pg_origin_join"):
        # origin = comm stream C; compute forked onto M; C waits on M's
        # event, RCCL on C, M waits C's event; end joined
        C = torch.cuda.Stream()
        M = torch.cuda.Stream()
        x = torch.randn(4096, device=dev)
        y = torch.empty_like(x)
        z = torch.empty_like(x)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=C, capture_error_mode="thread_local"):
            M.wait_stream(C)
            with torch.cuda.stream(M):
                x2 = x * 2.0
            C.wait_stream(M)
            if mode.endswith("tok"):
                with torch.cuda.stream(M):
                    t = torch.ops.tdfo.rccl_all_to_all(h, y, x2, [], [], True)
                    torch.ops.tdfo.rccl_wait(h, t)
            else:
                torch.ops.tdfo.rccl_all_to_all(h, y, x2, [], [], False)
            M.wait_stream(C)
            with torch.cuda.stream(M):
                z.copy_(y + 1.0)
            C.wait_stream(M)
        print(mode, "captured", flush=True)
        with torch.cuda.stream(C):
            g.replay()
        torch.cuda.synchronize()
        print(mode, "replay ok", bool(torch.equal(z, x * 2 + 1)), flush=True)
        return
    if mode == "pg_loopback_fork":
        from tdfo_amd.parallel.comm import LoopbackComm
        lb = LoopbackComm(4, 0, dev)
        x = torch.randn(4096, device=dev)
        y = torch.empty_like(x)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            w = lb.all_to_all(y, x, async_op=True)
            w.wait()
            y.add_(1.0)
        g.replay()
        torch.cuda.synchronize()
        print(mode, "replay ok", flush=True)
        return
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
