#!/usr/bin/env python
"""How does HIP run three per-stream composed graphs with cross-stream event
nodes (the multi-rank step's structure)? Segments are spin kernels of known
length with device timestamps around them; prints per-segment start/end
(us from the step's first stamp) for a few steady-state steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from tdfo_amd import ops
    from tdfo_amd.ops import _ext
    assert _ext.load()
    dev = torch.device("cuda", 0)
    order = os.environ.get("ORDER", "M,D,EC").split(",")
    steps = 8
    # segment name -> (stream, duration us)
    segs = {"M1": ("M", 30), "M2": ("M", 200), "M4": ("M", 70), "M3": ("M", 100),
            "D0": ("D", 80), "Dp": ("D", 60), "Da": ("D", 20), "Db": ("D", 80),
            "EC1": ("EC", 120), "ECu": ("EC", 30), "ECl": ("EC", 15), "ECb1": ("EC", 40),
            "ECb2": ("EC", 150)}
    names = list(segs)
    NS = len(names)
    buf = torch.zeros(steps * NS * 2 + 64, dtype=torch.int64, device=dev)
    cnt = torch.zeros(NS, dtype=torch.int64, device=dev)
    streams = {k: torch.cuda.Stream() for k in ("M", "D", "EC")}
    ev = {k: ops.SyncEvent(2) for k in ("e3", "d", "c5", "c4", "m2", "m3", "m4", "e0", "dp")}
    graphs = {}
    for i, (name, (st, us)) in enumerate(segs.items()):
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, stream=streams[st]):
            ops.stamp(buf, cnt, i, NS, 0)
            ops.spin_us(us)
            ops.stamp(buf, cnt, i, NS, 1)
        graphs[name] = g
    torch.cuda.synchronize()
    buf.zero_()
    cnt.zero_()

    def chain(parts):
        return ops.ComposedGraph([(k, graphs[v] if k == "graph" else ev[v]) for k, v in parts])
    comp = {
        "M": chain([("wait", "e3"), ("wait", "d"), ("graph", "M1"), ("wait", "c5"), ("graph", "M2"),
                    ("record", "m2"), ("graph", "M4"), ("record", "m4"), ("graph", "M3"),
                    ("record", "m3")]),
        "D": chain([("wait", "c4"), ("graph", "D0"), ("record", "e0"), ("wait", "m2"), ("graph", "Dp"),
                    ("record", "dp"), ("wait", "m4"), ("graph", "Da"), ("wait", "m3"), ("graph", "Db"),
                    ("record", "d")]),
        "EC": chain([("wait", "m2"), ("graph", "EC1"), ("wait", "e0"), ("wait", "dp"), ("graph", "ECu"),
                     ("wait", "m4"), ("graph", "ECl"), ("record", "e3"), ("graph", "ECb1"),
                     ("record", "c4"), ("graph", "ECb2"), ("record", "c5")]),
    }
    torch.cuda.synchronize()
    for step in range(steps):
        for k in order:
            with torch.cuda.stream(streams[k]):
                comp[k].replay()
    torch.cuda.synchronize()
    b = buf[: steps * NS * 2].view(steps, NS, 2).cpu()
    for step in range(2, steps):
        t0 = int(b[step, 0, 0])
        row = [f"{n}:{(int(b[step, i, 0]) - t0) / 100:.0f}-{(int(b[step, i, 1]) - t0) / 100:.0f}"
               for i, n in enumerate(names)]
        print(f"step {step}: " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
