#!/usr/bin/env python
"""Cross-stream hand-off latency on MI355X: event record/wait vs signal-memory
value write/wait (ops.SignalFlag), eager and as executable-graph nodes
(ops.ComposedGraph). A producer stream spins ~50 us then stamps the device
wall clock and signals; a consumer stream waits, then stamps. The latency is
consumer stamp - producer stamp (100 MHz clock), median over the repeats.

Also checks that a value-wait graph launched BEFORE its producer graph waits
for it (an event wait node would bind to the previous record instead).
"""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402
from tdfo_amd.ops import _ext  # noqa: E402
from tdfo_amd.utils.capture import graph_capture  # noqa: E402

N = 40


def lat(buf):
    b = buf.cpu().view(-1, 2, 2)          # [k][seg][which]
    d = [(int(b[k, 1, 0]) - int(b[k, 0, 1])) / 100.0 for k in range(N)]
    return round(statistics.median(d[2:]), 2), round(min(d[2:]), 2), round(max(d[2:]), 2)


def fresh(dev):
    return (torch.zeros(N * 4 + 8, dtype=torch.int64, device=dev),
            torch.zeros(2, dtype=torch.int64, device=dev))


def main():
    assert _ext.load(), "native library missing"
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}

    # eager events
    buf, cnt = fresh(dev)
    for k in range(N):
        ev = ops.SyncEvent(2)
        with torch.cuda.stream(s1):
            ops.spin_us(50.0)
            ops.stamp(buf, cnt, 0, 2, 0)
            ops.stamp(buf, cnt, 0, 2, 1)
            ev.record()
        with torch.cuda.stream(s2):
            ev.wait()
            ops.stamp(buf, cnt, 1, 2, 0)
            ops.stamp(buf, cnt, 1, 2, 1)
        torch.cuda.synchronize()
    out["eager_event_us"] = lat(buf)
    print(json.dumps(out), flush=True)

    # eager value flags (consumer enqueued first: it must wait for the write)
    buf, cnt = fresh(dev)
    f = ops.SignalFlag()
    for k in range(1, N + 1):
        with torch.cuda.stream(s2):
            f.wait(k)
            ops.stamp(buf, cnt, 1, 2, 0)
            ops.stamp(buf, cnt, 1, 2, 1)
        with torch.cuda.stream(s1):
            ops.spin_us(50.0)
            ops.stamp(buf, cnt, 0, 2, 0)
            ops.stamp(buf, cnt, 0, 2, 1)
            f.write(k)
        torch.cuda.synchronize()
    out["eager_value_us"] = lat(buf)
    print(json.dumps(out), flush=True)

    # graphs: producer [spin, stamps] + signal, consumer wait + [stamps]
    def capture(fn, stream):
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with graph_capture(g, stream=stream):
            fn()
        return g

    buf, cnt = fresh(dev)
    gp = capture(lambda: (ops.spin_us(50.0), ops.stamp(buf, cnt, 0, 2, 0),
                          ops.stamp(buf, cnt, 0, 2, 1)), s1)
    gc = capture(lambda: (ops.stamp(buf, cnt, 1, 2, 0), ops.stamp(buf, cnt, 1, 2, 1)), s2)
    ev = ops.SyncEvent(2)
    P = ops.ComposedGraph([("graph", gp), ("record", ev)])
    C = ops.ComposedGraph([("wait", ev), ("graph", gc)])
    cnt.zero_()
    torch.cuda.synchronize()
    for k in range(N):
        with torch.cuda.stream(s1):
            P.replay()
        with torch.cuda.stream(s2):
            C.replay()
        torch.cuda.synchronize()
    out["graph_event_us"] = lat(buf)
    print(json.dumps(out), flush=True)

    # graphs with value nodes, consumer launched first; the consumer resets
    # the flag after its wait (the next producer write follows it)
    buf2, cnt2 = fresh(dev)
    gp2 = capture(lambda: (ops.spin_us(50.0), ops.stamp(buf2, cnt2, 0, 2, 0),
                           ops.stamp(buf2, cnt2, 0, 2, 1)), s1)
    gc2 = capture(lambda: (ops.stamp(buf2, cnt2, 1, 2, 0), ops.stamp(buf2, cnt2, 1, 2, 1)), s2)
    f2 = ops.SignalFlag()
    try:
        P2 = ops.ComposedGraph([("graph", gp2), ("writeval", (f2, 1))])
        C2 = ops.ComposedGraph([("waitval", (f2, 1)), ("writeval", (f2, 0)), ("graph", gc2)])
        out["value_nodes"] = "explicit"
    except RuntimeError as e:
        out["memop_node_error"] = str(e)[:200]
        # the same operations stream-captured into child graphs instead
        gw = capture(lambda: f2.write(1), s1)
        gq = capture(lambda: (f2.wait(1), f2.write(0)), s2)
        P2 = ops.ComposedGraph([("graph", gp2), ("graph", gw)])
        C2 = ops.ComposedGraph([("graph", gq), ("graph", gc2)])
        out["value_nodes"] = "captured"
    print(json.dumps(out), flush=True)
    cnt2.zero_()
    torch.cuda.synchronize()
    for k in range(N):
        with torch.cuda.stream(s2):
            C2.replay()
        with torch.cuda.stream(s1):
            P2.replay()
        torch.cuda.synchronize()
    out["graph_value_us"] = lat(buf2)
    b = buf2.cpu().view(-1, 2, 2)
    out["graph_value_order_ok"] = all(int(b[k, 1, 0]) >= int(b[k, 0, 1]) for k in range(N))

    # the same operations stream-captured into child graphs
    buf3, cnt3 = fresh(dev)
    gp3 = capture(lambda: (ops.spin_us(50.0), ops.stamp(buf3, cnt3, 0, 2, 0),
                           ops.stamp(buf3, cnt3, 0, 2, 1)), s1)
    gc3 = capture(lambda: (ops.stamp(buf3, cnt3, 1, 2, 0), ops.stamp(buf3, cnt3, 1, 2, 1)), s2)
    f3 = ops.SignalFlag()
    try:
        gw = capture(lambda: f3.write(1), s1)
        gq = capture(lambda: (f3.wait(1), f3.write(0)), s2)
        P3 = ops.ComposedGraph([("graph", gp3), ("graph", gw)])
        C3 = ops.ComposedGraph([("graph", gq), ("graph", gc3)])
        cnt3.zero_()
        torch.cuda.synchronize()
        for k in range(N):
            with torch.cuda.stream(s2):
                C3.replay()
            with torch.cuda.stream(s1):
                P3.replay()
            torch.cuda.synchronize()
        out["captured_value_us"] = lat(buf3)
        b = buf3.cpu().view(-1, 2, 2)
        out["captured_value_order_ok"] = all(int(b[k, 1, 0]) >= int(b[k, 0, 1])
                                             for k in range(N))
    except RuntimeError as e:
        out["captured_value_error"] = str(e)[:200]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
