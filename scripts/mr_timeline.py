#!/usr/bin/env python
"""Per-segment device timeline of the multi-rank stream graphs (emulated
rank RANK of W, modelled links GBPS per rank): stamps around every captured
segment, printed per step in us from the step's M1 start; with HOST=1 also
when the host launched each step (host clock mapped onto the device clock by
a stamp taken right after a synchronize)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, DLRMConfig, DLRMTrainer
    from tdfo_amd.parallel.comm import LoopbackComm
    from tdfo_amd.train.loop import StepLoop, make_source
    from tdfo_amd.ops import _ext
    assert _ext.load()
    dev = torch.device("cuda", 0)
    W = int(os.environ.get("W", 8))
    R = int(os.environ.get("RANK_EMU", 0))
    gbps = float(os.environ.get("GBPS", min(W - 1, 7) * 153.0))
    # SHARDING=data_parallel: config 3's plan (replicated + row-wise tables)
    cfg = DLRMConfig(table_rows=list(CRITEO_1TB_ROWS), pipeline=True,
                     sharding=os.environ.get("SHARDING", "auto"))
    cfg.ids_stream = False
    tr = DLRMTrainer(cfg, 8192, dev, group=LoopbackComm(W, R, dev, gbps, 10.0), rank=R,
                     world_size=W)
    steps = int(os.environ.get("STEPS", 12))
    nseg = 16
    buf = torch.zeros((steps + 4) * nseg * 2, dtype=torch.int64, device=dev)
    cnt = torch.zeros(nseg, dtype=torch.int64, device=dev)
    tr._mr_stamp = (buf, cnt)
    src = make_source(cfg.table_rows, 8192, dev, cfg.pooling_factors(), 1, R, kind="fresh")
    loop = StepLoop(tr, src)
    loop.run(4)
    tr.capture_graph(warmup=0)
    torch.cuda.synchronize()
    # host -> device clock: a stamp right after a synchronize ~ now
    from tdfo_amd import ops
    cal = torch.zeros(4, dtype=torch.int64, device=dev)
    ccnt = torch.zeros(1, dtype=torch.int64, device=dev)
    h0 = time.perf_counter()
    ops.stamp(cal, ccnt, 0, 1, 0)
    torch.cuda.synchronize()
    host = []
    for _ in range(steps):
        host.append(time.perf_counter())
        loop.run(1)
    torch.cuda.synchronize()
    d0 = int(cal[0].item())
    names = tr._mr["names"]
    n = len(names)
    b = buf[: steps * n * 2].view(steps, n, 2).cpu()
    for s in range(2, steps):
        t0 = int(b[s, names.index("M1"), 0])
        row = [f"{nm}:{(int(b[s, i, 0]) - t0) / 100:.0f}-{(int(b[s, i, 1]) - t0) / 100:.0f}"
               for i, nm in enumerate(names)]
        nxt = (int(b[s + 1, names.index("M1"), 0]) - t0) / 100 if s + 1 < steps else float("nan")
        hl = ((host[s] - h0) * 1e6 - (t0 - d0) / 100) if os.environ.get("HOST") else None
        hs = f" host launch {hl:+.0f} us vs M1 start" if hl is not None else ""
        print(f"step {s} (period {nxt:.0f} us){hs}: " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
