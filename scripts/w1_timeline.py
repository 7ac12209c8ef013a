#!/usr/bin/env python
"""Per-segment device timeline of the one-GPU DLRM step (per-stream composed
graphs, fresh device batches, the bench.py step): stamps around every
captured segment, printed per step in us from the step's M1 start, plus the
per-segment mean over the steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import json
    from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, DLRMConfig, DLRMTrainer
    from tdfo_amd.ops import _ext
    from tdfo_amd.train.loop import StepLoop, make_source
    assert _ext.load()
    dev = torch.device("cuda", 0)
    kind = sys.argv[1] if len(sys.argv) > 1 else "fresh"        # fresh | pool
    over = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}  # DLRMConfig overrides
    cfg = DLRMConfig(table_rows=list(CRITEO_1TB_ROWS), **over)
    tr = DLRMTrainer(cfg, 8192, dev)
    print(f"data={kind} cfg={over}")
    steps, nseg = 40, 8
    buf = torch.zeros((steps + 8) * nseg * 2, dtype=torch.int64, device=dev)
    cnt = torch.zeros(nseg, dtype=torch.int64, device=dev)
    tr._ms_stamp = (buf, cnt)
    if kind == "pool":
        from tdfo_amd.data.synthetic import SyntheticCriteo
        from tdfo_amd.train.loop import PoolBatches
        data = SyntheticCriteo(cfg.table_rows, 8192, pooling=cfg.pooling_factors(), device=dev,
                               seed=1)
        src = PoolBatches([data.next() for _ in range(8)])
    else:
        src = make_source(cfg.table_rows, 8192, dev, cfg.pooling_factors(), 1, 0, kind="fresh")
    loop = StepLoop(tr, src)
    loop.run(9)
    tr.capture_graph(warmup=1)
    torch.cuda.synchronize()
    cnt.zero_()
    loop.run(steps)
    torch.cuda.synchronize()
    names = tr._ms["names"]
    n = len(names)
    b = buf[: steps * n * 2].view(steps, n, 2).cpu().double() / 100.0   # 100 MHz wall clock
    m1 = names.index("M1")
    rows = []
    for s in range(4, steps - 1):
        t0 = b[s, m1, 0]
        rows.append([(float(b[s, i, 0] - t0), float(b[s, i, 1] - t0)) for i in range(n)]
                    + [float(b[s + 1, m1, 0] - t0)])
    for r in rows[-5:]:
        print(f"period {r[-1]:.0f} us: " + "  ".join(
            f"{nm}:{a:.0f}-{e:.0f}" for nm, (a, e) in zip(names, r[:-1])), flush=True)
    import statistics as st
    print("mean period %.1f us" % st.mean(r[-1] for r in rows))
    for i, nm in enumerate(names):
        print(f"  {nm}: start {st.mean(r[i][0] for r in rows):7.1f}  end {st.mean(r[i][1] for r in rows):7.1f}"
              f"  dur {st.mean(r[i][1] - r[i][0] for r in rows):6.1f}")


if __name__ == "__main__":
    main()
