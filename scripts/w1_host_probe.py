#!/usr/bin/env python
"""One-GPU bench step (fresh device batches, per-stream graphs): host time to
issue a burst of steps from an idle queue vs the device time of the burst.
If the issue time per step approaches the device step, the host is on the
critical path."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, DLRMConfig, DLRMTrainer
    from tdfo_amd.train.loop import StepLoop, make_source
    dev = torch.device("cuda", 0)
    cfg = DLRMConfig(table_rows=list(CRITEO_1TB_ROWS))
    tr = DLRMTrainer(cfg, 8192, dev)
    src = make_source(cfg.table_rows, 8192, dev, cfg.pooling_factors(), 1, 0, kind="fresh")
    loop = StepLoop(tr, src)
    loop.run(9)
    tr.capture_graph(warmup=1)
    loop.run(3)
    torch.cuda.synchronize()
    out = {"graph": tr.graph}
    for n in (5, 20, 100):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.run(n)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[f"n{n}"] = {"issue_us_per_step": round((t1 - t0) / n * 1e6, 1),
                        "total_us_per_step": round((t2 - t0) / n * 1e6, 1)}
    # per-call host costs of one step
    import cProfile
    import pstats
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    loop.run(50)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(15)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
