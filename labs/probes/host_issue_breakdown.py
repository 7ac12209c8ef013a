"""Host time per call of the one-GPU DLRM-1TB step loop (bench.py's path:
fresh device batches, per-stream composed graphs): the batch producer's
next(), load_batch() and step(), over 100 steps after capture, no host
synchronisation inside the window (us per call, mean / median)."""
import os
import statistics as st
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, DLRMConfig, DLRMTrainer
    from tdfo_amd.train.loop import StepLoop, make_source
    dev = torch.device("cuda", 0)
    cfg = DLRMConfig(table_rows=list(CRITEO_1TB_ROWS), ids_stream=False)
    tr = DLRMTrainer(cfg, 8192, dev)
    src = make_source(cfg.table_rows, 8192, dev, cfg.pooling_factors(), 1, 0, kind="fresh")
    loop = StepLoop(tr, src)
    loop.run(9)
    tr.capture_graph(warmup=1)
    loop.run(20)
    torch.cuda.synchronize()
    t = {"next": [], "load": [], "step": []}
    for _ in range(100):
        a = time.perf_counter()
        batch, slot = loop._next()
        b = time.perf_counter()
        tr.load_batch(*batch, on_device=True)
        c = time.perf_counter()
        tr.step()
        d = time.perf_counter()
        t["next"].append(b - a)
        t["load"].append(c - b)
        t["step"].append(d - c)
    torch.cuda.synchronize()
    for k, v in t.items():
        print(f"{k}: mean {st.mean(v) * 1e6:.1f} us  median {st.median(v) * 1e6:.1f} us", flush=True)


if __name__ == "__main__":
    main()
