#!/usr/bin/env python
"""Host cost of the multi-rank stream-graph launches (emulated W=8 rank 0):
per-graph hipGraphLaunch time, and whether the device runs behind the host."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, DLRMConfig, DLRMTrainer
    from tdfo_amd.parallel.comm import LoopbackComm
    from tdfo_amd.ops import _ext
    assert _ext.load()
    dev = torch.device("cuda", 0)
    W = int(os.environ.get("W", 8))
    cfg = DLRMConfig(table_rows=list(CRITEO_1TB_ROWS), pipeline=True)
    tr = DLRMTrainer(cfg, 8192, dev, group=LoopbackComm(W, 0, dev, 300.0, 10.0), rank=0,
                     world_size=W)
    data = SyntheticCriteo(cfg.table_rows, 8192, device=dev, seed=1)
    pool = [data.next() for _ in range(4)]
    tr.prime(*pool[0])
    for i in range(3):
        tr.set_next_batch(*pool[(i + 1) % 4])
        tr.step()
    tr.capture_graph(warmup=0)
    for i in range(3):
        tr.set_next_batch(*pool[i % 4])
        tr.step()
    torch.cuda.synchronize()
    mr = tr._mr
    print("nodes/graph:", {k: None for k in mr["composed"]}, flush=True)
    for trial in range(2):
        lt = {"M": 0.0, "D": 0.0, "EC": 0.0, "stage": 0.0}
        n = 20
        t0 = time.perf_counter()
        for i in range(n):
            a = time.perf_counter()
            tr.set_next_batch(*pool[i % 4])
            lt["stage"] += time.perf_counter() - a
            s, g = mr["streams"], mr["composed"]
            cur = torch.cuda.current_stream()
            s["EC"].wait_stream(cur)
            for k in ("M", "D", "EC"):
                a = time.perf_counter()
                with torch.cuda.stream(s[k]):
                    g[k].replay()
                lt[k] += time.perf_counter() - a
        host = time.perf_counter() - t0
        tr.sync_streams()
        torch.cuda.synchronize()
        dev_t = time.perf_counter() - t0
        print({k: round(v / n * 1e6, 1) for k, v in lt.items()},
              "host us/step", round(host / n * 1e6, 1), "device us/step", round(dev_t / n * 1e6, 1),
              flush=True)


if __name__ == "__main__":
    main()
