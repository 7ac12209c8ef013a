#!/usr/bin/env python
"""A/B of DLRMConfig variants on one GPU, the bench.py step (fresh device
batches, captured graphs): each variant is built, warmed, captured and timed
in turn, twice over (A B A B), in one process.

usage: python labs/cfg_ab.py '{"defer_wgrad": true}' '{"defer_wgrad": false}' [--model dcnv2]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(over, model, steps=50, warmup=10):
    from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, MLPERF_MULTIHOT, DLRMConfig, DLRMTrainer
    from tdfo_amd.train.loop import StepLoop, make_source
    dev = torch.device("cuda", 0)
    kw = dict(table_rows=list(CRITEO_1TB_ROWS))
    if model == "dcnv2":
        kw.update(interaction="dcn", pooling=list(MLPERF_MULTIHOT), top=[1024, 1024, 512, 256, 1])
    kw.update(over)
    cfg = DLRMConfig(**kw)
    tr = DLRMTrainer(cfg, 8192, dev)
    src = make_source(cfg.table_rows, 8192, dev, cfg.pooling_factors(), 1, 0, kind="fresh")
    loop = StepLoop(tr, src)
    loop.run(warmup - 1)
    tr.capture_graph(warmup=1)
    loop.run(3)
    torch.cuda.synchronize()
    t = time.perf_counter()
    loop.run(steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / steps * 1e3
    del tr, loop, src
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return ms


def main():
    from tdfo_amd.ops import _ext
    assert _ext.load()
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    model = "dcnv2" if "--model" in sys.argv and sys.argv[sys.argv.index("--model") + 1] == "dcnv2" else "dlrm"
    args = [a for a in args if a != "dcnv2"]
    variants = [json.loads(a) for a in args]
    res = {i: [] for i in range(len(variants))}
    for rep in range(2):
        for i, v in enumerate(variants):
            res[i].append(round(run(v, model), 4))
            print(json.dumps({"variant": v, "ms": res[i][-1]}), flush=True)
    for i, v in enumerate(variants):
        print(json.dumps({"variant": v, "ms_runs": res[i], "model": model}), flush=True)


if __name__ == "__main__":
    main()
