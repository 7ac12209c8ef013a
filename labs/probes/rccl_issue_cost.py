#!/usr/bin/env python
"""Host cost of issuing the multi-rank step's collectives through
torch.distributed + RCCL, measured on a one-rank RCCL group (one GPU box):
per-call host microseconds of async all_to_all_single (with splits),
all_reduce, all_gather_into_tensor and reduce_scatter_tensor at the DLRM-1TB
W=8 rank-0 sizes, next to a hipGraph replay and an event wait. Combined with
``bench.py --emulate-world 8`` (whose loopback collectives are cheaper to
issue) it prices the real W=8 step's host issue time.

    python labs/probes/rccl_issue_cost.py [--iters 200]
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def timed(fn, iters):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    host = (time.perf_counter() - t) / iters * 1e6
    torch.cuda.synchronize()
    dev = (time.perf_counter() - t) / iters * 1e6
    return round(host, 2), round(dev, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    B, D = 8192, 128
    bf = torch.bfloat16
    # W=8 rank-0 shapes: pooled rows of ~4 tables for 8 sources, 2.7 M fp32 grads
    pooled = torch.zeros(8 * B * 4 * D, dtype=bf, device=dev)
    pooled_o = torch.zeros_like(pooled)
    ids = torch.zeros(8 * B * 4, dtype=torch.int64, device=dev)
    ids_o = torch.zeros_like(ids)
    grads = torch.zeros(2_700_000, dtype=torch.float32, device=dev)
    ag_in = torch.zeros(B * D, dtype=bf, device=dev)
    ag_out = torch.zeros(B * D, dtype=bf, device=dev)
    res = {}

    def a2a(o, i):
        def f():
            w = dist.all_to_all_single(o, i, output_split_sizes=[o.numel()],
                                       input_split_sizes=[i.numel()], async_op=True)
            w.wait()
        return f

    res["all_to_all_ids"] = timed(a2a(ids_o, ids), a.iters)
    res["all_to_all_pooled"] = timed(a2a(pooled_o, pooled), a.iters)

    def ar():
        dist.all_reduce(grads, async_op=True).wait()
    res["all_reduce_grads"] = timed(ar, a.iters)

    def ag():
        dist.all_gather_into_tensor(ag_out, ag_in, async_op=True).wait()
    res["all_gather"] = timed(ag, a.iters)

    def rs():
        dist.reduce_scatter_tensor(ag_out, ag_in, async_op=True).wait()
    res["reduce_scatter"] = timed(rs, a.iters)

    x = torch.zeros(1024, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        x.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(8):
            x.add_(1)
    res["graph_replay_8_kernels"] = timed(g.replay, a.iters)
    side = torch.cuda.Stream()

    def evw():
        side.wait_stream(torch.cuda.current_stream())
        torch.cuda.current_stream().wait_stream(side)
    res["stream_fork_join"] = timed(evw, a.iters)
    print(json.dumps({"host_us_and_wall_us_per_call": res,
                      "note": "one-rank RCCL group: host issue cost of the c10d path; the "
                              "device work is a local copy"}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
