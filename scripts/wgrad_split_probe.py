#!/usr/bin/env python
"""Split-K count of the small weight grads (bot0: dW [512, 64] over B=8192;
bot1/top3: [256, 512]): graph-timed GEMM into the fp32 slab per split."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, it=20, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=st):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (it * reps) * 1e3


def main():
    from tdfo_amd import ops
    B = 8192
    for out, inn in [(512, 64), (256, 512), (128, 256), (512, 256)]:
        dy = torch.randn(B, out, device="cuda").bfloat16()
        x = torch.randn(B, inn, device="cuda").bfloat16()
        res = {}
        for S in (8, 16, 32, 64, 128):
            if (B // 64) % S:
                continue
            sl = torch.zeros(S * out * inn, device="cuda")
            res[S] = round(timeit(lambda: ops.gemm(dy, True, x, True, None, False, None, None, sl,
                                                   S, ldc32=inn)), 2)
        print(json.dumps({"out": out, "in": inn, "us_by_splits": res}), flush=True)


if __name__ == "__main__":
    main()
