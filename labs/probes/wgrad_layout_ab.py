"""A/B: a weight grad dW = dy^T x read from the activations as they are
(col-layout operands, transposing LDS reads) vs from K-major copies dy^T /
x^T (row-layout operands, plain 16-B fragment reads). Same split-K slabs,
same kernel library; us per call over 200 calls (events), median of 3."""
import sys
import torch
sys.path.insert(0, ".")
from tdfo_amd import ops

B = 8192
dev = "cuda:0"
shapes = [(1024, 512), (1024, 1024), (512, 1024), (256, 512), (512, 3456), (3456, 512), (1024, 3456)]


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(3):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n * 1000)
    return sorted(ts)[1]


for N, K in shapes:
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.randn(B, N, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(B, K, device=dev, generator=g).to(torch.bfloat16)
    dyT, xT = dy.t().contiguous(), x.t().contiguous()
    S = ops.wgrad_splits(N, K, B, 256)
    res = {}
    for s in sorted({S, max(1, S // 2), S * 2}):
        sl_c = torch.zeros(s, N, K, device=dev)
        sl_r = torch.zeros(s, N, K, device=dev)
        tc = timeit(lambda: ops.gemm(dy, True, x, True, None, False, None, None, sl_c, s))
        tr = timeit(lambda: ops.gemm(dyT, False, xT, False, None, False, None, None, sl_r, s))
        ok = torch.allclose(sl_c.sum(0), sl_r.sum(0), rtol=1e-3, atol=1e-2)
        res[s] = (round(tc, 2), round(tr, 2), ok)
    print(f"N={N} K={K} default_splits={S} " + " ".join(f"s{s}: col {c} row {r} {'ok' if o else 'MISMATCH'}" for s, (c, r, o) in res.items()), flush=True)
