"""Embedding backward at the world-8 table-wise layout (R = 8 runs of Tp
tables, B = 8192 one-hot ids each): per-table LDS sort + run merge vs the
device-wide radix sort. CUDA-event timing, same process."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from tdfo_amd import ops  # noqa: E402

dev = "cuda"
for R, Tp, rows in [(1, 26, 4_000_000), (8, 3, 40_000_000), (8, 4, 4_000_000), (2, 13, 10_000_000)]:
    B, D = 8192, 128
    T = R * Tp
    ro = (torch.arange(Tp, dtype=torch.int64) * rows).repeat(R).to(dev)
    ids = torch.randint(0, rows, (T * B,), device=dev)
    offs = torch.arange(T * B + 1, device=dev)
    goff = torch.arange(T, device=dev) * D
    W = torch.zeros(Tp * rows, D, device=dev)
    s1 = torch.zeros(Tp * rows, device=dev)
    grad = torch.randn(B * T * D, device=dev).to(torch.bfloat16)
    hyper = torch.tensor([0.01, 1.0], device=dev)
    res = {}
    for seg in (R, 0, R, 0):
        f = lambda: ops.embedding_bwd(W, ro, ids, offs, goff, T, B, grad, T * D,  # noqa: E731
                                      ops.EMB_ROWWISE_ADAGRAD, hyper, state1=s1, segsort=seg)
        for _ in range(3):
            f()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            f()
        b.record()
        torch.cuda.synchronize()
        res["segsort" if seg else "radix"] = round(a.elapsed_time(b) / 20 * 1e3, 1)
    print(json.dumps({"runs": R, "tables": Tp, "rows": rows, "B": B, **res}), flush=True)
