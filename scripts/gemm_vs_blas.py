#!/usr/bin/env python
"""Our HIP GEMM vs torch.matmul (hipBLASLt) on the DLRM MLP shapes, bf16,
same process. Device time: each op is captured 20x into a hipGraph and the
graph replayed (no host launch cost in either number; eager torch.matmul
carries ~17 us of host overhead per call on this image, which the round-1/2
tables measured instead of the GEMM)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402

# (M, N, K) of every DLRM-1TB Linear forward (B = 8192); the dgrad of the
# same layer is (M, K, N) and the wgrad (N, K, M)
SHAPES = [(8192, 512, 64), (8192, 256, 512), (8192, 128, 256), (8192, 1024, 512),
          (8192, 1024, 1024), (8192, 512, 1024), (8192, 256, 512)]
# DCN-v2 (--model dcnv2, GEMM policy 5): cross-layer V (d=3456 -> r=512) and
# U (512 -> 3456), top-0 (3456 -> 1024)
DCN_SHAPES = [(8192, 512, 3456), (8192, 3456, 512), (8192, 1024, 3456)]


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
    bf = torch.bfloat16
    shapes = SHAPES
    if "--model" in sys.argv and sys.argv[sys.argv.index("--model") + 1] == "dcnv2":
        shapes = DCN_SHAPES
        ops.gemm_policy(5)
    for M, N, K in shapes:
        x = torch.randn(M, K, device="cuda").to(bf)
        w = torch.randn(N, K, device="cuda").to(bf)
        b = torch.randn(N, device="cuda").to(bf)
        y = torch.empty(M, N, device="cuda", dtype=bf)
        dy = torch.randn(M, N, device="cuda").to(bf)
        dx = torch.empty(M, K, device="cuda", dtype=bf)
        gw = torch.empty(N * K, device="cuda")
        ours = timeit(lambda: ops.linear_fwd(x, w, None, True, out=y))
        ours_d = timeit(lambda: ops.linear_dgrad(dy, w, mask=x, out=dx))
        ours_w = timeit(lambda: ops.linear_wgrad(dy, x, gw))
        blas = timeit(lambda: torch.nn.functional.linear(x, w, b))
        blas_relu = timeit(lambda: torch.relu(torch.nn.functional.linear(x, w, b)))
        blas_d = timeit(lambda: dy @ w)
        blas_w = timeit(lambda: dy.t() @ x)
        wo = torch.empty(N, K, device="cuda", dtype=bf)
        blas_w = min(blas_w, timeit(lambda: torch.mm(dy.t(), x, out=wo)))
        tf = 2 * M * N * K / 1e12
        print(json.dumps({"M": M, "N": N, "K": K, "ours_fwd_us": round(ours, 2),
                          "blas_fwd_us": round(blas, 2), "blas_fwd_relu_us": round(blas_relu, 2),
                          "ours_dgrad_us": round(ours_d, 2), "blas_dgrad_us": round(blas_d, 2),
                          "ours_wgrad_us": round(ours_w, 2), "blas_wgrad_us": round(blas_w, 2),
                          "ours_fwd_tflops": round(tf / ours * 1e6, 1),
                          "blas_fwd_tflops": round(tf / blas * 1e6, 1),
                          "ours_dgrad_tflops": round(tf / ours_d * 1e6, 1),
                          "blas_dgrad_tflops": round(tf / blas_d * 1e6, 1),
                          "ours_wgrad_tflops": round(tf / ours_w * 1e6, 1),
                          "blas_wgrad_tflops": round(tf / blas_w * 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
