"""Debug: per-table max |diff| of the 2-rank row-wise step vs one process on
the GPU (shared cuda:0 over gloo), for graph/eager x bf16/fp32 comm."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from tests.dist_harness import run_distributed  # noqa: E402
from tests.test_gpu_multirank import _worker, B  # noqa: E402

if __name__ == "__main__":
    single = run_distributed(_worker, 1, 2 * B, "table_wise", True, "fp32", device="cuda")[0]
    p1, tabs1, loss1 = single
    for graph in (True, False):
        for comm in ("bf16", "fp32"):
            multi = run_distributed(_worker, 2, B, "row_wise", graph, comm, device="cuda")
            for rank in range(2):
                p, tabs, loss = multi[rank]
                d = {t: round(float((w - tabs1[t][2][lo:lo + w.shape[0], c0:c0 + w.shape[1]])
                                    .abs().max()), 5) for t, (lo, c0, w) in tabs.items()}
                print("graph", graph, comm, "rank", rank, "dense",
                      round(float((p - p1).abs().max()), 5), d, flush=True)
