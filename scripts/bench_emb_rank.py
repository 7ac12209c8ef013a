"""Per-rank embedding cost at the table-wise multi-rank layout, on one GPU.

A rank that owns tables ``rows`` at world size W looks up W runs (one per
source rank) of B one-hot ids per table, then runs the fused sort-based
backward + row-wise Adagrad. This times exactly that work (forward gather +
backward) for:

  1. single tables of increasing row count (the planner's cost curve), and
  2. every rank of the planner's W = 4 / 8 plans for the Criteo-1TB tables,

so the max-over-ranks embedding time of each plan is measured, not guessed.
CUDA-event timing, median of 5 x 10 back-to-back iterations.
"""
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from tdfo_amd import ops  # noqa: E402
from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, DLRMConfig  # noqa: E402
from tdfo_amd.sparse import planner  # noqa: E402
from tdfo_amd.sparse.tables import EmbOptimConfig, TableBatchedEmbedding  # noqa: E402

dev = "cuda"
B, D = 8192, 128
OPT = EmbOptimConfig("rowwise_adagrad")


def rank_us(rows, W):
    """(fwd us, bwd us) for one rank owning tables ``rows`` at world size W."""
    if not rows:
        return 0.0, 0.0
    st = TableBatchedEmbedding(rows, D, dev, OPT, seed=1)
    Tp = len(rows)
    T = W * Tp
    ids = torch.cat([torch.randint(0, rows[i], (B,), device=dev)
                     for _ in range(W) for i in range(Tp)])
    offs = torch.arange(T * B + 1, device=dev)
    row_off = torch.tensor([st.row_offset_host[i] for _ in range(W) for i in range(Tp)],
                           dtype=torch.int64, device=dev)
    out_off = torch.tensor([s * B * Tp * D + i * D for s in range(W) for i in range(Tp)],
                           dtype=torch.int64, device=dev)
    out = torch.empty(W * B * Tp * D, dtype=torch.bfloat16, device=dev)
    grad = torch.randn(W * B * Tp * D, device=dev).to(torch.bfloat16)
    hyper = torch.tensor([0.01, 1.0], device=dev)
    seg = W if W <= 2 else 0

    def fwd():
        st.forward(ids, offs, row_off, T, B, out, out_off, Tp * D, onehot=True)

    def bwd():
        st.backward_update(ids, offs, row_off, T, B, grad, out_off, Tp * D, hyper, segsort=seg)

    res = []
    for f in (fwd, bwd):
        for _ in range(3):
            f()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                f()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / 10 * 1e3)
        res.append(round(statistics.median(ts), 1))
    del st
    torch.cuda.empty_cache()
    return tuple(res)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "all"
    if mode in ("all", "sweep"):
        for W in (1, 8):
            for r in (4, 100, 2000, 20000, 400000, 3_000_000, 25_000_000, 40_000_000):
                f, b = rank_us([r], W)
                print(json.dumps({"sweep": True, "W": W, "rows": r, "fwd_us": f, "bwd_us": b,
                                  "us_per_kid": round((f + b) / (W * B / 1000), 3)}), flush=True)
    if mode in ("all", "plans"):
        tables = DLRMConfig(table_rows=CRITEO_1TB_ROWS).tables()
        models = {"batch_only": lambda r: 1.0}
        for W in (4, 8):
            for name, rc in models.items():
                p = planner.plan_sharding(tables, W, OPT, row_cost=rc)
                per = []
                for r in range(W):
                    rows = [CRITEO_1TB_ROWS[t] for t in p.tables_on(r)]
                    f, b = rank_us(rows, W)
                    per.append({"rows": rows, "fwd_us": f, "bwd_us": b, "sum": round(f + b, 1)})
                print(json.dumps({"plan": name, "W": W, "max_us": max(x["sum"] for x in per),
                                  "mean_us": round(sum(x["sum"] for x in per) / W, 1),
                                  "ranks": per}), flush=True)


if __name__ == "__main__":
    main()
