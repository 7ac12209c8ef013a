"""Diagnostic (inexact by design): the one-GPU DLRM bench step with one stage
left out of the captured graphs, to price what each stage's presence costs
the step (a stage that is off the critical path still slows its neighbours
through shared CUs / HBM). The stage runs normally in the eager warm-up
steps (so every workspace it fills is valid) and is dropped from the
capture onward. Usage: python labs/probes/step_skip.py <stage> [bench
args]; stage in none | dense_opt | emb_sort | emb_update | emb_lookup."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
stage = sys.argv.pop(1)
import bench  # noqa: E402  (sets the one-GPU runtime mode from sys.argv)
from tdfo_amd.models.dlrm import DLRMTrainer  # noqa: E402
from tdfo_amd.sparse.sharded import ShardedEmbeddingBags  # noqa: E402

EAGER = 2          # calls that run for real (bench --warmup 5: two eager steps)


def _skip_after(cls, name):
    real = getattr(cls, name)
    count = {"n": 0}

    def f(self, *a, **k):
        count["n"] += 1
        if count["n"] <= EAGER:
            return real(self, *a, **k)
        return None
    setattr(cls, name, f)


target = {"dense_opt": (DLRMTrainer, "_s_dense_update"),
          "emb_sort": (ShardedEmbeddingBags, "stage_bwd_prepare"),
          "emb_update": (ShardedEmbeddingBags, "stage_bwd_update"),
          "emb_lookup": (ShardedEmbeddingBags, "stage_fwd_lookup")}.get(stage)
if target is not None:
    _skip_after(*target)
print(f"step_skip: {stage}", file=sys.stderr, flush=True)
bench.main(sys.argv[1:])
