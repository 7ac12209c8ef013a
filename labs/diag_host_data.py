"""Diagnose the host data plane: CPU time per step in the prefetcher vs the
step, GPU time of an H2D batch, and the step time with/without H2D."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd.data.prefetch import host_prefetcher  # noqa: E402
from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, DLRMConfig, DLRMTrainer  # noqa: E402

B = 8192
cfg = DLRMConfig()
tr = DLRMTrainer(cfg, B, "cuda:0")
pf = host_prefetcher(cfg.table_rows, B, "cuda:0", seed=1,
                     threads=int(os.environ.get("GEN_THREADS", "12")))
for _ in range(5):
    b, s = pf.next()
    tr.load_batch(*b)
    pf.release(s)
    tr.step()
tr.capture_graph(warmup=1)
torch.cuda.synchronize()
jobs = []
_orig = pf.gen.batch


def timed(j):
    a = time.perf_counter()
    r = _orig(j)
    jobs.append((a, time.perf_counter()))
    return r


pf.gen.batch = timed
t_next = t_load = t_step = 0.0
n = 50
t0 = time.perf_counter()
for _ in range(n):
    a = time.perf_counter()
    b, s = pf.next()
    c = time.perf_counter()
    tr.load_batch(*b)
    pf.release(s)
    d = time.perf_counter()
    tr.step()
    e = time.perf_counter()
    t_next += c - a
    t_load += d - c
    t_step += e - d
torch.cuda.synchronize()
el = time.perf_counter() - t0
dur = sorted(b - a for a, b in jobs[-n:])
print(f"worker job ms (in the timed loop): median {dur[len(dur) // 2] * 1e3:.3f} "
      f"max {dur[-1] * 1e3:.3f}", flush=True)
pf.gen.batch = _orig
print(f"total {el / n * 1e3:.3f} ms/step; cpu: next {t_next / n * 1e3:.3f} load {t_load / n * 1e3:.3f}"
      f" step {t_step / n * 1e3:.3f}; in next: wait-gen {pf.t_wait_gen / n * 1e3:.3f}"
      f" submit {pf.t_submit / n * 1e3:.3f}", flush=True)
# pure H2D of one batch (pinned)
h = pf.gen.batch(0)
dd = [x.to("cuda:0") for x in h]
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(20):
    for x, y in zip(dd, h):
        x.copy_(y, non_blocking=True)
ev1.record()
torch.cuda.synchronize()
print(f"H2D per batch {ev0.elapsed_time(ev1) / 20 * 1e3:.1f} us, pinned={h[1].is_pinned()}", flush=True)
# generator only
t = time.perf_counter()
for i in range(20):
    pf.gen.batch(i)
print(f"gen {((time.perf_counter() - t) / 20) * 1e3:.3f} ms", flush=True)
pf.close()
