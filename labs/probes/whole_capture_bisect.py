#!/usr/bin/env python
"""Find the first stage of the whole-step capture that breaks
hipStreamEndCapture: capture the first N stages (+ joins) in a child
process per N (a crash ends only that child)."""
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(n: int, strategy: str):
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    from tdfo_amd.parallel.comm import LoopbackComm

    rows = [5000, 7, 30000, 1000, 3, 800, 64, 129]
    cfg = DLRMConfig(embedding_dim=64, table_rows=rows, bottom=[128, 64], top=[128, 64, 1],
                     sharding=strategy, pipeline=True, pooling=[1, 2, 1, 3, 1, 1, 1, 1], seed=3)
    dev = torch.device("cuda", 0)
    tr = DLRMTrainer(cfg, 256, dev, group=LoopbackComm(4, 0, dev), rank=0, world_size=4)
    data = SyntheticCriteo(rows, 256, pooling=cfg.pooling_factors(), device="cuda:0", seed=9)
    b = [data.next() for _ in range(4)]
    tr.prime(*b[0])
    tr.set_next_batch(*b[1])
    tr.step()
    full = tr._whole_stages()
    emb = tr.emb

    def cleanup():
        emb.ids_exchange_wait()
        for w in emb._pending or ():
            w.wait()
        emb._pending = None
        bw = getattr(emb, "_bw", None)
        if bw is not None and bw[0] is not None:
            emb.backward_wait()
        tr._m_allreduce_wait()

    mode = os.environ.get("BISECT_MODE", "")
    if mode:
        def ps_only():
            cur = torch.cuda.current_stream()
            tr._ps.wait_stream(cur)
            with torch.cuda.stream(tr._ps):
                emb.stage_bwd_prepare()
            cur.wait_stream(tr._ps)

        def prep_inline():
            emb.stage_bwd_prepare()

        def top_nops():
            tr._ps = None
            tr._s_top()

        def top_a_nops():
            tr._ps = None
            tr._s_top_a()

        def fork_kernel_only():
            cur = torch.cuda.current_stream()
            tr._ps.wait_stream(cur)
            with torch.cuda.stream(tr._ps):
                tr.x0.mul_(1.0)
            cur.wait_stream(tr._ps)

        fn = {"ps_only": ps_only, "prep_inline": prep_inline, "top_nops": top_nops,
              "top_a_nops": top_a_nops, "fork_kernel_only": fork_kernel_only}[mode]
        tr._whole_stages = lambda: full[:2] + [("c", fn), ("m", cleanup), ("j", None)]
    elif n < len(full):
        tr._whole_stages = lambda: full[:n] + [("m", cleanup), ("j", None)]
    names = [f"{k}:{getattr(f, '__name__', f)}" for k, f in full]
    print("stages", len(full), names[:n][-1:] if n else [], flush=True)
    tr.capture_graph(warmup=0)
    print("captured", n, flush=True)
    tr.set_next_batch(*b[2])
    tr.step()
    torch.cuda.synchronize()
    print("replayed", n, flush=True)


def main():
    if len(sys.argv) > 2:
        child(int(sys.argv[1]), sys.argv[2])
        return
    strategy = sys.argv[1] if len(sys.argv) > 1 else "table_wise"
    if len(sys.argv) > 1 and sys.argv[1] == "modes":
        for m in ["fork_kernel_only", "prep_inline", "ps_only", "top_a_nops", "top_nops"]:
            r = subprocess.run([sys.executable, "-u", __file__, "3", "table_wise"],
                               capture_output=True, text=True, timeout=120,
                               env=dict(os.environ, BISECT_MODE=m))
            out = [l for l in r.stdout.splitlines() if l.split()[:1] in (["captured"], ["replayed"])]
            print(m, "rc", r.returncode, out, flush=True)
        return
    for n in range(0, 40):
        r = subprocess.run([sys.executable, "-u", __file__, str(n), strategy],
                           capture_output=True, text=True, timeout=120)
        out = [l for l in r.stdout.splitlines() if l.split()[:1] in (["stages"], ["captured"],
                                                                      ["replayed"])]
        print(n, "rc", r.returncode, out, flush=True)
        if r.returncode != 0 and "Traceback" in r.stderr:
            print(r.stderr[-1500:], flush=True)
        if out and out[0].startswith("stages") and int(out[0].split()[1]) <= n:
            break


if __name__ == "__main__":
    main()
