"""Isolated timing of the DLRM bottom MLP forward: the fused one-launch
kernel (csrc/kernels/mlp_fused.hip) vs the three per-layer GEMMs, B = 8192,
500 back-to-back calls (events), plus a bitwise check of the two."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer
    B = int(os.environ.get("BB", 8192))
    tr = DLRMTrainer(DLRMConfig(table_rows=[1000, 20, 5000]), B, "cuda:0")
    g = torch.Generator().manual_seed(3)
    tr.x0[:, :13] = torch.randn(B, 13, generator=g).to("cuda:0", torch.bfloat16)
    outs = []
    for fused in (True, False):
        tr._fused_bottom = fused
        tr._s_bottom_fwd()
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (tr.bot_in[1], tr.bot_in[2], tr.h_out)])
    print("bitwise equal:", all(torch.equal(a, b) for a, b in zip(*outs)), flush=True)
    for fused in (True, False, True, False):
        tr._fused_bottom = fused
        for _ in range(20):
            tr._s_bottom_fwd()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(500):
            tr._s_bottom_fwd()
        e1.record()
        torch.cuda.synchronize()
        print("fused" if fused else "per-layer", "us/call", round(e0.elapsed_time(e1) / 500 * 1000, 2),
              flush=True)


if __name__ == "__main__":
    main()
