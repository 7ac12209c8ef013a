"""Run the fused embedding backward at DLRM-1TB scale N times (for rocprofv3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tdfo_amd import ops  # noqa: E402

T, B, D = 26, 8192, 128
rows = [39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 38532951, 2953546, 403346, 10,
        2208, 11938, 155, 4, 976, 14, 39979771, 25641295, 39664984, 585935, 12972, 108, 36]
dev = "cuda"
W = torch.empty(sum(rows), D, device=dev).uniform_(-0.01, 0.01)
ro = torch.zeros(T, dtype=torch.long)
ro[1:] = torch.tensor(rows[:-1]).cumsum(0)
ro = ro.to(dev)
ids = torch.cat([torch.randint(0, r, (B,), device=dev) for r in rows])
offs = torch.arange(T * B + 1, device=dev)
oo = torch.tensor([t * D for t in range(T)], device=dev)
grad = torch.randn(B * T * D, device=dev).to(torch.bfloat16) * 0.01
st = torch.zeros(W.shape[0], device=dev)
hyper = torch.tensor([0.01, 1.0], device=dev)
out = torch.empty(B * T * D, device=dev, dtype=torch.bfloat16)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    ops.embedding_bag_fwd(W, ro, ids, offs, oo, T, B, out, T * D)
    ops.embedding_bwd(W, ro, ids, offs, oo, T, B, grad, T * D, ops.EMB_ROWWISE_ADAGRAD, hyper,
                      state1=st)
torch.cuda.synchronize()
print("done")
