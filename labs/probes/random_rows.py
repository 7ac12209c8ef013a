"""Random-row gather bandwidth vs table size (the floor under the embedding
lookup / update kernels): the one-hot lookup kernel gathers N random 512-B
rows (D = 128 fp32) of a table of R rows into a bf16 output, graph-replayed;
effective bytes / s counts the row reads + the output writes. If the rate
falls as the table grows past what the address-translation caches cover, the
DLRM / DCN-v2 lookups and updates over their 90-96 GB tables are held by that,
not by HBM bandwidth. One JSON line per size."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from tdfo_amd import ops  # noqa: E402


def main():
    D, N = 128, 1 << 21
    dev = "cuda"
    for gib in [1, 4, 16, 48, 96]:
        R = (gib << 30) // (D * 4)
        W = torch.empty(R, D, dtype=torch.float32, device=dev)
        W[:: max(1, R // 1024)].fill_(1.0)
        g = torch.Generator(device=dev).manual_seed(gib)
        ids = torch.randint(0, R, (N,), device=dev, generator=g)
        offs = torch.arange(N + 1, dtype=torch.int64, device=dev)
        ro = torch.zeros(1, dtype=torch.int64, device=dev)
        oo = torch.zeros(1, dtype=torch.int64, device=dev)
        out = torch.empty(N, D, dtype=torch.bfloat16, device=dev)
        run = lambda: ops.embedding_bag_fwd(W, ro, ids, offs, oo, 1, N, out, D, onehot=True)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(10):
                run()
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        nbytes = N * D * 4 + N * D * 2 + N * 8
        print(json.dumps({"table_GiB": gib, "rows": R, "gathers": N, "us": round(us, 1),
                          "TBps": round(nbytes / us / 1e6, 2)}), flush=True)
        del W, gr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
