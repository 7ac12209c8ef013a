"""Probe: graphs captured with keep_graph chained by explicit cross-stream
event nodes (ops.ComposedGraph); prints each stage so a crash names it."""
import torch
from tdfo_amd import ops

x = torch.zeros(1 << 20, device="cuda")
y = torch.zeros(1 << 20, device="cuda")
main = torch.cuda.current_stream()
se = torch.cuda.Stream()
e1, e2 = ops.SyncEvent(2), ops.SyncEvent(2)
gs = []
for fn in (lambda: x.add_(1), lambda: x.add_(y), lambda: x.mul_(2)):
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        fn()
    gs.append(g)
print("captured", flush=True)
cg = ops.ComposedGraph([("graph", gs[0]), ("wait", e1), ("graph", gs[1]), ("record", e2),
                        ("graph", gs[2])])
print("composed", flush=True)
ref = torch.zeros(1 << 20, device="cuda")
for i in range(3):
    with torch.cuda.stream(se):
        torch.cuda._sleep(2000000)
        y.fill_(i + 1)
        e1.record(se)
    cg.replay()
    e2.wait(se)
    ref = (ref + 1 + (i + 1)) * 2
torch.cuda.synchronize()
print("replayed", x[:2].tolist(), ref[:2].tolist(), flush=True)
assert torch.equal(x, ref)
print("ok")
