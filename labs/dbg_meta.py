import os, sys, torch
sys.path.insert(0, os.getcwd())
from tdfo_amd import ops
from tests.test_gpu_kernels import _emb_case
DEV = "cuda"
B, T, D = 8192, 3, 128
rows = [50, 9000, 70000]
W, ro, idx, offs = _emb_case(T, B, rows, D, 1, False, seed=7)
W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
goff = torch.tensor([t * D for t in range(T)], device=DEV)
grad = torch.randn(B * T * D, device=DEV)
hyper = torch.tensor([0.05, 3.0], device=DEV)
opt = ops.EMB_ROWWISE_ADAGRAD
s1 = torch.rand(W.shape[0], device=DEV)
res = []
for seg in (1, 0):
    Wn, a1 = W.clone(), s1.clone()
    ops.embedding_bwd(Wn, ro, idx, offs, goff, T, B, grad, T * D, opt, hyper, state1=a1, segsort=seg)
    res.append((Wn, a1))
torch.cuda.synchronize()
d = (res[0][0] - res[1][0]).abs().amax(1)
bad = torch.nonzero(d > 0).flatten()
print("rows differing:", bad.numel(), "of", W.shape[0], "max", float(d.max()))
print("first bad rows:", bad[:20].tolist())
ch = (W - res[1][0]).abs().amax(1) > 0
ch0 = (W - res[0][0]).abs().amax(1) > 0
print("rows updated radix", int(ch.sum()), "segsort", int(ch0.sum()))
for r in bad[:5].tolist():
    print(r, float(d[r]), float((res[0][0][r]-W[r]).abs().max()), float((res[1][0][r]-W[r]).abs().max()))
# per table counts of ids
for t in range(T):
    u = torch.unique(idx[t*B:(t+1)*B])
    print("table", t, "unique", u.numel())
