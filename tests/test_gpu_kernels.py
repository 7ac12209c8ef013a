"""HIP kernel numerics vs the fp32 torch references (run on MI355X).

Each test builds inputs on the GPU, runs the native op (torch.ops.tdfo.*),
and compares against tdfo_amd.ops.reference on the same data in fp32.
"""
import pytest
import torch

from tdfo_amd import ops
from tdfo_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    from tdfo_amd.ops import _ext

    assert _ext.load(), "native library must load on the GPU box"


def bf(x):
    return x.to(torch.bfloat16)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


# ------------------------------------------------------------------ GEMM
@pytest.fixture(params=[0, 1, 2, 3, 4, 8],
                ids=["auto", "twostage", "deep", "pingpong", "big", "p8"])
def gemm_pol(request):
    """Run a GEMM test once per kernel (auto, and each kernel forced)."""
    old = ops.gemm_policy(request.param)
    yield request.param
    ops.gemm_policy(old)


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 200, 192), (8192, 1024, 512),
                                   (1000, 72, 128), (64, 512, 1024), (777, 264, 320),
                                   (2048, 1032, 128)])
@pytest.mark.parametrize("a_col,b_col", [(False, False), (False, True), (True, True)])
def test_gemm_layouts(M, N, K, a_col, b_col, gemm_pol):
    if a_col and M % 8:
        pytest.skip("col A needs M%8")
    if b_col and N % 8:
        pytest.skip("col B needs N%8")
    torch.manual_seed(0)
    A = bf(torch.randn(K, M, device=DEV) if a_col else torch.randn(M, K, device=DEV))
    B = bf(torch.randn(K, N, device=DEV) if b_col else torch.randn(N, K, device=DEV))
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    out32 = torch.empty(M * N, device=DEV)
    ops.gemm(A, a_col, B, b_col, None, False, None, out, out32, 1)
    exp = torch.empty(M * N, device=DEV)
    ref.gemm(A, a_col, B, b_col, None, False, None, None, exp, 1)
    assert rel_err(out32.view(M, N), exp.view(M, N)) < 1e-4
    assert rel_err(out, exp.view(M, N)) < 1e-2


def test_gemm_asymmetric_identity(gemm_pol):
    # A = I with asymmetric B catches row/col swaps in the C map (guide §3)
    n = 128
    A = bf(torch.eye(n, device=DEV))                       # [M=128, K=128]
    Bs = bf(torch.arange(64 * n, device=DEV, dtype=torch.float32).view(64, n) % 97)  # [N][K]
    out32 = torch.empty(n * 64, device=DEV)
    ops.gemm(A, False, Bs, False, None, False, None, None, out32, 1)
    assert torch.equal(out32.view(n, 64), Bs.float().t())
    # col-layout B ([K][N]) and col-layout A ([K][M]) with the same data
    out32b = torch.empty(n * 64, device=DEV)
    ops.gemm(A, True, Bs.t().contiguous(), True, None, False, None, None, out32b, 1)
    assert torch.equal(out32b.view(n, 64), Bs.float().t())


def test_gemm_epilogue_bias_relu_mask(gemm_pol):
    torch.manual_seed(1)
    M, N, K = 513, 256, 128
    A = bf(torch.randn(M, K, device=DEV))
    W = bf(torch.randn(N, K, device=DEV))
    bias = torch.randn(N, device=DEV)
    mask = bf(torch.randn(M, N, device=DEV))
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm(A, False, W, False, bias, True, mask, out, None, 1)
    exp = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ref.gemm(A, False, W, False, bias, True, mask, exp, None, 1)
    assert rel_err(out, exp) < 1e-2


@pytest.mark.parametrize("M,N,K,S", [(1024, 1024, 8192, 8), (128, 256, 8192, 16),
                                     (200, 64, 640, 1), (512, 320, 4096, 3)])
def test_gemm_wgrad_pitched_slabs_with_colsum(M, N, K, S, gemm_pol):
    """Weight-grad GEMM into [S][M][ldc32] slabs with the A column sums (the
    bias gradient) in column csum_col; the pad columns stay untouched."""
    torch.manual_seed(3)
    ld = N + 64
    dy = bf(torch.randn(K, M, device=DEV))
    x = bf(torch.randn(K, N + 64, device=DEV))
    slab = torch.full((S * M * ld,), 7.0, device=DEV)
    ops.gemm(dy, True, x[:, :N], True, None, False, None, None, slab, S, ldc32=ld, csum_col=N)
    sl = slab.view(S, M, ld)
    exp = dy.float().t() @ x[:, :N].float()
    assert rel_err(sl[:, :, :N].sum(0), exp) < 1e-4
    assert rel_err(sl[:, :, N].sum(0), dy.float().sum(0)) < 1e-4
    assert torch.all(sl[:, :, N + 1:] == 7.0)
    exp_s = torch.full((S * M * ld,), 7.0, device=DEV)
    ref.gemm(dy, True, x[:, :N], True, None, False, None, None, exp_s, S, ldc32=ld, csum_col=N)
    assert rel_err(exp_s.view(S, M, ld)[:, :, :N + 1].sum(0), sl[:, :, :N + 1].sum(0)) < 1e-4


def test_gemm_strided_out_and_splitk(gemm_pol):
    torch.manual_seed(2)
    M, N, K = 256, 512, 8192
    dy = bf(torch.randn(K, M, device=DEV))
    x = bf(torch.randn(K, N, device=DEV))
    out = torch.empty(M * N, device=DEV)
    ops.linear_wgrad(dy, x, out, splits=8)
    exp = dy.float().t() @ x.float()
    assert rel_err(out.view(M, N), exp) < 1e-4
    big = torch.zeros(64, 1024, dtype=torch.bfloat16, device=DEV)
    view = big[:, 256:512]
    a = bf(torch.randn(64, 128, device=DEV))
    w = bf(torch.randn(256, 128, device=DEV))
    ops.linear_fwd(a, w, None, False, out=view)
    assert rel_err(view, a.float() @ w.float().t()) < 1e-2
    assert big[:, :256].abs().sum() == 0 and big[:, 512:].abs().sum() == 0


# ----------------------------------------------------------- interaction
@pytest.mark.parametrize("D", [16, 32, 64, 128])
@pytest.mark.parametrize("B", [1, 37, 1024])
def test_interaction(D, B):
    torch.manual_seed(3)
    F = 27
    T = F - 1
    dense = bf(torch.randn(B, D, device=DEV)).abs()
    dense[:, ::3] = -dense[:, ::3]
    emb = bf(torch.randn(B * T * D, device=DEV))
    off = [0] + [t * D for t in range(T)]
    stride = [0] + [T * D] * T
    ldo = ((D + F * (F - 1) // 2 + 63) // 64) * 64
    out = torch.full((B, ldo), 7.0, dtype=torch.bfloat16, device=DEV)
    ops.interaction_fwd(dense, emb, off, stride, F, D, out)
    exp = torch.empty_like(out)
    ref.interaction_fwd(dense, emb, off, stride, F, D, exp)
    assert rel_err(out, exp) < 1e-2
    dz = bf(torch.randn(B, ldo, device=DEV))
    dd = torch.zeros(B, D, dtype=torch.bfloat16, device=DEV)
    de = torch.zeros_like(emb)
    ops.interaction_bwd(dz, dense, emb, off, stride, F, D, dd, de, off, stride, True)
    edd = torch.zeros_like(dd)
    ede = torch.zeros_like(emb)
    ref.interaction_bwd(dz, dense, emb, off, stride, F, D, edd, ede, off, stride, True)
    assert rel_err(dd, edd) < 2e-2
    assert rel_err(de, ede) < 2e-2


# ------------------------------------------------------------- embedding
def _emb_case(T, B, rows, D, L, skew, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    lens = torch.randint(0, L + 1, (T * B,), generator=g) if L > 1 else torch.ones(T * B, dtype=torch.long)
    offsets = torch.zeros(T * B + 1, dtype=torch.long)
    offsets[1:] = lens.cumsum(0)
    nnz = int(offsets[-1])
    idx = []
    for j in range(T * B):
        t = j // B
        n = int(lens[j])
        if skew:
            idx.append(torch.randint(0, min(3, rows[t]), (n,), generator=g))
        else:
            idx.append(torch.randint(0, rows[t], (n,), generator=g))
    indices = torch.cat(idx) if nnz else torch.zeros(0, dtype=torch.long)
    ro = torch.zeros(T, dtype=torch.long)
    ro[1:] = torch.tensor(rows[:-1]).cumsum(0)
    W = torch.randn(sum(rows), D, generator=g)
    return W, ro, indices, offsets


@pytest.mark.parametrize("D", [16, 64, 128])
@pytest.mark.parametrize("L,mean", [(1, False), (5, False), (5, True)])
def test_embedding_fwd(D, L, mean):
    T, B = 4, 300
    rows = [100, 7, 5000, 1]
    W, ro, idx, offs = _emb_case(T, B, rows, D, L, False)
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    out_off = torch.tensor([t * D for t in range(T)], device=DEV)
    out = torch.zeros(B * T * D, dtype=torch.bfloat16, device=DEV)
    ops.embedding_bag_fwd(W, ro, idx, offs, out_off, T, B, out, T * D, mean=mean)
    exp = torch.zeros(B * T * D, device=DEV)
    ref.embedding_bag_fwd(W, ro, idx, offs, out_off, None, T, B, mean, exp, T * D)
    assert rel_err(out, exp) < 1e-2


@pytest.mark.parametrize("D", [16, 128])
@pytest.mark.parametrize("bf16_out,use_psw", [(True, False), (False, True)])
def test_embedding_fwd_onehot_path(D, bf16_out, use_psw):
    """onehot=True (no offsets loads, two bags in flight) == the general kernel."""
    T, B = 5, 3001
    rows = [100, 7, 5000, 1, 70000]
    W, ro, idx, offs = _emb_case(T, B, rows, D, 1, False, seed=3)
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    out_off = torch.tensor([t * D for t in range(T)], device=DEV)
    psw = torch.rand(idx.numel(), device=DEV) if use_psw else None
    dt = torch.bfloat16 if bf16_out else torch.float32
    outs = []
    for oh in (True, False):
        out = torch.zeros(B * T * D, dtype=dt, device=DEV)
        ops.embedding_bag_fwd(W, ro, idx, offs, out_off, T, B, out, T * D, psw=psw, onehot=oh)
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("opt", [ops.EMB_SGD, ops.EMB_ROWWISE_ADAGRAD, ops.EMB_ADAM,
                                 ops.EMB_ADAGRAD, ops.EMB_DENSE_GRAD])
@pytest.mark.parametrize("skew", [False, True])
@pytest.mark.parametrize("D", [32, 128])
def test_embedding_bwd_fused(opt, skew, D):
    T, B, L = 3, 700, 3
    rows = [50, 9000, 4]
    W, ro, idx, offs = _emb_case(T, B, rows, D, L, skew, seed=1)
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    goff = torch.tensor([t * D for t in range(T)], device=DEV)
    grad = torch.randn(B * T * D, device=DEV)
    hyper = torch.tensor([0.05, 3.0], device=DEV)

    def states():
        s1 = s2 = dg = None
        if opt == ops.EMB_ROWWISE_ADAGRAD:
            s1 = torch.rand(W.shape[0], device=DEV)
        elif opt in (ops.EMB_ADAGRAD, ops.EMB_ADAM):
            s1 = torch.rand(W.numel(), device=DEV)
        if opt == ops.EMB_ADAM:
            s2 = torch.rand(W.numel(), device=DEV)
        if opt == ops.EMB_DENSE_GRAD:
            dg = torch.zeros(W.numel(), device=DEV)
        return s1, s2, dg

    s1, s2, dg = states()
    Wn = W.clone()
    e1 = s1.clone() if s1 is not None else None
    e2 = s2.clone() if s2 is not None else None
    edg = dg.clone() if dg is not None else None
    ops.embedding_bwd(Wn, ro, idx, offs, goff, T, B, grad, T * D, opt, hyper, state1=s1,
                      state2=s2, weight_decay=0.01, dense_grad=dg)
    We = W.clone()
    ref.embedding_bwd(We, ro, idx, offs, goff, None, T, B, False, 20, grad, T * D, opt, e1, e2,
                      hyper, 1e-8, 0.9, 0.999, 0.01, edg)
    torch.cuda.synchronize()
    assert (Wn - We).abs().max() < 1e-4 * max(1.0, We.abs().max().item())
    if s1 is not None:
        assert (s1 - e1).abs().max() < 1e-3 * max(1.0, e1.abs().max().item())
    if dg is not None:
        assert (dg - edg).abs().max() < 1e-4 * max(1.0, edg.abs().max().item())


@pytest.mark.parametrize("opt", [ops.EMB_SGD, ops.EMB_ROWWISE_ADAGRAD, ops.EMB_ADAM,
                                 ops.EMB_ADAGRAD, ops.EMB_DENSE_GRAD])
def test_embedding_bwd_long_runs(opt):
    """Hot rows whose runs span hundreds of chunks (a 3-row table under a
    multi-hot batch: ~16 k ids per row, ~500 chunks) take the block-wide
    combine: equal to the fp32 reference and bitwise reproducible."""
    T, B, L, D = 2, 8192, 12, 128
    rows = [3, 5000]
    W, ro, idx, offs = _emb_case(T, B, rows, D, L, True, seed=5)
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    goff = torch.tensor([t * D for t in range(T)], device=DEV)
    grad = torch.randn(B * T * D, device=DEV) * 0.01
    hyper = torch.tensor([0.05, 3.0], device=DEV)
    n1 = W.shape[0] if opt == ops.EMB_ROWWISE_ADAGRAD else W.numel()
    s1 = torch.rand(n1, device=DEV) if opt in (ops.EMB_ROWWISE_ADAGRAD, ops.EMB_ADAGRAD,
                                                ops.EMB_ADAM) else None
    s2 = torch.rand(W.numel(), device=DEV) if opt == ops.EMB_ADAM else None
    res = []
    for _ in range(2):
        Wn = W.clone()
        a1 = s1.clone() if s1 is not None else None
        a2 = s2.clone() if s2 is not None else None
        dg = torch.zeros(W.numel(), device=DEV) if opt == ops.EMB_DENSE_GRAD else None
        ops.embedding_bwd(Wn, ro, idx, offs, goff, T, B, grad, T * D, opt, hyper, state1=a1,
                          state2=a2, dense_grad=dg)
        res.append((Wn, a1, dg))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0])
    if opt == ops.EMB_DENSE_GRAD:
        assert torch.equal(res[0][2], res[1][2])
    We = W.clone()
    e1 = s1.clone() if s1 is not None else None
    e2 = s2.clone() if s2 is not None else None
    edg = torch.zeros(W.numel(), device=DEV) if opt == ops.EMB_DENSE_GRAD else None
    ref.embedding_bwd(We, ro, idx, offs, goff, None, T, B, False, 20, grad, T * D, opt, e1, e2,
                      hyper, 1e-8, 0.9, 0.999, 0.0, edg)
    assert (res[0][0] - We).abs().max() < 1e-4 * max(1.0, We.abs().max().item())
    if edg is not None:
        assert (res[0][2] - edg).abs().max() < 1e-4 * max(1.0, edg.abs().max().item())
    if e1 is not None:
        assert (res[0][1] - e1).abs().max() < 1e-3 * max(1.0, e1.abs().max().item())


@pytest.mark.parametrize("B", [700, 8192])
@pytest.mark.parametrize("skew", [False, True])
@pytest.mark.parametrize("opt", [ops.EMB_ROWWISE_ADAGRAD, ops.EMB_ADAM])
def test_embedding_bwd_onehot_segsort(B, skew, opt):
    """One id per bag: the per-table LDS sort must give bit-identical updates
    to the device-wide radix sort, and match the fp32 reference."""
    T, D = 3, 128
    rows = [50, 9000, 70000]
    W, ro, idx, offs = _emb_case(T, B, rows, D, 1, skew, seed=7)
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    goff = torch.tensor([t * D for t in range(T)], device=DEV)
    grad = torch.randn(B * T * D, device=DEV)
    hyper = torch.tensor([0.05, 3.0], device=DEV)
    n1 = W.shape[0] if opt == ops.EMB_ROWWISE_ADAGRAD else W.numel()
    s1 = torch.rand(n1, device=DEV)
    s2 = torch.rand(W.numel(), device=DEV) if opt == ops.EMB_ADAM else None
    res = []
    for seg in (1, 0):
        Wn, a1 = W.clone(), s1.clone()
        a2 = s2.clone() if s2 is not None else None
        ops.embedding_bwd(Wn, ro, idx, offs, goff, T, B, grad, T * D, opt, hyper, state1=a1,
                          state2=a2, segsort=seg)
        res.append((Wn, a1))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    We, e1 = W.clone(), s1.clone()
    e2 = s2.clone() if s2 is not None else None
    ref.embedding_bwd(We, ro, idx, offs, goff, None, T, B, False, 20, grad, T * D, opt, e1, e2,
                      hyper, 1e-8, 0.9, 0.999, 0.0, None)
    assert (res[0][0] - We).abs().max() < 1e-4 * max(1.0, We.abs().max().item())


@pytest.mark.parametrize("B", [8192, 1000])
def test_fused_bottom_mlp_matches_per_layer_gemms(B):
    """The fused bottom-MLP forward (one launch, activations chained through
    LDS) writes bitwise the same three activations as the per-layer GEMMs,
    including a batch that is not a multiple of the 32-row tile."""
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    cfg = DLRMConfig(table_rows=[1000, 20, 5000])
    tr = DLRMTrainer(cfg, B, DEV)
    assert tr._fused_bottom
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, 13, generator=g)
    tr.x0[:, :13] = x.to(DEV, torch.bfloat16)
    outs = []
    for fused in (True, False):
        tr._fused_bottom = fused
        for t in (tr.bot_in[1], tr.bot_in[2], tr.h_out):
            t[:, : t.shape[1] - (64 if t is not tr.h_out else 0)].fill_(7.0)
        tr._s_bottom_fwd()
        torch.cuda.synchronize()
        outs.append([tr.bot_in[1].clone(), tr.bot_in[2].clone(), tr.h_out.clone()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert float(outs[0][2].float().abs().sum()) > 0
    # and against an fp32 torch oracle of the same layers (bf16 operands,
    # fp32 products, the activations rounded to bf16 between layers)
    h = tr.bot_in[0].float()
    for i, L in enumerate(tr.bottom_layers):
        W = tr.fp.bf16(L.name + ".w")[:, :L.in_k].float()
        y = (h[:, :L.in_k] @ W.t())[:, :L.out]
        if not L.bias_in_k:
            y = y + tr.fp.param(L.name + ".w")[:L.out, L.bcol].float()
        y = torch.relu(y).to(torch.bfloat16).float()
        if i + 1 < len(tr.bottom_layers):
            # the next layer's augmented input (its ones column for an in-K bias)
            h = tr.bot_in[i + 1].float().clone()
            h[:, :L.out] = y
        else:
            h = y
    got = outs[0][2].float()[:, : h.shape[1]]
    rel = float((got - h).abs().max() / h.abs().max())
    assert rel < 2e-2, rel


@pytest.mark.parametrize("B", [8192, 1000])
def test_fused_bottom_mlp_batch_load_fold(B):
    """The batch load folded into the fused bottom-MLP launch (fp32 dense
    features + labels from a staging buffer) gives bitwise what batch_load
    followed by the plain fused launch gives: x0, labels and the three
    activations."""
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    cfg = DLRMConfig(table_rows=[1000, 20, 5000])
    tr = DLRMTrainer(cfg, B, DEV)
    assert tr._fused_bottom
    g = torch.Generator().manual_seed(5)
    dense = (torch.randn(B, 13, generator=g) * 3).to(DEV)
    label = (torch.rand(B, generator=g) < 0.3).float().to(DEV)
    res = []
    for fold in (True, False):
        tr.x0[:, :13].fill_(5.0)
        tr.label.fill_(-1.0)
        for t in (tr.bot_in[1], tr.bot_in[2], tr.h_out):
            t[:, : t.shape[1] - (64 if t is not tr.h_out else 0)].fill_(7.0)
        if fold:
            tr._s_bottom_fwd(staged=(dense, label))
        else:
            ops.batch_load(dense, tr.x0, tr.ids[:0], tr.ids[:0], label, tr.label)
            tr._s_bottom_fwd()
        torch.cuda.synchronize()
        res.append([t.clone() for t in (tr.x0, tr.label, tr.bot_in[1], tr.bot_in[2], tr.h_out)])
    for a, b in zip(*res):
        assert torch.equal(a, b)
    assert torch.equal(res[0][1][:B], label)


def test_embedding_dense_grad_replicated_tables():
    """The replicated tables' backward at W > 1 (dense fp32 gradient, one id
    per bag, per-table LDS sort): the tiny tables' runs span tens of chunks
    and take the block-wide walk -- equal to the fp32 reference and bitwise
    reproducible."""
    T, B, D = 6, 8192, 128
    rows = [3, 4, 14, 155, 976, 2208]
    W, ro, idx, offs = _emb_case(T, B, rows, D, 1, False, seed=11)
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    goff = torch.tensor([t * D for t in range(T)], device=DEV)
    grad = torch.randn(B * T * D, device=DEV) * 0.01
    hyper = torch.tensor([0.05, 3.0], device=DEV)
    res = []
    for _ in range(2):
        dg = torch.zeros(W.numel(), device=DEV)
        ops.embedding_bwd(W.clone(), ro, idx, offs, goff, T, B, grad, T * D,
                          ops.EMB_DENSE_GRAD, hyper, dense_grad=dg, segsort=1)
        res.append(dg)
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1])
    edg = torch.zeros(W.numel(), device=DEV)
    ref.embedding_bwd(W.clone(), ro, idx, offs, goff, None, T, B, False, 20, grad, T * D,
                      ops.EMB_DENSE_GRAD, None, None, hyper, 1e-8, 0.9, 0.999, 0.0, edg)
    assert (res[0] - edg).abs().max() < 1e-4 * max(1.0, edg.abs().max().item())


@pytest.mark.parametrize("R,B", [(2, 2048), (3, 2048), (8, 2048), (8, 8192)])
def test_embedding_bwd_onehot_multirun(R, B):
    """World > 1 layout: each physical table's ids arrive as R runs (virtual
    tables v = run * Tp + table sharing the table's rows). Per-run LDS sorts +
    run merge must match the radix-sort path bit for bit."""
    Tp, D = 3, 128
    rows = [50, 9000, 70000]
    g = torch.Generator().manual_seed(11)
    T = R * Tp
    ro_p = torch.tensor([0, 50, 9050])
    ro = ro_p.repeat(R).to(DEV)
    ids = torch.cat([torch.randint(0, min(rows[v % Tp], 40 if v % 2 else 10 ** 9), (B,), generator=g)
                     for v in range(T)]).to(DEV)
    offs = torch.arange(T * B + 1, device=DEV)
    goff = torch.tensor([v * D for v in range(T)], device=DEV)
    W = torch.randn(sum(rows), D, generator=g).to(DEV)
    grad = torch.randn(B * T * D, generator=g).to(DEV)
    hyper = torch.tensor([0.05, 3.0], device=DEV)
    s1 = torch.rand(W.shape[0], device=DEV)
    res = []
    for seg in (R, 0):
        Wn, a1 = W.clone(), s1.clone()
        ops.embedding_bwd(Wn, ro, ids, offs, goff, T, B, grad, T * D, ops.EMB_ROWWISE_ADAGRAD,
                          hyper, state1=a1, segsort=seg)
        res.append((Wn, a1))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("segsort", [0, 1])
def test_embedding_bwd_prepare_apply_matches_fused(segsort):
    """The two-phase backward (ids-only prepare on another stream, then apply)
    gives the fused result bit for bit."""
    T, B, D = 3, 4096, 128
    rows = [50, 9000, 70000]
    W, ro, idx, offs = _emb_case(T, B, rows, D, 1 if segsort else 3, False, seed=9)
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    goff = torch.tensor([t * D for t in range(T)], device=DEV)
    grad = torch.randn(B * T * D, device=DEV)
    hyper = torch.tensor([0.05, 3.0], device=DEV)
    s1 = torch.rand(W.shape[0], device=DEV)
    Wf, sf = W.clone(), s1.clone()
    ops.embedding_bwd(Wf, ro, idx, offs, goff, T, B, grad, T * D, ops.EMB_ROWWISE_ADAGRAD, hyper,
                      state1=sf, segsort=segsort)
    Wp, sp = W.clone(), s1.clone()
    ws = torch.empty(ops.embedding_bwd_workspace(idx.numel(), D), dtype=torch.uint8, device=DEV)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ops.embedding_bwd_prepare(Wp, ro, idx, offs, goff, T, B, T * D, ws, segsort=segsort)
    torch.cuda.current_stream().wait_stream(side)
    ops.embedding_bwd_apply(Wp, ro, idx, offs, goff, T, B, grad, T * D, ops.EMB_ROWWISE_ADAGRAD,
                            hyper, ws, state1=sp, segsort=segsort)
    torch.cuda.synchronize()
    assert torch.equal(Wf, Wp) and torch.equal(sf, sp)


@pytest.mark.parametrize("mean", [False, True])
def test_embedding_bwd_fixed_bag_len_keys(mean):
    """Fixed multi-hot (every bag of table t holds L[t] ids, DCN-v2's MLPerf
    pooling): the keys pass with ``bag_len`` (bag by division) prepares the
    same workspace as the bag-offset search -- identical update."""
    T, B, D = 4, 2048, 128
    rows = [3, 40000, 900, 1 << 20]
    L = [1, 7, 3, 100]
    g = torch.Generator().manual_seed(4)
    idx = torch.cat([torch.randint(0, rows[t], (B * L[t],), generator=g) for t in range(T)])
    lens = torch.tensor(L).repeat_interleave(B)
    offs = torch.zeros(T * B + 1, dtype=torch.long)
    offs[1:] = lens.cumsum(0)
    ro = torch.zeros(T, dtype=torch.long)
    ro[1:] = torch.tensor(rows[:-1]).cumsum(0)
    W = torch.randn(sum(rows), D, generator=g) * 0.1
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    goff = torch.tensor([t * D for t in range(T)], device=DEV)
    grad = torch.randn(B * T * D, device=DEV)
    hyper = torch.tensor([0.05, 3.0], device=DEV)
    s1 = torch.rand(W.shape[0], device=DEV)
    bl = torch.tensor(L, dtype=torch.int32, device=DEV)
    out = []
    for bag_len in (None, bl):
        Wp, sp = W.clone(), s1.clone()
        ws = torch.empty(ops.embedding_bwd_workspace(idx.numel(), D), dtype=torch.uint8,
                         device=DEV)
        ops.embedding_bwd_prepare(Wp, ro, idx, offs, goff, T, B, T * D, ws, mean=mean,
                                  bag_len=bag_len)
        ops.embedding_bwd_apply(Wp, ro, idx, offs, goff, T, B, grad, T * D,
                                ops.EMB_ROWWISE_ADAGRAD, hyper, ws, state1=sp, mean=mean)
        torch.cuda.synchronize()
        out.append((Wp, sp))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    assert not torch.equal(out[0][0], W)


def test_embedding_bwd_deterministic():
    T, B, D = 2, 4096, 128
    rows = [3, 100000]
    W, ro, idx, offs = _emb_case(T, B, rows, D, 4, True, seed=5)
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    goff = torch.tensor([0, D], device=DEV)
    grad = torch.randn(B * T * D, device=DEV)
    hyper = torch.tensor([0.1, 1.0], device=DEV)
    outs = []
    for _ in range(2):
        Wn = W.clone()
        s1 = torch.zeros(W.shape[0], device=DEV)
        ops.embedding_bwd(Wn, ro, idx, offs, goff, T, B, grad, T * D, ops.EMB_ROWWISE_ADAGRAD,
                          hyper, state1=s1)
        outs.append(Wn)
    assert torch.equal(outs[0], outs[1])


# ------------------------------------------------------------ loss/optim
@pytest.mark.parametrize("K", [64, 256])
def test_head_bce(K):
    torch.manual_seed(4)
    B = 1000
    H = bf(torch.randn(B, K, device=DEV))
    w = torch.randn(K, device=DEV)
    b = torch.randn(1, device=DEV)
    y = (torch.rand(B, device=DEV) > 0.5).float()
    np_ = ops.head_parts(B)
    logits = torch.empty(B, device=DEV)
    dH = torch.empty_like(H)
    part = torch.empty(np_ * (K + 2), device=DEV)
    ops.head_bce(H, w, b, y, 1.0 / B, True, logits, dH, part)
    red = torch.empty(K + 2, device=DEV)
    ops.reduce_rows(part, np_, K + 2, K + 2, red)
    el, edH, ep = torch.empty_like(logits), torch.empty_like(dH), torch.zeros(np_ * (K + 2), device=DEV)
    ref.head_bce(H, w, b, y, 1.0 / B, True, el, edH, ep)
    assert rel_err(logits, el) < 1e-4
    assert rel_err(dH, edH) < 1e-2
    assert rel_err(red, ep[: K + 2]) < 1e-4


def test_colsum_reduce():
    x = bf(torch.randn(1000, 512, device=DEV))
    out = torch.empty(512, device=DEV)
    ops.colsum(x, out)
    assert rel_err(out, x.float().sum(0)) < 1e-4


@pytest.mark.parametrize("opt", [ops.OPT_ADAMW, ops.OPT_ADAM, ops.OPT_SGD, ops.OPT_ADAGRAD])
def test_dense_optimizer(opt):
    n = 4096 + 64
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.rand(n, device=DEV)
    v = torch.rand(n, device=DEV)
    hyper = torch.tensor([1e-2, 5.0, 0.5], device=DEV)
    pb = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    P, M, V = p.clone(), m.clone(), v.clone()
    ops.dense_optimizer(p, g, m, v, pb, opt, hyper, wd=0.01, momentum=0.9 if opt == ops.OPT_SGD else 0.0)
    ref.dense_optimizer(P, g, M, V, None, opt, hyper, 0.9, 0.999, 1e-8, 0.01,
                        0.9 if opt == ops.OPT_SGD else 0.0, None)
    assert (p - P).abs().max() < 1e-5
    assert torch.equal(pb, p.to(torch.bfloat16))


def test_auc_hist():
    logits = torch.randn(10000, device=DEV)
    y = (torch.rand(10000, device=DEV) < torch.sigmoid(logits)).float()
    h = torch.zeros(2 * 200, dtype=torch.long, device=DEV)
    ops.auc_hist(logits, y, 200, h)
    e = torch.zeros_like(h)
    ref.auc_hist(logits, y, 200, e)
    assert torch.equal(h, e)
    assert abs(ref.hist_auc(h) - ref.exact_auc(logits, y)) < 5e-3


# ---------------------------------------------------------- end-to-end
def test_dlrm_step_matches_cpu():
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    cfg = DLRMConfig(embedding_dim=64, table_rows=[1000, 20, 5000, 300, 3], bottom=[128, 64],
                     top=[128, 64, 1], dense_lr=3e-3, emb_lr=0.05)
    B = 256
    gpu = DLRMTrainer(cfg, B, DEV)
    cpu = DLRMTrainer(cfg, B, "cpu")
    cpu.emb.tw_store.weight.copy_(gpu.emb.tw_store.weight.cpu())
    cpu.fp.p.copy_(gpu.fp.p.cpu())
    cpu.fp.sync_bf16()
    data = SyntheticCriteo(cfg.table_rows, B, device="cpu", seed=3)
    lg, lc = [], []
    for _ in range(20):
        batch = data.next()
        gpu.load_batch(*(x.to(DEV) for x in batch))
        cpu.load_batch(*batch)
        gpu.step()
        cpu.step()
        lg.append(gpu.pop_loss() / B)
        lc.append(cpu.pop_loss() / B)
    for a, b in zip(lg, lc):
        assert abs(a - b) < 0.02, (lg, lc)
    assert sum(lg[-5:]) < sum(lg[:5])


def test_dlrm_head_reduce_side_blocks_bit_identical():
    """The head's reduce run by extra blocks of the first top backward GEMM
    pair (parked head_reduce) gives the bits of its own launch."""
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    cfg = DLRMConfig(embedding_dim=128, table_rows=[1000, 20, 5000], bottom=[128],
                     top=[512, 256, 1])
    B = 1024
    a = DLRMTrainer(cfg, B, DEV)
    b = DLRMTrainer(cfg, B, DEV)
    a._head_side, b._head_side = True, False
    data = SyntheticCriteo(cfg.table_rows, B, device=DEV, seed=9)
    for _ in range(5):
        x = data.next()
        for t in (a, b):
            t.load_batch(*x)
            t.step()
    torch.cuda.synchronize()
    assert torch.equal(a.fp.p, b.fp.p)
    assert torch.equal(a.emb.tw_store.weight, b.emb.tw_store.weight)
    assert torch.equal(a.dense_hyper, b.dense_hyper) and torch.equal(a.emb_hyper, b.emb_hyper)
    assert a.pop_loss() == b.pop_loss()


@pytest.mark.parametrize("staged,one", [(False, "0"), (False, "1"), (False, "ids0"),
                                        (True, "0"), (False, "defer")])
def test_dlrm_graph_replay_matches_eager(staged, one):
    """Graph-replayed steps match eager ones: per-stream graphs (one=1: each
    stream's step as composed graphs joined by in-graph event nodes, with
    device-resident batches whose ids are copied on a third stream behind the
    sort; ids0: without that stream; defer: as 1, with the top weight grads
    after the interaction backward) and the staged multi-rank capture at one
    rank."""
    import dataclasses

    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    cfg = DLRMConfig(embedding_dim=128, table_rows=[1000, 20, 5000], bottom=[128],
                     top=[256, 1], composed_graphs=one != "0",
                     ids_stream=one in ("1", "defer"))
    B = 512
    a = DLRMTrainer(cfg, B, DEV)
    cfg_b = dataclasses.replace(cfg, defer_wgrad=True if one == "defer" else None)
    b = DLRMTrainer(cfg_b, B, DEV)
    data = SyntheticCriteo(cfg.table_rows, B, device=DEV, seed=4)
    batches = [data.next() for _ in range(6)]
    torch.cuda.synchronize()          # device-resident batches, ready for every stream
    for t in (a, b):
        t.load_batch(*batches[0])
    b.capture_graph(warmup=1, staged=staged)
    if not staged:
        assert b.graph == "streams" and ("M" in b._ms["graphs"]) == (one != "0")
        assert (b._ms["cstream"] is not None) == (one in ("1", "defer"))
    if staged:
        # one rank: the prep stage is a no-op and is not captured (no empty graph)
        assert all(kind in ("m", "em", "j") or g[0] is not None for kind, g in b.graph)
        assert not b.emb.fwd_prep_noop or len(b._stages()) == 15
    a.step()  # replicate the capture warmup on the eager trainer
    for x in batches[1:]:
        a.load_batch(*x)
        b.load_batch(*x, on_device=not staged)
        a.step()
        b.step()
    torch.cuda.synchronize()
    b.sync_streams()
    torch.cuda.synchronize()
    assert torch.allclose(a.fp.p, b.fp.p, atol=1e-5)
    assert torch.allclose(a.emb.tw_store.weight, b.emb.tw_store.weight, atol=1e-5)


def test_dlrm_graph_replay_matches_eager_without_packet_capture():
    """bench.py's one-GPU runtime mode (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0: graph
    nodes dispatched at launch) replays the composed per-stream graphs to the
    same result as eager steps. A child process: the mode is read when the
    HIP runtime initialises."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DEBUG_CLR_GRAPH_PACKET_CAPTURE="0")
    code = ("import tests.test_gpu_kernels as t; "
            "t.test_dlrm_graph_replay_matches_eager(False, '1'); print('ok')")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


@pytest.mark.parametrize("mean", [False, True])
def test_embedding_bwd_multihot_large(mean):
    """DCN-v2-shaped multi-hot backward (variable and empty bags, ~0.7M ids:
    the per-bag keys kernel + the 4096-item-tile radix sort) matches the fp32
    reference, and matches the 1024-item-tile sort bit for bit."""
    T, B, D = 4, 8192, 128
    rows = [5, 300_000, 1_000, 2_000_000]
    g = torch.Generator(device="cpu").manual_seed(3)
    maxlen = [1, 100, 8, 60]
    lens = torch.cat([torch.randint(0, m + 1, (B,), generator=g) for m in maxlen])
    offs = torch.zeros(T * B + 1, dtype=torch.long)
    offs[1:] = lens.cumsum(0)
    idx = torch.cat([torch.randint(0, rows[t], (int(lens[t * B:(t + 1) * B].sum()),),
                                   generator=g) for t in range(T)])
    assert idx.numel() > (1 << 19)
    ro = torch.zeros(T, dtype=torch.long)
    ro[1:] = torch.tensor(rows[:-1]).cumsum(0)
    W = torch.randn(sum(rows), D, generator=g) * 0.1
    W, ro, idx, offs = (x.to(DEV) for x in (W, ro, idx, offs))
    goff = torch.tensor([t * D for t in range(T)], device=DEV)
    grad = torch.randn(B * T * D, device=DEV)
    hyper = torch.tensor([0.05, 3.0], device=DEV)
    res = []
    for tiled in (1, 0):
        old = ops.radix_sort_tiled(tiled)
        try:
            Wn, s1 = W.clone(), torch.zeros(W.shape[0], device=DEV)
            ops.embedding_bwd(Wn, ro, idx, offs, goff, T, B, grad, T * D,
                              ops.EMB_ROWWISE_ADAGRAD, hyper, state1=s1, mean=mean)
            torch.cuda.synchronize()
        finally:
            ops.radix_sort_tiled(old)
        res.append((Wn, s1))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    We, e1 = W.clone(), torch.zeros(W.shape[0], device=DEV)
    ref.embedding_bwd(We, ro, idx, offs, goff, None, T, B, mean, 20, grad, T * D,
                      ops.EMB_ROWWISE_ADAGRAD, e1, None, hyper, 1e-8, 0.9, 0.999, 0.0, None)
    assert (res[0][0] - We).abs().max() < 1e-4 * max(1.0, We.abs().max().item())
    assert (res[0][1] - e1).abs().max() < 1e-3 * max(1.0, e1.abs().max().item())


def test_embedding_bwd_graph_replay_large():
    """Bench-scale fused backward (213k ids, skewed + uniform tables) captured
    in a hipGraph and replayed must match eager execution bit for bit."""
    T, B, D = 26, 8192, 128
    rows = [3, 10, 4000, 2_000_000] + [50_000] * 22
    g = torch.Generator(device="cpu").manual_seed(7)
    idx = torch.cat([torch.randint(0, r, (B,), generator=g) for r in rows]).to(DEV)
    offs = torch.arange(T * B + 1, device=DEV)
    ro = torch.zeros(T, dtype=torch.long)
    ro[1:] = torch.tensor(rows[:-1]).cumsum(0)
    ro = ro.to(DEV)
    W0 = torch.randn(sum(rows), D, device=DEV) * 0.01
    goff = torch.tensor([t * D for t in range(T)], device=DEV)
    grad = (torch.randn(B * T * D, device=DEV) * 0.01).to(torch.bfloat16)
    hyper = torch.tensor([0.05, 1.0], device=DEV)
    We, se = W0.clone(), torch.zeros(W0.shape[0], device=DEV)
    for _ in range(3):
        ops.embedding_bwd(We, ro, idx, offs, goff, T, B, grad, T * D, ops.EMB_ROWWISE_ADAGRAD,
                          hyper, state1=se)
    Wg, sg = W0.clone(), torch.zeros(W0.shape[0], device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.embedding_bwd(Wg, ro, idx, offs, goff, T, B, grad, T * D, ops.EMB_ROWWISE_ADAGRAD,
                          hyper, state1=sg)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ops.embedding_bwd(Wg, ro, idx, offs, goff, T, B, grad, T * D, ops.EMB_ROWWISE_ADAGRAD,
                          hyper, state1=sg)
    graph.replay()
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(We, Wg)
    assert torch.equal(se, sg)


def test_gemm_out2_mul_add(gemm_pol):
    torch.manual_seed(5)
    M, N, K = 300, 256, 128
    A = bf(torch.randn(M, K, device=DEV))
    W = bf(torch.randn(N, K, device=DEV))
    bias = torch.randn(N, device=DEV)
    mul = bf(torch.randn(M, N, device=DEV))
    add = bf(torch.randn(M, N, device=DEV))
    y, o2 = (torch.empty(M, N, dtype=torch.bfloat16, device=DEV) for _ in range(2))
    ops.gemm(A, False, W, False, bias, False, None, y, None, 1, mul=mul, add=add, out2=o2)
    ey, eo2 = (torch.empty(M, N, dtype=torch.bfloat16, device=DEV) for _ in range(2))
    ref.gemm(A, False, W, False, bias, False, None, ey, None, 1, mul=mul, add=add, out2=eo2)
    assert rel_err(y, ey) < 1e-2 and rel_err(o2, eo2) < 2e-2


def test_concat_split_cross_bwd():
    torch.manual_seed(6)
    B, F, D = 100, 5, 64
    T = F - 1
    dense = bf(torch.randn(B, D, device=DEV))
    emb = bf(torch.randn(B * T * D, device=DEV))
    off = [0] + [t * D for t in range(T)]
    stride = [0] + [T * D] * T
    out = torch.empty(B, F * D, dtype=torch.bfloat16, device=DEV)
    ops.concat_features(dense, emb, off, stride, F, D, out)
    exp = torch.empty_like(out)
    ref.concat_features(dense, emb, off, stride, F, D, exp)
    assert torch.equal(out, exp)
    dd, de = torch.zeros_like(dense), torch.zeros_like(emb)
    ops.split_features(out, F, D, dense, dd, de, off, stride, True)
    edd, ede = torch.zeros_like(dense), torch.zeros_like(emb)
    ref.split_features(out, F, D, dense, edd, ede, off, stride, True)
    assert torch.equal(dd, edd) and torch.equal(de, ede)
    a, b, c = (bf(torch.randn(B * 64, device=DEV)) for _ in range(3))
    dy, dx0 = bf(torch.randn(B * 64, device=DEV)), bf(torch.randn(B * 64, device=DEV))
    e_dy, e_dx0 = dy.clone(), dx0.clone()
    ops.cross_bwd(a, b, c, dy, dx0, True, True)
    ref.cross_bwd(a, b, c, e_dy, e_dx0, True, True)
    assert rel_err(dy, e_dy) < 1e-2 and rel_err(dx0, e_dx0) < 1e-2


def test_dcn_step_matches_cpu():
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    cfg = DLRMConfig(embedding_dim=64, table_rows=[1000, 20, 5000, 300], bottom=[128, 64],
                     top=[128, 64, 1], interaction="dcn", dcn_layers=2, dcn_rank=64,
                     pooling=[2, 1, 3, 1], dense_lr=1e-3, emb_lr=0.05)
    B = 256
    gpu = DLRMTrainer(cfg, B, DEV)
    cpu = DLRMTrainer(cfg, B, "cpu")
    cpu.emb.tw_store.weight.copy_(gpu.emb.tw_store.weight.cpu())
    cpu.fp.p.copy_(gpu.fp.p.cpu())
    cpu.fp.sync_bf16()
    data = SyntheticCriteo(cfg.table_rows, B, pooling=cfg.pooling, device="cpu", seed=3)
    for _ in range(10):
        batch = data.next()
        gpu.load_batch(*(x.to(DEV) for x in batch))
        cpu.load_batch(*batch)
        gpu.step()
        cpu.step()
        a, b = gpu.pop_loss() / B, cpu.pop_loss() / B
        assert abs(a - b) < 0.02, (a, b)


# 3 M keys: 2 tiles per thread in the tiled column scan; 16.8 M: past its
# 4096-tile limit (the single-thread-per-column scan fallback)
@pytest.mark.parametrize("n", [1, 1000, 4096, 4097, 213_000, 1_500_000, 3_000_000, 16_800_000])
@pytest.mark.parametrize("dtype,bits", [(torch.int32, 28), (torch.int64, 40), (torch.int32, 5)])
@pytest.mark.parametrize("tiled", [0, 2])
def test_radix_sort_matches_stable_torch_sort(n, dtype, bits, tiled):
    g = torch.Generator(device="cpu").manual_seed(n)
    keys = torch.randint(0, 1 << bits, (n,), generator=g, dtype=torch.int64)
    keys[: n // 3] = keys[: n // 3] % 7          # heavy duplicates
    keys = keys.to(dtype).to(DEV)
    vals = torch.arange(n, dtype=torch.int32, device=DEV)
    old = ops.radix_sort_tiled(tiled)
    try:
        k, v = ops.sort_pairs(keys, vals, bits)
    finally:
        ops.radix_sort_tiled(old)
    ek, ei = torch.sort(keys, stable=True)
    assert torch.equal(k, ek)
    assert torch.equal(v, ei.to(torch.int32))


def test_dlrm_small_hidden_layers_match_cpu():
    """Hidden widths below the 64-wide K padding (augmented bias inside K)."""
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    cfg = DLRMConfig(embedding_dim=16, table_rows=[300, 40, 500, 70], bottom=[32, 16],
                     top=[32, 1], dense_lr=3e-3, emb_lr=0.05)
    B = 64
    gpu = DLRMTrainer(cfg, B, DEV)
    cpu = DLRMTrainer(cfg, B, "cpu")
    cpu.emb.tw_store.weight.copy_(gpu.emb.tw_store.weight.cpu())
    cpu.fp.p.copy_(gpu.fp.p.cpu())
    cpu.fp.sync_bf16()
    data = SyntheticCriteo(cfg.table_rows, B, device="cpu", seed=3)
    for _ in range(10):
        batch = data.next()
        gpu.load_batch(*(x.to(DEV) for x in batch))
        cpu.load_batch(*batch)
        gpu.step()
        cpu.step()
        assert abs(gpu.pop_loss() - cpu.pop_loss()) / B < 0.02


@pytest.mark.parametrize("K", [16, 32, 100])
@pytest.mark.parametrize("a_col,b_col", [(False, False), (False, True), (True, True)])
def test_gemm_k_tail_padding(K, a_col, b_col, gemm_pol):
    torch.manual_seed(K)
    M, N = 96, 80
    A = bf(torch.randn(K, M, device=DEV) if a_col else torch.randn(M, K, device=DEV))
    Bm = bf(torch.randn(K, N, device=DEV) if b_col else torch.randn(N, K, device=DEV))
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.gemm(A, a_col, Bm, b_col, out=out)
    a = A.float().t() if a_col else A.float()
    b = Bm.float() if b_col else Bm.float().t()
    assert rel_err(out, a @ b) < 2e-2


@pytest.mark.parametrize("D", [1, 16, 6])
def test_jagged_dense_roundtrip(D):
    torch.manual_seed(D)
    lens = torch.randint(0, 30, (37,))
    off = torch.zeros(38, dtype=torch.int64)
    off[1:] = torch.cumsum(lens, 0)
    nnz = int(off[-1])
    vals = torch.randn(nnz, D)
    T = 20
    out = torch.empty(37, T, D, device=DEV)
    ops.jagged_to_dense(vals.to(DEV), off.to(DEV), T, -2.0, out)
    ref_out = torch.empty(37, T, D)
    ref.jagged_to_dense(vals, off, T, -2.0, ref_out)
    assert torch.equal(out.cpu(), ref_out)
    g = torch.randn(37, T, D)
    vg = torch.empty(nnz, D, device=DEV)
    ops.dense_to_jagged(g.to(DEV), off.to(DEV), vg)
    rg = torch.empty(nnz, D)
    ref.dense_to_jagged(g, off, rg)
    assert torch.equal(vg.cpu(), rg)
    ids = torch.randint(0, 1000, (nnz,))
    oi = torch.empty(37, T, dtype=torch.int64, device=DEV)
    ops.jagged_ids_to_dense(ids.to(DEV), off.to(DEV), 0, oi)
    ri = torch.empty(37, T, dtype=torch.int64)
    ref.jagged_ids_to_dense(ids, off, 0, ri)
    assert torch.equal(oi.cpu(), ri)


def test_head_reduce_and_step_bumps():
    torch.manual_seed(11)
    nparts, K = 37, 256
    part = torch.randn(nparts * (K + 2), device=DEV)
    grad = torch.empty(K + 1, device=DEV)
    loss = torch.tensor([1.5], device=DEV)
    h1 = torch.tensor([0.1, 4.0, 1.0], device=DEV)
    h2 = torch.tensor([0.2, 9.0], device=DEV)
    ops.head_reduce(part, nparts, K, grad, loss, (h1, h2))
    p = part.view(nparts, K + 2).double()
    assert torch.allclose(grad.double(), p[:, : K + 1].sum(0), atol=1e-4)
    assert abs(float(loss) - (1.5 + float(p[:, K + 1].sum()))) < 1e-3
    assert float(h1[1]) == 5.0 and float(h2[1]) == 10.0 and float(h1[0]) == pytest.approx(0.1)


def _fixed_order_column_sums(p, PH=16):
    """head_reduce's summation order in fp32: per column, row phase ph sums
    rows ph, ph + PH, ... into four accumulators (groups of four rows, a
    partial last group into the first), then the phases are added in order."""
    n = p.shape[0]
    out = torch.zeros(p.shape[1], dtype=torch.float32)
    for ph in range(PH):
        s = [torch.zeros(p.shape[1], dtype=torch.float32) for _ in range(4)]
        r = ph
        while r + 3 * PH < n:
            for q in range(4):
                s[q] = s[q] + p[r + q * PH]
            r += 4 * PH
        while r < n:
            s[0] = s[0] + p[r]
            r += PH
        out = out + ((s[0] + s[1]) + (s[2] + s[3]))
    return out


@pytest.mark.parametrize("nparts", [37, 512, 600])
def test_head_reduce_fixed_order(nparts):
    """The preloaded head_reduce adds the partial rows in the plain loop's
    order: bit-identical to that order for <= 512 rows and past it."""
    torch.manual_seed(17)
    K = 256
    part = torch.randn(nparts * (K + 2), device=DEV)
    grad = torch.empty(K + 1, device=DEV)
    loss = torch.zeros(1, device=DEV)
    ops.head_reduce(part, nparts, K, grad, loss)
    want = _fixed_order_column_sums(part.view(nparts, K + 2).cpu())
    assert torch.equal(grad.cpu(), want[: K + 1])
    assert torch.equal(loss.cpu(), want[K + 1:])


@pytest.mark.parametrize("opt", ["adamw", "sgd_momentum", "adagrad"])
def test_dense_optimizer_slab_segments(opt):
    """Split-K weight-grad slabs summed inside the optimizer == reduce then step
    (segments of 1, 3, 9 and 17 slabs: partial and several 8-slab groups)."""
    torch.manual_seed(12)
    n = 8192
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    segs = [(0, 512, 1), (1024, 1024, 3), (2048, 2048, 9), (5120, 1536, 17)]
    slabs = [torch.randn(S * ln, device=DEV) for _, ln, S in segs]
    hyper = torch.tensor([1e-2, 2.0, 1.0], device=DEV)
    code = {"adamw": ops.OPT_ADAMW, "sgd_momentum": ops.OPT_SGD,
            "adagrad": ops.OPT_ADAGRAD}[opt]
    kw = {"momentum": 0.9} if opt == "sgd_momentum" else {}
    g2 = g.clone()
    for (st, ln, S), sl in zip(segs, slabs):
        g2[st:st + ln] = sl.view(S, ln).sum(0)
    m0, v0 = torch.rand(n, device=DEV), torch.rand(n, device=DEV)
    res = []
    for grad, sg in ((g, [(st, sl, S) for (st, _, S), sl in zip(segs, slabs)]), (g2, ())):
        p1 = p.clone()
        m1 = m0.clone()
        v1 = v0.clone() if opt == "adamw" else None
        ops.dense_optimizer(p1, grad, m1, v1, None, code, hyper, wd=0.01, segments=sg, **kw)
        res.append((p1, m1))
    assert torch.allclose(res[0][0], res[1][0], atol=1e-5)
    assert torch.allclose(res[0][1], res[1][1], atol=1e-4)


def test_gather_columns_matches_index_select():
    torch.manual_seed(13)
    N, n = 5000, 777
    src = [torch.randint(-100, 100, (N,), device=DEV, dtype=dt)
           for dt in (torch.int8, torch.int16, torch.int32, torch.int64)]
    src.append(torch.randn(N, device=DEV))
    idx = torch.randperm(N, device=DEV)[:n]
    outi = torch.zeros(4, n, dtype=torch.int64, device=DEV)
    X = torch.zeros(n, 9, device=DEV)
    dst = [outi[i] for i in range(4)] + [X.view(-1)[5:]]
    ops.gather_columns(src, idx, 0, n, dst, [1, 1, 1, 1, 9])
    for i in range(4):
        assert torch.equal(outi[i], src[i].index_select(0, idx).long())
    assert torch.equal(X[:, 5], src[4].index_select(0, idx))
    ops.gather_columns(src[:1], None, 100, n, [outi[0]], [1])   # contiguous range
    assert torch.equal(outi[0], src[0][100:100 + n].long())


# ------------------------------------------------------------------ batch load
@pytest.mark.parametrize("n", [8192 * 26, 4097])
def test_batch_load_matches_copies(n):
    B, nd, ldx = 1024, 13, 32
    g = torch.Generator(device=DEV).manual_seed(3)
    dense = torch.rand(B, nd, device=DEV, generator=g) * 5
    ids = torch.randint(0, 1 << 40, (n,), device=DEV, generator=g)
    label = (torch.rand(B, device=DEV, generator=g) > 0.5).float()
    x0 = torch.full((B, ldx), 7.0, device=DEV, dtype=torch.bfloat16)
    ids_dst = torch.empty_like(ids)
    label_dst = torch.empty_like(label)
    torch.ops.tdfo.batch_load(dense, x0, ids, ids_dst, label, label_dst)
    torch.cuda.synchronize()
    assert torch.equal(ids_dst, ids)
    assert torch.equal(label_dst, label)
    assert torch.equal(x0[:, :nd], dense.to(torch.bfloat16))
    assert torch.all(x0[:, nd:] == 7.0)          # pad / bias columns untouched


def test_load_batch_any_input_dtype_and_offset_views():
    """DLRMTrainer.load_batch must take int32 ids, float64 labels and an ids
    view at an odd int64 offset (e.g. a rank's slice of a global id tensor):
    the fused kernel is used only when its contract holds, else copies."""
    from tdfo_amd.models.dlrm import DLRMConfig, DLRMTrainer

    cfg = DLRMConfig(embedding_dim=64, table_rows=[100, 50], bottom=[64], top=[64, 1])
    B = 128
    tr = DLRMTrainer(cfg, B, DEV)
    g = torch.Generator(device=DEV).manual_seed(1)
    dense = torch.rand(B, 13, device=DEV, generator=g)
    ids = torch.randint(0, 50, (2 * B,), device=DEV, generator=g)
    label = (torch.rand(B, device=DEV, generator=g) > 0.5).double()
    tr.load_batch(dense, ids.int(), label)
    big = torch.cat([torch.zeros(1, dtype=torch.int64, device=DEV), ids])
    torch.cuda.synchronize()
    assert torch.equal(tr.ids, ids) and torch.equal(tr.label, label.float())
    tr.ids.zero_()
    tr.load_batch(dense, big[1:], label.float())               # 8-B aligned, not 16
    torch.cuda.synchronize()
    assert torch.equal(tr.ids, ids)
    assert torch.equal(tr.x0[:, :13], dense.to(torch.bfloat16))
    tr.step()
    torch.cuda.synchronize()


@pytest.mark.parametrize("opt", [ops.EMB_ROWWISE_ADAGRAD, ops.EMB_SGD, ops.EMB_ADAGRAD,
                                 ops.EMB_ADAM])
@pytest.mark.parametrize("D", [32, 128])
def test_embedding_dense_update_matches_reference(opt, D):
    """Replicated tables' step from an all-reduced dense gradient (half the
    rows untouched: they must not move for SGD / Adagrad variants)."""
    rows = 3000
    g = torch.Generator().manual_seed(D + opt)
    W0 = torch.randn(rows, D, generator=g)
    grad = torch.randn(rows, D, generator=g) * 0.1
    grad[::2] = 0.0
    s1 = s2 = None
    if opt == ops.EMB_ROWWISE_ADAGRAD:
        s1 = torch.rand(rows, generator=g)
    elif opt == ops.EMB_ADAGRAD:
        s1 = torch.rand(rows, D, generator=g)
    elif opt == ops.EMB_ADAM:
        s1, s2 = torch.zeros(rows, D), torch.zeros(rows, D)
    hyper = torch.tensor([0.05, 3.0])
    Wg = W0.to(DEV)
    sg1 = s1.to(DEV) if s1 is not None else None
    sg2 = s2.to(DEV) if s2 is not None else None
    ops.embedding_dense_update(Wg, grad.to(DEV), rows, opt, hyper.to(DEV), state1=sg1, state2=sg2)
    We, se1 = W0.clone(), s1.clone() if s1 is not None else None
    se2 = s2.clone() if s2 is not None else None
    ref.embedding_dense_update(We, grad, rows, opt, se1, se2, hyper, 1e-8, 0.9, 0.999, 0.0)
    assert torch.allclose(Wg.cpu(), We, atol=1e-5, rtol=1e-5)
    if opt != ops.EMB_ADAM:
        assert torch.equal(Wg.cpu()[::2], W0[::2])


@pytest.mark.parametrize("M", [8192, 1000])
@pytest.mark.parametrize("N,K", [(1024, 512), (256, 512), (512, 256), (512, 3456), (3456, 512)])
@pytest.mark.parametrize("policy", [0, 3, 5, 8])
def test_gemm_batch_pairs_wgrad_dgrad(M, N, K, policy):
    """A layer's weight grad (split-K slabs + column sums) and dgrad (ReLU
    mask) recorded under ops.gemm_batch go out as one paired launch with the
    same numbers as two launches, bit for bit."""
    torch.manual_seed(7)
    dy = bf(torch.randn(M, N, device=DEV))
    x = bf(torch.randn(M, K + 64, device=DEV))
    W = bf(torch.randn(N, K + 64, device=DEV))
    S = ops.wgrad_splits(N, K, M)
    res = []
    oldp = ops.gemm_policy(policy)
    for pair in (1, 2, 0):
        old = ops.gemm_pairing(pair)
        try:
            slab = torch.zeros(S * N * (K + 64), device=DEV)
            dx = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
            with ops.gemm_batch():
                ops.gemm(dy, True, x[:, :K], True, None, False, None, None, slab, S,
                         ldc32=K + 64, csum_col=K)
                ops.gemm(dy, False, W[:, :K], True, None, False, x[:, :K], dx, None, 1)
            torch.cuda.synchronize()
        finally:
            ops.gemm_pairing(old)
        res.append((slab, dx))
    ops.gemm_policy(oldp)
    # same numbers however the two problems were launched (the deep and the
    # 256x128 kernels reduce K in the same order)
    for r in res[1:]:
        assert torch.equal(res[0][0], r[0]) and torch.equal(res[0][1], r[1])
    sl = res[0][0].view(S, N, K + 64).sum(0)
    assert rel_err(sl[:, :K], dy.float().t() @ x[:, :K].float()) < 1e-3
    exp = (dy.float() @ W[:, :K].float()) * (x[:, :K].float() > 0)
    assert rel_err(res[0][1], exp) < 1e-2


@pytest.mark.parametrize("policy", [0, 3, 5])
def test_gemm_batch_pairs_two_wgrads(policy):
    """Two independent weight grads (a multi-rank step's deferred ones) share
    one paired launch, bit-identical to two launches."""
    torch.manual_seed(9)
    M = 4096
    dys = [bf(torch.randn(M, n, device=DEV)) for n in (1024, 512)]
    xs = [bf(torch.randn(M, k, device=DEV)) for k in (512, 1024)]
    oldp = ops.gemm_policy(policy)
    res = []
    for pair in (1, 0):
        old = ops.gemm_pairing(pair)
        try:
            outs = [torch.zeros(dy.shape[1] * x.shape[1], device=DEV) for dy, x in zip(dys, xs)]
            with ops.gemm_batch():
                for dy, x, o in zip(dys, xs, outs):
                    ops.gemm(dy, True, x, True, None, False, None, None, o, 1)
            torch.cuda.synchronize()
        finally:
            ops.gemm_pairing(old)
        res.append(outs)
    ops.gemm_policy(oldp)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
    for dy, x, o in zip(dys, xs, res[0]):
        assert rel_err(o.view(dy.shape[1], x.shape[1]), dy.float().t() @ x.float()) < 1e-3
