"""Row-wise sharding kernels (csrc/kernels/rowwise.hip + the RW owner backward
in embedding.hip) vs the torch references in tdfo_amd.ops.reference.

One process plays every rank: the kernels never communicate (the exchange is
an RCCL all-to-all of the [W][cap+1] buffers), so bucketize at world W, the
owner-side pooling of a [W][cap+1] receive buffer and the owner backward are
all checked at W = 1..8 on one GPU.
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


def make_meta(rows, L, B, W):
    """meta of an engine whose rw tables are ``rows`` (pooling L), ids laid
    out table-major in the input, owner-local stores of ceil(rows/W) rows."""
    nrw = len(rows)
    in_base, acc = [], 0
    for j in range(nrw):
        in_base.append(acc)
        acc += B * L[j]
    blk = [-(-r // W) for r in rows]
    lrow, a = [], 0
    for b_ in blk:
        lrow.append(a)
        a += b_
    cum = [0]
    for j in range(nrw):
        cum.append(cum[-1] + B * L[j])
    meta = torch.tensor(in_base + list(L) + blk + lrow + cum, dtype=torch.int64)
    return meta, cum[-1], a


def rand_ids(rows, L, B, g, dev):
    return torch.cat([torch.randint(0, r, (B * l_,), generator=g) for r, l_ in zip(rows, L)]).to(dev)


@pytest.mark.parametrize("W", [1, 2, 3, 8])
@pytest.mark.parametrize("rows,L,B", [([1000, 37, 50000], [1, 3, 2], 257),
                                      ([40000] * 4, [1, 1, 1, 1], 4096),
                                      ([9999, 123456], [7, 100], 64)])
def test_rw_bucketize_matches_reference(W, rows, L, B):
    g = torch.Generator().manual_seed(W * 7 + B)
    ids = rand_ids(rows, L, B, g, DEV)
    meta, n, _ = make_meta(rows, L, B, W)
    meta = meta.to(DEV)
    cap = n
    send = torch.full((W * (cap + 1),), -7, dtype=torch.int64, device=DEV)
    ws = torch.empty(ops.rw_bucketize_workspace(n, W), dtype=torch.uint8, device=DEV)
    ovf = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.rw_bucketize(ids, meta, len(rows), W, B, cap, n, send, ws, ovf)
    exp = torch.full_like(send, -7).cpu()
    eovf = torch.zeros(1, dtype=torch.int32)
    ref.rw_bucketize(ids.cpu(), meta.cpu(), len(rows), W, B, cap, n, exp, eovf)
    got = send.cpu().view(W, cap + 1)
    exp = exp.view(W, cap + 1)
    assert int(ovf) == 0
    assert torch.equal(got[:, cap], exp[:, cap])
    for o in range(W):
        c = int(exp[o, cap])
        assert torch.equal(got[o, :c], exp[o, :c]), o      # stable: exact order


def test_rw_bucketize_overflow_flag():
    rows, L, B, W = [1000], [4], 512, 4
    g = torch.Generator().manual_seed(0)
    ids = torch.zeros(B * 4, dtype=torch.int64, device=DEV)     # every id owned by rank 0
    ids[::2] = torch.randint(0, 250, (B * 2,), generator=g).to(DEV)
    meta, n, _ = make_meta(rows, L, B, W)
    cap = 600                                                     # < n ids for owner 0
    send = torch.zeros(W * (cap + 1), dtype=torch.int64, device=DEV)
    ws = torch.empty(ops.rw_bucketize_workspace(n, W), dtype=torch.uint8, device=DEV)
    ovf = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.rw_bucketize(ids, meta.to(DEV), 1, W, B, cap, n, send, ws, ovf)
    assert int(ovf) == 1
    seg = send.view(W, cap + 1).cpu()
    assert int(seg[0, cap]) == cap                               # clamped count, no OOB write
    exp = torch.zeros_like(seg).view(-1)
    ref.rw_bucketize(ids.cpu(), meta, 1, W, B, cap, n, exp, torch.zeros(1, dtype=torch.int32))
    assert torch.equal(seg[0, :cap], exp.view(W, cap + 1)[0, :cap])


def _recv_from(rows, L, B, W, owner, seed, dev):
    """The receive buffer of ``owner`` after an exchange: every requester's
    segment for this owner (built with the reference bucketize)."""
    meta, n, total = make_meta(rows, L, B, W)
    cap = n
    recv = torch.zeros(W, cap + 1, dtype=torch.int64)
    for r in range(W):
        g = torch.Generator().manual_seed(seed + r)
        ids = rand_ids(rows, L, B, g, "cpu")
        send = torch.zeros(W * (cap + 1), dtype=torch.int64)
        ref.rw_bucketize(ids, meta, len(rows), W, B, cap, n, send, torch.zeros(1, dtype=torch.int32))
        recv[r] = send.view(W, cap + 1)[owner]
    return recv.view(-1).to(dev), meta.to(dev), cap, total


@pytest.mark.parametrize("W", [1, 4])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,L,B,D", [([5000, 300], [1, 4], 128, 128), ([777] * 3, [2, 1, 9], 64, 64)])
def test_rw_pool_matches_reference(W, out_dtype, rows, L, B, D):
    recv, meta, cap, total = _recv_from(rows, L, B, W, owner=W - 1, seed=3, dev=DEV)
    nrw = len(rows)
    Wt = torch.randn(total + 1, D, device=DEV)
    starts = torch.zeros(W * (nrw * B + 1), dtype=torch.int32, device=DEV)
    out = torch.full((W * B * nrw * D,), 5.0, dtype=out_dtype, device=DEV)
    ops.rw_pool(Wt, recv, meta, nrw, W, B, cap, False, starts, out, nrw * D)
    exp = torch.zeros(W * B * nrw * D, dtype=torch.float32)
    ref.rw_pool(Wt.cpu(), recv.cpu(), meta.cpu(), nrw, W, B, cap, False, exp, nrw * D)
    tol = 2e-2 if out_dtype == torch.bfloat16 else 1e-5
    assert torch.allclose(out.float().cpu(), exp, atol=tol, rtol=tol)


@pytest.mark.parametrize("opt", [ops.EMB_ROWWISE_ADAGRAD, ops.EMB_SGD, ops.EMB_ADAM])
@pytest.mark.parametrize("W,mean", [(1, False), (4, False), (3, True)])
def test_rw_owner_backward_matches_reference(opt, W, mean):
    rows, L, B, D = [2000, 50, 30000], [3, 1, 2], 96, 64
    recv, meta, cap, total = _recv_from(rows, L, B, W, owner=0, seed=11, dev=DEV)
    nrw = len(rows)
    g = torch.Generator().manual_seed(5)
    W0 = torch.randn(total + 1, D, generator=g).to(DEV)          # + scratch row
    s1 = s2 = None
    if opt == ops.EMB_ROWWISE_ADAGRAD:
        s1 = torch.rand(total + 1, generator=g).to(DEV)
    elif opt == ops.EMB_ADAM:
        s1 = torch.zeros(total + 1, D, device=DEV)
        s2 = torch.zeros(total + 1, D, device=DEV)
    grad = (torch.randn(W * B * nrw * D, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    hyper = torch.tensor([0.05, 1.0], device=DEV)
    kb = ops.key_bits_for(total + 1)
    Wg = W0.clone()
    sg1 = s1.clone() if s1 is not None else None
    sg2 = s2.clone() if s2 is not None else None
    ws = torch.empty(ops.embedding_bwd_workspace(W * cap, D), dtype=torch.uint8, device=DEV)
    ops.embedding_bwd_prepare_rw(Wg, recv, meta, nrw, W, B, cap, mean, kb, nrw * D, total, ws)
    ops.embedding_bwd_apply_rw(Wg, recv, meta, nrw, W, B, cap, mean, kb, grad, nrw * D, opt, hyper,
                               ws, state1=sg1, state2=sg2)
    We = W0.clone().cpu()
    se1 = s1.clone().cpu() if s1 is not None else None
    se2 = s2.clone().cpu() if s2 is not None else None
    ref.rw_embedding_bwd(We, recv.cpu(), meta.cpu(), nrw, W, B, cap, mean, grad.cpu(), nrw * D,
                         opt, se1, se2, hyper.cpu(), 1e-8, 0.9, 0.999, 0.0)
    # every real row matches; the scratch row (last) is junk by design. Adam's
    # first step is ~lr * sign(g): a row-gradient that cancels to ~0 may flip
    # sign under a different fp32 summation order, so allow a few elements
    diff = (Wg[:total].cpu() - We[:total]).abs() > 1e-5 + 1e-4 * We[:total].abs()
    if opt == ops.EMB_ADAM:
        assert float(diff.float().mean()) < 1e-3, int(diff.sum())
    else:
        assert not bool(diff.any()), int(diff.sum())
    if se1 is not None:
        assert torch.allclose(sg1[:total].cpu(), se1[:total], atol=1e-5, rtol=1e-4)
