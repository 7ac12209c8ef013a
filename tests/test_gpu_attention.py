"""Fused Bert4Rec encoder kernels (attention core, LayerNorm) vs fp32 torch
references of the same ops, on MI355X."""
import math

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


def _mha_reference(qkv, ids, H):
    """The reference model's math (torchrec/models.py:11-28) on [B,T,3E]."""
    B, T, E3 = qkv.shape
    E = E3 // 3
    dk = E // H
    q, k, v = qkv.view(B, T, 3, H, dk).permute(2, 0, 3, 1, 4)
    scores = q @ k.transpose(-2, -1) / math.sqrt(dk)
    mask = (ids != 0).view(B, 1, 1, T).repeat(1, 1, T, 1)
    scores = scores.masked_fill(mask == 0, -1e9)
    p = torch.softmax(scores, dim=-1)
    return (p @ v).transpose(1, 2).reshape(B, T, E)


@pytest.mark.parametrize("B,T,E,H", [(16, 20, 16, 2), (3, 64, 64, 4), (5, 7, 32, 1)])
def test_attention_no_dropout_matches_reference(B, T, E, H):
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3 * E, device=DEV)
    ids = torch.randint(1, 50, (B, T), device=DEV)
    ids[:, : T // 3] = 0                       # left padding
    ids[0] = 0                                 # a fully padded row (uniform softmax)
    out = torch.empty(B, T, E, device=DEV)
    ops.attention_fwd(qkv, ids, H, 0.0, 1, None, 0, out)
    x = qkv.clone().requires_grad_(True)
    exp = _mha_reference(x, ids, H)
    assert torch.allclose(out, exp, atol=1e-5, rtol=1e-4)
    g = torch.randn_like(exp)
    exp.backward(g)
    dqkv = torch.empty_like(qkv)
    ops.attention_bwd(qkv, ids, g, H, 0.0, 1, None, 0, dqkv)
    assert torch.allclose(dqkv, x.grad, atol=1e-4, rtol=1e-3)


def test_attention_dropout_matches_hash_reference():
    torch.manual_seed(1)
    B, T, E, H, rate = 16, 20, 16, 2, 0.1
    qkv = torch.randn(B, T, 3 * E, device=DEV)
    ids = torch.randint(0, 30, (B, T), device=DEV)
    step = torch.tensor([7], dtype=torch.int64, device=DEV)
    out = torch.empty(B, T, E, device=DEV)
    ops.attention_fwd(qkv, ids, H, rate, 123, step, 0, out)
    exp = torch.empty_like(out)
    ref.attention_fwd(qkv, ids, H, rate, 123, step.cpu(), 0, exp)
    assert torch.allclose(out, exp, atol=1e-5, rtol=1e-4)
    g = torch.randn_like(out)
    d = torch.empty_like(qkv)
    ops.attention_bwd(qkv, ids, g, H, rate, 123, step, 0, d)
    e = torch.empty_like(qkv)
    ref.attention_bwd(qkv, ids, g, H, rate, 123, step.cpu(), 0, e)
    assert torch.allclose(d, e, atol=1e-4, rtol=1e-3)
    # a different step draws a different mask
    step2 = torch.tensor([8], dtype=torch.int64, device=DEV)
    out2 = torch.empty_like(out)
    ops.attention_fwd(qkv, ids, H, rate, 123, step2, 0, out2)
    assert not torch.allclose(out, out2)


@pytest.mark.parametrize("M,n", [(320, 16), (16, 320), (1000, 1024), (7, 100)])
def test_layernorm_fwd_bwd(M, n):
    torch.manual_seed(2)
    x = torch.randn(M, n, device=DEV) * 3 + 1
    gamma = torch.randn(n, device=DEV)
    beta = torch.randn(n, device=DEV)
    y = torch.empty_like(x)
    mean = torch.empty(M, device=DEV)
    rstd = torch.empty(M, device=DEV)
    ops.layernorm_fwd(x, n, 1e-5, gamma, beta, y, mean, rstd)
    xr = x.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    exp = torch.nn.functional.layer_norm(xr, (n,), gr, br, 1e-5)
    assert torch.allclose(y, exp, atol=1e-4, rtol=1e-4)
    g = torch.randn_like(x)
    exp.backward(g)
    dx = torch.empty_like(x)
    part = torch.empty(ops.layernorm_parts(M) * 2 * n, device=DEV)
    dgb = torch.empty(2 * n, device=DEV)
    ops.layernorm_bwd(x, g, n, gamma, mean, rstd, dx, part, dgb)
    assert torch.allclose(dx, xr.grad, atol=1e-4, rtol=1e-3)
    assert torch.allclose(dgb[:n], gr.grad, atol=1e-3, rtol=1e-3)
    assert torch.allclose(dgb[n:], br.grad, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("M,n,rate", [(512, 320, 0.0), (512, 320, 0.1), (37, 100, 0.3)])
def test_seq_prologue_fwd_bwd(M, n, rate):
    """Fused dropout(LN(x + pos)): kernel vs the fp32 reference (same hash mask)
    and, at rate 0, vs torch autograd of the unfused ops."""
    from tdfo_amd.ops import reference as ref

    torch.manual_seed(4)
    x = torch.randn(M, n, device=DEV) * 2 + 0.5
    pos = torch.randn(n, device=DEV)
    gamma, beta = torch.randn(n, device=DEV), torch.randn(n, device=DEV)
    step = torch.tensor([7], dtype=torch.int64, device=DEV)
    y, mean, rstd = torch.empty_like(x), torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ops.seq_prologue_fwd(x, pos, n, 1e-5, gamma, beta, rate, 1234, step, y, mean, rstd)
    ey, em, er = torch.empty_like(x), torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ref.seq_prologue_fwd(x, pos, n, 1e-5, gamma, beta, rate, 1234, step, ey, em, er)
    assert torch.allclose(y, ey, atol=1e-4, rtol=1e-4)
    g = torch.randn_like(x)
    dx = torch.empty_like(x)
    part = torch.empty(ops.layernorm_parts(M) * 3 * n, device=DEV)
    out3 = torch.empty(3 * n, device=DEV)
    ops.seq_prologue_bwd(x, pos, g, n, gamma, mean, rstd, rate, 1234, step, dx, part, out3)
    edx, eo3 = torch.empty_like(x), torch.empty(3 * n, device=DEV)
    ref.seq_prologue_bwd(x, pos, g, n, gamma, em, er, rate, 1234, step, edx, eo3)
    assert torch.allclose(dx, edx, atol=1e-4, rtol=1e-3)
    assert torch.allclose(out3, eo3, atol=2e-3, rtol=1e-3)
    if rate > 0:
        assert 0.0 < float((y == 0).float().mean()) < 2 * rate
        return
    xr, pr = x.clone().requires_grad_(True), pos.clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    e = torch.nn.functional.layer_norm(xr + pr, (n,), gr, br, 1e-5)
    e.backward(g)
    assert torch.allclose(dx, xr.grad, atol=1e-4, rtol=1e-3)
    assert torch.allclose(out3[:n], gr.grad, atol=2e-3, rtol=1e-3)
    assert torch.allclose(out3[n:2 * n], br.grad, atol=2e-3, rtol=1e-3)
    assert torch.allclose(out3[2 * n:], pr.grad, atol=2e-3, rtol=1e-3)


def test_bert4rec_fused_encoder_matches_torch_path():
    """Whole encoder fwd+bwd: fused HIP path vs the torch reference path (dropout 0)."""
    from tdfo_amd.models import bert4rec as m

    torch.manual_seed(3)
    model = m.Bert4Rec(1000, 20, 16, 2, 2, dropout=0.0).to(DEV)
    seqs = torch.randint(0, 1000, (16, 20), device=DEV)
    seqs[:, :5] = 0
    emb = torch.randn(16, 20, 16, device=DEV, requires_grad=True)
    grads = []
    outs = []
    for fused in (True, False):
        m.USE_FUSED = fused
        model.zero_grad()
        emb.grad = None
        h = model.encode(emb, seqs)
        h.square().sum().backward()
        outs.append(h.detach())
        grads.append([emb.grad.clone()] + [p.grad.clone() for p in model.parameters()
                                           if p.grad is not None])
    m.USE_FUSED = True
    assert torch.allclose(outs[0], outs[1], atol=1e-4, rtol=1e-4)
    for a, b in zip(grads[0], grads[1]):
        assert torch.allclose(a, b, atol=1e-3, rtol=1e-3)


def _enc_params(E, FF, dev, g):
    def r(*s, sc=0.3):
        return (torch.randn(*s, generator=g) * sc).to(dev)
    return [r(3 * E, E), r(3 * E, sc=0.1), r(E, E), r(E, sc=0.1), 1 + r(E, sc=0.1), r(E, sc=0.1),
            1 + r(E, sc=0.1), r(E, sc=0.1), r(FF, E), r(FF, sc=0.1), r(E, FF), r(E, sc=0.1)]


def test_fused_encoder_layer_separate_qkv_matches_concatenated():
    """The block with Q / K / V weights and biases as 16 separate tensors
    (what the Bert4Rec trainer passes: no per-step concatenation) equals the
    12-tensor form with [W_qkv] / [b_qkv] concatenated, bit for bit."""
    from tdfo_amd.models import bert4rec as m

    B, T, E, H = 16, 20, 16, 2
    g = torch.Generator().manual_seed(7)
    params = _enc_params(E, 4 * E, DEV, g)
    x = torch.randn(B, T, E, generator=g).to(DEV)
    ids = torch.randint(1, 50, (B, T), generator=g).to(DEV)
    step = torch.tensor([3], dtype=torch.int64, device=DEV)
    dy = torch.randn(B, T, E, generator=g).to(DEV)
    outs = []
    for sep in (False, True):
        xa = x.clone().requires_grad_(True)
        if sep:
            ps = (list(params[0].split(E, 0)) + list(params[1].split(E, 0)) + list(params[2:]))
        else:
            ps = list(params)
        pa = [p.clone().contiguous().requires_grad_(True) for p in ps]
        y = m._EncoderLayerFn.apply(xa, ids, step, H, 0.1, 0x5EED, 1e-5, None, *pa)
        y.backward(dy)
        grads = [p.grad for p in pa]
        if sep:
            grads = [torch.cat(grads[0:3], 0), torch.cat(grads[3:6], 0)] + grads[6:]
        outs.append((y.detach(), xa.grad, grads))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    for a, b in zip(outs[0][2], outs[1][2]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,T,E,H,rate", [(16, 20, 16, 2, 0.1), (16, 20, 16, 2, 0.0),
                                          (3, 24, 32, 4, 0.1), (5, 7, 16, 1, 0.2)])
def test_fused_encoder_layer_matches_reference(B, T, E, H, rate):
    """Whole transformer block (encoder.hip) fwd + bwd vs the torch reference
    with the same hash dropout masks."""
    from tdfo_amd.models import bert4rec as m

    g = torch.Generator().manual_seed(B * 100 + T)
    FF = 4 * E
    params = _enc_params(E, FF, DEV, g)
    x = torch.randn(B, T, E, generator=g).to(DEV)
    ids = torch.randint(1, 50, (B, T), generator=g).to(DEV)
    ids[:, : T // 4] = 0
    ids[0] = 0
    step = torch.tensor([5], dtype=torch.int64, device=DEV)
    seed = 0x5EED + 7919
    xa = x.clone().requires_grad_(True)
    pa = [p.clone().requires_grad_(True) for p in params]
    y = m._EncoderLayerFn.apply(xa, ids, step, H, rate, seed, 1e-5, None, *pa)
    xr = x.clone().requires_grad_(True)
    pr = [p.clone().requires_grad_(True) for p in params]
    yr = ref.encoder_layer(xr, ids, pr, H, rate, seed, 5, 0, 1e-5)
    assert torch.allclose(y, yr, atol=1e-4, rtol=1e-4), (y - yr).abs().max()
    dy = torch.randn(B, T, E, generator=g).to(DEV)
    y.backward(dy)
    yr.backward(dy)
    assert torch.allclose(xa.grad, xr.grad, atol=2e-4, rtol=1e-3), (xa.grad - xr.grad).abs().max()
    for i, (a, b) in enumerate(zip(pa, pr)):
        err = float((a.grad - b.grad).abs().max() / (b.grad.abs().max() + 1e-6))
        assert err < 1e-4, (i, err)
