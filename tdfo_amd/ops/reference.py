"""Pure-torch fp32 reference implementations of every native op.

These are (a) the CPU execution path of the framework (BASELINE config 1:
DLRM-tiny on CPU through the same engine code) and (b) the numerical oracles
the GPU tests compare the HIP kernels against. Semantics mirror the kernels
exactly, including bf16 rounding of bf16 outputs and the optimizer formulas.
"""
from __future__ import annotations

import math

import torch

EMB_SGD, EMB_ROWWISE_ADAGRAD, EMB_ADAM, EMB_ADAGRAD, EMB_DENSE_GRAD = range(5)
OPT_ADAMW, OPT_ADAM, OPT_SGD, OPT_ADAGRAD = range(4)


def _f(t: torch.Tensor) -> torch.Tensor:
    return t.float()


def gemm(a, a_col, b, b_col, bias=None, relu=False, mask=None, out=None, out32=None, splits=1,
         mul=None, add=None, out2=None, ldc32=0, csum_col=-1):
    A = _f(a).t() if a_col else _f(a)          # [M, K]
    Bm = _f(b) if b_col else _f(b).t()         # [K, N]
    c = A @ Bm
    if bias is not None:
        c = c + bias.float()
    if relu:
        c = c.clamp_min(0)
    if mask is not None:
        c = c * (mask.float() > 0)
    if out is not None:
        out.copy_(c.to(out.dtype))
    if out2 is not None:
        c2 = c * mul.float() if mul is not None else c
        if add is not None:
            c2 = c2 + add.float()
        out2.copy_(c2.to(out2.dtype))
    if out32 is not None:
        M, N = c.shape
        ld = ldc32 or N
        # split-K semantics: slice 0 holds the full sum, other slices zero
        sl = out32.view(-1)[: splits * M * ld].view(splits, M, ld)
        sl[0, :, :N].copy_(c)
        sl[1:, :, :N].zero_()
        if csum_col >= 0:                      # column sums of A (bias grads)
            sl[0, :, csum_col].copy_(A.sum(1))
            sl[1:, :, csum_col].zero_()


def interaction_fwd(dense, emb, off, stride, F, D, out, ones_col=-1):
    B = dense.shape[0]
    rows = [_f(dense[:, :D])]
    flat = emb.reshape(-1)
    ar = torch.arange(B, device=dense.device)
    for i in range(1, F):
        idx = off[i] + ar[:, None] * stride[i] + torch.arange(D, device=dense.device)[None, :]
        rows.append(_f(flat[idx]))
    X = torch.stack(rows, 1)                   # [B, F, D]
    Z = torch.bmm(X, X.transpose(1, 2))
    li, lj = torch.tril_indices(F, F, offset=-1, device=dense.device)
    tri = Z[:, li, lj]
    out.zero_()
    out[:, :D] = dense[:, :D].to(out.dtype)
    out[:, D:D + tri.shape[1]] = tri.to(out.dtype)
    if ones_col >= 0:
        out[:, ones_col] = 1.0


def interaction_bwd(dz, dense, emb, off, stride, F, D, d_dense, d_emb, doff, dstride, relu_mask):
    B = dense.shape[0]
    dev = dense.device
    flat = emb.reshape(-1)
    ar = torch.arange(B, device=dev)
    cols = torch.arange(D, device=dev)
    rows = [_f(dense[:, :D])]
    for i in range(1, F):
        rows.append(_f(flat[off[i] + ar[:, None] * stride[i] + cols[None, :]]))
    X = torch.stack(rows, 1)
    P = F * (F - 1) // 2
    li, lj = torch.tril_indices(F, F, offset=-1, device=dev)
    S = torch.zeros(B, F, F, device=dev)
    g = _f(dz[:, D:D + P])
    S[:, li, lj] = g
    S[:, lj, li] = g
    dX = torch.bmm(S, X)
    dd = dX[:, 0] + _f(dz[:, :D])
    if relu_mask:
        dd = dd * (X[:, 0] > 0)
    d_dense[:, :D] = dd.to(d_dense.dtype)
    dflat = d_emb.reshape(-1)
    for i in range(1, F):
        idx = doff[i] + ar[:, None] * dstride[i] + cols[None, :]
        dflat[idx.reshape(-1)] = dX[:, i].reshape(-1).to(d_emb.dtype)


def embedding_bag_fwd(W, row_offset, indices, offsets, out_off, psw, T, B, mean, out, out_stride):
    D = W.shape[1]
    dev = W.device
    lengths = offsets[1:] - offsets[:-1]
    bag = torch.repeat_interleave(torch.arange(T * B, device=dev), lengths)
    t = bag // B
    rows = row_offset[t] + indices
    vals = W[rows].float()
    if psw is not None:
        vals = vals * psw.float()[:, None]
    pooled = torch.zeros(T * B, D, device=dev)
    pooled.index_add_(0, bag, vals)
    if mean:
        pooled = pooled / lengths.clamp_min(1).float()[:, None]
    tt = torch.arange(T, device=dev).repeat_interleave(B)
    bb = torch.arange(B, device=dev).repeat(T)
    base = bb * out_stride + out_off[tt]
    idx = base[:, None] + torch.arange(D, device=dev)[None, :]
    out.view(-1)[idx.reshape(-1)] = pooled.reshape(-1).to(out.dtype)


def embedding_grad_rows(W, row_offset, indices, offsets, grad_off, psw, T, B, mean, grad, grad_stride):
    """Return (unique global rows [U], summed fp32 grads [U, D])."""
    D = W.shape[1]
    dev = W.device
    lengths = offsets[1:] - offsets[:-1]
    bag = torch.repeat_interleave(torch.arange(T * B, device=dev), lengths)
    t = bag // B
    b = bag - t * B
    keys = row_offset[t] + indices
    base = b * grad_stride + grad_off[t]
    g = grad.reshape(-1)[(base[:, None] + torch.arange(D, device=dev)[None, :]).reshape(-1)]
    g = g.float().view(-1, D)
    scale = torch.ones(keys.shape[0], device=dev)
    if psw is not None:
        scale = scale * psw.float()
    if mean:
        scale = scale / lengths[bag].float()
    g = g * scale[:, None]
    uniq, inv = torch.unique(keys, return_inverse=True)
    acc = torch.zeros(uniq.shape[0], D, device=dev)
    acc.index_add_(0, inv, g)
    return uniq, acc


def embedding_bwd(W, row_offset, indices, offsets, grad_off, psw, T, B, mean, key_bits, grad,
                  grad_stride, opt, state1, state2, hyper, eps, beta1, beta2, weight_decay,
                  dense_grad):
    if hyper.numel() > 3 and float(hyper[3]) > 0:          # dynamic loss scale: skipped step
        return
    rows, g = embedding_grad_rows(W, row_offset, indices, offsets, grad_off, psw, T, B, mean,
                                  grad, grad_stride)
    if rows.numel() == 0:
        return
    if hyper.numel() > 2:
        g = g * float(hyper[2])                             # loss-scale unscale
    lr = float(hyper[0])
    w = W[rows]
    if opt == EMB_SGD:
        w = w - lr * (g + weight_decay * w)
    elif opt == EMB_ROWWISE_ADAGRAD:
        gg = g + weight_decay * w
        st = state1[rows] + (gg * gg).mean(1)
        state1[rows] = st
        w = w - (lr / (st.sqrt() + eps))[:, None] * gg
    elif opt == EMB_ADAGRAD:
        gg = g + weight_decay * w
        st = state1.view(W.shape)[rows] + gg * gg
        state1.view(W.shape)[rows] = st
        w = w - lr * gg / (st.sqrt() + eps)
    elif opt == EMB_ADAM:
        step = float(hyper[1])
        m = state1.view(W.shape)[rows] * beta1 + (1 - beta1) * g
        v = state2.view(W.shape)[rows] * beta2 + (1 - beta2) * g * g
        state1.view(W.shape)[rows] = m
        state2.view(W.shape)[rows] = v
        bc1 = 1 - beta1 ** step
        bc2 = 1 - beta2 ** step
        w = w - lr * ((m / bc1) / ((v / bc2).sqrt() + eps) + weight_decay * w)
    elif opt == EMB_DENSE_GRAD:
        dense_grad.view(W.shape)[rows] += g
        return
    else:
        raise ValueError(f"unknown embedding optimizer {opt}")
    W[rows] = w


def embedding_dense_update(W, grad, rows, opt, state1, state2, hyper, eps, beta1, beta2,
                           weight_decay):
    """Dense step over rows [0, rows) from a dense [rows, D] gradient; rows with
    an all-zero gradient are skipped like the kernel's no-op update (exact for
    SGD / Adagrad / row-wise Adagrad without weight decay)."""
    D = W.shape[1]
    g = grad.reshape(-1)[: rows * D].view(rows, D).float()
    if opt in (EMB_SGD, EMB_ROWWISE_ADAGRAD, EMB_ADAGRAD) and weight_decay == 0.0:
        idx = torch.nonzero(g.abs().sum(1) > 0).view(-1)
    else:
        idx = torch.arange(rows, device=W.device)
    n = int(idx.numel())
    if n == 0:
        return
    z = torch.zeros(1, dtype=torch.int64, device=W.device)
    embedding_bwd(W, z, idx, torch.arange(n + 1, device=W.device), z, None, 1, n, False, 64,
                  g[idx].contiguous(), D, opt, state1, state2, hyper, eps, beta1, beta2,
                  weight_decay, None)


def rw_unpack_meta(meta, nrw):
    m = meta.to(torch.int64)
    return m[:nrw], m[nrw:2 * nrw], m[2 * nrw:3 * nrw], m[3 * nrw:4 * nrw], m[4 * nrw:5 * nrw + 1]


def rw_bucketize(ids, meta, nrw, W, B, cap, n, send, overflow):
    """Reference of the row-wise bucketize (rowwise.hip): stable per-owner
    segments (owner = id mod W, local row = id div W) of packed (bag key << 32
    | owner-local row) entries, the count in slot ``cap`` of each [cap + 1]
    segment, overflow flagged (sticky) in overflow[0], the largest per-owner
    count in overflow[1] (when it has two elements)."""
    dev = ids.device
    in_base, L, blk, lrow, cum = rw_unpack_meta(meta, nrw)
    q = torch.arange(n, device=dev)
    j = torch.searchsorted(cum[1:], q, right=True)
    off = q - cum[j]
    b = off // L[j]
    gid = ids[in_base[j] + off]
    owner = gid % W
    row = lrow[j] + gid // W
    packed = ((j * B + b) << 32) | row
    seg = send.view(W, cap + 1)
    most = 0
    for o in range(W):
        sel = packed[owner == o]
        c = int(sel.numel())
        most = max(most, c)
        if c > cap:
            overflow.view(-1)[0] = 1
            c = cap
        seg[o, :c] = sel[:c]
        seg[o, cap] = c
    if overflow.numel() >= 2:
        overflow.view(-1)[1] = most


def _rw_entries(recv, meta, nrw, W, B, cap, slots=False):
    """(requester, bag key, row key) of every valid received entry (and its
    slot index in the requester's segment with ``slots``)."""
    seg = recv.view(W, cap + 1)
    rs, keys, rows, idx = [], [], [], []
    for r in range(W):
        c = int(seg[r, cap])
        v = seg[r, :c]
        rs.append(torch.full((c,), r, dtype=torch.int64, device=recv.device))
        keys.append(v >> 32)
        rows.append(v & 0xFFFFFFFF)
        idx.append(torch.arange(c, device=recv.device))
    if slots:
        return torch.cat(rs), torch.cat(keys), torch.cat(rows), torch.cat(idx)
    return torch.cat(rs), torch.cat(keys), torch.cat(rows)


def rw_rows_gather(Wt, recv, W, cap, out):
    """Reference of rw_rows_gather (rowwise.hip): the owner's row per received
    entry, [W][cap + 1][D] (slots past a segment's count untouched)."""
    D = Wt.shape[1]
    seg = recv.view(W, cap + 1)
    o = out.view(-1)[: W * (cap + 1) * D].view(W, cap + 1, D)
    for r in range(W):
        c = min(int(seg[r, cap]), cap)
        if c:
            o[r, :c] = Wt[seg[r, :c] & 0xFFFFFFFF].to(out.dtype)


def rw_rows_scatter(send, W, cap, B, D, rows, region, ld, smap, nrw):
    """Reference of rw_rows_scatter: each of this requester's slots (o, i)
    writes its received row to its bag's column block and its offset to the
    slot map (count in slot cap)."""
    seg = send.view(W, cap + 1)
    R = rows.view(-1)[: W * (cap + 1) * D].view(W, cap + 1, D)
    m = smap.view(-1)[: W * (cap + 1)].view(W, cap + 1)
    reg = region.view(-1)
    ar = torch.arange(D, device=send.device)
    for o in range(W):
        c = min(int(seg[o, cap]), cap)
        m[o, cap] = c
        if c:
            k = seg[o, :c] >> 32
            off = (k % B) * ld + (k // B) * D
            m[o, :c] = off.to(torch.int32)
            reg[(off[:, None] + ar).reshape(-1)] = R[o, :c].reshape(-1).to(reg.dtype)


def rw_grads_gather(smap, W, cap, D, dregion, gsend):
    """Reference of rw_grads_gather: gradient rows of the slots in the map."""
    m = smap.view(-1)[: W * (cap + 1)].view(W, cap + 1)
    G = gsend.view(-1)[: W * (cap + 1) * D].view(W, cap + 1, D)
    reg = dregion.reshape(-1)
    ar = torch.arange(D, device=smap.device)
    for o in range(W):
        c = int(m[o, cap])
        if c:
            off = m[o, :c].long()
            G[o, :c] = reg[(off[:, None] + ar).reshape(-1)].view(c, D).to(G.dtype)


def rw_pool(Wt, recv, meta, nrw, W, B, cap, mean, out, out_ld):
    D = Wt.shape[1]
    _, L, _, _, _ = rw_unpack_meta(meta, nrw)
    r, k, row = _rw_entries(recv, meta, nrw, W, B, cap)
    j, b = k // B, k % B
    acc = torch.zeros(W * B * nrw, D, device=Wt.device)
    vals = Wt[row].float()
    if mean:
        vals = vals / L[j].float()[:, None]
    acc.index_add_(0, (r * B + b) * nrw + j, vals)
    o = out.view(-1)[: W * B * out_ld].view(W * B, out_ld)
    o[:, : nrw * D] = acc.view(W * B, nrw * D).to(out.dtype)


def rw_embedding_bwd(Wt, recv, meta, nrw, W, B, cap, mean, grad, grad_ld, opt, state1, state2,
                     hyper, eps, beta1, beta2, weight_decay, rows=False):
    """Owner-side fused backward of the row-wise exchange: every received
    entry (r, (j, b), row) takes gradient row grad[(r*B + b)*grad_ld + j*D:]
    (``rows``: the row of its slot, grad[(r*(cap + 1) + i)*grad_ld:])."""
    D = Wt.shape[1]
    _, L, _, _, _ = rw_unpack_meta(meta, nrw)
    r, k, row, i = _rw_entries(recv, meta, nrw, W, B, cap, slots=True)
    n = int(row.numel())
    if n == 0:
        return
    j, b = k // B, k % B
    base = (r * (cap + 1) + i) * grad_ld if rows else (r * B + b) * grad_ld + j * D
    g = grad.reshape(-1)[(base[:, None] + torch.arange(D, device=Wt.device)).reshape(-1)]
    g = g.float().view(n, D).contiguous()
    psw = (1.0 / L[j].float()) if mean else None
    z = torch.zeros(1, dtype=torch.int64, device=Wt.device)
    embedding_bwd(Wt, z, row, torch.arange(n + 1, device=Wt.device), z, psw, 1, n, False, 64,
                  g, D, opt, state1, state2, hyper, eps, beta1, beta2, weight_decay, None)


def dense_optimizer(p, g, m, v, p_bf16, opt, hyper, beta1, beta2, eps, wd, momentum, found_inf):
    if found_inf is not None and float(found_inf.reshape(-1)[0]) > 0:
        return
    lr, step, gs = (float(x) for x in hyper[:3])
    gg = g * gs
    if opt in (OPT_ADAMW, OPT_ADAM):
        if opt == OPT_ADAM:
            gg = gg + wd * p
        else:
            p.mul_(1 - lr * wd)
        m.mul_(beta1).add_(gg, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(gg, gg, value=1 - beta2)
        bc1 = 1 - beta1 ** step
        bc2 = 1 - beta2 ** step
        p.sub_(lr * (m / bc1) / ((v / bc2).sqrt() + eps))
    elif opt == OPT_SGD:
        gg = gg + wd * p
        if momentum != 0:
            if step > 1:
                m.mul_(momentum).add_(gg)
            else:
                m.copy_(gg)
            gg = m
        p.sub_(lr * gg)
    elif opt == OPT_ADAGRAD:
        gg = gg + wd * p
        m.addcmul_(gg, gg)
        p.sub_(lr * gg / (m.sqrt() + eps))
    else:
        raise ValueError(opt)
    if p_bf16 is not None:
        p_bf16.copy_(p.to(torch.bfloat16))


def check_finite(g, found):
    if not torch.isfinite(g).all():
        found.fill_(1.0)


def head_parts(B: int) -> int:
    return (B + 15) // 16


def head_bce(H, w, b, label, inv_n, relu_mask, logits, dH, part):
    h = _f(H)
    x = h @ w.float() + b.float()
    y = label.float()
    logits.copy_(x)
    loss = x.clamp_min(0) - x * y + torch.log1p(torch.exp(-x.abs()))
    g = (torch.sigmoid(x) - y) * inv_n
    dh = g[:, None] * w.float()[None, :]
    if relu_mask:
        dh = dh * (h > 0)
    dH.copy_(dh.to(dH.dtype))
    K = h.shape[1]
    part.view(-1)[: part.numel()].zero_()
    pv = part.view(-1)[: K + 2]
    pv[:K] = (g[:, None] * h).sum(0)
    pv[K] = g.sum()
    pv[K + 1] = loss.sum()


def reduce_rows(inp, rows, n, ld, out, accumulate, scale):
    flat = inp.reshape(-1)
    s = torch.zeros(n, device=inp.device)
    for r in range(rows):
        s += flat[r * ld: r * ld + n]
    s *= scale
    o = out.view(-1)[:n]
    if accumulate:
        o += s
    else:
        o.copy_(s)


def head_reduce(part, nparts, K, grad, loss_acc, bumps=()):
    p = part[: nparts * (K + 2)].view(nparts, K + 2)
    grad[: K + 1].copy_(p[:, : K + 1].sum(0))
    loss_acc[:1] += p[:, K + 1].sum()
    for b in bumps:
        b[1:2] += 1.0


def colsum(x, out, accumulate):
    s = _f(x).sum(0)
    if accumulate:
        out += s
    else:
        out.copy_(s)


def auc_hist(logits, labels, nb, hist):
    p = torch.sigmoid(logits.float())
    bkt = (p * nb).long().clamp(0, nb - 1)
    pos = labels.float() > 0.5
    hist[:nb] += torch.bincount(bkt[~pos], minlength=nb)
    hist[nb:] += torch.bincount(bkt[pos], minlength=nb)


def cast_bf16(x, y):
    y.copy_(x.to(torch.bfloat16))


def exact_auc(scores: torch.Tensor, labels: torch.Tensor) -> float:
    """Rank-based (Mann-Whitney) ROC-AUC with tie handling."""
    s = scores.double().cpu()
    y = labels.double().cpu() > 0.5
    n_pos = int(y.sum())
    n_neg = y.numel() - n_pos
    if n_pos == 0 or n_neg == 0:
        return float("nan")
    order = torch.argsort(s)
    ranks = torch.empty_like(s)
    ranks[order] = torch.arange(1, s.numel() + 1, dtype=torch.float64)
    # average ranks for ties
    uniq, inv, counts = torch.unique(s, return_inverse=True, return_counts=True)
    sums = torch.zeros(uniq.numel(), dtype=torch.float64).index_add_(0, inv, ranks)
    ranks = (sums / counts)[inv]
    return float((ranks[y].sum() - n_pos * (n_pos + 1) / 2) / (n_pos * n_neg))


def hist_auc(hist: torch.Tensor) -> float:
    """AUC from a [neg | pos] bucket histogram (trapezoid over thresholds)."""
    h = hist.double().cpu()
    nb = h.numel() // 2
    neg, pos = h[:nb], h[nb:]
    tp = torch.cat([pos.flip(0).cumsum(0), pos.new_zeros(0)])
    fp = neg.flip(0).cumsum(0)
    P, N = pos.sum(), neg.sum()
    if P == 0 or N == 0:
        return float("nan")
    tpr = torch.cat([torch.zeros(1, dtype=torch.float64), tp / P])
    fpr = torch.cat([torch.zeros(1, dtype=torch.float64), fp / N])
    return float(torch.trapz(tpr, fpr))


def key_bits_for(rows: int) -> int:
    return max(1, math.ceil(math.log2(max(2, rows))))


def _gather_slots(emb, off, stride, F, D, B, dev):
    flat = emb.reshape(-1)
    ar = torch.arange(B, device=dev)
    cols = torch.arange(D, device=dev)
    return [flat[off[i] + ar[:, None] * stride[i] + cols[None, :]] for i in range(1, F)]


def concat_features(dense, emb, off, stride, F, D, out):
    B = dense.shape[0]
    parts = [dense[:, :D]] + _gather_slots(emb, off, stride, F, D, B, dense.device)
    out.view(B, F * D).copy_(torch.cat([p.to(out.dtype) for p in parts], 1))


def split_features(dx, F, D, dense, d_dense, d_emb, doff, dstride, relu_mask):
    B = dense.shape[0]
    x = dx[:, :F * D].reshape(B, F, D) if dx.dim() == 2 else dx.reshape(B, F, D)
    d0 = x[:, 0].float()
    if relu_mask:
        d0 = d0 * (dense[:, :D].float() > 0)
    d_dense[:, :D] = d0.to(d_dense.dtype)
    dflat = d_emb.reshape(-1)
    ar = torch.arange(B, device=dx.device)
    cols = torch.arange(D, device=dx.device)
    for i in range(1, F):
        idx = doff[i] + ar[:, None] * dstride[i] + cols[None, :]
        dflat[idx.reshape(-1)] = x[:, i].reshape(-1).to(d_emb.dtype)


def cross_bwd(dout, x0, y, dy, dx0, accumulate, add_dout=False):
    a = dout.float()
    dy.copy_((a * x0.float()).to(dy.dtype))
    base = dx0.float() if accumulate else torch.zeros_like(a)
    res = base + a * y.float()
    if add_dout:
        res = res + a
    dx0.copy_(res.to(dx0.dtype))


TT_NPARAM = 2400
TT_PART_LD = 2432
TT_SPB = 16          # samples per kernel block (two_tower.hip SPB)


def two_tower_unpack(P):
    """Flat TwoTower params -> dict of Flax-convention tensors (kernel [in, out])."""
    E = 16
    o = 0
    out = {}
    for name, rows in (("user_fc1", 16), ("user_fc2", 16), ("item_fc1", 98), ("item_fc2", 16)):
        out[name + ".kernel"] = P[o: o + rows * E].view(rows, E)
        o += rows * E
        out[name + ".bias"] = P[o: o + E]
        o += E
    return out


def two_tower_forward(X, P):
    """fp32 forward of the towers (jax-flax/models.py:72-102). X [B, >=114]."""
    p = two_tower_unpack(P)
    xu, xi = X[:, :16], X[:, 16:114]
    hu = xu @ p["user_fc1.kernel"] + p["user_fc1.bias"]
    u = torch.nn.functional.silu(hu) @ p["user_fc2.kernel"] + p["user_fc2.bias"]
    hi = xi @ p["item_fc1.kernel"] + p["item_fc1.bias"]
    iv = torch.nn.functional.silu(hi) @ p["item_fc2.kernel"] + p["item_fc2.bias"]
    return (u * iv).sum(1)


def two_tower(X, P, labels, inv_n, logits, dX=None, part=None, loss_scale=None, half=False):
    """Oracle of tdfo::two_tower via autograd. part rows follow the kernel:
    one row per TT_SPB-sample block, [dP | loss_sum]. ``half``: the towers run
    in float16 (autograd through fp16 ops); ``loss_scale`` scales the loss."""
    dt = torch.float16 if half else torch.float32
    if dX is None:
        with torch.no_grad():
            logits.copy_(two_tower_forward(X.float().to(dt), P.float().to(dt)).float())
        return
    B = X.shape[0]
    ls = float(loss_scale.reshape(-1)[0]) if loss_scale is not None else 1.0
    with torch.enable_grad():
        Xr = X[:, :114].detach().float().clone().requires_grad_(True)
        Pr = P[:TT_NPARAM].detach().float().clone().requires_grad_(True)
        lg = two_tower_forward(Xr.to(dt), Pr.to(dt)).float()
        y = labels.float()
        per = torch.nn.functional.binary_cross_entropy_with_logits(lg, y, reduction="none")
        (per.sum() * (inv_n * ls)).backward()
    logits.copy_(lg.detach())
    dX[:, :112].copy_(Xr.grad[:, :112])
    nparts = (B + TT_SPB - 1) // TT_SPB
    pv = part.view(-1)[: nparts * TT_PART_LD].view(nparts, TT_PART_LD)
    pv.zero_()
    pv[0, :TT_NPARAM] = Pr.grad
    pv[0, TT_NPARAM] = per.detach().sum()


def linear_xent(H, W, bias, labels, eps, ignore, dH, lossv, dW=None, db=None):
    """Oracle: logits = H W^T + b; CrossEntropy(ignore_index, label_smoothing)
    mean over non-ignored tokens; per-token loss in lossv, grads of the mean."""
    with torch.enable_grad():
        Hr = H.detach().float().clone().requires_grad_(True)
        Wr = W.detach().float().clone().requires_grad_(True)
        br = bias.detach().float().clone().requires_grad_(True)
        logits = Hr @ Wr.t() + br
        per = torch.nn.functional.cross_entropy(logits, labels, ignore_index=ignore,
                                                label_smoothing=eps, reduction="none")
        nv = max(1, int((labels != ignore).sum()))
        (per.sum() / nv).backward()
    lossv.copy_(per.detach())
    dH.copy_(Hr.grad)
    if dW is not None:
        dW.copy_(Wr.grad)
        db.copy_(br.grad)


def _bag_positions(offsets, T):
    lens = (offsets[1:] - offsets[:-1])
    B = lens.numel()
    nnz = int(offsets[-1])
    bag = torch.repeat_interleave(torch.arange(B, device=offsets.device), lens)
    pos = torch.arange(nnz, device=offsets.device) - offsets[:-1][bag]
    return bag, pos


def jagged_to_dense(values, offsets, T, pad, out):
    out.fill_(pad)
    bag, pos = _bag_positions(offsets, T)
    keep = pos < T
    out[bag[keep], pos[keep]] = values[keep].to(out.dtype)


def dense_to_jagged(dense, offsets, vgrad):
    T = dense.shape[1]
    bag, pos = _bag_positions(offsets, T)
    vgrad.zero_()
    keep = pos < T
    vgrad[keep] = dense[bag[keep], pos[keep]]


def jagged_ids_to_dense(values, offsets, pad, out):
    T = out.shape[1]
    out.fill_(pad)
    bag, pos = _bag_positions(offsets, T)
    keep = pos < T
    out[bag[keep], pos[keep]] = values[keep]


# ------------------------------------------------ Bert4Rec attention / LN
_M32 = 0xFFFFFFFF


def _hash3(a, b, c):
    """Same counter hash as csrc/kernels/attention.hip (uint32 arithmetic in int64)."""
    h = ((a * 0x9E3779B1) & _M32) ^ (((b + 0x7F4A7C15) * 0x85EBCA77) & _M32) ^ \
        (((c + 0x165667B1) * 0xC2B2AE3D) & _M32)
    h = h & _M32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    h = h ^ (h >> 16)
    return h


def attn_keep_scale(B: int, H: int, T: int, rate: float, seed: int, step: int, device):
    """[B, H, T, T] dropout multiplier (keep / (1 - rate) or 0) of the fused kernel."""
    if rate <= 0:
        return torch.ones(B, H, T, T, device=device)
    a = (seed ^ ((step * 0x632BE5AB) & _M32)) & _M32
    bh = torch.arange(B * H, dtype=torch.int64, device=device).view(B, H, 1, 1)
    i = torch.arange(T, dtype=torch.int64, device=device).view(1, 1, T, 1)
    j = torch.arange(T, dtype=torch.int64, device=device).view(1, 1, 1, T)
    r = _hash3(torch.full((1,), a, dtype=torch.int64, device=device), bh * 64 + i, j)
    keep = (r >> 8).to(torch.float32) * (1.0 / 16777216.0) >= rate
    return keep.to(torch.float32) / (1.0 - rate)


def attention_core(qkv, ids, H, rate, seed, step, pad_id):
    """Differentiable torch reference of the fused kernel: qkv [B,T,3E] -> [B,T,E]."""
    B, T, E3 = qkv.shape
    E = E3 // 3
    dk = E // H
    q, k, v = qkv.view(B, T, 3, H, dk).permute(2, 0, 3, 1, 4)
    s = (q / math.sqrt(dk)) @ k.transpose(-2, -1)
    mask = (ids != pad_id).view(B, 1, 1, T)
    s = s.masked_fill(~mask, -1e9)
    p = torch.softmax(s, dim=-1) * attn_keep_scale(B, H, T, rate, seed, step, qkv.device)
    return (p @ v).transpose(1, 2).reshape(B, T, E)


def attention_fwd(qkv, ids, H, rate, seed, step, pad_id, out):
    out.copy_(attention_core(qkv, ids, H, rate, seed, int(step[0]) if step is not None else 0,
                             pad_id))


def attention_bwd(qkv, ids, dout, H, rate, seed, step, pad_id, dqkv):
    x = qkv.detach().requires_grad_(True)
    with torch.enable_grad():
        o = attention_core(x, ids, H, rate, seed, int(step[0]) if step is not None else 0,
                           pad_id)
        (g,) = torch.autograd.grad(o, x, dout)
    dqkv.copy_(g)


def layernorm_fwd(x, n, eps, gamma, beta, y, mean, rstd):
    xv = x.reshape(-1, n)
    mu = xv.mean(1)
    var = xv.var(1, unbiased=False)
    rs = torch.rsqrt(var + eps)
    y.view(-1, n).copy_((xv - mu[:, None]) * rs[:, None] * gamma.view(1, n) + beta.view(1, n))
    mean[: mu.numel()].copy_(mu)
    rstd[: rs.numel()].copy_(rs)


def layernorm_bwd(x, g, n, gamma, mean, rstd, dx, dgb):
    xv, gv = x.reshape(-1, n), g.reshape(-1, n)
    M = xv.shape[0]
    xh = (xv - mean[:M, None]) * rstd[:M, None]
    gg = gv * gamma.view(1, n)
    dxv = rstd[:M, None] * (gg - gg.mean(1, keepdim=True) - xh * (gg * xh).mean(1, keepdim=True))
    dx.view(-1, n).copy_(dxv)
    dgb[:n].copy_((gv * xh).sum(0))
    dgb[n:].copy_(gv.sum(0))


def rank_metrics(h, W, bias, cand, ks, out):
    wr = W[cand]                                                    # [B, C, E]
    scores = (wr * h[:, None, :]).sum(-1) + bias[cand]
    rank = (scores[:, 1:] >= scores[:, :1]).sum(1)
    rec = [(rank < k).float().sum() for k in ks]
    g = 1.0 / torch.log2(rank.float() + 2.0)
    ndcg = [torch.where(rank < k, g, torch.zeros_like(g)).sum() for k in ks]
    out.copy_(torch.stack(rec + ndcg + [torch.tensor(float(h.shape[0]), device=h.device)]))


def seq_prologue_mul(M: int, n: int, rate: float, seed: int, step: int, device):
    """[M, n] dropout multiplier of the fused sequence prologue
    (csrc/kernels/layernorm.hip::pro_mul)."""
    if rate <= 0:
        return torch.ones(M, n, device=device)
    sd = ((seed & _M32) ^ ((step * 0x632BE5AB) & _M32) ^ 0x51ED270B) & _M32
    r = _hash3(torch.full((1,), sd, dtype=torch.int64, device=device),
               torch.arange(M, dtype=torch.int64, device=device).view(M, 1),
               torch.arange(n, dtype=torch.int64, device=device).view(1, n))
    keep = (r >> 8).to(torch.float32) * (1.0 / 16777216.0) >= rate
    return keep.to(torch.float32) / (1.0 - rate)


def seq_prologue_fwd(x, pos, n, eps, gamma, beta, rate, seed, step, y, mean, rstd):
    v = x.reshape(-1, n) + pos.reshape(1, n)
    M = v.shape[0]
    mu = v.mean(1)
    rs = torch.rsqrt(v.var(1, unbiased=False) + eps)
    o = (v - mu[:, None]) * rs[:, None] * gamma.view(1, n) + beta.view(1, n)
    st = int(step.reshape(-1)[0]) if step is not None else 0
    y.view(-1, n).copy_(o * seq_prologue_mul(M, n, rate, seed, st, x.device))
    mean[:M].copy_(mu)
    rstd[:M].copy_(rs)


def seq_prologue_bwd(x, pos, g, n, gamma, mean, rstd, rate, seed, step, dx, out3):
    v = x.reshape(-1, n) + pos.reshape(1, n)
    M = v.shape[0]
    st = int(step.reshape(-1)[0]) if step is not None else 0
    gv = g.reshape(-1, n) * seq_prologue_mul(M, n, rate, seed, st, x.device)
    xh = (v - mean[:M, None]) * rstd[:M, None]
    gg = gv * gamma.view(1, n)
    dxv = rstd[:M, None] * (gg - gg.mean(1, keepdim=True) - xh * (gg * xh).mean(1, keepdim=True))
    dx.view(-1, n).copy_(dxv)
    out3[:n].copy_((gv * xh).sum(0))
    out3[n:2 * n].copy_(gv.sum(0))
    out3[2 * n:].copy_(dxv.sum(0))


# ------------------------------------------------------------ encoder layer
ENC_SITE_A, ENC_SITE_F, ENC_SITE_G, ENC_SITE_BLK = 1, 2, 3, 4


def enc_site_mul(B: int, T: int, N: int, rate: float, seed: int, step: int, site: int, device):
    """[B, T, N] dropout multiplier of sublayer site ``site`` in the fused
    encoder-layer kernel (csrc/kernels/encoder.hip::site_mul)."""
    if rate <= 0:
        return torch.ones(B, T, N, device=device)
    sd = (seed ^ ((step * 0x632BE5AB) & _M32)) & _M32
    a = (sd ^ ((site * 0x27D4EB2F) & _M32)) & _M32
    bt = (torch.arange(B, dtype=torch.int64, device=device).view(B, 1, 1) * 64 +
          torch.arange(T, dtype=torch.int64, device=device).view(1, T, 1))
    n = torch.arange(N, dtype=torch.int64, device=device).view(1, 1, N)
    r = _hash3(torch.full((1,), a, dtype=torch.int64, device=device), bt, n)
    keep = (r >> 8).to(torch.float32) * (1.0 / 16777216.0) >= rate
    return keep.to(torch.float32) / (1.0 - rate)


def encoder_layer(x, ids, params, H, rate, seed, step, pad_id=0, eps=1e-5):
    """Differentiable torch reference of the fused pre-norm transformer block
    (same math and dropout masks as csrc/kernels/encoder.hip)."""
    if len(params) == 16:                 # Q / K / V weights and biases as separate tensors
        params = ([torch.cat(params[0:3], 0), torch.cat(params[3:6], 0)] + list(params[6:]))
    wqkv, bqkv, wo, bo, g1, be1, g2, be2, w1, b1, w2, b2 = params
    B, T, E = x.shape
    dev = x.device
    m = lambda site, N: enc_site_mul(B, T, N, rate, seed, step, site, dev)  # noqa: E731
    h1 = torch.nn.functional.layer_norm(x, (E,), g1, be1, eps)
    qkv = h1 @ wqkv.t() + bqkv
    ctx = attention_core(qkv, ids, H, rate, seed, step, pad_id)
    x1 = x + (ctx @ wo.t() + bo) * m(ENC_SITE_A, E)
    h2 = torch.nn.functional.layer_norm(x1, (E,), g2, be2, eps)
    f = torch.relu(h2 @ w1.t() + b1) * m(ENC_SITE_F, w1.shape[0])
    x2 = x1 + (f @ w2.t() + b2) * m(ENC_SITE_G, E)
    return x2 * m(ENC_SITE_BLK, E)


