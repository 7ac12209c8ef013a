"""Bert4Rec: ETL transforms, fused linear+xent oracle,
metrics, trainer, checkpoint layout, DDP/DMP over gloo."""
import math

import numpy as np
import pytest
import torch

from tdfo_amd import ops
from tdfo_amd.data import bert4rec_etl as E
from tdfo_amd.models.bert4rec import (METRIC_NAMES, Bert4RecTrainer, linear_cross_entropy,
                                      recall_ndcg_sums)
from tdfo_amd.utils.checkpoint import bert4rec_ckpt_name, load_state_dict, save_state_dict
from tests.dist_harness import run_distributed


def test_sliding_windows_match_reference_padding():
    seq = np.arange(1, 26)
    _, w = E.sliding_windows(seq, np.array([25]), 20, 10)
    assert w.shape == (3, 20)
    assert w[0].tolist() == list(range(1, 21))
    assert w[1].tolist() == list(range(11, 26)) + [0] * 5
    assert w[2].tolist() == list(range(21, 26)) + [0] * 15
    # two users, lengths 10 and 11 (reference _get_pad_size semantics)
    u, w = E.sliding_windows(np.arange(1, 22), np.array([10, 11]), 20, 10)
    assert u.tolist() == [0, 1, 1]
    assert w[0].tolist() == list(range(1, 11)) + [0] * 10
    assert w[2].tolist() == [21] + [0] * 19


def test_masking_last_item_always_masked():
    rng = np.random.default_rng(0)
    b = np.arange(1, 31, dtype=np.int32)
    starts, lens = np.array([0, 10]), np.array([8, 18])
    masked, labels = E.mask_train(b, starts, lens, 0.2, 99, rng)
    assert len(masked) == 26
    assert masked[7] == 99 and masked[25] == 99          # last items
    assert ((masked == 99) == (labels != 0)).all()
    items = np.concatenate([b[0:8], b[10:28]])
    assert (labels[labels != 0] == items[labels != 0]).all()


def test_eval_seqs_and_negatives():
    b = np.arange(1, 41, dtype=np.int32)
    starts, train_len = np.array([0, 20]), np.array([18, 3])
    ev = E.eval_seqs(b, starts, train_len, 5, 99)
    assert ev[0].tolist() == [15, 16, 17, 18, 99]
    assert ev[1].tolist() == [0, 21, 22, 23, 99]
    items = np.arange(1, 400)
    probs = np.ones(len(items)) / len(items)
    negs = E.sample_negatives(b, starts, train_len, np.array([19, 24]), items, probs,
                              np.random.default_rng(1))
    assert negs.shape == (2, 100)
    assert not set(negs[0]) & set(range(1, 20))
    assert len(set(negs[1])) == 100 and 24 not in set(negs[1])


def test_etl_end_to_end(tmp_path):
    from tdfo_amd.data.goodreads import make_synthetic_raw
    make_synthetic_raw(tmp_path, 120, 400, seed=3, mean_inter=40)
    info = E.run_etl(tmp_path, verbose=False)
    tr = E.read_columns(str(tmp_path / "parquet_bert4rec" / "train_part_*.parquet"))
    ev = E.read_columns(str(tmp_path / "parquet_bert4rec" / "eval_part_*.parquet"))
    assert tr["train_interactions"].shape[1] == 20 and tr["labels"].shape[1] == 20
    assert ev["candidate_items"].shape == (info["n_users"], 101)
    mask_id = info["n_items"] + 1
    assert tr["train_interactions"].max() <= mask_id and tr["labels"].max() <= info["n_items"]
    assert (ev["eval_seqs"][:, -1] == mask_id).all()
    assert len(list((tmp_path / "parquet_bert4rec").glob("*.parquet"))) == 4


@pytest.mark.parametrize("V,N", [(50, 24), (1100, 40)])
def test_linear_xent_oracle_matches_naive(V, N):
    torch.manual_seed(V)
    H, W, b = torch.randn(N, 16), torch.randn(V, 16) * 0.3, torch.randn(V) * 0.1
    y = torch.randint(0, V, (N,))
    y[::3] = 0
    dH, lv, dW, db = torch.zeros(N, 16), torch.zeros(N), torch.zeros(V, 16), torch.zeros(V)
    ops.linear_xent(H, W, b, y, 0.1, 0, dH, lv, dW, db)
    # naive formula: lse - (1-eps) z_y - eps mean z
    z = H @ W.t() + b
    lse = torch.logsumexp(z, 1)
    per = lse - 0.9 * z.gather(1, y[:, None])[:, 0] - 0.1 * z.mean(1)
    per[y == 0] = 0
    torch.testing.assert_close(lv, per, rtol=1e-4, atol=1e-5)
    # dH closed form = (softmax @ W - 0.9 W_y - 0.1 mean W) / n_valid
    nv = int((y != 0).sum())
    g = (torch.softmax(z, 1) @ W - 0.9 * W[y] - 0.1 * W.mean(0)) / nv
    g[y == 0] = 0
    torch.testing.assert_close(dH, g, rtol=1e-4, atol=1e-6)
    loss = linear_cross_entropy(H, W, b, y)
    torch.testing.assert_close(loss, per.sum() / nv)


def test_metrics_match_reference_formula():
    torch.manual_seed(0)
    scores = torch.randn(64, 101)
    got = recall_ndcg_sums(scores) / 64
    labels = torch.zeros(64, 101)
    labels[:, 0] = 1
    _, cut = torch.sort(-scores, dim=1)
    for i, k in enumerate((10, 20, 50)):
        hits = torch.gather(labels, 1, cut[:, :k])
        rec = hits.sum(1).mean()
        w = 1 / torch.log2(torch.arange(2, 2 + k).float())
        ndcg = (hits * w).sum(1).mean()          # idcg = 1 for one positive
        assert abs(float(got[i]) - float(rec)) < 1e-6
        assert abs(float(got[3 + i]) - float(ndcg)) < 1e-6


def test_metrics_ties_count_against_positive():
    # an untrained / degenerate model scores every candidate the same: the
    # positive must then rank last, not first (no optimistic hits)
    scores = torch.zeros(4, 101)
    got = recall_ndcg_sums(scores)
    assert float(got.sum()) == 0.0
    scores[:, 0] = 1.0
    scores[:, 1:10] = 1.0               # 9 ties ahead -> rank 9: a hit at @10 only
    got = recall_ndcg_sums(scores) / 4
    assert float(got[0]) == 1.0
    assert abs(float(got[3]) - 1.0 / math.log2(11)) < 1e-6


def _batch(g, B, T, n_items, n_mask=3):
    base = torch.randint(1, n_items - T, (B, 1), generator=g)
    seqs = base + torch.arange(T)
    labels = torch.zeros_like(seqs)
    labels[:, -n_mask:] = seqs[:, -n_mask:]
    seqs = seqs.clone()
    seqs[:, -n_mask:] = n_items + 1
    return seqs, labels


def test_bert4rec_cpu_learns_and_checkpoint(tmp_path):
    torch.manual_seed(0)
    tr = Bert4RecTrainer(150, 20, 16, 2, 2, 16, lr=5e-3, device="cpu", seed=1)
    g = torch.Generator().manual_seed(0)
    losses = []
    for i in range(150):
        tr.load_batch(*_batch(g, 16, 20, 150))
        tr.step()
        if i % 50 == 49:
            losses.append(tr.pop_loss())
    assert losses[-1] < losses[0] - 0.3, losses
    seqs, _ = _batch(g, 16, 20, 150)
    tr.eval_batch(seqs, torch.randint(1, 151, (16, 101), generator=g))
    m = tr.pop_metrics()
    assert set(m) == set(METRIC_NAMES)
    sd = tr.state_dict()
    assert "history.embed_collection.embeddings.item_embedding.weight" in sd
    assert sd["out.weight"].shape == (152, 16)
    assert sd["history.layernorm.weight"].shape == (20, 16)        # LayerNorm([T, E]) quirk
    p = tmp_path / bert4rec_ckpt_name(10)
    assert p.name == "bert4recepoch_10_model.pth"
    save_state_dict(sd, str(p))
    back = load_state_dict(str(p))
    assert set(back) == set(sd)


def _dist_worker(rank, world, mode, steps):
    from tdfo_amd.parallel.dist import get_info
    info = get_info()
    B, T, n = 8, 20, 120
    tr = Bert4RecTrainer(n, T, 16, 2, 2, B, lr=3e-3, device="cpu", mode=mode,
                         group=info.group, rank=rank, world=world, dropout=0.0, seed=5)
    g = torch.Generator().manual_seed(11)
    for _ in range(steps):
        s, l = _batch(g, B * world, T, n)
        tr.load_batch(s[rank * B:(rank + 1) * B], l[rank * B:(rank + 1) * B])
        tr.step()
    out = {k: v.detach().clone() for k, v in tr.state_dict().items()}
    return {"sd": {k.replace("module.", ""): v for k, v in out.items()}, "loss": tr.pop_loss()}


@pytest.mark.parametrize("mode", ["ddp", "dmp"])
def test_bert4rec_distributed_matches_single(mode):
    steps, world = 3, 2
    tr = Bert4RecTrainer(120, 20, 16, 2, 2, 8 * world, lr=3e-3, device="cpu", dropout=0.0,
                         seed=5)
    g = torch.Generator().manual_seed(11)
    for _ in range(steps):
        tr.load_batch(*_batch(g, 8 * world, 20, 120))
        tr.step()
    ref_sd = tr.state_dict()
    outs = run_distributed(_dist_worker, world, mode, steps)
    tol = 2e-5    # dmp: fp32 pooled rows (ShardedEmbeddingModule recv_dtype="fp32")
    for o in outs:
        for k, v in ref_sd.items():
            d = (o["sd"][k] - v).abs()
            if mode == "dmp" and "embedding" in k:
                # the owner sums a row's gradient contributions in another
                # order: a row whose fp32 sum cancels to ~0 takes a different
                # Adam sign step (<= lr) -- allowed for a handful of elements
                assert (d > tol).float().mean() < 0.01 and d.max() <= 3e-3, (k, d.max())
            else:
                torch.testing.assert_close(o["sd"][k], v, rtol=tol, atol=tol,
                                           msg=lambda m, k=k: f"{k}: {m}")


def test_reference_attention_core_matches_model_math():
    """CPU: the fused kernels' torch reference (hash dropout off) equals the
    reference model's attention (masked_fill(-1e9), softmax, P.V)."""
    import math

    from tdfo_amd.ops import reference as ref

    torch.manual_seed(0)
    B, T, E, H = 4, 20, 16, 2
    qkv = torch.randn(B, T, 3 * E)
    ids = torch.randint(0, 9, (B, T))
    out = torch.empty(B, T, E)
    ref.attention_fwd(qkv, ids, H, 0.0, 1, None, 0, out)
    dk = E // H
    q, k, v = qkv.view(B, T, 3, H, dk).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-2, -1) / math.sqrt(dk)).masked_fill((ids == 0).view(B, 1, 1, T), -1e9)
    exp = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, T, E)
    assert torch.allclose(out, exp, atol=1e-6)
    keep = ref.attn_keep_scale(B, H, T, 0.1, 5, 3, "cpu")
    frac = float((keep == 0).float().mean())
    assert 0.05 < frac < 0.15                  # ~rate of the elements dropped


def test_encoder_layer_reference_matches_block():
    """ops.reference.encoder_layer (the fused kernel's oracle) is the same math
    as the module path of TransformerBlock when dropout is off."""
    import torch

    from tdfo_amd.models import bert4rec as m
    from tdfo_amd.ops import reference as ref

    torch.manual_seed(0)
    B, T, E, H = 4, 9, 16, 2
    blk = m.TransformerBlock(E, H, 0.0).eval()
    x = torch.randn(B, T, E)
    ids = torch.randint(0, 5, (B, T))
    mask = (ids != 0).unsqueeze(1).unsqueeze(1)
    exp = blk(x, mask)
    got = ref.encoder_layer(x, ids, blk._fused_params(), H, 0.0, 1, 0, 0,
                            blk.input_sublayer.norm.eps)
    assert torch.allclose(got, exp, atol=1e-5, rtol=1e-5)


def test_seq_prologue_reference_matches_autograd():
    """CPU reference of the fused Bert4Rec input block (dropout(LN(x + pos)))
    vs torch autograd of the unfused ops at rate 0, and mask statistics."""
    from tdfo_amd.ops import reference as ref

    torch.manual_seed(0)
    M, n = 64, 320
    x, pos = torch.randn(M, n), torch.randn(n)
    gamma, beta = torch.randn(n), torch.randn(n)
    y, mean, rstd = torch.empty(M, n), torch.empty(M), torch.empty(M)
    ref.seq_prologue_fwd(x, pos, n, 1e-5, gamma, beta, 0.0, 5, None, y, mean, rstd)
    xr, pr = x.clone().requires_grad_(True), pos.clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    e = torch.nn.functional.layer_norm(xr + pr, (n,), gr, br, 1e-5)
    assert torch.allclose(y, e, atol=1e-5)
    g = torch.randn(M, n)
    e.backward(g)
    dx, out3 = torch.empty(M, n), torch.empty(3 * n)
    ref.seq_prologue_bwd(x, pos, g, n, gamma, mean, rstd, 0.0, 5, None, dx, out3)
    assert torch.allclose(dx, xr.grad, atol=1e-5)
    assert torch.allclose(out3[:n], gr.grad, atol=1e-4)
    assert torch.allclose(out3[n:2 * n], br.grad, atol=1e-4)
    assert torch.allclose(out3[2 * n:], pr.grad, atol=1e-4)
    m = ref.seq_prologue_mul(M, n, 0.25, 5, 3, "cpu")
    assert abs(float((m == 0).float().mean()) - 0.25) < 0.02


def test_rank_metrics_reference_matches_recall_ndcg():
    """ops.rank_metrics (CPU reference of the fused eval kernel) equals the
    trainer's scores -> recall_ndcg_sums path, ties included."""
    from tdfo_amd import ops
    from tdfo_amd.models.bert4rec import METRICS_K, recall_ndcg_sums

    torch.manual_seed(0)
    B, C, E, V = 37, 101, 16, 500
    h, W, b = torch.randn(B, E), torch.randn(V, E), torch.randn(V)
    cand = torch.randint(0, V, (B, C))
    cand[:5, 7] = cand[:5, 0]                      # exact ties with the positive
    out = torch.empty(2 * len(METRICS_K) + 1)
    ops.rank_metrics(h, W, b, cand, METRICS_K, out)
    scores = torch.einsum("bce,be->bc", W[cand], h) + b[cand]
    exp = recall_ndcg_sums(scores)
    assert torch.allclose(out[:-1], exp, atol=1e-4)
    assert float(out[-1]) == B


def test_bert4rec_step_counters_bumped_once_per_step():
    """The trainer bumps the dense / embedding optimizer step numbers and the
    dropout RNG step with one ops.bump per step (the optimizers skip their own)."""
    tr = Bert4RecTrainer(n_items=30, max_len=6, embed_dim=16, n_heads=2, n_layers=1,
                         batch_size=4, device="cpu")
    g = torch.Generator().manual_seed(0)
    for i in range(3):
        seqs = torch.randint(1, 31, (4, 6), generator=g)
        labels = torch.where(torch.rand(4, 6, generator=g) < 0.5, seqs, torch.zeros_like(seqs))
        tr.load_batch(seqs, labels)
        tr.step()
        assert float(tr.opt.hyper[1]) == i + 1
        assert float(tr.item.hyper[1]) == i + 1
        assert int(tr.model.rng_step) == i + 1
