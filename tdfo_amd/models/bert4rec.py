"""Bert4Rec (reference torchrec/models.py + torchrec/train.py), MI355X layout.

Architecture (kept 1:1, including the reference's quirks):
  item embedding (V = n_items + 2, uniform[-1, 1], PAD id 0 embedded: Q9)
  + learned positional encoding randn(T, E)
  -> LayerNorm over [T, E] jointly (Q10) -> dropout
  -> n_layers x pre-norm transformer block
       x + drop(MHA(LN(x)))   (key-padding mask, masked_fill(-1e9), softmax, dropout)
       x + drop(FFN(LN(x)))   (E -> 4E ReLU dropout -> E), then block dropout
  -> Linear(E, V) + CrossEntropy(ignore_index=0, label_smoothing=0.1)

What is different on MI355X:
  * the output projection + loss is ``tdfo::linear_xent``: online softmax
    over vocab splits, forward and backward fused, the [B*T, V] logits are
    never written (the reference's largest tensor);
  * the item table lives in a table-batched fp32 store updated by the
    sort-based fused Adam inside backward (TorchRec DMP ``fused_params``
    semantics) — locally, replicated with a sparse (ids, row-grad)
    all-gather for DDP mode, or sharded (``model_parallel``) through the
    all-to-all embedding engine;
  * all dense parameters sit in one flat buffer updated by one fused Adam
    launch (torch.optim.Adam semantics: L2 weight decay added to the grad);
  * the whole single-GPU step (encoder fwd/bwd included) is captured into
    one hipGraph (the encoder is ~100 tiny ops at E=16, T=20).
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..utils.capture import graph_capture
from .. import ops
from ..optim.flat import FlatOptimizer
from ..sparse.tables import EmbOptimConfig, TableBatchedEmbedding, TableConfig

PAD_ID = 0
METRICS_K = (10, 20, 50)


# ---------------------------------------------------- fused HIP encoder ops
# On GPU the attention core (scores, key-padding mask, softmax, dropout, P.V)
# and every LayerNorm run as hand-written kernels (csrc/kernels/attention.hip,
# layernorm.hip); on CPU the same modules run the torch reference ops.
USE_FUSED = True
# whole transformer block in one fwd / one bwd kernel (encoder.hip); False
# keeps the per-op path (fused attention core + LayerNorm kernels, torch GEMMs)
USE_FUSED_BLOCK = True
# the step counters' bump inside the item lookup launch (TDFO_B4R_FOLD_BUMP=0:
# a launch of its own)
_FOLD_BUMP = os.environ.get("TDFO_B4R_FOLD_BUMP", "1") != "0"


def _fused(x: torch.Tensor) -> bool:
    return USE_FUSED and x.is_cuda


class _AttnCoreFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, ids, H, rate, seed, step):
        qkv = qkv.contiguous()
        B, T, E3 = qkv.shape
        out = torch.empty(B, T, E3 // 3, dtype=qkv.dtype, device=qkv.device)
        ops.attention_fwd(qkv, ids, H, rate, seed, step, PAD_ID, out)
        ctx.save_for_backward(qkv, ids, step)
        ctx.cfg = (H, rate, seed)
        return out

    @staticmethod
    def backward(ctx, g):
        qkv, ids, step = ctx.saved_tensors
        H, rate, seed = ctx.cfg
        dqkv = torch.empty_like(qkv)
        ops.attention_bwd(qkv, ids, g.contiguous(), H, rate, seed, step, PAD_ID, dqkv)
        return dqkv, None, None, None, None, None


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, n, eps):
        x = x.contiguous()
        M = x.numel() // n
        y = torch.empty_like(x)
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        ops.layernorm_fwd(x, n, eps, gamma, beta, y, mean, rstd)
        ctx.save_for_backward(x, gamma, mean, rstd)
        ctx.n = n
        return y

    @staticmethod
    def backward(ctx, g):
        x, gamma, mean, rstd = ctx.saved_tensors
        n = ctx.n
        M = x.numel() // n
        dx = torch.empty_like(x)
        part = torch.empty(ops.layernorm_parts(M) * 2 * n, dtype=torch.float32, device=x.device)
        dgb = torch.empty(2 * n, dtype=torch.float32, device=x.device)
        ops.layernorm_bwd(x, g.contiguous(), n, gamma, mean, rstd, dx, part, dgb)
        return dx, dgb[:n].view_as(gamma), dgb[n:].view_as(gamma), None, None


class _EncoderLayerFn(torch.autograd.Function):
    """Whole pre-norm transformer block as two HIP kernels (encoder.hip)."""

    @staticmethod
    def forward(ctx, x, ids, step, H, rate, seed, eps, gdst, *params):
        x = x.contiguous()
        B, T, E = x.shape
        FF = params[-4].shape[0]
        ctx.gdst = gdst
        dev = x.device
        saved = [torch.empty(B, T, 3 * E, device=dev), torch.empty(B, T, E, device=dev),
                 torch.empty(B, T, E, device=dev), torch.empty(B, T, FF, device=dev)]
        y = torch.empty_like(x)
        params = [p.contiguous() for p in params]
        ops.encoder_layer_fwd(x, ids, step, params, H, rate, seed, PAD_ID, eps, saved, y)
        ctx.save_for_backward(x, ids, step, *params, *saved)
        ctx.cfg = (H, rate, seed, eps)
        return y

    @staticmethod
    def backward(ctx, dy):
        t = ctx.saved_tensors
        npar = len(t) - 7                   # x, ids, step, params..., 4 saved
        x, ids, step = t[0], t[1], t[2]
        params, saved = list(t[3:3 + npar]), list(t[3 + npar:])
        H, rate, seed, eps = ctx.cfg
        B, T, E = x.shape
        FF = params[-4].shape[0]
        P = ops.encoder_param_count(E, FF)
        part = torch.empty(B * P, device=x.device)
        dx = torch.empty_like(x)
        if ctx.gdst is not None:
            # every parameter gradient straight into the flat gradient buffer
            # by the kernel's reduction (gidx: flat positions in packed order):
            # no cat-backward, no AccumulateGrad adds, no scatter launch
            flat, idx = ctx.gdst
            # the reduction over sequences rides in the next backward launch
            # (layer below / sequence prologue); `part` stays referenced
            # until that launch is issued (no allocator reuse under it)
            defer = _DEFER_ENC_RED and x.is_cuda
            ops.encoder_layer_bwd(x, ids, step, params, H, rate, seed, PAD_ID, eps, saved,
                                  dy.contiguous(), dx, part, flat, gidx=idx, defer=defer)
            _PARKED[0] = part if defer else None
            return (dx, None, None, None, None, None, None, None) + (None,) * len(params)
        grad = torch.empty(P, device=x.device)
        ops.encoder_layer_bwd(x, ids, step, params, H, rate, seed, PAD_ID, eps, saved,
                              dy.contiguous(), dx, part, grad)
        grads, o = [], 0
        for p in params:
            grads.append(grad[o:o + p.numel()].view_as(p))
            o += p.numel()
        return (dx, None, None, None, None, None, None, None, *grads)


class _SeqPrologueFn(torch.autograd.Function):
    """dropout(LN_[T,E](item_emb + pos)) as one HIP kernel each way
    (layernorm.hip seq_prologue_*): replaces the add, LayerNorm, dropout and
    their backward library ops, incl. the positional-encoding grad reduction."""

    @staticmethod
    def forward(ctx, x, pos, gamma, beta, eps, rate, seed, step, gdst=None):
        x = x.contiguous()
        n = pos.numel()
        ctx.gdst = gdst
        M = x.numel() // n
        y = torch.empty_like(x)
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        ops.seq_prologue_fwd(x, pos.contiguous(), n, eps, gamma.contiguous(), beta.contiguous(),
                             rate, seed, step, y, mean, rstd)
        ctx.save_for_backward(x, pos, gamma, mean, rstd, step)
        ctx.cfg = (n, rate, seed)
        return y

    @staticmethod
    def backward(ctx, g):
        x, pos, gamma, mean, rstd, step = ctx.saved_tensors
        n, rate, seed = ctx.cfg
        M = x.numel() // n
        dx = torch.empty_like(x)
        part = torch.empty(ops.layernorm_parts(M) * 3 * n, dtype=torch.float32, device=x.device)
        if ctx.gdst is not None:            # [gamma | beta | pos] -> the flat gradients
            flat, idx = ctx.gdst
            ops.seq_prologue_bwd(x, pos.contiguous(), g.contiguous(), n, gamma.contiguous(),
                                 mean, rstd, rate, seed, step, dx, part, flat, gidx=idx)
            _PARKED[0] = None               # (a parked encoder reduction ran in it)
            return (dx, None, None, None, None, None, None, None, None)
        out3 = torch.empty(3 * n, dtype=torch.float32, device=x.device)
        ops.seq_prologue_bwd(x, pos.contiguous(), g.contiguous(), n, gamma.contiguous(), mean,
                             rstd, rate, seed, step, dx, part, out3)
        return (dx, out3[2 * n:].view_as(pos), out3[:n].view_as(gamma),
                out3[n:2 * n].view_as(gamma), None, None, None, None, None)


_ENC_OK: Dict[tuple, bool] = {}
# encoder reductions parked into the next backward launch (TDFO_B4R_DEFER_ENC_RED)
_DEFER_ENC_RED = os.environ.get("TDFO_B4R_DEFER_ENC_RED", "1") != "0"
_PARKED: list = [None]             # the parked reduction's partials, kept alive


def _fused_block_ok(T: int, E: int, H: int, FF: int) -> bool:
    k = (T, E, H, FF)
    if k not in _ENC_OK:
        _ENC_OK[k] = ops.encoder_layer_supported(T, E, H, FF)
    return _ENC_OK[k]


def layer_norm(x: torch.Tensor, ln: nn.LayerNorm) -> torch.Tensor:
    if _fused(x):
        n = ln.weight.numel()
        return _LayerNormFn.apply(x, ln.weight, ln.bias, n, ln.eps)
    return ln(x)


class KeyPad:
    """Attention context of the fused path: item ids (key-padding mask is
    ids != PAD) and the device step counter that keys the dropout hash."""

    def __init__(self, ids: torch.Tensor, step: Optional[torch.Tensor]):
        self.ids, self.step = ids, step


# ------------------------------------------------------------------ encoder
class MultiHeadedAttention(nn.Module):
    def __init__(self, num_heads: int, dim: int, dropout: float = 0.1):
        super().__init__()
        assert dim % num_heads == 0          # torchrec/models.py:40
        self.d_k = dim // num_heads
        self.h = num_heads
        self.linear_layers = nn.ModuleList([nn.Linear(dim, dim) for _ in range(3)])
        self.output_linear = nn.Linear(dim, dim)
        self.dropout = nn.Dropout(dropout)
        self.seed = 0x5EED                 # per-layer dropout-hash seed (set by Bert4Rec)

    def forward(self, x, mask):
        B, T, _ = x.shape
        w = torch.cat([l.weight for l in self.linear_layers], 0)       # one QKV GEMM
        b = torch.cat([l.bias for l in self.linear_layers], 0)
        if isinstance(mask, KeyPad):
            rate = self.dropout.p if self.training else 0.0
            core = _AttnCoreFn.apply(F.linear(x, w, b), mask.ids, self.h, rate, self.seed,
                                     mask.step)
            return self.output_linear(core)
        qkv = F.linear(x, w, b).view(B, T, 3, self.h, self.d_k).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(self.d_k)
        scores = scores.masked_fill(~mask, -1e9)
        p = self.dropout(torch.softmax(scores, dim=-1))
        out = torch.matmul(p, v).transpose(1, 2).reshape(B, T, self.h * self.d_k)
        return self.output_linear(out)


class FeedForward(nn.Module):
    def __init__(self, dim: int, dropout: float = 0.1):
        super().__init__()
        self.w_1 = nn.Linear(dim, 4 * dim)
        self.w_2 = nn.Linear(4 * dim, dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        return self.w_2(self.dropout(F.relu(self.w_1(x))))


class SublayerConnection(nn.Module):
    def __init__(self, dim: int, dropout: float):
        super().__init__()
        self.norm = nn.LayerNorm(dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, fn):
        return x + self.dropout(fn(layer_norm(x, self.norm)))   # pre-norm (torchrec/models.py:102-106)


class TransformerBlock(nn.Module):
    def __init__(self, dim: int, heads: int, dropout: float):
        super().__init__()
        self.attention = MultiHeadedAttention(heads, dim, dropout)
        self.feed_forward = FeedForward(dim, dropout)
        self.input_sublayer = SublayerConnection(dim, dropout)
        self.output_sublayer = SublayerConnection(dim, dropout)
        self.dropout = nn.Dropout(dropout)

    def _fused_params(self):
        # Q / K / V as the module's own tensors (the kernel stages them apart:
        # no concatenated copy per step)
        att, ff = self.attention, self.feed_forward
        return [l.weight for l in att.linear_layers] + [l.bias for l in att.linear_layers] + [
                att.output_linear.weight, att.output_linear.bias,
                self.input_sublayer.norm.weight, self.input_sublayer.norm.bias,
                self.output_sublayer.norm.weight, self.output_sublayer.norm.bias,
                ff.w_1.weight, ff.w_1.bias, ff.w_2.weight, ff.w_2.bias]

    def forward(self, x, mask):
        att = self.attention
        if (USE_FUSED_BLOCK and isinstance(mask, KeyPad) and x.is_cuda
                and _fused_block_ok(x.shape[1], x.shape[2], att.h, self.feed_forward.w_1.out_features)):
            rate = self.dropout.p if self.training else 0.0
            return _EncoderLayerFn.apply(x, mask.ids, mask.step, att.h, rate, att.seed,
                                         self.input_sublayer.norm.eps,
                                         getattr(self, "gdst", None), *self._fused_params())
        x = self.input_sublayer(x, lambda y: self.attention(y, mask))
        x = self.output_sublayer(x, self.feed_forward)
        return self.dropout(x)


# ---------------------------------------------------------- item embedding
class _SeqEmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, anchor, owner):
        ctx.owner = owner
        return owner._lookup(ids)

    @staticmethod
    def backward(ctx, grad):
        ctx.owner._update(grad.contiguous())
        return None, None, None


class ItemEmbedding(nn.Module):
    """Replicated item table with the fused sparse Adam in backward.
    ``group``/``world`` > 1: DDP semantics (row grads averaged over ranks)
    via one all-gather of ids and row grads instead of a dense all-reduce."""

    def __init__(self, vocab: int, dim: int, n_tokens: int, optim: EmbOptimConfig, device,
                 group=None, world: int = 1, seed: int = 0):
        super().__init__()
        self.store = TableBatchedEmbedding([vocab], dim, device, optim, init_ranges=[1.0],
                                           seed=seed)
        self.D = dim
        self.N = n_tokens
        self.group, self.world = group, world
        self.hyper = torch.tensor([optim.lr, 0.0], dtype=torch.float32, device=device)
        self.step_bumped_by_caller = False
        self.offsets = torch.arange(n_tokens * world + 1, dtype=torch.int64, device=device)
        self.zero = torch.zeros(1, dtype=torch.int64, device=device)
        if world > 1:
            self.g_ids = torch.zeros(world * n_tokens, dtype=torch.int64, device=device)
            self.g_grad = torch.zeros(world * n_tokens, dim, dtype=torch.float32, device=device)
        self._anchor = nn.Parameter(torch.zeros(1, device=device))
        self._ids = None
        self.fwd_bumps = ()              # counters the next lookup launch advances

    @property
    def weight(self):
        return self.store.weight

    def _lookup(self, ids):
        n = ids.numel()
        # a fresh output (the caller's autograd saves it): the lookup writes it
        # directly, no copy of a static buffer
        out = torch.empty(n, self.D, dtype=torch.float32, device=self.store.weight.device)
        # the trainer's step counters ride in this first launch of the step
        bumps, self.fwd_bumps = self.fwd_bumps, ()
        self.store.forward(ids, self.offsets[: n + 1], self.zero, 1, n, out, self.zero, self.D,
                           onehot=True, bumps=bumps)
        self._ids = ids
        return out

    def _update(self, grad):
        ids = self._ids
        n = ids.numel()
        if not self.step_bumped_by_caller:
            self.hyper[1:2].add_(1.0)
        if self.world > 1:
            dist.all_gather_into_tensor(self.g_ids[: self.world * n], ids, group=self.group)
            dist.all_gather_into_tensor(self.g_grad[: self.world * n], grad, group=self.group)
            self.g_grad.mul_(1.0 / self.world)
            ids, grad, n = self.g_ids[: self.world * n], self.g_grad[: self.world * n], self.world * n
        # one id per position of the single table: the per-table LDS sort
        # (device-wide radix sort past 8192 ids, embedding.hip onehot_path)
        self.store.backward_update(ids, self.offsets[: n + 1], self.zero, 1, n, grad, self.zero,
                                   self.D, self.hyper, segsort=1)

    def forward(self, ids):
        if self.training and torch.is_grad_enabled():
            return _SeqEmbFn.apply(ids, self._anchor, self)
        return self._lookup(ids)


class _LinearXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, H, W, b, labels, eps, loss_acc, unit_grad, step=None):
        N = H.shape[0]
        dH = torch.empty_like(H)
        lossv = torch.empty(N, dtype=torch.float32, device=H.device)
        # unit gradient and W / b used nowhere else in the graph: the kernel
        # writes their gradients straight into the (zeroed) .grad buffers
        # instead of autograd accumulating returned tensors into them
        direct = bool(unit_grad and W.grad is not None and b.grad is not None and
                      W.grad.is_contiguous() and b.grad.is_contiguous())
        dW = W.grad if direct else torch.empty_like(W)
        db = b.grad if direct else torch.empty_like(b)
        loss = torch.empty(1, dtype=torch.float32, device=H.device)
        # the kernel also reduces the mean loss (and adds it to loss_acc)
        ops.linear_xent(H, W, b, labels, eps, PAD_ID, dH, lossv, dW, db, loss=loss,
                        loss_acc=loss_acc, step=step if direct else None)
        ctx.save_for_backward(dH, dW, db)
        ctx.unit_grad = unit_grad
        ctx.direct = direct
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        dH, dW, db = ctx.saved_tensors
        if ctx.unit_grad:      # caller's promise: the loss is backward()'s root (g == 1)
            if ctx.direct:
                return dH, None, None, None, None, None, None, None
            return dH, dW, db, None, None, None, None, None
        return dH * g, dW * g, db * g, None, None, None, None, None


def linear_cross_entropy(H, W, b, labels, eps=0.1, loss_acc=None, unit_grad=False, step=None):
    """mean CE(ignore_index=0, label_smoothing=eps) of H @ W^T + b, fused.
    loss_acc (fp64 [1]): the kernel adds the loss to it. unit_grad: the
    returned loss is the root of backward() (gradient exactly 1) and W / b
    feed nothing else, so the saved gradients are returned without the
    scaling launches -- and when W.grad / b.grad exist (the trainer's flat
    gradient views, zeroed each step) they are written there directly.
    step: the optimizer step of W / b fused into the kernels (see
    ops.linear_xent; only with unit_grad and direct gradient buffers)."""
    return _LinearXentFn.apply(H.contiguous(), W, b, labels.contiguous(), eps, loss_acc,
                               unit_grad, step)


class Bert4Rec(nn.Module):
    """Reference parameter names are preserved (state_dict() keys match
    torchrec's Bert4Rec except the item table, exported by the trainer)."""

    def __init__(self, vocab_size: int, max_len: int, embed_dim: int, num_heads: int,
                 num_layers: int, dropout: float = 0.1):
        super().__init__()
        self.vocab_size, self.max_len, self.emb_dim = vocab_size, max_len, embed_dim
        self.positional_encoding = nn.Parameter(torch.randn(max_len, embed_dim))
        self.layernorm = nn.LayerNorm([max_len, embed_dim])
        self.emb_dropout = nn.Dropout(dropout)
        self.transformer_blocks = nn.ModuleList(
            [TransformerBlock(embed_dim, num_heads, dropout) for _ in range(num_layers)])
        self.out = nn.Linear(embed_dim, vocab_size)
        for i, blk in enumerate(self.transformer_blocks):
            blk.attention.seed = 0x5EED + 7919 * i
        # device step counter for the fused attention's dropout hash (advanced
        # once per training step by the trainer, inside the captured graph)
        self.register_buffer("rng_step", torch.zeros(1, dtype=torch.int64), persistent=False)

    def encode(self, item_emb: torch.Tensor, seqs: torch.Tensor) -> torch.Tensor:
        """item_emb [B, T, E] (looked-up rows), seqs [B, T] ids -> hidden [B, T, E]."""
        if _fused(item_emb):
            mask = KeyPad(seqs.contiguous(), self.rng_step)
        else:
            mask = (seqs != PAD_ID).unsqueeze(1).unsqueeze(1)      # [B, 1, 1, T] key mask
        if _fused(item_emb):
            rate = self.emb_dropout.p if self.training else 0.0
            x = _SeqPrologueFn.apply(item_emb, self.positional_encoding, self.layernorm.weight,
                                     self.layernorm.bias, self.layernorm.eps, rate,
                                     0x5EED0E3B, self.rng_step, getattr(self, "gdst", None))
        else:
            x = self.emb_dropout(layer_norm(item_emb + self.positional_encoding, self.layernorm))
        for blk in self.transformer_blocks:
            x = blk(x, mask)
        return x


# ------------------------------------------------------------------ metrics
def recall_ndcg_sums(scores: torch.Tensor) -> torch.Tensor:
    """scores [B, 1 + negs], positive in column 0 (torchrec/train.py:52-78).
    Returns per-metric SUMS over the batch in the order
    [Recall@10, Recall@20, Recall@50, NDCG@10, NDCG@20, NDCG@50].

    Tie rule: a negative scoring EQUAL to the positive ranks ahead of it
    (pessimistic), so ties never inflate Recall/NDCG. The reference sorts
    with torch.sort(-scores), whose order among ties is unspecified; no
    reference fixture pins it (parity unpinned)."""
    rank = (scores[:, 1:] >= scores[:, :1]).sum(1)                    # 0-based rank of the positive
    rec = [(rank < k).float().sum() for k in METRICS_K]
    ndcg = [torch.where(rank < k, 1.0 / torch.log2(rank.float() + 2.0),
                        torch.zeros_like(rank, dtype=torch.float32)).sum() for k in METRICS_K]
    return torch.stack(rec + ndcg)


METRIC_NAMES = [f"Recall@{k}" for k in METRICS_K] + [f"NDCG@{k}" for k in METRICS_K]


# ------------------------------------------------------------------ trainer
class Bert4RecTrainer:
    """One rank of Bert4Rec training. mode: "local" | "ddp" | "dmp"."""

    def __init__(self, n_items: int, max_len: int = 20, embed_dim: int = 16, n_heads: int = 2,
                 n_layers: int = 2, batch_size: int = 16, lr: float = 3e-4, wd: float = 1e-4,
                 device="cpu", mode: str = "local", group=None, rank: int = 0, world: int = 1,
                 dropout: float = 0.1, seed: int = 42, label_smoothing: float = 0.1):
        self.V = n_items + 2                     # 0 = PAD, n_items + 1 = MASK
        self.T, self.E, self.B = max_len, embed_dim, batch_size
        self.device = dev = torch.device(device)
        self.mode, self.group, self.rank, self.world = mode, group, rank, world
        self.eps = label_smoothing
        torch.manual_seed(seed)
        self.model = Bert4Rec(self.V, max_len, embed_dim, n_heads, n_layers, dropout).to(dev)
        emb_opt = EmbOptimConfig("adam", lr=lr, weight_decay=wd)
        ntok = batch_size * max_len
        if mode == "dmp":
            from ..sparse.modules import ShardedEmbeddingModule
            tab = TableConfig("item_embedding", self.V, embed_dim, init_range=1.0)
            self.item = ShardedEmbeddingModule([tab], ntok, [1], emb_opt, dev, world_size=world,
                                               rank=rank, group=group, seed=seed)
            full = TableBatchedEmbedding([self.V], embed_dim, dev, emb_opt, init_ranges=[1.0],
                                         seed=seed)
            self.item.set_table_weight(0, full.weight)      # identical init on every rank
            del full
        else:
            self.item = ItemEmbedding(self.V, embed_dim, ntok, emb_opt, dev,
                                      group=group if mode == "ddp" else None,
                                      world=world if mode == "ddp" else 1, seed=seed)
        if world > 1:     # identical dense init on all ranks (DDP broadcasts from rank 0)
            for p in self.model.parameters():
                dist.broadcast(p.data, 0, group=group)
        self.opt = FlatOptimizer(self.model.parameters(), "adam", lr=lr, weight_decay=wd,
                                 group=group if world > 1 else None)
        # One rank: the output layer's Adam step runs inside the fused
        # Linear+CE kernels, which hold its complete gradient (no 17 M-element
        # gradient written and re-read by the flat optimizer, no zero fill);
        # the flat optimizer steps the rest. More ranks all-reduce the
        # gradient first. TDFO_XENT_FUSED_STEP=0: the unfused path (A/B).
        self._xent_step = None
        if (world == 1 and dev.type == "cuda" and not self.opt.dynamic_scale
                and os.environ.get("TDFO_XENT_FUSED_STEP", "1") != "0"):
            out = self.model.out
            mw, vw = self.opt.moments(out.weight)
            mb, vb = self.opt.moments(out.bias)
            self._xent_step = (self.opt.opt, [mw, vw, mb, vb], self.opt.hyper, self.opt.beta1,
                               self.opt.beta2, self.opt.eps, self.opt.wd)
            self.opt.exclude([out.weight, out.bias])
        # Fused encoder kernels write their parameter gradients into the flat
        # gradient buffer through one index_copy each (maps built once from the
        # flat views), so autograd accumulates nothing there (the QKV cat's
        # backward and 35 AccumulateGrad adds per step before)
        self._zero_ranges = None
        if dev.type == "cuda" and os.environ.get("TDFO_B4R_DIRECT_GRADS", "1") != "0":
            self._attach_direct_grads()
        self.seqs = torch.zeros(batch_size, max_len, dtype=torch.int64, device=dev)
        self.labels = torch.zeros(batch_size, max_len, dtype=torch.int64, device=dev)
        self.loss_sum = torch.zeros(1, dtype=torch.float64, device=dev)
        self.steps = 0
        self.metric_sums = torch.zeros(len(METRIC_NAMES) + 1, dtype=torch.float64, device=dev)
        self.graph = None
        self._static_loss = None
        # the step's counters (dense / embedding optimizer step numbers, the
        # dropout RNG step) bumped by one launch at the start of the step
        # (three library add kernels before)
        self.opt.step_bumped_by_caller = True
        self.item.step_bumped_by_caller = True
        eh = self.item.engine._hyper if mode == "dmp" else self.item.hyper
        self._counters = [self.opt.hyper[1:2], eh[1:2], self.model.rng_step]

    def _flat_index(self, params) -> torch.Tensor:
        return ops.flat_scatter_index(self.opt.grad, [p.grad for p in params])

    def _attach_direct_grads(self):
        m = self.model
        m.gdst = (self.opt.grad, self._flat_index([m.layernorm.weight, m.layernorm.bias,
                                                   m.positional_encoding]))
        idxs = [m.gdst[1]]
        for blk in m.transformer_blocks:
            att, ff = blk.attention, blk.feed_forward
            order = ([l.weight for l in att.linear_layers] + [l.bias for l in att.linear_layers]
                     + [att.output_linear.weight, att.output_linear.bias,
                        blk.input_sublayer.norm.weight, blk.input_sublayer.norm.bias,
                        blk.output_sublayer.norm.weight, blk.output_sublayer.norm.bias,
                        ff.w_1.weight, ff.w_1.bias, ff.w_2.weight, ff.w_2.bias])
            blk.gdst = (self.opt.grad, self._flat_index(order))
            idxs.append(blk.gdst[1])
        # flat ranges the direct writes do not cover: the only ones a step
        # must still zero while the fused kernels run (none when the output
        # layer's step is fused too: no fill launches)
        cov = torch.ones(self.opt.numel, dtype=torch.bool)    # (alignment gaps: never written)
        for _, off, n in self.opt._views:
            cov[off:off + n] = False
        cov[torch.cat(idxs).cpu()] = True
        self._zero_ranges = []
        for lo, hi in self.opt._ranges:
            c = cov[lo:hi]
            j = lo
            while j < hi:
                if bool(c[j - lo]):
                    j += 1
                    continue
                k = j
                while k < hi and not bool(c[k - lo]):
                    k += 1
                self._zero_ranges.append((j, k))
                j = k

    def _zero_grads(self):
        m = self.model
        ff = m.transformer_blocks[0].feed_forward.w_1.out_features if len(m.transformer_blocks) else 0
        direct = (self._zero_ranges is not None and USE_FUSED and USE_FUSED_BLOCK and
                  _fused_block_ok(self.T, self.E, m.transformer_blocks[0].attention.h, ff)
                  if len(m.transformer_blocks) else False)
        if not direct:
            self.opt.zero_grads()
            return
        for lo, hi in self._zero_ranges:
            self.opt.grad[lo:hi].zero_()

    # ------------------------------------------------------------ train
    def _embed(self, seqs):
        B, T = seqs.shape
        flat = seqs.reshape(-1)
        if self.mode == "dmp":
            return self.item(flat)[0].view(B, T, self.E)
        return self.item(flat).view(B, T, self.E)

    def _fwd_bwd(self, seqs, labels):
        self.model.train()
        self.item.train()
        x = self._embed(seqs)
        h = self.model.encode(x, seqs)
        loss = linear_cross_entropy(h.reshape(-1, self.E), self.model.out.weight,
                                    self.model.out.bias, labels.reshape(-1), self.eps,
                                    loss_acc=self.loss_sum, unit_grad=True, step=self._xent_step)
        # the root gradient from a persistent 1 (implicit backward() fills a
        # fresh ones tensor every step: one fill launch)
        one = getattr(self, "_one", None)
        if one is None or one.shape != loss.shape or one.device != loss.device:
            one = self._one = torch.ones_like(loss)
        loss.backward(one)
        return loss

    def _step_body(self, seqs, labels):
        if self.mode != "dmp" and self.device.type == "cuda" and _FOLD_BUMP:
            self.item.fwd_bumps = self._counters     # advanced by the step's lookup launch
        else:
            ops.bump(self._counters)
        self._zero_grads()
        loss = self._fwd_bwd(seqs, labels)
        if self.device.type == "cuda":
            ops.encoder_reduce_flush()      # (a no-op unless nothing took it)
            _PARKED[0] = None
        self.opt.all_reduce_grads(average=True)
        self.opt.step()
        return loss          # (already added to loss_sum by the fused loss kernel)

    def load_batch(self, seqs, labels):
        b = seqs.shape[0]
        assert b == self.B, "Bert4Rec steps use full batches"
        self.seqs.copy_(seqs, non_blocking=True)
        self.labels.copy_(labels, non_blocking=True)

    def step(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self._step_body(self.seqs, self.labels)
        self.steps += 1

    def capture_graph(self, warmup: int = 2):
        """Whole step (encoder fwd/bwd, fused xent, fused embedding Adam,
        flat Adam) in one hipGraph; single process only."""
        if self.device.type != "cuda" or self.world > 1:
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._step_body(self.seqs, self.labels)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            self._step_body(self.seqs, self.labels)
        torch.cuda.synchronize()
        self.graph = g

    def pop_loss(self) -> float:
        """Average training loss since the last call, averaged over ranks."""
        v = torch.stack([self.loss_sum[0], torch.tensor(float(self.steps), dtype=torch.float64,
                                                        device=self.device)])
        if self.world > 1:
            dist.all_reduce(v, group=self.group)
        self.loss_sum.zero_()
        self.steps = 0
        return float(v[0] / max(1.0, float(v[1])))

    # ------------------------------------------------------------ eval
    @torch.no_grad()
    def eval_batch(self, seqs: torch.Tensor, candidates: torch.Tensor):
        """Score the last position against 1 + 100 candidates (no [B, V]
        logits: gathered output rows only) and accumulate metric sums."""
        self.model.eval()
        self.item.eval()
        B = seqs.shape[0]
        if self.mode == "dmp" and B < self.B:     # sharded engine has a static shape
            pad = torch.zeros(self.B - B, self.T, dtype=seqs.dtype, device=seqs.device)
            seqs_p = torch.cat([seqs, pad])
        else:
            seqs_p = seqs
        h = self.model.encode(self._embed(seqs_p), seqs_p)[:B, -1, :]         # [B, E]
        if h.is_cuda and self.E in (16, 32, 64):
            # one fused scoring + ranking kernel (ranking.hip): no [B, C] scores
            out = torch.empty(2 * len(METRICS_K) + 1, dtype=torch.float32, device=h.device)
            ops.rank_metrics(h.contiguous(), self.model.out.weight.detach(),
                             self.model.out.bias.detach(), candidates.contiguous(), METRICS_K, out)
            self.metric_sums += out.double()
            return
        w = self.model.out.weight[candidates]                                # [B, C, E]
        scores = torch.einsum("bce,be->bc", w, h) + self.model.out.bias[candidates]
        self.metric_sums[:-1] += recall_ndcg_sums(scores).double()
        self.metric_sums[-1] += B

    def pop_metrics(self) -> Dict[str, float]:
        v = self.metric_sums.clone()
        if self.world > 1:
            dist.all_reduce(v, group=self.group)
        self.metric_sums.zero_()
        n = max(1.0, float(v[-1]))
        return {k: float(v[i]) / n for i, k in enumerate(METRIC_NAMES)}

    # ------------------------------------------------------------ state
    def item_table(self) -> torch.Tensor:
        if self.mode == "dmp":
            full = torch.zeros(self.V, self.E, dtype=torch.float32, device=self.device)
            part = self.item.engine.get_table_weight(0)
            if part is not None:
                rows, w = part
                full[rows].copy_(w)
            if self.world > 1:
                dist.all_reduce(full, group=self.group)
            return full
        return self.item.weight[: self.V]

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """torchrec Bert4Rec key layout (torchrec/models.py:132-223)."""
        sd = {}
        for k, v in self.model.state_dict().items():
            if k == "positional_encoding":
                k = "history.positional_encoding"
            elif k.startswith("layernorm."):
                k = "history." + k
            sd[k] = v
        sd["history.embed_collection.embeddings.item_embedding.weight"] = self.item_table()
        if self.mode == "ddp":
            sd = {"module." + k: v for k, v in sd.items()}
        return sd
