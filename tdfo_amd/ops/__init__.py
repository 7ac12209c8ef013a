"""Device-dispatching functional ops.

GPU tensors -> hand-written HIP kernels (``torch.ops.tdfo``, must be built);
CPU tensors -> fp32 torch references (``tdfo_amd.ops.reference``). All ops
are out-variants so engines can preallocate buffers and capture hipGraphs.
"""
from __future__ import annotations

import os

import torch

from . import reference as ref
from ._ext import available as native_available  # noqa: F401
from ._ext import ops as _native
from .reference import (EMB_ADAGRAD, EMB_ADAM, EMB_DENSE_GRAD, EMB_ROWWISE_ADAGRAD,  # noqa: F401
                        EMB_SGD, OPT_ADAGRAD, OPT_ADAM, OPT_ADAMW, OPT_SGD, key_bits_for)


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def bottom_mlp_fwd_ok(k0: int, n0: int, n1: int, n2: int) -> bool:
    """The fused bottom-MLP forward covers this stack (csrc/kernels/mlp_fused.hip)."""
    return bool(native_available() and _native().bottom_mlp_fwd_ok(int(k0), int(n0), int(n1),
                                                                    int(n2)))


def bottom_mlp_fwd(x, w0, w1, w2, b0, b1, b2, y0, y1, y2, dense=None, label=None):
    """Three Linear + ReLU layers in one launch (GPU only): y0 = relu(x w0^T
    (+ b0)), y1 = relu(y0 w1^T + b1), y2 = relu(y1 w2^T + b2), the first K
    columns of each weight; bitwise equal to three ``gemm`` calls.
    ``dense`` (fp32 [M, nd]): ``batch_load``'s dense part folded in --
    x[:, :nd] = bf16(dense) first (written back to x); ``label = (src, dst)``
    also copied."""
    ls, ld = label if label is not None else (None, None)
    _native().bottom_mlp_fwd(x, w0, w1, w2, b0, b1, b2, y0, y1, y2, dense, ls, ld)


def gemm(a, a_col, b, b_col, bias=None, relu=False, mask=None, out=None, out32=None, splits=1,
         mul=None, add=None, out2=None, ldc32=0, csum_col=-1):
    """C = A B (+ epilogue). out32: fp32 split-K slabs [splits][M][ldc32]
    (ldc32 0 = N); csum_col >= 0 (col-layout A): each slab's column csum_col
    also gets the sum over that split's K range of A's column m."""
    if _gpu(a):
        _native().gemm(a, a_col, b, b_col, bias, relu, mask, out, out32, splits, mul, add, out2,
                       ldc32, csum_col)
    else:
        ref.gemm(a, a_col, b, b_col, bias, relu, mask, out, out32, splits, mul, add, out2,
                 ldc32, csum_col)


class SyncEvent:
    """A cross-stream event with a chosen release scope (mode 0: default
    system-scope fence, 1: device-scope release, 2: no system fence).
    record()/wait() act on the current stream, like torch.cuda.Event."""

    def __init__(self, mode: int = 1):
        self._h = int(_native().sync_event_create(mode))
        self._pinned = False     # referenced by a ComposedGraph's event node

    def record(self, stream=None):
        # (an explicit stream goes down as its raw handle: no torch stream
        # context switch on the host per call)
        _native().sync_event_record(self._h, -1 if stream is None else stream.cuda_stream)

    def wait(self, stream=None):
        _native().sync_event_wait(self._h, -1 if stream is None else stream.cuda_stream)

    def query(self) -> bool:
        """True once the work before the latest record has completed."""
        return bool(_native().sync_event_query(self._h))

    @property
    def handle(self) -> int:
        return self._h

    def __del__(self):
        # an event an executable graph's node refers to is never destroyed: a
        # cyclic garbage collection finalizes objects in any order, and the
        # HIP runtime aborts when a graph exec outlives its node's event
        if self._pinned:
            return
        try:
            _native().sync_event_destroy(self._h)
        except Exception:
            pass


def copy_on(dst, src, stream=None):
    """dst <- src (same dtype / size, contiguous, GPU) as one async device
    copy on ``stream`` (default: the current one), passed as its raw handle."""
    _native().copy_on(dst, src, -1 if stream is None else stream.cuda_stream)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class ComposedGraph:
    """Captured graphs chained with cross-stream event nodes and instantiated
    as one executable graph. parts: ("graph", torch.cuda.CUDAGraph captured
    with keep_graph=True), ("wait", SyncEvent), ("record", SyncEvent). The
    torch graphs (and the memory pool their kernels use) must outlive this."""

    def __init__(self, parts):
        kinds, handles = [], []
        self._keep = []
        for kind, obj in parts:
            if kind == "graph":
                kinds.append(0)
                handles.append(int(obj.raw_cuda_graph()))
            elif kind in ("wait", "record"):
                kinds.append(1 if kind == "wait" else 2)
                handles.append(obj.handle)
                obj._pinned = True
            else:
                raise ValueError(kind)
            self._keep.append(obj)
        self._ex = int(_native().graph_compose(kinds, handles))

    def replay(self, stream=None):
        """Launch on ``stream`` (default: the current stream)."""
        _native().graph_exec_launch(self._ex, -1 if stream is None else stream.cuda_stream)

    def __del__(self):
        try:
            _native().graph_exec_destroy(self._ex)
        except Exception:
            pass


def graph_num_nodes(g: torch.cuda.CUDAGraph) -> int:
    """Nodes of a graph captured with keep_graph=True (0: it captured no work)."""
    return int(_native().graph_num_nodes(int(g.raw_cuda_graph())))


def upload_graphs(graphs):
    """hipGraphUpload every executable graph (torch CUDAGraph or
    ComposedGraph) on the current stream, so their first launches do not
    set them up (TDFO_GRAPH_UPLOAD=0: skip; A/B of the first-replays
    transient, profiles/r04/notes.md)."""
    import os
    if os.environ.get("TDFO_GRAPH_UPLOAD", "1") == "0":
        return
    for g in graphs:
        if isinstance(g, ComposedGraph):
            _native().graph_exec_upload(g._ex)
        elif isinstance(g, torch.cuda.CUDAGraph):
            try:                  # (a keep_graph capture has no executable yet)
                ex = int(g.raw_cuda_graph_exec())
            except RuntimeError:
                ex = 0
            if ex:
                _native().graph_exec_upload(ex)


class gemm_batch:
    """Context manager: GEMMs issued inside are recorded and enqueued in
    order on exit, consecutive (weight grad, dgrad) pairs on the small-tile
    kernel as ONE launch (the MLP backward). Only ops.gemm calls may be
    issued inside (other ops would be enqueued ahead of the recorded GEMMs).
    No-op off the GPU."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled

    def __enter__(self):
        if self.enabled:
            _native().gemm_batch_begin()
        return self

    def __exit__(self, *exc):
        if self.enabled:
            _native().gemm_batch_end()
        return False


def gemm_pairing(v: int = -1) -> int:
    """Paired launches inside gemm_batch: 1 on (default; a dgrad the deep
    128x128 kernel would take alone moves to 256x128 tiles beside its 256x128
    weight grad), 2 on without that move, 0 off; v < 0 only reads it.
    Returns the previous value."""
    return int(_native().gemm_pairing(v))


def gemm_policy(p: int = -1) -> int:
    """GEMM tile-shape policy of the native library (process-global): 0 auto,
    1-4 one kernel forced (2-stage, deep, ping-pong, 256x128), 5 DCN-v2
    (256x128 tiles for every GEMM without column sums except the long-K deep
    ones). p < 0 only reads it. Returns the previous one."""
    return int(_native().gemm_policy(p))


def encoder_layer_supported(T: int, E: int, H: int, FF: int) -> bool:
    return bool(_native().encoder_layer_supported(T, E, H, FF))


def encoder_param_count(E: int, FF: int) -> int:
    return int(_native().encoder_param_count(E, FF))


def encoder_layer_fwd(x, ids, step, params, H, rate, seed, pad_id, eps, saved, y):
    """Fused pre-norm transformer block forward (GPU only); saved = [qkv, ctx,
    x1, f] buffers the backward reads."""
    _native().encoder_layer_fwd(x, ids, step, list(params), H, rate, seed, pad_id, eps,
                                list(saved), y)


def encoder_layer_bwd(x, ids, step, params, H, rate, seed, pad_id, eps, saved, dy, dx, part,
                      grad, gidx=None, defer=False):
    """dx and the packed parameter gradient (summed over sequences in order);
    with ``gidx`` (see ``flat_scatter_index``) gradient c lands in
    grad[gidx[c]] -- a trainer's flat gradient buffer -- instead.
    ``defer``: the reduction over sequences is parked and run by extra blocks
    of the next encoder / sequence-prologue backward launch (one launch
    fewer); the caller keeps ``part`` alive until then and calls
    ``encoder_reduce_flush`` before reading ``grad``."""
    _native().encoder_layer_bwd(x, ids, step, list(params), H, rate, seed, pad_id, eps,
                                list(saved), dy, dx, part, grad, gidx, defer)


def encoder_reduce_flush():
    """Launch a parked encoder reduction (no-op when none is parked; GPU
    callers only: deferral exists on the native path)."""
    _native().encoder_reduce_flush()


def flat_scatter_index(flat: torch.Tensor, views) -> torch.Tensor:
    """int64 positions in ``flat`` of every element of ``views`` (contiguous
    views into ``flat``, in order), on flat's device: the ``gidx`` that makes
    a kernel write a packed gradient straight into a flat gradient buffer.
    Bounds-checked here, once, so the kernels can trust it."""
    base, esz, idx = flat.data_ptr(), flat.element_size(), []
    for v in views:
        off = (v.data_ptr() - base) // esz
        if not (v.is_contiguous() and 0 <= off and off + v.numel() <= flat.numel()):
            raise ValueError("flat_scatter_index: every view must be a contiguous view of flat")
        idx.append(torch.arange(off, off + v.numel(), dtype=torch.int64))
    return torch.cat(idx).to(flat.device)


def embedding_segsort(v: int = -1) -> int:
    """One-hot embedding backward sort: 1 per-table LDS sort (default), 0 the
    device-wide radix sort; v < 0 only reads it. Returns the previous one.
    Resolved into each backward's ``segsort`` argument when the backward is
    prepared (``effective_segsort``), so toggling it between the prepare and
    apply halves cannot change the workspace layout apply reads."""
    return int(_native().embedding_segsort(v))


def radix_sort_tiled(v: int = -1) -> int:
    """Device-wide radix sort variant: 0 1024-item tiles / 10-bit digits,
    1 4096-item tiles / <=8-bit digits from 2^19 keys up (default), 2 always
    4096-item tiles; v < 0 only reads it. Returns the previous one."""
    return int(_native().radix_sort_tiled(v))


def effective_segsort(segsort: int) -> int:
    return int(segsort) if segsort and embedding_segsort() else 0


def linear_xent_impl(p: int = -1) -> int:
    """Fused Linear+CE kernel family: 2 3-pass bf16 MFMA (default; env
    TDFO_XENT_IMPL), 1 f32-input MFMA, 0 VALU; p < 0 only reads it. Returns
    the previous one."""
    return int(_native().linear_xent_impl(p))


def linear_fwd(x, w, bias=None, relu=False, out=None):
    """out = act(x @ w^T + bias); x [M,K] bf16, w [N,K] bf16."""
    if out is None:
        out = torch.empty(x.shape[0], w.shape[0], dtype=torch.bfloat16, device=x.device)
    gemm(x, False, w, False, bias, relu, None, out, None, 1)
    return out


def linear_dgrad(dy, w, mask=None, out=None):
    """out = (dy @ w) * (mask > 0); dy [M,N], w [N,K]."""
    if out is None:
        out = torch.empty(dy.shape[0], w.shape[1], dtype=torch.bfloat16, device=dy.device)
    gemm(dy, False, w, True, None, False, mask, out, None, 1)
    return out


# split-K block target for weight grads (DLRMTrainer passes its own per
# workload: profiles/gemm_step_ab.md). Round-1 in-step A/B (XCD-remapped split-K,
# direct fp32 slab stores): DLRM 0.621 ms at 256 vs 0.636-0.641 at 512, 0.646
# at 1024, 0.670 at 128; DCN-v2 2.902 vs 3.003 (512), 3.200 (128).
_WGRAD_TARGET = 512
_WGRAD_MINKT = 8


def wgrad_splits(M: int, N: int, K: int, target_blocks: int = 0, slots: int = 0) -> int:
    """Split-K count for a weight-grad GEMM (K = batch): ~target_blocks blocks
    of 128x128 tiles, but every split keeps >= 8 K tiles (measured on
    MI355X: bot/top3 wgrads run 18.8 us at 16 splits vs 22.7 us at 64; top1
    is best at 8).

    slots > 0: the GEMM runs on the 256x128 one-block-per-CU kernel (DCN-v2,
    GEMM policy 5) with `slots` resident blocks. A 128x128-tile target then
    leaves CUs idle (U wgrad: 70 tiles x 2 splits = 140 blocks), so the split
    minimises (block rounds x K tiles per split) + the fp32 slab traffic each
    extra split adds (written here, read by the optimizer / reduce; priced in
    K-tile times of ~0.6 us at ~5 TB/s)."""
    kt = K // 64
    # (round 5: K ranges down to 2 tiles for the few-tile bottom-0 / bottom-2
    # weight grads measured slower in the DLRM-1TB step, 0.435-0.436 vs
    # 0.429-0.431 ms, profiles/r05/notes.md)
    smax = max(1, kt // _WGRAD_MINKT)
    if slots > 0:
        tiles = ((M + 255) // 256) * ((N + 127) // 128)
        pen = M * N * 8 / 5e12 / 0.6e-6
        best, best_s = None, 1
        for s in range(1, smax + 1):
            cost = -(-tiles * s // slots) * -(-kt // s) + pen * (s - 1)
            if best is None or cost < best:
                best, best_s = cost, s
        return best_s
    target_blocks = target_blocks or _WGRAD_TARGET
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    return max(1, min(smax, -(-target_blocks // tiles)))

def linear_wgrad(dy, x, out, slab=None, splits=None, accumulate=False):
    """out[N,K] (fp32) = dy^T @ x with dy [M,N], x [M,K]; split-K over M."""
    N, K, M = dy.shape[1], x.shape[1], dy.shape[0]
    if splits is None:
        splits = wgrad_splits(N, K, M)
    if splits == 1 and not accumulate:
        gemm(dy, True, x, True, None, False, None, None, out, 1)
        return out
    if slab is None:
        slab = torch.empty(splits * N * K, dtype=torch.float32, device=dy.device)
    gemm(dy, True, x, True, None, False, None, None, slab, splits)
    reduce_rows(slab, splits, N * K, N * K, out, accumulate, 1.0)
    return out


def interaction_fwd(dense, emb, off, stride, F, D, out, ones_col=-1):
    if _gpu(dense):
        _native().interaction_fwd(dense, emb, list(off), list(stride), F, D, out, ones_col)
    else:
        ref.interaction_fwd(dense, emb, off, stride, F, D, out, ones_col)


def interaction_bwd(dz, dense, emb, off, stride, F, D, d_dense, d_emb, doff, dstride, relu_mask):
    if _gpu(dz):
        _native().interaction_bwd(dz, dense, emb, list(off), list(stride), F, D, d_dense, d_emb,
                                  list(doff), list(dstride), relu_mask)
    else:
        ref.interaction_bwd(dz, dense, emb, off, stride, F, D, d_dense, d_emb, doff, dstride,
                            relu_mask)


def embedding_bag_fwd(W, row_offset, indices, offsets, out_off, T, B, out, out_stride, mean=False,
                      psw=None, onehot=False, bumps=()):
    """onehot=True promises offsets == arange (one id per bag): the kernel then
    skips the offsets loads and keeps two bags' row gathers in flight.
    ``bumps``: fp32 / int64 step counters advanced by one inside the launch."""
    bumps = list(bumps)
    if _gpu(W):
        _native().embedding_bag_fwd(W, row_offset, indices, offsets, out_off, psw, T, B, mean, out,
                                    out_stride, bool(onehot), bumps)
    else:
        ref.embedding_bag_fwd(W, row_offset, indices, offsets, out_off, psw, T, B, mean, out,
                              out_stride)
        for t in bumps:
            t.view(-1)[:1].add_(1)


def embedding_bwd(W, row_offset, indices, offsets, grad_off, T, B, grad, grad_stride, opt, hyper,
                  state1=None, state2=None, eps=1e-8, beta1=0.9, beta2=0.999, weight_decay=0.0,
                  key_bits=None, mean=False, psw=None, dense_grad=None, segsort=0):
    """Fused sort-based backward + optimizer. segsort=R > 0 promises one id
    per bag and that the T virtual tables are R runs (run-major) of T/R
    physical tables, only runs of the same table sharing rows; then per-table
    LDS sorts (+ a run merge for R > 1) replace the device-wide radix sort."""
    if key_bits is None:
        key_bits = key_bits_for(W.shape[0])
    if _gpu(W):
        segsort = effective_segsort(segsort)
        _native().embedding_bwd(W, row_offset, indices, offsets, grad_off, psw, T, B, mean,
                                key_bits, grad, grad_stride, opt, state1, state2, hyper, eps,
                                beta1, beta2, weight_decay, dense_grad, int(segsort))
    else:
        ref.embedding_bwd(W, row_offset, indices, offsets, grad_off, psw, T, B, mean, key_bits,
                          grad, grad_stride, opt, state1, state2, hyper, eps, beta1, beta2,
                          weight_decay, dense_grad)


def embedding_bwd_workspace(nnz: int, D: int) -> int:
    return int(_native().embedding_bwd_workspace(int(nnz), int(D)))


def embedding_bwd_prepare(W, row_offset, indices, offsets, grad_off, T, B, grad_stride, workspace,
                          key_bits=None, mean=False, psw=None, segsort=0, bag_len=None):
    """First half of the fused embedding backward (GPU): keys, sort and
    gradient offsets into ``workspace`` -- needs only the ids, so it can run
    on a side stream before the gradient exists. ``bag_len`` (int32 [T],
    optional): every bag of virtual table v holds bag_len[v] ids (fixed
    multi-hot) -- the keys pass then divides instead of searching."""
    if key_bits is None:
        key_bits = key_bits_for(W.shape[0])
    _native().embedding_bwd_prepare(W, row_offset, indices, offsets, grad_off, psw, T, B, mean,
                                    key_bits, grad_stride, int(segsort), workspace, bag_len)


def embedding_bwd_apply(W, row_offset, indices, offsets, grad_off, T, B, grad, grad_stride, opt,
                        hyper, workspace, state1=None, state2=None, eps=1e-8, beta1=0.9,
                        beta2=0.999, weight_decay=0.0, key_bits=None, mean=False, psw=None,
                        dense_grad=None, segsort=0):
    """Second half: segment reduction + optimizer from a prepared workspace."""
    if key_bits is None:
        key_bits = key_bits_for(W.shape[0])
    _native().embedding_bwd_apply(W, row_offset, indices, offsets, grad_off, psw, T, B, mean,
                                  key_bits, grad, grad_stride, opt, state1, state2, hyper, eps,
                                  beta1, beta2, weight_decay, dense_grad, int(segsort), workspace)


def embedding_dense_update(W, grad, rows, opt, hyper, state1=None, state2=None, eps=1e-8,
                           beta1=0.9, beta2=0.999, weight_decay=0.0, clear_grad=False):
    """Optimizer step over rows [0, rows) of W from a dense fp32 gradient
    (data-parallel tables after their gradient all-reduce). ``clear_grad``:
    zero grad rows [0, rows) as they are read (also on a skipped step)."""
    if _gpu(W):
        _native().embedding_dense_update(W, grad, int(rows), int(opt), state1, state2, hyper, eps,
                                         beta1, beta2, weight_decay, bool(clear_grad))
    else:
        ref.embedding_dense_update(W, grad, rows, opt, state1, state2, hyper, eps, beta1, beta2,
                                   weight_decay)
        if clear_grad:
            grad.view(-1)[: int(rows) * W.shape[1]].zero_()


def rw_bucketize_workspace(n: int, W: int) -> int:
    return int(_native().rw_bucketize_workspace(int(n), int(W))) if native_available() else 1


def rw_bucketize(ids, meta, nrw, W, B, cap, n, send, workspace, overflow):
    """Row-wise bucketize into fixed-capacity per-owner segments (see
    csrc/include/tdfo_kernels.h, "row-wise shards")."""
    if _gpu(ids):
        _native().rw_bucketize(ids, meta, int(nrw), int(W), int(B), int(cap), int(n), send,
                               workspace, overflow)
    else:
        ref.rw_bucketize(ids, meta, nrw, W, B, cap, n, send, overflow)


def rw_pool(Wt, recv, meta, nrw, W, B, cap, mean, starts, out, out_ld):
    if _gpu(Wt):
        _native().rw_pool(Wt, recv, meta, int(nrw), int(W), int(B), int(cap), bool(mean), starts,
                          out, int(out_ld))
    else:
        ref.rw_pool(Wt, recv, meta, nrw, W, B, cap, mean, out, out_ld)


def embedding_bwd_prepare_rw(Wt, recv, meta, nrw, W, B, cap, mean, key_bits, grad_ld, dummy_row,
                             workspace, rows=False):
    """GPU: keys + sort of the received row-wise entries (ids only). CPU: no-op
    (``embedding_bwd_apply_rw`` does everything). ``rows``: the gradients
    arrive per slot ([W][cap + 1][grad_ld], the "rows" exchange)."""
    if _gpu(Wt):
        _native().embedding_bwd_prepare_rw(Wt, recv, meta, int(nrw), int(W), int(B), int(cap),
                                           bool(mean), int(key_bits), int(grad_ld),
                                           int(dummy_row), workspace, int(bool(rows)))


def embedding_bwd_apply_rw(Wt, recv, meta, nrw, W, B, cap, mean, key_bits, grad, grad_ld, opt,
                           hyper, workspace, state1=None, state2=None, eps=1e-8, beta1=0.9,
                           beta2=0.999, weight_decay=0.0, rows=False):
    if _gpu(Wt):
        _native().embedding_bwd_apply_rw(Wt, int(W), int(B), int(cap), bool(mean), int(key_bits),
                                         grad, int(opt), state1, state2, hyper, eps, beta1, beta2,
                                         weight_decay, workspace)
    else:
        ref.rw_embedding_bwd(Wt, recv, meta, nrw, W, B, cap, mean, grad, grad_ld, opt, state1,
                             state2, hyper, eps, beta1, beta2, weight_decay, rows=rows)


def rw_rows_gather(Wt, recv, W, cap, out):
    """One-hot row-wise "rows" exchange, owner side: bf16 row per received
    entry into ``out`` [W][cap + 1][D] (csrc/kernels/rowwise.hip)."""
    if _gpu(Wt):
        _native().rw_rows_gather(Wt, recv, int(W), int(cap), out)
    else:
        ref.rw_rows_gather(Wt, recv, W, cap, out)


def rw_rows_scatter(send, W, cap, B, D, rows, region, ld, smap, nrw):
    """Requester side: received rows into the pooled region (row stride
    ``ld``) and the slot -> offset map the backward gathers with."""
    if _gpu(send):
        _native().rw_rows_scatter(send, int(W), int(cap), int(B), int(D), rows, region, int(ld),
                                  smap, int(nrw))
    else:
        ref.rw_rows_scatter(send, W, cap, B, D, rows, region, ld, smap, nrw)


def rw_grads_gather(smap, W, cap, D, dregion, gsend):
    """Requester side of the backward: each slot's gradient row, [W][cap + 1][D]."""
    if _gpu(smap):
        _native().rw_grads_gather(smap, int(W), int(cap), int(D), dregion, gsend)
    else:
        ref.rw_grads_gather(smap, W, cap, D, dregion, gsend)


def dense_optimizer(p, g, m, v, p_bf16, opt, hyper, beta1=0.9, beta2=0.999, eps=1e-8, wd=0.0,
                    momentum=0.0, found_inf=None, segments=()):
    """Fused flat optimizer. ``segments``: (start, slab, splits) triples whose
    elements take sum_s slab.view(splits, -1)[s] as their gradient (split-K
    weight-grad partials reduced inside the optimizer pass)."""
    if _gpu(p):
        _native().dense_optimizer(p, g, m, v, p_bf16, opt, hyper, beta1, beta2, eps, wd, momentum,
                                  found_inf, [s[1] for s in segments],
                                  [int(s[0]) for s in segments], [int(s[2]) for s in segments])
    else:
        if segments:
            g = g.clone()
            for start, slab, splits in segments:
                n = slab.numel() // splits
                g[start:start + n] = slab.view(splits, n).sum(0)
        ref.dense_optimizer(p, g, m, v, p_bf16, opt, hyper, beta1, beta2, eps, wd, momentum,
                            found_inf)


def check_finite(g, found):
    if _gpu(g):
        _native().check_finite(g, found)
    else:
        ref.check_finite(g, found)


def head_parts(B: int) -> int:
    return (B + 15) // 16


def head_bce(H, w, b, label, inv_n, relu_mask, logits, dH, part):
    if _gpu(H):
        _native().head_bce(H, w, b, label, inv_n, relu_mask, logits, dH, part)
    else:
        ref.head_bce(H, w, b, label, inv_n, relu_mask, logits, dH, part)


def reduce_rows(inp, rows, n, ld, out, accumulate=False, scale=1.0):
    if _gpu(inp):
        _native().reduce_rows(inp, rows, n, ld, out, accumulate, scale)
    else:
        ref.reduce_rows(inp, rows, n, ld, out, accumulate, scale)


class SegmentMap:
    """A static permutation of an int64 buffer made of contiguous pieces
    ``(src_off, dst_off, length)``: ``apply(src, dst)`` copies every piece in
    one native launch on the GPU (seg_copy_kernel: one block per <= 4096-id
    chunk, offsets from a device table built here once), or one index_select
    on the CPU."""

    CHUNK = 4096

    def __init__(self, pieces, device):
        self.device = torch.device(device)
        pieces = [(int(a), int(b), int(n)) for a, b, n in pieces if int(n) > 0]
        self.src_n = max([a + n for a, _, n in pieces], default=0)
        self.dst_n = max([b + n for _, b, n in pieces], default=0)
        self.n = sum(n for _, _, n in pieces)
        if self.device.type == "cuda":
            ch = []
            for a, b, n in pieces:
                for o in range(0, n, self.CHUNK):
                    ch.append((a + o, b + o, min(self.CHUNK, n - o)))
            self.chunks = torch.tensor(ch if ch else [[0, 0, 0]], dtype=torch.int64,
                                       device=self.device).view(-1, 3)
            self.nchunks = len(ch)
        else:
            idx = torch.zeros(self.dst_n, dtype=torch.int64)
            for a, b, n in pieces:
                idx[b:b + n] = torch.arange(a, a + n)
            self.index = idx

    def apply(self, src: torch.Tensor, dst: torch.Tensor):
        if src.is_cuda:
            if self.nchunks:
                _native().seg_copy(src, dst, self.chunks, self.src_n, self.dst_n)
        else:
            torch.index_select(src, 0, self.index, out=dst[:self.dst_n])

    @staticmethod
    def from_index(index: torch.Tensor, device):
        """The pieces of a gather index that is a union of contiguous runs."""
        ix = index.to("cpu", torch.int64).view(-1)
        pieces, start = [], 0
        for i in range(1, ix.numel() + 1):
            if i == ix.numel() or int(ix[i]) != int(ix[i - 1]) + 1:
                pieces.append((int(ix[start]), start, i - start))
                start = i
        return SegmentMap(pieces, device)


class PieceCopy:
    """Static B x w block copies between strided views of one bf16 buffer,
    pieces ``(src_off, src_ld, dst_off, dst_ld)`` in elements: one native
    launch for all of them on the GPU (piece_copy_kernel), strided torch
    copies on the CPU. ``reverse()`` swaps source and destination."""

    def __init__(self, pieces, B: int, w: int, device):
        self.pieces = [tuple(int(v) for v in p) for p in pieces]
        self.B, self.w = int(B), int(w)
        self.device = torch.device(device)
        self.extent = max([max(a + (self.B - 1) * la, c + (self.B - 1) * lc) + self.w
                           for a, la, c, lc in self.pieces], default=0)
        if self.device.type == "cuda" and self.pieces:
            ok = self.w % 8 == 0 and all(v % 8 == 0 for p in self.pieces for v in p)
            if not ok:
                raise ValueError("PieceCopy: offsets, strides and width must be multiples of 8")
            self.table = torch.tensor(self.pieces, dtype=torch.int64, device=self.device)

    def reverse(self) -> "PieceCopy":
        return PieceCopy([(c, lc, a, la) for a, la, c, lc in self.pieces], self.B, self.w,
                         self.device)

    def apply(self, buf: torch.Tensor):
        if not self.pieces:
            return
        if buf.is_cuda:
            _native().piece_copy(buf, self.table, self.B, self.w, self.extent)
            return
        for a, la, c, lc in self.pieces:
            buf.as_strided((self.B, self.w), (lc, 1), c).copy_(
                buf.as_strided((self.B, self.w), (la, 1), a))


def slab_reduce(segs):
    """segs: [(slabs, S, out)]: out = sum of the S consecutive out-sized fp32
    slabs in ``slabs`` (split order), every segment in one launch."""
    if not segs:
        return
    if _gpu(segs[0][0]):
        for i in range(0, len(segs), 16):
            part = segs[i:i + 16]
            _native().slab_reduce([x[0] for x in part], [int(x[1]) for x in part],
                                  [x[2] for x in part])
    else:
        for sl, S, out in segs:
            n = out.numel()
            out.view(-1).copy_(sl.view(-1)[:S * n].view(S, n).sum(0))


def head_reduce(part, nparts, K, grad, loss_acc, bumps=(), defer=False):
    """grad[:K+1] = column sums of part[:, :K+1]; loss_acc += sum part[:, K+1];
    bump[1] += 1 for each step-counter vector in ``bumps`` (one launch).
    ``defer`` (GPU): run by extra blocks of the next paired 128x128 GEMM
    launch (the first top-MLP backward pair); ``flush_side_job()`` launches it
    if none took it."""
    if _gpu(part):
        _native().head_reduce(part, int(nparts), int(K), grad, loss_acc, list(bumps),
                              bool(defer))
    else:
        ref.head_reduce(part, nparts, K, grad, loss_acc, bumps)


def colsum(x, out, accumulate=False):
    if _gpu(x):
        _native().colsum(x, out, accumulate)
    else:
        ref.colsum(x, out, accumulate)


def auc_hist(logits, labels, nb, hist):
    if _gpu(logits):
        _native().auc_hist(logits, labels, nb, hist)
    else:
        ref.auc_hist(logits, labels, nb, hist)


def cast_bf16(x, y):
    if _gpu(x):
        _native().cast_bf16(x, y)
    else:
        ref.cast_bf16(x, y)


def synth_criteo(seed, rank, batch_index, B, rows, pooling, base, dist, alpha, w_dense,
                 table_bias, dense, ids, label):
    """One fresh synthetic Criteo batch on the device (csrc/kernels/synthetic.hip),
    the twin of the C++ host generator; GPU only."""
    n = int(sum(int(B) * int(x) for x in pooling.tolist())) if not pooling.is_cuda else None
    if n is not None and ids.numel() != n:
        raise ValueError(f"synth_criteo: ids has {ids.numel()} entries, batch needs {n}")
    _native().synth_criteo(int(seed), int(rank), int(batch_index), int(B), rows, pooling, base,
                           int(dist), float(alpha), w_dense, table_bias, dense, ids, label)


def stamp(buf, cnt, seg: int, nseg: int, which: int):
    """Device timestamp of segment ``seg``'s current run (see stamp_kernel)."""
    _native().stamp(buf, cnt, int(seg), int(nseg), int(which))


def bump(counters):
    """counters[i].view(-1)[0] += 1 for each float32 / int64 tensor (one launch
    on the GPU)."""
    counters = list(counters)
    if counters and _gpu(counters[0]):
        _native().bump(counters)
    else:
        for t in counters:
            t.view(-1)[:1].add_(1)


def burn_us(us: float):
    """MFMA load on every CU for ``us`` microseconds (device warm-up)."""
    _native().burn_us(float(us))


def spin_us(us: float):
    """Occupy the current stream for ``us`` microseconds (one sleeping wave):
    the modelled link time of an emulated collective."""
    _native().spin_us(float(us))


def batch_load(dense, x0, ids, ids_dst, label, label_dst):
    """x0[:, :nd] = bf16(dense), ids_dst = ids, label_dst = label (one launch on GPU)."""
    # the fused kernel needs fp32 row-major dense, int64 ids at a 16-B aligned
    # address, fp32 labels and exactly matching sizes; anything else copies
    if (_gpu(x0) and dense.is_cuda and ids.is_cuda and label.is_cuda
            and dense.dtype == torch.float32 and dense.dim() == 2 and dense.stride(-1) == 1
            and dense.shape[0] == x0.shape[0] and dense.shape[1] <= x0.shape[1]
            and ids.dtype == torch.int64 and ids.is_contiguous() and ids.data_ptr() % 16 == 0
            and ids.numel() == ids_dst.numel() and ids_dst.dtype == torch.int64
            and label.dtype == torch.float32 and label.numel() == label_dst.numel()
            and label_dst.dtype == torch.float32):
        _native().batch_load(dense, x0, ids.contiguous(), ids_dst, label.contiguous(), label_dst)
    else:
        x0[:, :dense.shape[1]].copy_(dense, non_blocking=True)
        ids_dst.copy_(ids, non_blocking=True)
        label_dst.copy_(label, non_blocking=True)


def concat_features(dense, emb, off, stride, F, D, out):
    if _gpu(dense):
        _native().concat_features(dense, emb, list(off), list(stride), F, D, out)
    else:
        ref.concat_features(dense, emb, off, stride, F, D, out)


def split_features(dx, F, D, dense, d_dense, d_emb, doff, dstride, relu_mask):
    if _gpu(dx):
        _native().split_features(dx, F, D, dense, d_dense, d_emb, list(doff), list(dstride),
                                 relu_mask)
    else:
        ref.split_features(dx, F, D, dense, d_dense, d_emb, doff, dstride, relu_mask)


def cross_bwd(dout, x0, y, dy, dx0, accumulate, add_dout=False):
    if _gpu(dout):
        _native().cross_bwd(dout, x0, y, dy, dx0, accumulate, add_dout)
    else:
        ref.cross_bwd(dout, x0, y, dy, dx0, accumulate, add_dout)


def sort_pairs(keys, vals, key_bits):
    """Stable radix sort of (keys, int32 vals) on the low key_bits bits."""
    if _gpu(keys):
        return _native().sort_pairs(keys, vals, key_bits)
    mask = (1 << key_bits) - 1
    k = keys & mask if key_bits < 63 else keys
    order = torch.sort(k, stable=True).indices
    return keys[order], vals[order]


TT_NPARAM = ref.TT_NPARAM
TT_PART_LD = ref.TT_PART_LD


def two_tower_parts(B: int) -> int:
    return (B + ref.TT_SPB - 1) // ref.TT_SPB


def flush_side_job():
    """Launch a ``two_tower(defer=True)`` / ``reduce_adam(defer=True)`` job no
    embedding backward took (GPU callers only: deferral exists on the native
    path)."""
    _native().flush_side_job()


def two_tower(X, P, labels, inv_n, logits, dX=None, part=None, loss_scale=None, half=False,
              bumps=(), emb=None, defer=False):
    """Fused TwoTower forward (+ BCE + backward when dX/part given).
    ``half``: fp16 compute (mixed precision); ``loss_scale``: device scalar
    multiplying the loss gradient (dynamic loss scaling). ``bumps`` (train):
    step counters ([lr, step, ...]) advanced by one inside the launch.
    ``emb = (weight [rows, 16], ids [7 * B] table-major, row_offset [7])``:
    the kernel gathers X[:, :112] itself (X then holds only the two dense
    features) -- the lookup launch folded in. ``defer`` (GPU, fp32 train
    step): co-launched with the next ``embedding_bwd``'s per-table sort (or
    launched first by it); ``flush_side_job()`` after that backward."""
    bumps = list(bumps)
    if _gpu(X):
        w, ids, ro = emb if emb is not None else (None, None, None)
        _native().two_tower(X, P, labels, float(inv_n), logits, dX, part, loss_scale, bool(half),
                            bumps, w, ids, ro, bool(defer))
    else:
        if emb is not None:
            w, ids, ro = emb
            B = X.shape[0]
            X = X.clone()
            for t in range(7):
                X[:, 16 * t:16 * (t + 1)] = w[ro[t] + ids[t * B:(t + 1) * B]]
        ref.two_tower(X, P, labels, inv_n, logits, dX, part, loss_scale, half)
        for b in bumps:
            b[1:2] += 1.0


def reduce_adam(part, nparts, n, ld, grad, p, m, v, hyper, beta1=0.9, beta2=0.999, eps=1e-8,
                wd=0.0, adamw=True, loss_acc=None, logits=None, labels=None, nb=0, hist=None,
                defer=False):
    """grad[:n + 1] = fixed-order sum of ``nparts`` partial rows (stride ``ld``),
    one Adam(W) step of p[:n] from grad[:n] and loss_acc (fp64) += grad[n]:
    ``reduce_rows`` + ``dense_optimizer`` + the loss add in one launch; with
    ``hist`` also ``auc_hist(logits, labels, nb, hist)`` (a block of its own).
    ``defer`` (GPU): run it as side blocks of the next ``embedding_bwd``'s
    sort launch instead (it reads nothing that backward writes); call
    ``flush_side_job()`` after that backward (launches it if none took it)."""
    if _gpu(part):
        _native().reduce_adam(part, int(nparts), int(n), int(ld), grad, p, m, v, hyper,
                              float(beta1), float(beta2), float(eps), float(wd), bool(adamw),
                              loss_acc, logits, labels, int(nb), hist, bool(defer))
    else:
        if hist is not None:
            ref.auc_hist(logits, labels, nb, hist)
        ref.reduce_rows(part, nparts, n + 1, ld, grad, False, 1.0)
        loss_acc += grad[n:n + 1].double()
        ref.dense_optimizer(p[:n], grad[:n], m[:n], v[:n], None, OPT_ADAMW if adamw else OPT_ADAM,
                            hyper, beta1, beta2, eps, wd, 0.0, None)


def linear_xent(H, W, bias, labels, eps, ignore, dH, lossv, dW=None, db=None, loss=None,
                loss_acc=None, step=None):
    """Fused Linear(16->V) + label-smoothed CrossEntropy, fwd+bwd (no logits).
    loss (fp32 [1]): mean loss over the non-ignored tokens; loss_acc (fp64
    [1]): += that loss (device running sum). step = (opt, [mW, vW, mb, vb],
    hyper, beta1, beta2, eps, weight_decay): apply the flat optimizer's
    Adam / AdamW step to W and bias in place inside the kernels (dW / db are
    then scratch and are not the gradient on return)."""
    if _gpu(H):
        if step is None:
            _native().linear_xent(H, W, bias, labels, float(eps), int(ignore), dH, lossv, dW, db,
                                  loss, loss_acc, [], None, [], -1)
        else:
            opt, st, hyper, b1, b2, oeps, wd = step
            _native().linear_xent(H, W, bias, labels, float(eps), int(ignore), dH, lossv, dW, db,
                                  loss, loss_acc, list(st), hyper,
                                  [float(b1), float(b2), float(oeps), float(wd)], int(opt))
    else:
        ref.linear_xent(H, W, bias, labels, eps, ignore, dH, lossv, dW, db)
        if loss is not None:
            nv = (labels != ignore).sum().clamp_min(1).to(torch.float32)
            loss.view(-1)[0] = lossv.sum() / nv
            if loss_acc is not None:
                loss_acc.view(-1)[0] += loss.view(-1)[0].double()
        if step is not None:
            opt, st, hyper, b1, b2, oeps, wd = step
            for p, g, m, v in ((W, dW, st[0], st[1]), (bias, db, st[2], st[3])):
                ref.dense_optimizer(p.view(-1), g.view(-1), m.view(-1), v.view(-1), None, opt,
                                    hyper, b1, b2, oeps, wd, 0.0, None)


def jagged_to_dense(values, offsets, T, pad, out):
    """values [nnz, D] fp32 + offsets [B+1] -> out [B, T, D] (pad fill)."""
    if _gpu(values):
        _native().jagged_to_dense(values, offsets, int(T), float(pad), out)
    else:
        ref.jagged_to_dense(values, offsets, T, pad, out)


def dense_to_jagged(dense, offsets, vgrad):
    if _gpu(dense):
        _native().dense_to_jagged(dense, offsets, vgrad)
    else:
        ref.dense_to_jagged(dense, offsets, vgrad)


def jagged_ids_to_dense(values, offsets, pad, out):
    if _gpu(values):
        _native().jagged_ids_to_dense(values, offsets, int(pad), out)
    else:
        ref.jagged_ids_to_dense(values, offsets, pad, out)


def attention_fwd(qkv, ids, H, rate, seed, step, pad_id, out):
    """Fused small-T MHA core: qkv [B,T,3E] fp32 -> out [B,T,E] (key-padding
    mask from ids != pad_id, hash dropout keyed by (seed, step[0]))."""
    if _gpu(qkv):
        _native().attention_fwd(qkv, ids, int(H), float(rate), int(seed), step, int(pad_id), out)
    else:
        ref.attention_fwd(qkv, ids, H, rate, seed, step, pad_id, out)


def attention_bwd(qkv, ids, dout, H, rate, seed, step, pad_id, dqkv):
    if _gpu(qkv):
        _native().attention_bwd(qkv, ids, dout, int(H), float(rate), int(seed), step,
                                int(pad_id), dqkv)
    else:
        ref.attention_bwd(qkv, ids, dout, H, rate, seed, step, pad_id, dqkv)


def layernorm_parts(M: int) -> int:
    return int(_native().layernorm_parts(int(M))) if native_available() else 1


def layernorm_fwd(x, n, eps, gamma, beta, y, mean, rstd):
    if _gpu(x):
        _native().layernorm_fwd(x, int(n), float(eps), gamma, beta, y, mean, rstd)
    else:
        ref.layernorm_fwd(x, n, eps, gamma, beta, y, mean, rstd)


def rank_metrics(h, W, bias, cand, ks, out):
    """out[2 len(ks) + 1] = per-batch sums of [Recall@k.. | NDCG@k.. | count]
    for candidates cand [B, C] (column 0 = positive) scored h . W[c] + b[c]."""
    if _gpu(h):
        _native().rank_metrics(h, W, bias, cand, list(ks), out)
    else:
        ref.rank_metrics(h, W, bias, cand, ks, out)


def seq_prologue_fwd(x, pos, n, eps, gamma, beta, rate, seed, step, y, mean, rstd):
    """y = dropout(LN(x + pos)) over rows of n (Bert4Rec input block); the
    dropout mask is a counter hash of (seed, step[0], row, element)."""
    if _gpu(x):
        _native().seq_prologue_fwd(x, pos, int(n), float(eps), gamma, beta, float(rate),
                                   int(seed) & 0xFFFFFFFF, step, y, mean, rstd)
    else:
        ref.seq_prologue_fwd(x, pos, n, eps, gamma, beta, rate, seed, step, y, mean, rstd)


def seq_prologue_bwd(x, pos, g, n, gamma, mean, rstd, rate, seed, step, dx, part, out3,
                     gidx=None):
    """dx and out3 = [dgamma | dbeta | dpos] (3n) of seq_prologue_fwd; with
    ``gidx`` element j of that goes to out3[gidx[j]] (a flat gradient buffer)."""
    if _gpu(x):
        _native().seq_prologue_bwd(x, pos, g, int(n), gamma, mean, rstd, float(rate),
                                   int(seed) & 0xFFFFFFFF, step, dx, part, out3, gidx)
    elif gidx is not None:
        tmp = torch.empty(3 * n, dtype=torch.float32, device=x.device)
        ref.seq_prologue_bwd(x, pos, g, n, gamma, mean, rstd, rate, seed, step, dx, tmp)
        out3.index_copy_(0, gidx, tmp)
    else:
        ref.seq_prologue_bwd(x, pos, g, n, gamma, mean, rstd, rate, seed, step, dx, out3)


def layernorm_bwd(x, g, n, gamma, mean, rstd, dx, part, dgb):
    """dgb [2n] = [dgamma | dbeta]; part: layernorm_parts(M) * 2n scratch (GPU)."""
    if _gpu(x):
        _native().layernorm_bwd(x, g, int(n), gamma, mean, rstd, dx, part, dgb)
    else:
        ref.layernorm_bwd(x, g, n, gamma, mean, rstd, dx, dgb)


def gather_columns(src, idx, row0, n, dst, dst_stride):
    """dst[c].flatten()[i * dst_stride[c]] = src[c][idx[i] if idx is not None else row0 + i]
    (dtype-converting, one launch for all columns on GPU)."""
    if _gpu(src[0]):
        _native().gather_columns(list(src), idx, int(row0), int(n), list(dst),
                                 [int(s) for s in dst_stride])
    else:
        for s, d, st in zip(src, dst, dst_stride):
            v = s.index_select(0, idx[:n]) if idx is not None else s[row0: row0 + n]
            d.view(-1)[: (n - 1) * st + 1: st].copy_(v.to(d.dtype)) if n else None
