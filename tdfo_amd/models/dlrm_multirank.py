"""Multi-rank DLRM / DCN-v2 step as per-stream hipGraphs with the RCCL
collectives inside (mixin of ``DLRMTrainer``; W > 1, pipelined input dist).

Why this shape (all measured on this ROCm, labs/probes/rccl_capture_probe.py and
labs/probes/whole_capture_bisect.py):

* RCCL can only be captured on the capture's ORIGIN stream: a collective on a
  stream forked into a capture (torch's own async c10d collectives included)
  makes hipStreamEndCapture segfault, as does any fork whose source is itself
  a forked stream.
* One captured graph's independent branches are replayed mostly in order, so
  a single whole-step graph serialises the embedding work behind the MLP
  (emulated W=8: 0.95 ms/step vs 0.91 for the staged replay).

So each stream's share of the step is captured as segments with THAT stream
as origin (no forks at all), and the segments of a stream are chained with
explicit event record / wait nodes into one executable graph
(``ops.ComposedGraph``), launched on its own stream -- three launches per
step instead of ~20 Python stage issues and ~8 c10d calls:

  M  (MLP):      [wait dpp'] bottom fwd  [wait c5', d'] top fwd/bwd + interaction bwd
                 (m2)  [wait stg] bottom bwd, next batch's load from staging
                 (m4)  top weight grads (m3)
  D  (dense      [wait c5'] ids-only sort of this batch (e0)  [wait stg] next
      comm):     batch's sharded-table ids bucketed from the staging, row-wise
                 need all-reduced + published to the host (pre)  [wait m2]
                 replicated tables' dense grad + all-reduce + update (dp)
                 [wait m4] bottom-bucket all-reduce, next batch's replicated
                 ids, bottom-bucket optimizer (dpp)  [wait m3] top-bucket
                 all-reduce, top-bucket optimizer (d)
  EC (embedding  [wait m2] gradient all-to-all  [wait e0, dp] fused embedding
      + its      update  [wait pre, dpp] id all-to-all, lookup + pooled
      RCCL):     all-to-all (c5)

(stg: recorded by the host on the current stream after it staged the next
batch; TDFO_MR_EARLY_PREP=0 moves the bucketize back into M4 and the publish
into D's bottom-bucket segment.)

(primed events: the previous step's records). The embedding exchanges and
the dense all-reduces use two communicators so they run concurrently (the
role of TorchRec's input/output dists beside the DDP reducer,
torchrec/train.py:241-260). A wait node binds to the most recent record
enqueued before its graph is launched, so the per-step launch order M, D, EC
makes M's waits see the previous step's records and D's / EC's this step's
(D's c5 wait: the previous step's, EC has not been launched yet).
"""
from __future__ import annotations

import os
import warnings

import torch

from .. import ops
from ..utils.capture import graph_capture


# A/B knob: TDFO_MR_HEAD_WAIT=1 restores the wait for the current stream at
# the head of M (the staged batch before the bottom forward)
_HEAD_WAIT = os.environ.get("TDFO_MR_HEAD_WAIT", "0") == "1"
# A/B knob: TDFO_MR_EARLY_PREP=0 buckets the next batch's sharded ids in M4
# (from the loaded ids) and publishes the row-wise need in Da, as before
_EARLY_PREP = os.environ.get("TDFO_MR_EARLY_PREP", "1") != "0"
# A/B knob: TDFO_MR_SORT_EC=1 runs the ids-only sort and the early prep on
# the embedding stream (EC idles until the interaction backward) instead of
# D (which then only carries the dense side)
_SORT_EC = os.environ.get("TDFO_MR_SORT_EC", "0") == "1"


class MultiRankStreamsMixin:
    """Per-stream graph capture / replay for W > 1 (``capture_graph`` picks it
    when ``_mr_ok()``)."""

    # segments that always hold work (bottom / top MLP, the dense buckets'
    # all-reduces + optimizer); the others may be empty for a plan (e.g. Dp
    # without replicated tables, D0 / EC1 without sharded ones)
    _MR_WORK = ("M1", "M2", "M4", "Da", "Db")

    def _mr_ok(self) -> bool:
        """Pipelined with the lookup in the tail and every exchange
        enqueue-only (native RCCL or loopback). Row-wise tables qualify: their
        capacity check is lagged (no host read inside the step; the host reads
        the need the previous replay published when it issues the next)."""
        return (self.world > 1 and self.cfg.stream_graphs and self._pipe_lookup
                and getattr(self.comm, "capturable", False)
                and getattr(self.dcomm, "capturable", False)
                and (not (self.emb.rw_tables and self.emb.rw_dynamic) or self._rw_lagged))

    def _mr_drain(self):
        """Complete every exchange left in flight by eager stages (prime(),
        eager steps): nothing crosses into the graphs."""
        self.emb.ids_exchange_wait()
        if self.emb._pending:
            self.emb.forward_wait()
        se = self._side()
        if se is not None:
            torch.cuda.current_stream().wait_stream(se)
        self._mr_inflight = False

    def _mr_segments(self):
        emb = self.emb
        hyper = self.emb_hyper
        dp_dense = bool(emb.dp_tables) and emb.dp_dense

        def m2():
            emb.forward_wait()                  # post-exchange assembly only
            self._s_top()

        def dp_a():                             # replicated tables: dense grad, all-reduce,
            emb.stage_bwd_local(hyper)          # update (all on D, beside the exchange)
            emb.backward_start(exchange=False)
            if dp_dense:
                emb.stage_bwd_update(hyper, sharded=False)

        def ec_upd():
            emb.backward_wait()                 # (handles of stream-ordered enqueues)
            emb.stage_bwd_update(hyper, dp=not dp_dense)

        def ec_b1():
            # (row-wise need published on D, right after the bucketize)
            emb.stage_fwd_ids_exchange(lagged=self._rw_lagged, publish=False)

        def ec_b2():
            # (replicated tables with a dense update: looked up on D, right
            # after their update and their ids, see d_prep; on EC instead the
            # emulated W=8 step ran the same and config 3 slower, 0.96 vs
            # 0.85 ms, profiles/r04/notes.md)
            emb.stage_fwd_lookup(dp=not dp_dense)
            emb.stage_fwd_out_exchange()

        split_opt = os.environ.get("TDFO_MR_SPLIT_OPT", "1") != "0"     # A/B knob

        def d_b():
            # the top bucket (top MLP, DCN cross layers, head): all-reduce,
            # then the optimizer on its range only
            self._m_allreduce_top_start()
            if split_opt:
                self._m_allreduce_wait(("_ar_top",))
                self._dense_update_range(self._ar_split, self.fp.p.numel())
            else:
                self._m_allreduce_wait()
                self._s_dense_update()

        early = _EARLY_PREP and not emb.tw_identity

        def m4():
            self._s_bottom_bwd()
            self._m_load_next()                 # x0 / labels / ids free: next batch in
            # ... and its sharded tables' ids bucketed for the id exchange
            # (their send buffers' last reader was the previous exchange)
            if not early:
                emb.stage_fwd_prep(self.ids, dp=False)

        sort_ec = _SORT_EC and early and dp_dense

        def pre(comm):
            # early prep: the next batch's sharded-table ids bucketed on D
            # (or EC) straight from the host staging, as soon as the previous
            # id exchange (c5') has released the send buffers, and the
            # row-wise need published right after -- early in the step
            # instead of after the bottom backward (M4), so the host, which
            # reads it before it issues the next step, is not held until
            # mid-step (the need's all-reduce on that stream's communicator)
            emb.stage_fwd_prep(self._stg[1], dp=False)
            if emb.rw_tables:
                emb._rw_ids = self.ids          # a redo re-reads the batch from ids (M4 loads it)
            if self._rw_lagged:
                emb.rw_publish_need(comm)

        def d_prep():                           # the replicated tables' ids, once their
            emb.stage_fwd_prep(self.ids, sharded=False)   # dense grad (Dp) has read them
            if dp_dense:                        # ... and their lookup (updated in Dp)
                emb.stage_fwd_lookup(sharded=False)

        def ec_b():
            ec_b1()
            ec_b2()

        def d_a():
            # the next batch's all-reduced row-wise need to the host mailbox
            # first (the host reads it when it issues the next step), then the
            # bottom bucket and the replicated tables' ids
            if self._rw_lagged and not early:
                emb.rw_publish_need(self.dcomm)
            self._m_allreduce_start()
            d_prep()
            # DDP-style split of the dense optimizer: the bottom bucket is
            # updated as soon as its all-reduce lands, so the next step's
            # bottom forward (M1, waiting on dpp) runs while the top bucket
            # is still being reduced (before: M1 waited for the whole
            # optimizer behind the top bucket, profiles/r04/prof_w8r1_lanes)
            if split_opt:
                self._m_allreduce_wait(("_ar_work",))
                self._dense_update_range(0, self._ar_split)

        return {"M1": self._s_bottom_fwd, "M2": m2, "M4": m4,
                "M3": self._s_top_wgrad if self._defer_top_wgrad else None,
                "D0": None if sort_ec else emb.stage_bwd_prepare,
                "Dpre": (lambda: pre(self.dcomm)) if early and not sort_ec else None,
                "ECs": emb.stage_bwd_prepare if sort_ec else None,
                "ECpre": (lambda: pre(self.comm)) if sort_ec else None,
                "Dp": dp_a,
                "Da": d_a,
                "Db": d_b, "EC1": lambda: emb.backward_start(dp=False),
                "ECub": lambda: (ec_upd(), ec_b())}

    def _mr_capture(self, restage: bool = True):
        split_opt = os.environ.get("TDFO_MR_SPLIT_OPT", "1") != "0"
        """``restage`` False (re-capture between steps): keep the staging
        buffers and the next batch already staged in them."""
        assert self.device.type == "cuda"
        dev = self.device
        if restage or self._stg is None:
            self._stg = (self.x0.clone(), self.ids.clone(), self.label.clone())
        self._mr_drain()
        torch.cuda.synchronize()
        # (default priority: a high-priority M and/or EC stream ran the
        # emulated W=8 step at 1.93-2.26 vs 0.63-0.64 ms)
        streams = {k: torch.cuda.Stream(device=dev) for k in ("M", "D", "EC")}
        ev = {k: ops.SyncEvent(2) for k in ("d", "c5", "m2", "m3", "m4", "e0", "dp", "dpp",
                                            "stg", "pre")}
        seg = self._mr_segments()
        dp_dense = bool(self.emb.dp_tables) and self.emb.dp_dense
        early = _EARLY_PREP and not self.emb.tw_identity       # (as in _mr_segments)
        sort_ec = _SORT_EC and early and dp_dense
        home = lambda name: "EC" if name.startswith("EC") else name[0]  # noqa: E731
        pool = torch.cuda.graph_pool_handle()
        graphs = {}
        self._whole_capture = True       # staging load, no _ps fork, no event records
        was_mstream = self._mstream
        self._mstream = True             # the ids-only sort is its own segment (D0)
        # diagnostics (scripts/mr_timeline.py): device timestamps around
        # every segment of every replay
        stamp = getattr(self, "_mr_stamp", None)
        names = [n for n, f in seg.items() if f is not None]
        try:
            for name, fn in seg.items():
                if fn is None:
                    continue
                st = streams[home(name)]
                g = torch.cuda.CUDAGraph(keep_graph=True)
                routes = [c.capture_origin(st) for c in {id(self.comm): self.comm,
                                                          id(self.dcomm): self.dcomm}.values()
                          if hasattr(c, "capture_origin")]
                with warnings.catch_warnings():
                    # a plan without replicated (or without sharded) tables
                    # leaves some segments empty: checked and dropped below
                    warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
                    with graph_capture(g, pool=pool, stream=st,
                                       capture_error_mode="thread_local"):
                        for r in routes:
                            r.__enter__()
                        try:
                            if stamp is not None:
                                ops.stamp(stamp[0], stamp[1], names.index(name), len(names), 0)
                            fn()
                            if stamp is not None:
                                ops.stamp(stamp[0], stamp[1], names.index(name), len(names), 1)
                        finally:
                            for r in routes:
                                r.__exit__(None, None, None)
                if ops.graph_num_nodes(g) == 0:
                    if name in self._MR_WORK:
                        raise RuntimeError(f"multi-rank segment {name} captured no work")
                    continue                       # not chained (its events still are)
                graphs[name] = g
        finally:
            self._whole_capture = False
            self._mstream = was_mstream
        # the captured exchanges' handles are not real in-flight work
        self.emb._ids_works = []
        self.emb._pending = None
        self._ar_top = self._ar_work = None
        torch.cuda.synchronize()

        def chain(parts):
            return ops.ComposedGraph([(k, graphs[v] if k == "graph" else ev[v])
                                      for k, v in parts if k != "graph" or v in graphs])

        # M: the bottom backward before the top weight grads, so the next
        # batch may load (x0 free) and the bottom bucket reduce sooner
        # (every segment boundary costs ~8 us of queue idle and every
        # cross-stream wait ~15-23 us: labs/probes/mr_sched_probe.py)
        composed = {
            # M: the bottom backward (+ the next batch's load into x0 / ids /
            # labels, all of whose readers have run) before the top weight
            # grads, so the embedding side and the bottom bucket go sooner
            # (the host-staged next batch is waited for right before M4, its
            # only reader: the bottom forward does not wait for the host's
            # generator launch and staging copy, see _mr_step)
            "M": chain([("wait", "dpp" if split_opt else "d"), ("graph", "M1"), ("wait", "c5"),
                        ("wait", "d"), ("graph", "M2"), ("record", "m2"), ("wait", "stg"),
                        ("graph", "M4"), ("record", "m4"), ("graph", "M3"), ("record", "m3")]),
            # D: the ids-only sort of this batch (its ids arrived with the
            # previous step's exchanges), the replicated tables' dense grad +
            # all-reduce, the two dense buckets and the dense optimizer
            # (early prep: the next batch's sharded ids from the staging
            # right after the sort, Dpre)
            "D": chain(([] if sort_ec else
                        [("wait", "c5"), ("graph", "D0"), ("record", "e0")]
                        + ([("wait", "stg"), ("graph", "Dpre"), ("record", "pre")] if early
                           else []))
                       + [("wait", "m2"),
                          ("graph", "Dp"), ("record", "dp"), ("wait", "m4"), ("graph", "Da"),
                          ("record", "dpp"), ("wait", "m3"), ("graph", "Db"), ("record", "d")]),
            # EC: gradient all-to-all, fused embedding update, then the next
            # batch's bucketize, id all-to-all, lookup and pooled all-to-all
            # (the m4 wait sits before the update, not between it and the
            # exchange: it is long satisfied there, and a segment boundary
            # costs ~14 us of queue idle, scripts/mr_timeline.py; with a
            # dense replicated-table update D also looks those tables up, so
            # EC waits for none of D's replicated-table work)
            # (sort_ec: the sort and the early prep first on EC itself,
            # which otherwise idles until the interaction backward)
            "EC": (chain([("graph", "ECs"), ("record", "e0"), ("wait", "stg"),
                          ("graph", "ECpre"), ("record", "pre"), ("wait", "m2"),
                          ("graph", "EC1"), ("graph", "ECub"), ("record", "c5")]) if sort_ec else
                   chain([("wait", "m2"), ("graph", "EC1"), ("wait", "e0"),
                          ("wait", "pre" if early else "m4"),
                          ("graph", "ECub"), ("record", "c5")]) if dp_dense else
                   chain([("wait", "m2"), ("graph", "EC1"), ("wait", "e0"), ("wait", "dp"),
                          ("wait", "m4"), ("wait", "dpp"), ("graph", "ECub"),
                          ("record", "c5")])),
        }
        ops.upload_graphs(composed.values())
        self._mr = {"streams": streams, "events": ev, "graphs": graphs, "composed": composed,
                    "launched": False, "names": names, "full_wait": True,
                    "early": early}
        # the capture ran nothing: the batch handed in before it is the one
        # the first replay loads
        if restage and self._next is not None:
            d, i, l = self._next
            sx, si, sl = self._stg
            ops.batch_load(d, sx, i, si, l, sl)
        torch.cuda.synchronize()
        self.graph = "mstreams"
        self._graph_layout = self.emb.layout_version

    def _mr_stage_next(self, dense, ids, label):
        """Copy the next batch into the staging buffers on the current stream,
        after the previous step's graph has read them (its m4 record)."""
        cur = torch.cuda.current_stream()
        if self._mr["launched"]:
            self._mr["events"]["m4"].wait(cur)
            if self._mr["early"]:
                self._mr["events"]["pre"].wait(cur)     # D's early prep read it too
        sx, si, sl = self._stg
        ops.batch_load(dense, sx, ids, si, label, sl)

    def _mr_step(self):
        if getattr(self, "_mr_inflight", False):
            self._mr_drain()
        mr = self._mr
        s, g = mr["streams"], mr["composed"]
        cur = torch.cuda.current_stream()
        # M4 loads the staging this thread just wrote on the current stream:
        # an event recorded there, waited for inside M right before M4. Only
        # after a host-side reader / writer (sync_streams(), e.g. a state
        # load on the current stream) or on the first replay do the streams
        # wait for everything on the current stream before the step starts.
        # (Before: M waited at its head, so the bottom forward waited for the
        # host's generator launch and staging copy, which the host issues
        # only after the previous step's mailbox read -- emulated W=8: the
        # MLP queue idled ~270 us/step, profiles/r05/w8/step_lanes_before.txt)
        mr["events"]["stg"].record(cur)
        if mr["full_wait"] or not mr["launched"] or _HEAD_WAIT:
            for k in (("M", "D", "EC") if not mr["launched"] else ("M",)):
                s[k].wait_stream(cur)
            mr["full_wait"] = False
        # launch order M, D, EC: a wait node binds to the latest record
        # enqueued before its graph's launch (see the module docstring)
        for k in ("M", "D", "EC"):
            g[k].replay(s[k])
        if self._rw_lagged:
            self.emb.rw_note_replay()           # D published the next batch's need
        mr["launched"] = True

    def _mr_recapture(self):
        """Re-capture between two steps (a captured buffer was reallocated),
        keeping the next batch the caller already staged."""
        self.sync_streams()
        torch.cuda.synchronize()
        self._mr_capture(restage=False)

    def _mr_sync(self):
        cur = torch.cuda.current_stream()
        for st in self._mr["streams"].values():
            cur.wait_stream(st)
        self._mr["full_wait"] = True          # the caller may write on ``cur`` next
