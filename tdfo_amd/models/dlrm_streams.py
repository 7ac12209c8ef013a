"""One-process DLRM / DCN-v2 step as per-stream hipGraphs (mixin of
``DLRMTrainer``).

The HIP runtime replays one captured graph's independent branches mostly in
order on its own queue (the embedding lookup and the bottom MLP ran back to
back in a single whole-step graph), so one process instead captures the step
as graphs per stream and replays them on two streams joined by events: the
memory-bound embedding work (lookup, ids-only sort, fused update) runs on the
embedding stream concurrently with the MLP stream's GEMMs.

  embedding stream: E1 lookup -> (record ev1) -> E2 sort ......... E3 update
  MLP stream:       M1 bottom fwd -> (wait ev1) -> M2 top fwd+bwd -> (record
                    ev2) -> M3 bottom bwd + dense optimizer
                    (E3 waits for ev2: the embedding gradients)

With ``composed_graphs`` each stream's graphs are chained natively into one
executable graph with in-graph event nodes (``ops.ComposedGraph``;
``graph_compose`` in csrc/bindings.cpp): the queue idles ~8-10 us at an event
node instead of ~14 us at each graph boundary (DLRM-1TB 0.457 vs 0.463 ms/step;
DCN-v2 is faster without: 2.335 vs 2.362). The early lookup copies the next
batch's ids on the embedding stream (or, ``ids_stream``, on a third stream
right behind the sort), so the next lookup overlaps this step's bottom-MLP
backward; readers of tables / params outside ``step()`` call
``sync_streams()`` first.

Reader contract with a producer stream (``set_copy_stream``, the default
with the device generator): the step's embedding update (E3) is *deferred*
-- enqueued by the next ``load_batch`` / ``step`` / ``sync_streams()`` /
``flush_pending()``, after the wait for the next batch's ids copy. So after
a bare ``step()`` the update is not enqueued at all, and a device-wide
``torch.cuda.synchronize()`` alone does NOT make the tables current: call
``sync_streams()`` (or ``flush_pending()``) first. The trainer's own readers
do (``state_dict``, ``dense_state``, ``predict``, ``pop_loss``, checkpoints),
and ``StepLoop.run`` flushes at its end.
"""
from __future__ import annotations

import os

import torch

from .. import ops
from ..utils.capture import graph_capture


class StreamGraphsMixin:
    """Per-stream graph capture / replay for one process (``capture_graph``
    with ``streams=True``, the default at world size 1)."""

    def _ms_plan(self):
        emb = self.emb

        def e1():
            self._s_gen_ids()                # (in-step batches: this step's ids)
            if not emb.fwd_prep_noop:
                emb.stage_fwd_prep(self.ids)
            emb.stage_fwd_ids_exchange()
            emb.stage_fwd_lookup()
            emb.stage_fwd_out_exchange()
            emb.forward_wait()

        # "split_main" (DCN-v2): the top-MLP (+ head, cross layers) part of the
        # dense optimizer first on the MLP stream, beside the long multi-hot
        # embedding update (2.35 vs 2.40 ms/step); "one_pass" (DLRM): the
        # whole optimizer after the bottom backward (0.463 vs 0.471-0.479)
        split = self.cfg.opt_placement == "split_main"
        a, P = self._ar_split, self.fp.p.numel()

        def e3():
            emb.backward_start()
            emb.backward_wait()
            self._s_emb_update()

        def m2():
            self._s_top()

        def m3():
            if self._defer_top_wgrad:
                self._s_top_wgrad()          # beside the embedding update (E3)
            if split:
                self._dense_update_range(a, P)
            self._s_bottom_bwd()
            if split:
                self._dense_update_range(0, a)
            else:
                self._s_dense_update()

        def m1():
            self._s_gen_dense()              # (in-step batches: dense features / labels)
            if self._bstg is not None and self._fused_bottom and self._bot_load_fold:
                # this step's dense / labels from the staging, loaded by the
                # fused bottom-MLP launch itself (no batch_load launch)
                self._s_bottom_fwd(staged=self._bstg)
                return
            if self._bstg is not None:       # this step's dense / labels from the staging
                ops.batch_load(self._bstg[0], self.x0, self.ids[:0], self.ids[:0], self._bstg[1],
                               self.label)
            self._s_bottom_fwd()

        return {"E1": e1, "E2": emb.stage_bwd_prepare, "M1": m1,
                "M2": m2, "E3": e3, "M3": m3}

    def _capture_streams(self):
        assert self.world == 1
        self._mstream = True
        composed = self.cfg.composed_graphs
        if composed is None:
            composed = self.cfg.interaction == "dot"
        if os.environ.get("TDFO_COMPOSED") in ("0", "1"):     # A/B override
            composed = os.environ["TDFO_COMPOSED"] == "1"
        # cross-stream edges recorded without the system-scope fence a default
        # event record adds (the producing kernels already release to device
        # scope and no host reads these edges): DLRM-1TB 0.477-0.480 vs
        # 0.485-0.487 ms/step with torch events
        ev = [ops.SyncEvent(2) for _ in range(4)]
        ids_stream = self.cfg.ids_stream
        if ids_stream is None:
            ids_stream = composed
        # Staged batches (composed graphs + ids stream): a device batch is
        # copied (ids, dense, labels) on the ids stream into fixed buffers, and
        # the MLP graph converts dense / labels itself behind an in-graph wait
        # -- no eager launch and graph boundary on the MLP stream between
        # steps (that boundary idled it ~23-31 us per step,
        # profiles/r03/s3/w1_timeline/)
        self._bstg = None
        # (Rejected, round 5: staging on the batch producer's own copy stream
        # too, so the batch load stays inside the MLP graph instead of an eager
        # launch between two graph launches -- 0.433 vs 0.411-0.414 ms/step,
        # profiles/r05/notes.md)
        if composed and ids_stream and self._insrc is None:
            self._bstg = (torch.zeros(self.B, self.cfg.num_dense, device=self.device),
                          torch.zeros(self.B, device=self.device))
        ev_copy = ops.SyncEvent(2)
        ev_stg = ops.SyncEvent(2)
        plan = self._ms_plan()
        se = torch.cuda.Stream(device=self.device)
        pool = torch.cuda.graph_pool_handle()
        graphs = {}
        se.wait_stream(torch.cuda.current_stream())
        # diagnostics (scripts/w1_timeline.py): device timestamps around each
        # captured segment
        stamp = getattr(self, "_ms_stamp", None)
        names = list(plan)
        for name in plan:
            gr = torch.cuda.CUDAGraph(keep_graph=composed)
            # (the MLP graphs capture on torch's own side stream: capture is
            # not allowed on the default stream; replays run on any stream)
            with graph_capture(gr, pool=pool, stream=se if name[0] == "E" else None):
                if stamp is not None:
                    ops.stamp(stamp[0], stamp[1], names.index(name), len(names), 0)
                plan[name]()
                if stamp is not None:
                    ops.stamp(stamp[0], stamp[1], names.index(name), len(names), 1)
            graphs[name] = gr
        if composed:
            # (the ~20-us idle at every step boundary is the graph launch
            # boundary itself: dropping this wait measured the same,
            # 0.429-0.432 vs 0.431-0.434 ms/step, profiles/r05/notes.md)
            head = [("wait", ev_stg)] if self._bstg is not None else []
            graphs["M"] = ops.ComposedGraph(head + [("graph", graphs["M1"]), ("wait", ev[1]),
                                                    ("graph", graphs["M2"]), ("record", ev[2]),
                                                    ("graph", graphs["M3"])])
            graphs["EA"] = ops.ComposedGraph([("graph", graphs["E1"]), ("record", ev[1]),
                                              ("graph", graphs["E2"])])
            # the update with its wait / record as one launch
            graphs["EU"] = ops.ComposedGraph([("wait", ev[2]), ("graph", graphs["E3"]),
                                              ("record", ev[3])])
        ops.upload_graphs(graphs.values())
        torch.cuda.synchronize()
        cs = (torch.cuda.Stream(device=self.device) if ids_stream and self._insrc is None
              else None)
        src_cs = self._src_copy_stream is not None and self._insrc is None and self._bstg is None
        if src_cs:
            cs = self._src_copy_stream
        self._ms = {"graphs": graphs, "stream": se, "plan": plan, "composed": composed,
                    "names": names,
                    "cstream": cs, "ev_e2": ops.SyncEvent(2), "ev_copy": ev_copy,
                    "ev_stg": ev_stg,
                    "src_cs": src_cs, "pending_e3": False,
                    "defer_e3": src_cs and os.environ.get("TDFO_DEFER_E3", "1") != "0",
                    "e2_recorded": False, "events": ev}
        self.graph = "streams"

    def _ms_load_ids(self, ids: torch.Tensor, on_device: bool, dense=None, label=None) -> bool:
        """Per-stream mode: copy this step's ids on the embedding side (the
        lookup follows the previous step's embedding update on that stream),
        and with staged batches its dense features / labels too. Returns
        False when the caller must use the plain fused load."""
        if not (ids.is_cuda and ids.dtype == torch.int64 and ids.is_contiguous()
                and ids.numel() == self.ids.numel()):
            return False
        se, ev = self._ms["stream"], self._ms["events"][0]
        main = torch.cuda.current_stream()
        cs = self._ms.get("cstream")
        if self._ms.get("src_cs"):
            own = self._src_copy_owner
            if on_device and (own is None or own.owns(ids)):
                pass                           # the producer's batch: copy on its stream
            else:
                # another producer's batch (ordered on the MLP stream only)
                cs, on_device = None, False
        if cs is not None and on_device:
            # the ids copy on its own stream right behind this step's sort (E2,
            # the ids' last reader): the next lookup waits on an event that is
            # already signalled instead of queueing the copy behind the update
            if self._ms["e2_recorded"]:
                cs.wait_event(self._ms["ev_e2"])
            ops.copy_on(self.ids, ids, cs)
            self._ms["ev_copy"].record(cs)     # the ids: the embedding stream's edge
            stg = self._bstg
            if stg is not None:
                # the previous step's MLP graph read the staging in M1, before
                # its ev[2] record (a wait on a never-recorded event is a no-op);
                # after the ids' record, so the next lookup does not wait for it
                cs.wait_event(self._ms["events"][2])
                for dst, src in ((stg[0], dense), (stg[1], label.reshape(-1))):
                    if (src.dtype == dst.dtype and src.is_contiguous()
                            and src.numel() == dst.numel()):
                        ops.copy_on(dst, src, cs)
                    else:                      # (a converting copy)
                        with torch.cuda.stream(cs):
                            dst.copy_(src.reshape(dst.shape), non_blocking=True)
                self._ms["ev_stg"].record(cs)  # the MLP graph's head waits for this
            se.wait_event(self._ms["ev_copy"])
            self.flush_pending()
            return True
        if not on_device:
            se.wait_stream(main)               # e.g. an H2D the caller ordered on main
        with torch.cuda.stream(se):
            self.ids.copy_(ids, non_blocking=True)
            ev.record(se)
        if not on_device:
            main.wait_event(ev)                # dense / labels from the same source
        self.flush_pending()
        return True

    def _ms_step(self):
        if self._ms.get("pending_e3"):
            self._ms_issue_e3()              # (no load_batch since the last step)
        g, se, ev = self._ms["graphs"], self._ms["stream"], self._ms["events"]
        main = torch.cuda.current_stream()
        composed = self._ms["composed"]
        # (this step's ids were copied on the embedding side by load_batch, so
        # the lookup follows the previous step's embedding update there)
        # (Measured, round 5: replaying the next lookup before this update --
        # inexact, a bound on what an early lookup + stale-bag fix could
        # gain -- ran DCN-v2 at 2.40-2.42 vs 2.36-2.38 ms/step: the update and
        # lookup are HBM-bound and slow the GEMMs they overlap about as much
        # as they save, profiles/r05/notes.md)
        if composed:
            # (streams passed to the launches as raw handles: no host-side
            # torch stream switches on the step's issue path)
            g["EA"].replay(se)               # records ev[1] inside
        else:
            with torch.cuda.stream(se):
                g["E1"].replay()
                ev[1].record(se)
                g["E2"].replay()
        if self._ms.get("cstream") is not None:
            self._ms["ev_e2"].record(se)
            self._ms["e2_recorded"] = True
        if composed:
            g["M"].replay()                  # waits for ev[1], records ev[2] inside
        else:
            g["M1"].replay()
            main.wait_event(ev[1])           # pooled embeddings ready
            g["M2"].replay()
            ev[2].record(main)
        if self._ms.get("defer_e3"):
            # the embedding update is issued by the next load_batch, after the
            # wait for the next batch's ids copy: that wait then sits before
            # the update (which waits for the MLP stream anyway), not between
            # the update and the next lookup (flush_pending() / sync_streams()
            # / the next step issue it otherwise)
            self._ms["pending_e3"] = True
        else:
            self._ms_issue_e3()
        if not composed:
            g["M3"].replay()
        # no end-of-step join: the embedding stream's next work (ids copy,
        # lookup) is ordered behind this update on that stream, and the next
        # MLP graphs wait for the next lookup

    def _ms_issue_e3(self):
        g, se, ev = self._ms["graphs"], self._ms["stream"], self._ms["events"]
        if "EU" in g:
            g["EU"].replay(se)               # waits ev[2], records ev[3] inside
        else:
            with torch.cuda.stream(se):
                se.wait_event(ev[2])         # embedding gradients ready
                g["E3"].replay()
                ev[3].record(se)
        self._ms["pending_e3"] = False

    def flush_pending(self):
        """Issue a deferred embedding update (one-GPU per-stream graphs)."""
        if self._ms is not None and self._ms.get("pending_e3"):
            self._ms_issue_e3()

    def input_streams(self):
        """Streams that read a batch handed to load_batch (a producer orders
        its device copies on each, then passes on_device=True)."""
        main = torch.cuda.current_stream()
        if self.graph == "streams":
            if self._ms.get("src_cs"):
                # the ids are copied on the producer's own stream (in order
                # behind the batch there); only the MLP stream reads the rest
                return [main]
            cs = self._ms.get("cstream")
            return [main, self._ms["stream"]] + ([cs] if cs is not None else [])
        return [main]

    def sync_streams(self):
        """Order the current stream after all side-stream work of issued steps
        (embedding updates)."""
        if self._ms is not None:
            self.flush_pending()
            torch.cuda.current_stream().wait_stream(self._ms["stream"])
            if self._ms.get("cstream") is not None:
                torch.cuda.current_stream().wait_stream(self._ms["cstream"])
        if getattr(self, "_sides", None) is not None:
            torch.cuda.current_stream().wait_stream(self._sides)
        if getattr(self, "_mr", None) is not None:
            self._mr_sync()
