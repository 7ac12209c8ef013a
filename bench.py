#!/usr/bin/env python
"""Headline benchmark: DLRM training throughput (examples/sec, whole node) on
Criteo-1TB-shaped synthetic data at 1/2/4/8 MI355X (BASELINE.json metric).

Model (MLPerf DLRM / TorchRec-DLRM shape): 13 dense + 26 sparse features,
MLPerf Criteo-Terabyte cardinalities (max-ind-range 40M, 188M rows total),
embedding dim 128 (fp32 tables, ~96 GB), bottom MLP 13-512-256-128, dot
interaction, top MLP 479-1024-1024-512-256-1, bf16 compute / fp32 master.
Embeddings: table-wise sharded across ranks (all on one GPU at N=1), fused
row-wise Adagrad; dense: fused AdamW, all-reduced over RCCL.
Weak scaling: --batch is per GPU; value = global examples / second.

Launch: python bench.py [--gpus N]. With N > 1 and no WORLD_SIZE in the
environment, bench.py starts the N rank processes itself (a child
``torch.distributed.run`` on 127.0.0.1, before any GPU call) and exits with
its code; the driver's own ``torch.distributed.run ... bench.py --gpus N``
lands directly in the rank code. One rank per GPU over RCCL: N must not
exceed the visible GPUs (the multi-rank rehearsal on one GPU sets
TDFO_SHARE_DEVICE=1 TDFO_DIST_BACKEND=gloo explicitly).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time


def _one_gpu_run(argv) -> bool:
    """One process on one GPU, not an emulated rank (peeked before argparse:
    the runtime mode below must be set before any GPU call)."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return False
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    pre.add_argument("--emulate-world", type=int, default=0)
    a, _ = pre.parse_known_args(argv)
    return a.gpus <= 1 and a.emulate_world <= 1


# HIP runtime mode for one-GPU runs (utils/guarded.py: measured gain, why
# not for ranks); set before any GPU call and reported in the JSON line.
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tdfo_amd.utils.guarded import one_gpu_runtime_mode  # noqa: E402 (no GPU work)

RUNTIME_MODE = one_gpu_runtime_mode(_one_gpu_run(sys.argv[1:]))

import torch


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("TDFO_BENCH_BATCH", 8192)),
                    help="per-GPU batch (weak scaling)")
    ap.add_argument("--rows", default="1tb", choices=["1tb", "kaggle", "tiny", "gt1tb"])
    ap.add_argument("--model", default="dlrm", choices=["dlrm", "dcnv2"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--data", default="fresh", choices=["fresh", "instep", "pool", "host"],
                    help="fresh: a new batch every step from the one-launch device generator "
                         "on a side stream (default); instep (one GPU): the same batches "
                         "generated inside the step graphs (ids on the embedding stream, dense "
                         "features / labels on the MLP stream); pool: cycle --pool "
                         "pre-generated device batches; host: the C++ host generator through "
                         "pinned slots and a copy-stream H2D prefetcher")
    ap.add_argument("--pool", type=int, default=8, help="--data pool: batches in the pool")
    ap.add_argument("--dist", default="uniform", choices=["uniform", "zipf"])
    ap.add_argument("--rw-exchange", default="auto", choices=["auto", "pooled", "rows"],
                    help="row-wise exchange (DLRMConfig.rw_exchange): rows = one-hot tables "
                         "return looked-up rows by all-to-all instead of pooled partials")
    ap.add_argument("--dp-rule", default="cost", choices=["cost", "budget"],
                    help="--sharding data_parallel: replicate where the dense all-reduce is "
                         "cheaper than the row-wise exchange (cost) or smallest-first to 256 MB")
    ap.add_argument("--sharding", default="auto",
                    choices=["auto", "table_wise", "row_wise", "column_wise", "data_parallel",
                             "replicated"])
    ap.add_argument("--opt-placement", default=None,
                    choices=["one_pass", "split_main"],
                    help="one GPU: where the dense optimizer runs in the per-stream step "
                         "(DLRMConfig.opt_placement; default: the model's)")
    ap.add_argument("--defer-wgrad", default=None, choices=["0", "1"],
                    help="top / cross weight grads after the interaction / cross backward "
                         "(DLRMConfig.defer_wgrad; default: when N > 1)")
    ap.add_argument("--preheat-ms", type=float, default=30.0,
                    help="after the warm-up steps, this many ms of MFMA load on every CU "
                         "before the timed window (no training work: the chip's clock ramps "
                         "under sustained load, and host-launched eager warm-up steps leave "
                         "it idle; profiles/r04/notes.md); reported in the JSON lines; 0: off")
    ap.add_argument("--dense-comm", default="fp32", choices=["fp32", "bf16"],
                    help="N > 1: wire format of the dense-gradient all-reduce")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N > 1: exchange each batch's ids inside its own step instead of "
                         "during the previous step's dense update")
    ap.add_argument("--no-stream-graphs", action="store_true",
                    help="N > 1: replay graphs between eagerly issued exchanges instead of the "
                         "per-stream step graphs with the collectives inside")
    ap.add_argument("--host-data", action="store_true", help="same as --data host")
    ap.add_argument("--emulate-world", type=int, default=0, metavar="W",
                    help="one GPU runs one rank of the W-rank job: the real W-rank plan, layouts "
                         "and kernels, each collective replaced by device copies of the same "
                         "byte count (parallel/comm.py LoopbackComm); reports device ms/step, "
                         "host issue us/step and the collective volume (not the headline)")
    ap.add_argument("--emulate-rank", default="0", metavar="K[,K...]|max",
                    help="--emulate-world: the rank(s) to emulate, each in its own child "
                         "process (TDFO_EMU_INPROC=1: in turn in this one), or 'max': every "
                         "rank of the plan; the slowest is reported (a synchronous step runs "
                         "at the pace of its slowest rank)")
    ap.add_argument("--emulate-link-gbps", type=float, default=None,
                    help="--emulate-world: modelled per-rank xGMI injection bandwidth (GB/s); "
                         "each emulated collective also holds the comm stream for its link "
                         "bytes / this. Default: the planner's / SOL's link model, "
                         "min(W-1, 7) x 153 GB/s (one point-to-point link per peer); 0: local "
                         "copies only")
    ap.add_argument("--emulate-latency-us", type=float, default=10.0,
                    help="--emulate-world: modelled fixed cost per collective (us)")
    ap.add_argument("--no-preflight", action="store_true",
                    help="N > 1: skip the collective self-test before the trainer is built "
                         "(parallel/preflight.py; on a mismatch it switches to c10d + staged)")
    ap.add_argument("--watchdog-s", type=float, default=float(os.environ.get("TDFO_WATCHDOG_S",
                                                                          180)),
                    help="hang guard: a step whose heartbeat has not landed after this many "
                         "seconds (or a host that stops issuing steps) ends the rank with exit "
                         "code 3 and a diagnostic on stderr; 0 disables it")
    args = ap.parse_args(argv)
    if args.host_data:
        args.data = "host"
    return args


# Stock PyTorch-ROCm eager DLRM (nn.EmbeddingBag + nn.Linear, bf16 autocast,
# sparse Adagrad / AdamW) measured on one MI355X with the same shapes
# (scripts/baseline_torch_dlrm.py, profiles/torch_eager_baseline_dlrm.jsonl);
# BASELINE.md protocol item (a). For N GPUs it is scaled by N (perfect
# scaling assumed for the baseline).
EAGER_BASELINE_EX_S = {"1tb": 608463.1, "kaggle": 518563.4}


def parallelism(plan, world: int) -> str:
    """e.g. "dp8 dense + emb table_wise x8" (embedding sharding kinds from the plan)."""
    if world == 1:
        return "single-gpu"
    short = {"table_wise": "tw", "row_wise": "rw", "data_parallel": "dp", "column_wise": "cw"}
    kinds = "+".join(f"{short.get(k, k)}{n}" for k, n in sorted(plan.summary()["kinds"].items()))
    return f"dp{world} dense + emb[{kinds} tables] over {world} ranks"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(args, argv) -> int:
    """Start ``args.gpus`` rank processes (one per GPU) and return their exit
    code. Runs before anything touches the GPU (device_count() does not
    initialise HIP on this image)."""
    n = args.gpus
    share = os.environ.get("TDFO_SHARE_DEVICE") == "1"
    if share and os.environ.get("TDFO_DIST_BACKEND", "nccl") == "nccl":
        print(f"error: --gpus {n} with TDFO_SHARE_DEVICE=1 needs TDFO_DIST_BACKEND=gloo "
              "(RCCL cannot put two ranks on one GPU)", file=sys.stderr)
        return 2
    if not share:
        have = torch.cuda.device_count()
        if have < n:
            print(f"error: --gpus {n} but only {have} GPU(s) visible; bench.py runs one rank "
                  "per GPU over RCCL (RCCL cannot put two ranks on one GPU). Refusing to "
                  f"report an N=1 measurement as N={n}.", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def _cfg(args, rows, pipe):
    from tdfo_amd.models.dlrm import MLPERF_MULTIHOT, DLRMConfig
    kw = dict(table_rows=list(rows), sharding=args.sharding, pipeline=pipe,
              rw_exchange=args.rw_exchange, dp_rule=args.dp_rule,
              dense_comm=args.dense_comm, stream_graphs=not args.no_stream_graphs,
              opt_placement=args.opt_placement,
              defer_wgrad=None if args.defer_wgrad is None else args.defer_wgrad == "1")
    if args.model == "dlrm":
        return DLRMConfig(**kw)
    return DLRMConfig(interaction="dcn", pooling=list(MLPERF_MULTIHOT),
                      top=[1024, 1024, 512, 256, 1], **kw)


def measure(args, info, cfg, world: int, group, rank: int) -> dict:
    """Build the trainer of ``rank``, run the warm-up (eager steps, capture,
    first replays), then time ``args.steps`` steps between barriers + device
    synchronisations. Returns the measurement and the live trainer."""
    from tdfo_amd.models.dlrm import DLRMTrainer
    from tdfo_amd.data.synthetic import SyntheticCriteo
    from tdfo_amd.train.loop import PoolBatches, StepLoop, make_source
    from tdfo_amd.utils.watchdog import StepWatchdog

    B = args.batch
    t0 = time.time()
    tr = DLRMTrainer(cfg, B, info.device, group=group, rank=rank, world_size=world)
    if args.data == "pool":
        data = SyntheticCriteo(cfg.table_rows, B, pooling=cfg.pooling_factors(),
                               device=info.device, seed=1, rank=rank, dist=args.dist)
        src = PoolBatches([data.next() for _ in range(args.pool)])
    else:
        src = make_source(cfg.table_rows, B, info.device, cfg.pooling_factors(), 1, rank,
                          dist=args.dist, kind=args.data)
    wd = (StepWatchdog(info.device, args.watchdog_s, rank=info.rank, describe=tr.progress)
          if args.watchdog_s > 0 else None)
    loop = StepLoop(tr, src, watchdog=wd)
    torch.cuda.synchronize()
    setup_s = time.time() - t0
    use_graph = not args.no_graph

    # W untimed warm-up steps in all: eager ones, one inside the capture, and
    # two replays of the fresh graph (its first launches upload it)
    post = 2 if use_graph and args.warmup >= 4 else 0
    if use_graph and os.environ.get("TDFO_BENCH_POST"):     # diagnostics: more replays
        post = max(0, min(int(os.environ["TDFO_BENCH_POST"]), args.warmup - 1))
    loop.run(args.warmup - (1 + post if use_graph else 0))
    # one eager step's collectives (a whole-step graph issues none from the host)
    step_stats = None
    if tr.comm is not None:
        comms = [tr.comm] + ([tr.dcomm] if tr.dcomm is not tr.comm else [])
        for c in comms:
            c.reset_stats()
            if hasattr(c, "modelled_us"):
                c.modelled_us = 0.0
        loop.run(1)
        agg = {}
        for c in comms:
            for k, (n, b) in c.stats.items():
                a = agg.setdefault(k, [0, 0])
                a[0] += n
                a[1] += b
        step_stats = (agg, sum(getattr(c, "modelled_us", 0.0) for c in comms))
    if use_graph:
        tr.capture_graph(warmup=0 if step_stats is not None else 1)
        loop.run(post)
    torch.cuda.synchronize()
    tr.pop_loss()
    if args.preheat_ms > 0 and os.environ.get("TDFO_PREHEAT_KIND") == "copy":
        # diagnostics: an HBM-bound pre-heat (1 GiB copies, ~0.8 ms each)
        a = torch.empty(1 << 28, dtype=torch.float32, device=info.device)
        b = torch.empty_like(a)
        for _ in range(max(1, int(args.preheat_ms / 0.8))):
            b.copy_(a)
        del a, b
    elif args.preheat_ms > 0:
        from tdfo_amd import ops
        ops.burn_us(args.preheat_ms * 1e3)
    if info.world_size > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    mb = tr.emb._rw_mbox
    wait0 = mb.wait_s if mb is not None else 0.0
    grows0 = tr.emb.rw_grows if tr.emb.rw_tables else 0
    curve = int(os.environ.get("TDFO_BENCH_CURVE", "0"))
    marks = []
    t = time.perf_counter()
    if curve > 0:
        # diagnostics: device time of every `curve` timed steps (events on the
        # current stream between launches), to stderr
        hmarks = []
        for k in range(0, args.steps, curve):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks.append(e)
            hmarks.append(time.perf_counter())
            loop.run(min(curve, args.steps - k))
        hmarks.append(time.perf_counter())
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append(e)
    else:
        loop.run(args.steps)
    host_s = time.perf_counter() - t          # issue time (the device runs behind)
    torch.cuda.synchronize()
    if info.world_size > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t
    if marks:
        ms_w = [round(a.elapsed_time(b) / curve, 4) for a, b in zip(marks, marks[1:])]
        host_w = [round((b - a) * 1e3 / curve, 4) for a, b in zip(hmarks, hmarks[1:])]
        print(json.dumps({"ms_per_step_windows": ms_w, "host_ms_per_step_windows": host_w,
                          "window": curve}), file=sys.stderr, flush=True)
    if wd is not None:
        wd.close()
    if info.world_size > 1:
        x = torch.tensor([el], dtype=torch.float64, device=info.device)
        torch.distributed.all_reduce(x, op=torch.distributed.ReduceOp.MAX)
        el = float(x.item())
    wait_s = (mb.wait_s if mb is not None else 0.0) - wait0
    loss = tr.pop_loss() / max(1, args.steps * B)
    comm = ({k: {"calls_per_step": round(c, 2), "MB_per_step": round(b / 1e6, 3)}
             for k, (c, b) in sorted(step_stats[0].items())} if step_stats is not None else {})
    return {"tr": tr, "loop": loop, "el": el, "host_s": host_s, "wait_s": wait_s,
            "loss": loss, "setup_s": setup_s, "comm": comm,
            "modelled_us": step_stats[1] if step_stats is not None else 0.0,
            "rw_grows_timed": (tr.emb.rw_grows if tr.emb.rw_tables else 0) - grows0}


def _graph_name(tr):
    return tr.graph if isinstance(tr.graph, str) else ("staged" if tr.graph else None)


def emulate(args, info, rows):
    """--emulate-world: one (or, with --emulate-rank max, every) rank of the
    W-rank job on this GPU over loopback collectives."""
    import gc

    from tdfo_amd.parallel.comm import LoopbackComm
    from tdfo_amd.sparse.planner import LINK_GBS

    W = args.emulate_world
    link = (args.emulate_link_gbps if args.emulate_link_gbps is not None
            else min(W - 1, 7) * LINK_GBS)
    ranks = (list(range(W)) if args.emulate_rank == "max" else
             [int(x) for x in args.emulate_rank.split(",")])
    cfg = _cfg(args, rows, not args.no_pipeline)
    if args.data in ("host", "fresh", "instep"):
        cfg.ids_stream = False
    per = []
    comm0 = plan_summary = None
    for k in ranks:
        group = LoopbackComm(W, k, info.device, link_gbps=link, latency_us=args.emulate_latency_us)
        r = measure(args, info, cfg, W, group, k)
        tr = r["tr"]
        ms = r["el"] / args.steps * 1e3
        rec = {"rank": k, "ms_per_step": round(ms, 4),
               "host_issue_us_per_step": round((r["host_s"] - r["wait_s"]) / args.steps * 1e6, 1),
               "host_wait_us_per_step": round(r["wait_s"] / args.steps * 1e6, 1),
               "graph": _graph_name(tr), "plan_cost": round(tr.plan.cost[k], 1),
               "mem_GiB": round(tr.plan.mem_bytes[k] / 2**30, 1), "setup_s": round(r["setup_s"], 1)}
        if tr.emb.rw_tables:
            rec.update(rw_cap=tr.emb.rw_cap, rw_grows=tr.emb.rw_grows,
                       rw_grows_timed=r["rw_grows_timed"])
        print(json.dumps(rec), file=sys.stderr, flush=True)
        if plan_summary is None:
            plan_summary, comm0 = tr.plan.summary(), r["comm"]
        per.append((rec, r))
        if len(ranks) > 1:
            r["loop"].close()
            del tr, r, group
            per[-1] = (rec, None)
            gc.collect()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    rec = max((p[0] for p in per), key=lambda x: x["ms_per_step"])
    ms = rec["ms_per_step"]
    print(json.dumps({
        "metric": (f"emulated step of the {W}-rank job, slowest of ranks {ranks} "
                   "(loopback collectives)" if len(ranks) > 1 else
                   f"emulated rank-{ranks[0]} step of the {W}-rank job (loopback collectives)"),
        "value": ms, "unit": "ms/step", "higher_is_better": False,
        "emulated_world": W, "emulated_rank": rec["rank"], "steps": args.steps,
        "warmup": args.warmup, "per_rank_ms": {p[0]["rank"]: p[0]["ms_per_step"] for p in per},
        "host_issue_us_per_step": rec["host_issue_us_per_step"],
        "host_wait_us_per_step": rec["host_wait_us_per_step"],
        "examples_per_sec_whole_job_model": round(args.batch * W / (ms / 1e3), 1),
        "sol_ms_compute": round(cfg.sol(args.batch, 1)["sol_ms"], 4),
        "sol_comm_ms": round(cfg.sol(args.batch, W)["comm_ms"], 4),
        "comm": comm0,
        "comm_model": {"link_gbps": link, "latency_us": args.emulate_latency_us},
        "plan": plan_summary, "graph": rec["graph"], "pipeline": not args.no_pipeline,
        "dist": args.dist, "data": args.data,
        "config": {"model": "DLRM" if args.model == "dlrm" else "DCN-v2",
                   "tables": f"criteo-{args.rows}", "per_gpu_batch": args.batch,
                   "sharding": args.sharding}}), flush=True)


def emulate_ranks_isolated(args, argv) -> int:
    """--emulate-rank with several ranks: each rank in a fresh child process
    (started before this process touches the GPU), so no rank runs on memory
    another trainer freed -- in one process the 4th trainer of a sequence ran
    up to 1.35x slower whichever rank it was (profiles/r04/notes.md). Prints
    the slowest rank's line with every rank's ms/step."""
    W = args.emulate_world
    ranks = (list(range(W)) if args.emulate_rank == "max" else
             [int(x) for x in args.emulate_rank.split(",")])
    per = []
    for k in ranks:
        cmd = [sys.executable, os.path.abspath(__file__), *argv, "--emulate-rank", str(k)]
        p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            print(f"error: emulated rank {k} exited {p.returncode}", file=sys.stderr)
            return p.returncode or 1
        per.append(json.loads(lines[-1]))
    top = max(per, key=lambda x: x["value"])
    top["metric"] = (f"emulated step of the {W}-rank job, slowest of ranks {ranks} "
                     "(loopback collectives, one process per rank)")
    top["per_rank_ms"] = {x["emulated_rank"]: x["value"] for x in per}
    print(json.dumps(top), flush=True)
    return 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args, argv))
    from tdfo_amd.utils import supervise
    from tdfo_amd.utils.supervise import emit_result
    if (int(os.environ.get("WORLD_SIZE", "1")) > 1 and not supervise.is_child()
            and os.environ.get("TDFO_SUPERVISE", "1") == "1"):
        # every rank: a GPU-free supervisor runs the rank code as a child; if
        # any rank's child fails (watchdog exit 3, replica mismatch exit 4,
        # crash), all ranks rerun once on c10d collectives + staged replay
        sys.exit(supervise.supervise([sys.executable, os.path.abspath(__file__), *argv],
                                     attempts=[{}, {"TDFO_COMM": "torch"}],
                                     fallback_argv=[["--no-stream-graphs"]]))
    if (args.emulate_world > 1 and (args.emulate_rank == "max" or "," in args.emulate_rank)
            and os.environ.get("TDFO_EMU_INPROC") != "1"):
        sys.exit(emulate_ranks_isolated(args, argv))
    from tdfo_amd.parallel.dist import init_distributed, reset
    from tdfo_amd.models.dlrm import CRITEO_1TB_ROWS, CRITEO_KAGGLE_ROWS, DCN_GT1TB_ROWS
    from tdfo_amd.ops import _ext

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"error: --gpus {args.gpus} but WORLD_SIZE={world_env}")
    if args.emulate_world and args.gpus != 1:
        raise SystemExit("error: --emulate-world runs in one process (--gpus 1)")
    info = init_distributed("cuda")
    if not _ext.load():
        raise RuntimeError("native HIP library failed to load")
    if os.environ.get("TDFO_GEMM_POLICY"):      # override the trainer's per-model choice
        from tdfo_amd import ops
        ops.gemm_policy(int(os.environ["TDFO_GEMM_POLICY"]))
    rows = {"1tb": CRITEO_1TB_ROWS, "kaggle": CRITEO_KAGGLE_ROWS, "gt1tb": DCN_GT1TB_ROWS,
            "tiny": [1000] * 26}[args.rows]
    if args.emulate_world > 1:
        emulate(args, info, rows)
        reset()
        return
    world = info.world_size
    pf = None
    if world > 1 and not args.no_preflight:
        from tdfo_amd.parallel.preflight import preflight
        pf = preflight(info.group, info.device)
        print(json.dumps({"preflight": pf, "rank": info.rank}), file=sys.stderr, flush=True)
        if not pf["ok"]:
            args.no_stream_graphs = True          # c10d collectives, staged replay
    cfg = _cfg(args, rows, world > 1 and not args.no_pipeline)
    if args.data in ("host", "fresh", "instep"):
        # a streamed data source orders its batch on every input stream and
        # releases a slot after all of them: a third (ids) stream ties the
        # slot to the sort and stalls the prefetch (0.604 vs 0.470 ms/step)
        cfg.ids_stream = False
    B = args.batch
    r = measure(args, info, cfg, world, info.group, info.rank)
    tr, el = r["tr"], r["el"]
    ms = el / args.steps * 1e3
    value = B * world * args.steps / el
    sol = cfg.sol(B, world)
    consistent, per = True, {}
    if world > 1:
        # replicas must agree bit for bit before a throughput is reported
        from tdfo_amd.parallel.replicas import check_replicas
        inject = os.environ.get("TDFO_INJECT_DIVERGENCE")
        state = tr.replicated_state()
        att = os.environ.get("TDFO_ATTEMPT", "0")
        if inject is not None and int(inject) == info.rank and \
                os.environ.get("TDFO_INJECT_ATTEMPT", att) == att:
            state["dense.p"].view(-1)[0] += 1e-3          # test hook: one diverged replica
        consistent, per = check_replicas(state, info.group)
    comm_path = None
    if world > 1:
        from tdfo_amd.parallel.comm import RcclComm
        comm_path = ("native" if isinstance(tr.comm, RcclComm) else "c10d") + (
            "-graphs" if _graph_name(tr) == "mstreams" else "-staged")
    if not consistent:
        # no throughput for diverged replicas: nothing goes to stdout
        r["loop"].close()
        print(f"error: rank {info.rank}: replicated state differs across ranks ({per})",
              file=sys.stderr, flush=True)
        reset()
        sys.exit(4)
    if info.rank == 0:
        print(json.dumps({"plan": tr.plan.summary(), "setup_s": round(r["setup_s"], 1),
                          "train_loss": round(r["loss"], 4), "graph": _graph_name(tr),
                          "host_issue_us_per_step": round((r["host_s"] - r["wait_s"])
                                                          / args.steps * 1e6, 1),
                          "host_wait_us_per_step": round(r["wait_s"] / args.steps * 1e6, 1),
                          "comm": r["comm"], "preheat_ms": args.preheat_ms,
                          "ranks_consistent": consistent if world > 1 else None,
                          "preflight": pf,
                          "dense_tflops": round(cfg.dense_flops_per_example() * value / 1e12, 1),
                          "sol": {k: round(v, 4) for k, v in sol.items()}}),
              file=sys.stderr, flush=True)
        mname = "DLRM" if args.model == "dlrm" else "DCN-v2"
        rname = {"1tb": "1TB", "kaggle": "Kaggle", "gt1tb": "gt1TB", "tiny": "tiny"}[args.rows]
        src = {"fresh": "a fresh batch per step from the on-device generator (side stream)",
               "instep": "a fresh batch per step generated inside the step graphs",
               "pool": f"a pool of {args.pool} pre-generated device batches, cycled",
               "host": "C++ host generator + pinned copy-stream H2D"}[args.data]
        emit_result(json.dumps({
            "metric": f"examples/sec (whole node) {mname} on Criteo-{rname}-shaped synthetic",
            "value": round(value, 1), "unit": "examples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": (round(value / (EAGER_BASELINE_EX_S[args.rows] * world), 2)
                            if args.model == "dlrm" and args.rows in EAGER_BASELINE_EX_S
                            and args.batch == 8192 else None),
            "sol_ms": round(sol["sol_ms"], 4),
            "frac_of_sol": round(sol["sol_ms"] / ms, 3),
            "preheat_ms": args.preheat_ms,
            "hip_graph_packet_capture": RUNTIME_MODE,
            "comm_path": comm_path,
            "attempt": int(os.environ.get("TDFO_ATTEMPT", "0")),
            "ranks_consistent": consistent if world > 1 else None,
            "dtype": "bf16",
            "data": f"synthetic (Criteo-{args.rows}-shaped, {args.dist} ids, random-init "
                    f"embeddings, {src})",
            "config": {"model": mname,
                       "global_batch": B * world, "seq_len": None,
                       "parallelism": parallelism(tr.plan, world),
                       "tables": f"criteo-{args.rows}", "embedding_dim": cfg.embedding_dim,
                       "per_gpu_batch": B}}))
    r["loop"].close()
    reset()


if __name__ == "__main__":
    main()
