"""Streamed, reshardable checkpoints for TB-scale sharded embeddings.

The role of the reference's TF ``ModelCheckpoint`` / ``BackupAndRestore``
(tensorflow2/train_ps.py:148-157) and of the torchrec ``state_dict`` save
(torchrec/train.py:172-177), sized for tables that do not fit one host's
memory: DCN-v2's >1 TB row-wise set is ~145 GB of table + optimizer state
per rank at 8 ranks.

Layout (one directory per checkpoint)::

    manifest.json          written last (atomic rename) => the checkpoint is complete
    dense.pt               replicated dense params + optimizer moments + step counters (rank 0)
    rank_00003.json        index of the pieces rank 3 wrote
    t12.r0-2458261.c0-128.w.bin        fp32 [rows, cols] row-major, raw
    t12.r0-2458261.c0-128.s1.bin       optimizer state 1 ([rows] row-wise / [rows, cols])
    ...

Each rank streams every piece it owns -- (table, row range, column range)
of its table-wise / row-wise / column-wise shards; replicated tables only
from rank 0 -- device -> host -> file in bounded row chunks (``chunk_bytes``),
never materialising its shard on the host. Loading maps the pieces the
*current* plan gives this rank onto the saved pieces that overlap them and
reads just those rows through ``np.memmap``, again in bounded chunks, so a
checkpoint written at world size W (any plan) loads at any other world size
or plan. Row-wise Adagrad keeps one state per row per column block; when a
row's columns are re-split, the new block takes the width-weighted mean of
the saved blocks' states it covers.

Nothing in a checkpoint is executed on load: raw float32 files, JSON, and
``torch.load(weights_only=True)`` for the dense file.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

FORMAT = "tdfo-sharded-v2"


def _piece_name(t: int, lo: int, hi: int, step: int, c0: int, c1: int) -> str:
    rs = f"r{lo}-{hi}" + (f"s{step}" if step != 1 else "")
    return f"t{t}.{rs}.c{c0}-{c1}"


def _write_rows(path: Path, view: torch.Tensor, chunk_bytes: int):
    """Stream ``view`` ([rows] or [rows, cols], any device) to a raw fp32 file."""
    rows = view.shape[0]
    per_row = max(1, (view.numel() // max(1, rows)) * 4)
    step = max(1, chunk_bytes // per_row)
    tmp = path.with_suffix(path.suffix + ".tmp")
    with open(tmp, "wb") as f:
        for r0 in range(0, rows, step):
            view[r0: r0 + step].detach().to("cpu", torch.float32).contiguous().numpy().tofile(f)
    os.replace(tmp, path)


def local_pieces(emb) -> List[Dict]:
    """Pieces of the embedding tables this rank owns under its plan: dicts with
    table, global rows ``lo, lo + step, ... < hi`` (step 1: a contiguous range;
    W for a round-robin row-wise shard), cols [c0, c1), replicated flag, the
    weight view (one row per piece row, in that order) and the
    optimizer-state views (``state1`` row-wise [rows] or [rows, cols])."""
    out = []
    for t in range(emb.T):
        loc = emb._local_slices(t)
        if loc is None:
            continue
        store, i, sl = loc
        n = len(range(sl.start, sl.stop, sl.step))
        if n <= 0:
            continue
        c0, w = emb.table_cols(t)
        r0 = store.row_offset_host[i]
        states = {}
        for name in ("state1", "state2"):
            st = getattr(store, name)
            if st is None:
                continue
            states[name] = st[r0: r0 + n]
        out.append({"table": t, "lo": sl.start, "hi": sl.stop, "step": sl.step, "c0": c0,
                    "c1": c0 + w, "replicated": t in emb.dp_tables,
                    "weight": store.weight[r0: r0 + n], "states": states})
    return out


def save(tr, dirpath: str, step: int, rank: int, world: int, meta: Optional[Dict] = None,
         barrier: Optional[Callable[[], None]] = None, chunk_bytes: int = 256 << 20):
    """Write this rank's pieces (streamed), rank 0 the dense state and, after a
    barrier, the manifest (last, atomically)."""
    d = Path(dirpath)
    d.mkdir(parents=True, exist_ok=True)
    if hasattr(tr, "sync_streams"):
        tr.sync_streams()                  # side-stream table updates of issued steps
    index = []
    for p in local_pieces(tr.emb):
        if p["replicated"] and rank != 0:
            continue
        base = _piece_name(p["table"], p["lo"], p["hi"], p["step"], p["c0"], p["c1"])
        files = {"weight": base + ".w.bin"}
        _write_rows(d / files["weight"], p["weight"], chunk_bytes)
        for name, view in p["states"].items():
            files[name] = base + (".s1.bin" if name == "state1" else ".s2.bin")
            _write_rows(d / files[name], view, chunk_bytes)
        index.append({k: p[k] for k in ("table", "lo", "hi", "step", "c0", "c1")} |
                     {"files": files, "state1_rowwise": bool("state1" in p["states"] and
                                                             p["states"]["state1"].dim() == 1)})
    (d / f"rank_{rank:05d}.json").write_text(json.dumps(index))
    if rank == 0:
        dense = {k: v.detach().cpu() for k, v in tr.dense_state().items()}
        torch.save(dense, d / "dense.pt.tmp")
        os.replace(d / "dense.pt.tmp", d / "dense.pt")
    if barrier is not None:
        barrier()
    if rank == 0:
        emb = tr.emb
        man = {"format": FORMAT, "step": int(step), "world_size": int(world),
               "ranks": [f"rank_{r:05d}.json" for r in range(world)],
               "tables": [{"name": t.name, "rows": t.num_embeddings, "dim": t.embedding_dim}
                          for t in emb.tables],
               "optimizer": emb.optim.name,
               "plan": [{"table": s.table, "kind": s.kind, "ranks": list(s.ranks),
                         "row_blocks": list(s.row_blocks), "col_blocks": list(s.col_blocks)}
                        for s in emb.plan.shards],
               "meta": meta or {}}
        (d / "manifest.json.tmp").write_text(json.dumps(man, indent=1))
        os.replace(d / "manifest.json.tmp", d / "manifest.json")
    if barrier is not None:
        barrier()


def is_v2(dirpath: str) -> bool:
    p = Path(dirpath) / "manifest.json"
    return p.exists() and json.loads(p.read_text()).get("format") == FORMAT


def _saved_pieces(d: Path, man: Dict) -> Dict[int, List[Dict]]:
    by_table: Dict[int, List[Dict]] = {}
    for f in man["ranks"]:
        for p in json.loads((d / f).read_text()):
            by_table.setdefault(p["table"], []).append(p)
    return by_table


def _rows(sp: Dict) -> range:
    return range(sp["lo"], sp["hi"], sp.get("step", 1))


def _copy_region(dst: torch.Tensor, d: Path, sp: Dict, fname: str, lo: int, hi: int, c0: int,
                 c1: int, rowwise: bool, chunk_bytes: int, accumulate_weight: float = 0.0):
    """dst[rows lo..hi of the table, cols c0..c1] <- saved contiguous piece
    ``sp`` (the caller passes the intersection). ``rowwise``: dst is a [rows]
    state; with accumulate_weight > 0 it is accumulated (width-weighted mean)."""
    rows_s = sp["hi"] - sp["lo"]
    cols_s = sp["c1"] - sp["c0"]
    shape = (rows_s,) if rowwise else (rows_s, cols_s)
    mm = np.memmap(d / fname, dtype=np.float32, mode="r", shape=shape)
    per_row = max(1, (c1 - c0) * 4)
    step = max(1, chunk_bytes // per_row)
    for r0 in range(lo, hi, step):
        r1 = min(hi, r0 + step)
        if rowwise:
            src = torch.from_numpy(np.array(mm[r0 - sp["lo"]: r1 - sp["lo"]]))
        else:
            src = torch.from_numpy(np.array(mm[r0 - sp["lo"]: r1 - sp["lo"],
                                               c0 - sp["c0"]: c1 - sp["c0"]]))
        src = src.to(dst.device)
        if rowwise and accumulate_weight:
            dst[r0 - lo: r1 - lo] += accumulate_weight * src
        else:
            dst[r0 - lo: r1 - lo] = src
    del mm


def _copy_strided(p: Dict, d: Path, sp: Dict, chunk_bytes: int) -> int:
    """Local piece ``p`` <- every row it shares with saved piece ``sp`` when
    either is strided (round-robin row-wise shards): the local rows are
    walked in chunks, mapped to global ids, and the saved rows they hit are
    gathered from the memory-mapped files. Returns the elements covered."""
    pr, srows = _rows(p), _rows(sp)
    cl, ch = max(p["c0"], sp["c0"]), min(p["c1"], sp["c1"])
    if cl >= ch or not pr or not srows:
        return 0
    n_s, w_s = len(srows), sp["c1"] - sp["c0"]
    per_row = max(1, (p["c1"] - p["c0"]) * 4)
    chunk = max(1, chunk_bytes // per_row)
    covered = 0
    files = {"weight": (p["weight"], False)}
    for name, view in p["states"].items():
        if name not in sp["files"]:
            raise ValueError(f"checkpoint piece of table {p['table']} lacks {name}")
        files[name] = (view, view.dim() == 1)
    mms = {k: np.memmap(d / sp["files"][k], dtype=np.float32, mode="r",
                        shape=(n_s,) if rw else (n_s, w_s)) for k, (_, rw) in files.items()}
    sst = sp.get("step", 1)
    for k0 in range(0, len(pr), chunk):
        ids = torch.arange(pr.start + k0 * pr.step,
                           min(pr.stop, pr.start + (k0 + chunk) * pr.step), pr.step)
        hit = (ids >= sp["lo"]) & (ids < sp["hi"]) & ((ids - sp["lo"]) % sst == 0)
        if not bool(hit.any()):
            continue
        loc = (torch.nonzero(hit).view(-1) + k0).numpy()
        src = ((ids[hit] - sp["lo"]) // sst).numpy()
        covered += len(loc) * (ch - cl)
        for k, (view, rw) in files.items():
            li = torch.from_numpy(loc).to(view.device)
            if rw:
                vals = torch.from_numpy(np.asarray(mms[k][src])).to(view.device)
                view[li] += ((ch - cl) / (p["c1"] - p["c0"])) * vals
            else:
                vals = np.asarray(mms[k][src][:, cl - sp["c0"]: ch - sp["c0"]])
                view[li, cl - p["c0"]: ch - p["c0"]] = torch.from_numpy(vals).to(view.device)
    del mms
    return covered


def load(tr, dirpath: str, rank: int, world: int, expect_meta: Optional[Dict] = None,
         chunk_bytes: int = 256 << 20) -> int:
    """Load a v2 checkpoint written at any world size / plan into ``tr``'s
    current plan. Returns the step."""
    d = Path(dirpath)
    man = json.loads((d / "manifest.json").read_text())
    if man.get("format") != FORMAT:
        raise ValueError(f"{dirpath}: not a {FORMAT} checkpoint")
    if expect_meta:
        for k, v in expect_meta.items():
            if k in ("world_size", "strategy"):
                continue                   # resharding across world sizes / plans is supported
            if man["meta"].get(k) != v:
                raise ValueError(f"checkpoint {k}={man['meta'].get(k)!r} != current {v!r}")
    emb = tr.emb
    if [t["rows"] for t in man["tables"]] != [t.num_embeddings for t in emb.tables]:
        raise ValueError("checkpoint table cardinalities differ from the model's")
    if man["optimizer"] != emb.optim.name:
        raise ValueError(f"checkpoint optimizer {man['optimizer']} != {emb.optim.name}")
    saved = _saved_pieces(d, man)
    with torch.no_grad():
        for p in local_pieces(emb):
            t, lo, hi, c0, c1 = p["table"], p["lo"], p["hi"], p["c0"], p["c1"]
            cands = saved.get(t, [])
            covered = 0
            rw_state = p["states"].get("state1")
            rowwise = rw_state is not None and rw_state.dim() == 1
            if rowwise:
                rw_state.zero_()
            for sp in cands:
                if p["step"] != 1 or sp.get("step", 1) != 1:
                    covered += _copy_strided(p, d, sp, chunk_bytes)
                    continue
                rl, rh = max(lo, sp["lo"]), min(hi, sp["hi"])
                cl, ch = max(c0, sp["c0"]), min(c1, sp["c1"])
                if rl >= rh or cl >= ch:
                    continue
                covered += (rh - rl) * (ch - cl)
                _copy_region(p["weight"][rl - lo: rh - lo, cl - c0: ch - c0], d, sp,
                             sp["files"]["weight"], rl, rh, cl, ch, False, chunk_bytes)
                for name, view in p["states"].items():
                    if name not in sp["files"]:
                        raise ValueError(f"checkpoint piece of table {t} lacks {name}")
                    if view.dim() == 1:        # row-wise state: width-weighted mean
                        _copy_region(view[rl - lo: rh - lo], d, sp, sp["files"][name], rl, rh,
                                     sp["c0"], sp["c1"], True, chunk_bytes,
                                     accumulate_weight=(ch - cl) / (c1 - c0))
                    else:
                        _copy_region(view[rl - lo: rh - lo, cl - c0: ch - c0], d, sp,
                                     sp["files"][name], rl, rh, cl, ch, False, chunk_bytes)
            want = len(_rows(p)) * (c1 - c0)
            if covered != want:
                raise ValueError(f"checkpoint does not cover table {t} rows {_rows(p)} "
                                 f"cols [{c0},{c1}) ({covered} of {want})")
        dense = torch.load(d / "dense.pt", map_location="cpu", weights_only=True)
        tr.load_dense_state(dense)
    return int(man["step"])
