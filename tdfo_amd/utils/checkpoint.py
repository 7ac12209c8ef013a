"""Checkpoint formats.

1. Flax-compatible ``model_params.pt`` (jax-flax/models.py:128-131, written at
   jax-flax/train.py:164 / train_dp.py:247): ``flax.serialization.to_bytes``
   is msgpack of the nested param dict, each array packed as msgpack
   ExtType(1, msgpack((shape, dtype_name, C-order bytes))); arrays above 1 GiB
   are split into ``{"__msgpack_chunked_array__": True, "shape", "chunks"}``.
   Implemented here with ``msgpack`` directly (no flax/jax), byte-compatible
   so the reference's ``load_params`` (jax-flax/models.py:134-139) can read it.
   Unpacking never executes anything from the file (plain msgpack + frombuffer).

2. Torch ``.pth`` state dicts (torchrec/train.py:172-177): written with
   ``torch.save``; read back only with ``torch.load(weights_only=True)``.

3. Sharded resume checkpoints for TB-scale tables: one file per
   rank (its table shards + optimizer state, saved with torch.save of plain
   tensors) plus a JSON manifest (step, world size, plan summary, per-rank
   file names, RNG/loader positions). Loading verifies the manifest matches
   the current plan.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Any, Dict, Optional

import msgpack
import numpy as np
import torch

_EXT_NDARRAY = 1
_EXT_NPSCALAR = 3
_MAX_CHUNK = 2 ** 30
_CHUNK_KEY = "__msgpack_chunked_array__"


def _to_numpy(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu()
        if x.dtype == torch.bfloat16:
            x = x.float()
        return x.contiguous().numpy()
    return np.asarray(x)


def _nd_bytes(arr: np.ndarray) -> bytes:
    arr = np.ascontiguousarray(arr)
    return msgpack.packb((list(arr.shape), arr.dtype.name, arr.tobytes("C")), use_bin_type=True)


def _ext_pack(x):
    if isinstance(x, np.ndarray):
        return msgpack.ExtType(_EXT_NDARRAY, _nd_bytes(x))
    if isinstance(x, np.generic):
        return msgpack.ExtType(_EXT_NPSCALAR, _nd_bytes(np.asarray(x)))
    raise TypeError(f"cannot serialize {type(x)}")


def _prepare(tree):
    if isinstance(tree, dict):
        return {str(k): _prepare(v) for k, v in tree.items()}
    if isinstance(tree, (list, tuple)):
        # flax state dicts turn sequences into {"0": .., "1": ..}
        return {str(i): _prepare(v) for i, v in enumerate(tree)}
    arr = _to_numpy(tree) if isinstance(tree, (torch.Tensor, np.ndarray)) else tree
    if isinstance(arr, np.ndarray) and arr.nbytes > _MAX_CHUNK:
        flat = arr.reshape(-1)
        per = max(1, _MAX_CHUNK // arr.itemsize)
        chunks = {str(i): flat[s: s + per] for i, s in enumerate(range(0, flat.size, per))}
        return {_CHUNK_KEY: True, "shape": list(arr.shape), "chunks": chunks}
    return arr


def to_flax_bytes(tree: Dict[str, Any]) -> bytes:
    return msgpack.packb(_prepare(tree), default=_ext_pack, strict_types=True)


def _ext_unpack(code, data):
    if code in (_EXT_NDARRAY, _EXT_NPSCALAR):
        shape, dtype, buf = msgpack.unpackb(data, raw=False)
        arr = np.frombuffer(buf, dtype=np.dtype(dtype)).reshape(shape).copy()
        return arr if code == _EXT_NDARRAY else arr[()]
    return msgpack.ExtType(code, data)


def _unchunk(tree):
    if isinstance(tree, dict):
        if tree.get(_CHUNK_KEY):
            parts = [tree["chunks"][str(i)] for i in range(len(tree["chunks"]))]
            return np.concatenate(parts).reshape(tree["shape"])
        return {k: _unchunk(v) for k, v in tree.items()}
    return tree


def from_flax_bytes(data: bytes) -> Dict[str, Any]:
    return _unchunk(msgpack.unpackb(data, ext_hook=_ext_unpack, raw=False,
                                    max_bin_len=2 ** 62, max_str_len=2 ** 31))


def save_flax_params(params: Dict[str, Any], path: str = "model_params.pt"):
    with open(path, "wb") as f:
        f.write(to_flax_bytes(params))


def load_flax_params(path: str = "model_params.pt") -> Dict[str, Any]:
    with open(path, "rb") as f:
        return from_flax_bytes(f.read())


# ------------------------------------------------------------------ torch
def bert4rec_ckpt_name(epoch: int) -> str:
    """Reference quirk Q8 (torchrec/train.py:172-177): no separator."""
    return "bert4rec" + f"epoch_{epoch}_model.pth"


def save_state_dict(sd: Dict[str, torch.Tensor], path: str):
    torch.save({k: (v.detach().cpu() if isinstance(v, torch.Tensor) else v) for k, v in sd.items()},
               path)


def load_state_dict(path: str) -> Dict[str, torch.Tensor]:
    return torch.load(path, map_location="cpu", weights_only=True)


# ---------------------------------------------------------------- sharded
def save_sharded(dirpath: str, rank: int, world: int, step: int, tensors: Dict[str, torch.Tensor],
                 meta: Optional[Dict[str, Any]] = None, barrier=None):
    """Write this rank's shard; rank 0 writes the manifest after a barrier.
    The manifest is written last (atomically renamed), so a checkpoint with a
    manifest is complete."""
    d = Path(dirpath)
    d.mkdir(parents=True, exist_ok=True)
    fname = f"shard_{rank:05d}_of_{world:05d}.pt"
    tmp = d / (fname + ".tmp")
    torch.save({k: v.detach().cpu() for k, v in tensors.items()}, tmp)
    os.replace(tmp, d / fname)
    if barrier is not None:
        barrier()
    if rank == 0:
        man = {"step": int(step), "world_size": int(world),
               "files": [f"shard_{r:05d}_of_{world:05d}.pt" for r in range(world)],
               "meta": meta or {}}
        tmpm = d / "manifest.json.tmp"
        tmpm.write_text(json.dumps(man, indent=2))
        os.replace(tmpm, d / "manifest.json")
    if barrier is not None:
        barrier()


def load_manifest(dirpath: str) -> Optional[Dict[str, Any]]:
    p = Path(dirpath) / "manifest.json"
    if not p.exists():
        return None
    return json.loads(p.read_text())


def load_sharded(dirpath: str, rank: int, world: int,
                 expect_meta: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    man = load_manifest(dirpath)
    if man is None:
        raise FileNotFoundError(f"no complete checkpoint in {dirpath}")
    if man["world_size"] != world:
        raise ValueError(f"checkpoint has world_size {man['world_size']}, running with {world}")
    if expect_meta:
        for k, v in expect_meta.items():
            if man["meta"].get(k) != v:
                raise ValueError(f"checkpoint {k}={man['meta'].get(k)!r} != current {v!r}")
    tensors = torch.load(Path(dirpath) / man["files"][rank], map_location="cpu", weights_only=True)
    return {"step": man["step"], "meta": man["meta"], "tensors": tensors}
