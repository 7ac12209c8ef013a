"""Build the native HIP library of tdfo_amd for gfx950 (MI355X).

Kernels (``csrc/kernels/*.hip``) include no torch headers and compile in
seconds; ``csrc/bindings.cpp`` registers them as ``torch.ops.tdfo.*``. Objects
are built in parallel with ``hipcc --offload-arch=gfx950`` and linked in-tree
into ``tdfo_amd/lib/libtdfo_hip.so`` so the library travels with the repo
snapshot to the GPU box (no JIT cache, no site-packages install).

The C++ host data library (``csrc/data/*.cpp``) is linked into
``tdfo_amd/lib/libtdfo_data.so`` with plain g++ (no GPU code).

Usage: ``python -m tdfo_amd._build [--force] [--debug]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "lib"
BUILD = ROOT / "build" / "native"
HIP_LIB = LIBDIR / "libtdfo_hip.so"
DATA_LIB = LIBDIR / "libtdfo_data.so"
ARCH = os.environ.get("TDFO_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch  # noqa: F401  (only for paths)

    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    return inc, tdir / "lib"


def _digest(paths, extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    for p in sorted(paths):
        h.update(p.read_bytes())
    return h.hexdigest()


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def build_hip(force: bool = False, debug: bool = False, jobs: int = 8) -> Path:
    headers = list((CSRC / "include").glob("*.h"))
    kernels = sorted((CSRC / "kernels").glob("*.hip"))
    bindings = CSRC / "bindings.cpp"
    comm = sorted((CSRC / "comm").glob("*.cpp"))
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{CSRC / 'include'}",
             "-D__HIP_PLATFORM_AMD__=1", "-munsafe-fp-atomics"]
    if debug:
        flags += ["-g", "-DTDFO_DEBUG=1"]
    # A/B builds of compile-time kernel knobs (e.g. "-DTDFO_EMB_RIF=8")
    flags += os.environ.get("TDFO_HIPCC_EXTRA", "").split()
    inc, tlib = _torch_paths()
    tflags = [f"-I{p}" for p in inc] + ["-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1",
                                        "-DTORCH_EXTENSION_NAME=tdfo_hip"]
    key = _digest(headers + kernels + [bindings] + comm, " ".join(flags + tflags))
    stamp = BUILD / "hip.stamp"
    if not force and HIP_LIB.exists() and stamp.exists() and stamp.read_text() == key:
        return HIP_LIB
    BUILD.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)

    def compile_one(src: Path):
        # per-object stamp (source + every header + flags): an edit to one
        # kernel file recompiles that file only
        obj = BUILD / (src.parent.name + "_" + src.stem + ".o")
        extra = tflags if src.suffix == ".cpp" else []
        ostamp = obj.with_suffix(".stamp")
        okey = _digest(headers + [src], " ".join(flags + extra))
        if not force and obj.exists() and ostamp.exists() and ostamp.read_text() == okey:
            return obj
        lang = ["-x", "hip"] if src.suffix == ".cpp" else []
        _run([HIPCC, *flags, *extra, *lang, "-c", str(src), "-o", str(obj)])
        ostamp.write_text(okey)
        return obj

    srcs = kernels + [bindings] + comm
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = HIP_LIB.with_suffix(".so.tmp")
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp),
          f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
          "-lrccl", f"-Wl,-rpath,{tlib}"])
    os.replace(tmp, HIP_LIB)
    stamp.write_text(key)
    return HIP_LIB


def build_data(force: bool = False) -> Path | None:
    srcs = sorted((CSRC / "data").glob("*.cpp"))
    if not srcs:
        return None
    key = _digest(srcs + list((CSRC / "data").glob("*.h")), "data-v2")
    stamp = BUILD / "data.stamp"
    if not force and DATA_LIB.exists() and stamp.exists() and stamp.read_text() == key:
        return DATA_LIB
    BUILD.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    tmp = DATA_LIB.with_suffix(".so.tmp")
    _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", *map(str, srcs),
          "-o", str(tmp), "-lz"])
    os.replace(tmp, DATA_LIB)
    stamp.write_text(key)
    return DATA_LIB


def build_all(force: bool = False, debug: bool = False) -> None:
    build_data(force)
    build_hip(force, debug)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    args = ap.parse_args(argv)
    build_all(args.force, args.debug)
    print(f"built {HIP_LIB}")


if __name__ == "__main__":
    sys.exit(main())
