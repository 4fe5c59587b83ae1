"""Build libeggroll.so (HIP, gfx950) in-tree with plain hipcc — no torch in the C-ABI.

`python -m hyperscalees_t2i_amd.build_ext` (also run by `__graft_entry__.build()`).
The library lands in hyperscalees_t2i_amd/_build/ so it travels with the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
LIB = BUILD / "libeggroll.so"
SOURCES = ["eggroll_es.hip", "eggroll_lora.hip", "eggroll_model.hip"]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build libeggroll)")


STAMP = LIB.with_name(LIB.name + ".srcsha256")


def _stale() -> bool:
    """The library is current iff its stamp holds the digest of today's sources (content, not mtime:
    a snapshot copied to another machine keeps its bytes but not necessarily its timestamps)."""
    from ._lib import source_digest
    if not LIB.exists() or not STAMP.exists():
        return True
    return STAMP.read_text().strip() != source_digest()


def build(force: bool = False, verbose: bool = True) -> Path:
    from ._lib import source_digest
    if not force and not _stale():
        return LIB
    digest = source_digest()
    BUILD.mkdir(parents=True, exist_ok=True)
    objs, procs = [], []
    for s in SOURCES:   # the translation units compile in parallel (one hipcc each)
        obj = BUILD / (Path(s).stem + ".o")
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c",
               "-Wall", "-Wno-unused-function", f"-I{ROOT / 'include'}", str(CSRC / s), "-o", str(obj)]
        if verbose:
            print("[build]", " ".join(cmd), flush=True)
        procs.append((s, subprocess.Popen(cmd)))
        objs.append(str(obj))
    failed = [s for s, pr in procs if pr.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, f"hipcc {failed}")
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", str(tmp)]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    STAMP.write_text(digest + "\n")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(LIB)
