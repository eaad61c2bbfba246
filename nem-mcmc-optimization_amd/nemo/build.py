"""Build ``libnemo.so`` (HIP for gfx950) in-tree.

    python -m nemo.build            # from nem-mcmc-optimization_amd/

One hipcc invocation compiles the kernels and the C-ABI into a shared library
next to this file, so the built object travels with the repository snapshot to
the GPU box.  The build is skipped when the library is newer than every source.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC_DIR = os.path.join(os.path.dirname(PKG_DIR), "csrc")
REPO = os.path.dirname(os.path.dirname(PKG_DIR))
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG_DIR, "libnemo.so")
ARCH = os.environ.get("NEMO_OFFLOAD_ARCH", "gfx950")


def _sources():
    return sorted(glob.glob(os.path.join(SRC_DIR, "*.hip")) + glob.glob(os.path.join(SRC_DIR, "*.cpp")))


def _deps():
    return _sources() + glob.glob(os.path.join(SRC_DIR, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the engine needs ROCm's hipcc to build")


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in _deps())


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines=()) -> str:
    """Build the library (``out``/``defines``: instrumented variants for
    tools/ablate.sh; the product is the default in-tree ``libnemo.so``)."""
    target = out or LIB
    if not force and out is None and up_to_date():
        return LIB
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-I", INCLUDE, "-I", SRC_DIR,
           *[f"-D{d}" for d in defines], "-o", target + ".tmp"] + _sources()
    if verbose:
        print(" ".join(cmd), flush=True)
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"hipcc failed ({proc.returncode}):\n{proc.stdout}\n{proc.stderr}")
    if verbose and proc.stderr.strip():
        print(proc.stderr, file=sys.stderr)
    os.replace(target + ".tmp", target)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
