"""Build ``libnemo.so`` (HIP for gfx950) in-tree.

    python -m nemo.build            # from nem-mcmc-optimization_amd/

hipcc compiles each kernel / C-ABI source to an object (in parallel, one
process per source) and links them into a shared library next to this file,
so the built object travels with the repository snapshot to the GPU box.  The
build is skipped when the library is newer than every source.
"""
from __future__ import annotations

import glob
import hashlib
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

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


def build_id(defines=()) -> str:
    """Hash of every source and header the library is built from, the
    compile flags and the target: the same tree gives the same id on any
    host, so profiler records (profiles/*.json) can name the build they
    measured."""
    h = hashlib.sha256()
    for p in sorted(_deps()):
        h.update(os.path.relpath(p, REPO).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    h.update(repr((ARCH, list(defines), _FLAGS)).encode())
    return h.hexdigest()[:16]


_FLAGS = ("-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function")

# the translation unit each profiled kernel is compiled in (its device code
# is that file and what it includes, nothing else)
KERNEL_TU = {"i8l": "nemo_factored_i8.hip", "i8o": "nemo_factored_i8.hip", "i8s": "nemo_factored_i8.hip",
             "i8": "nemo_factored_i8.hip", "i8w": "nemo_factored_i8.hip", "factored": "nemo_factored.hip",
             "stream": "nemo_kernels.hip", "win": "nemo_window.hip", "win2": "nemo_window.hip"}


def _include_closure(src: str) -> list:
    """``src`` and every quoted #include it reaches in csrc/ or include/."""
    seen, todo = [], [src]
    while todo:
        p = todo.pop()
        if p in seen:
            continue
        seen.append(p)
        with open(p, encoding="utf-8", errors="replace") as fh:
            for line in fh:
                s = line.strip()
                if s.startswith("#include \""):
                    name = s.split('"')[1]
                    for d in (SRC_DIR, INCLUDE):
                        q = os.path.join(d, name)
                        if os.path.exists(q):
                            todo.append(q)
                            break
    return sorted(seen)


def code_id(tu: str, defines=()) -> str:
    """Hash of ONE translation unit's code (the source, its include closure,
    the flags and the target).  A profiler record of a kernel names the code
    id of the unit the kernel is compiled in: a change elsewhere in the
    library (the C ABI, another kernel file) leaves the kernel's machine code,
    and so its counters, unchanged."""
    h = hashlib.sha256()
    for p in _include_closure(os.path.join(SRC_DIR, tu)):
        h.update(os.path.relpath(p, REPO).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    h.update(repr((ARCH, list(defines), _FLAGS)).encode())
    return h.hexdigest()[:16]


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    if not all(os.path.getmtime(p) <= t for p in _deps()):
        return False
    with open(LIB, "rb") as fh:  # built from these very sources (mtimes lie after a checkout)
        return build_id().encode() in fh.read()


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines=()) -> str:
    """Build the library (``out``/``defines``: instrumented variants for
    tools/ablate.sh; the product is the default in-tree ``libnemo.so``)."""
    target = out or LIB
    if not force and out is None and up_to_date():
        return LIB
    flags = [f"--offload-arch={ARCH}", *_FLAGS, "-I", INCLUDE, "-I", SRC_DIR,
             f'-DNEMO_BUILD_ID="{build_id(defines)}"', *[f"-D{d}" for d in defines]]
    jobs = max(1, min(len(_sources()), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        proc = subprocess.run(cmd, capture_output=True, text=True)
        if proc.returncode != 0:
            raise RuntimeError(f"hipcc failed ({proc.returncode}):\n{proc.stdout}\n{proc.stderr}")
        if verbose and proc.stderr.strip():
            print(proc.stderr, file=sys.stderr)

    with tempfile.TemporaryDirectory(prefix="nemo_build_") as tmp:
        objs = [os.path.join(tmp, os.path.basename(src) + ".o") for src in _sources()]
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(run, [[hipcc(), *flags, "-c", src, "-o", o] for src, o in zip(_sources(), objs)]))
        run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-o", target + ".tmp", *objs])
    os.replace(target + ".tmp", target)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
