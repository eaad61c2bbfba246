"""The C-ABI's host logic under the sanitizers, on the CPU.

nem-mcmc-optimization_amd/csrc/nemo_host.h holds everything libnemo.so does
on the host without HIP: the pos checks, the staging validation (factored
form of a table, the knockdown chains), the fixed-point error bounds, the
InverseMethod level schedule (methods.py:117-129: levels must keep the
sequential loop's results) and the queue behind nemo_optimal_weights_begin /
_end.  tests/host/host_check.cpp drives all of it; here it is built with g++
under AddressSanitizer + UndefinedBehaviorSanitizer and under
ThreadSanitizer, and must run clean."""
import os
import shutil
import subprocess

import pytest
from conftest import REPO

SRC = os.path.join(REPO, "tests", "host", "host_check.cpp")
INC = os.path.join(REPO, "nem-mcmc-optimization_amd", "csrc")

SANITIZERS = {
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}


@pytest.mark.parametrize("kind", sorted(SANITIZERS))
def test_host_logic_clean_under_sanitizer(kind, tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / f"host_check_{kind}"
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-Wall", "-Wextra", "-Werror", "-pthread", *SANITIZERS[kind],
           "-I", INC, SRC, "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    res = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.startswith("ok "), res.stdout
    assert "runtime error" not in res.stderr and "WARNING: ThreadSanitizer" not in res.stderr, res.stderr
