"""The C-ABI library: builds for gfx950, loads without a GPU, exports every
entry point include/nemo.h declares, and fails loudly (no CPU fallback) when
no device is present."""
import ctypes
import os
import re

import numpy as np
import pytest
from conftest import REPO


def _declared():
    text = open(os.path.join(REPO, "include", "nemo.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nemo_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from nemo import _lib, build
    build.build()
    return _lib.load()


def test_header_and_binding_agree():
    from nemo import _lib
    assert _declared() == sorted(name for name, _, _ in _lib.SIGNATURES)


def test_library_exports_every_declared_symbol(lib):
    for name in _declared():
        assert hasattr(lib, name), name
    # and the symbols are plain C (unmangled) in the dynamic table
    raw = ctypes.CDLL(lib._name)
    for name in _declared():
        getattr(raw, name)


def test_no_device_means_loud_failure(lib):
    from nemo import _lib, engine
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible; this checks the CPU-only container")
    assert lib.nemo_version() >= 10000
    with pytest.raises(_lib.NemoError, match="no HIP device"):
        engine.Engine(np.zeros((3, 4)), np.zeros((2, 2, 4)))
    ctx = ctypes.c_void_p()
    assert lib.nemo_ctx_create(0, 1, 4, 0, ctypes.byref(ctx)) == _lib.NEMO_ERR_ARG
    assert b"num_s" in lib.nemo_last_error()
