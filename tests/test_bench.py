"""bench.py's bookkeeping on the CPU: the algorithmic figures the roofline is
priced with, the profile records it attaches, and the
multi-process CPU baseline's plumbing (a tiny run of the C2 model)."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402


def test_algorithmic_figures():
    # C3 fp64 streams 33,329,032 B per evaluation
    assert bench.algorithmic_bytes_per_eval(64, 2000, 0, 8) == 33_329_032
    # the factored contraction over the P = S(S-1)/2 permissible pairs
    assert bench.n_pairs(64, 0) == 2016
    assert bench.algorithmic_flops_per_eval(64, 2000, 0) == 2 * 2016 * 2000
    # C5: cap 6 -> 747 pairs (SURVEY.md 8 header)
    assert bench.n_pairs(128, 6) == 747


def test_profile_records_for_the_headline_kernel():
    t = bench.load_traffic("C3:i8l:b2048")
    assert t and t["bytes_per_launch"] > 6e7  # the w01 input, 2048 x 32 KB
    v = bench.load_valu_bound("C3:i8l:b2048")
    assert v and 0.0 < v["valu_busy"] < 1.0 and 0.0 < v["lds_busy"] < 1.0


@pytest.mark.timeout(180)
def test_cpu_baseline_procs_plumbing():
    r = bench.cpu_baseline_procs("C2", nproc=2, seconds=0.5)
    assert r["cores"] == 2 and r["kind"] == "port" and r["value"] > 0
