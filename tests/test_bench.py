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


def test_profile_records_are_tied_to_the_build(tmp_path, monkeypatch):
    # a PMC record names the libnemo.so build it measured; another build's
    # record is stale and never attached to a fresh timing
    import json
    (tmp_path / "profiles").mkdir()
    rec = {"C3:i8l:b2048": {"build_id": "aaaa", "bytes_per_launch": 6.66e7}}
    (tmp_path / "profiles" / "traffic.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    assert bench.load_record("traffic.json", "C3:i8l:b2048", "aaaa")["bytes_per_launch"] == 6.66e7
    assert bench.load_record("traffic.json", "C3:i8l:b2048", "bbbb") is None
    assert bench.load_record("valu.json", "C3:i8l:b2048", "aaaa") is None


def test_profile_record_holds_while_its_kernel_unit_is_unchanged(tmp_path, monkeypatch):
    # a record of another library build still holds when it names the code id
    # of the kernel's own translation unit as the tree has it now, and the
    # loaded library is this tree's build; a changed unit drops it
    import json
    sys.path.insert(0, os.path.join(HERE, "nem-mcmc-optimization_amd"))
    from nemo import build as nb
    (tmp_path / "profiles").mkdir()
    cid = nb.code_id(nb.KERNEL_TU["i8l"])
    assert cid == nb.code_id("nemo_factored_i8.hip") and cid != nb.code_id("nemo_kernels.hip")
    rec = {"C3:i8l:b2048": {"build_id": "old", "code_id": cid, "bytes_per_launch": 6.66e7},
           "C3:i8w:b2048": {"build_id": "old", "code_id": "feedfeedfeedfeed", "bytes_per_launch": 1.0}}
    (tmp_path / "profiles" / "traffic.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    tree = nb.build_id()
    assert bench.load_record("traffic.json", "C3:i8l:b2048", tree)["bytes_per_launch"] == 6.66e7
    assert bench.load_record("traffic.json", "C3:i8l:b2048", "a-library-of-another-tree") is None
    assert bench.load_record("traffic.json", "C3:i8w:b2048", tree) is None


def test_roofline_is_a_hardware_fraction(monkeypatch):
    # with the PMC record of the build: bound = VALU issue, frac <= 1 against
    # the max-clock issue peak, the int8 matrix cores and HBM beside it <= 1
    valu = {"build_id": "x", "SQ_ACTIVE_INST_VALU": 68724736.0, "SQ_LDS_IDX_ACTIVE": 51627709.0,
            "SQ_LDS_BANK_CONFLICT": 21046973.0, "valu_busy": 0.766, "mfma_busy": 0.322}
    traffic = {"build_id": "x", "bytes_per_launch": 66.6e6}
    monkeypatch.setattr(bench, "load_record", lambda name, key, bid: valu if name == "valu.json" else traffic)
    r = bench.score_roofline("C3", 64, 2000, 0, 2048, 10, 0.1466, 0.149, "x")
    assert r["bound"] == "valu" and 0.5 < r["frac"] <= 1.0
    assert abs(r["frac"] - 4 * 68724736.0 / 0.1466e-3 / (1024 * 2.4e9)) < 1e-12
    for k, v in r["secondary"].items():
        assert 0.0 < v["frac"] <= 1.0, k
    assert 0.25 < r["secondary"]["int8_mfma"]["frac"] < 0.4
    assert r["fp64_equivalent"]["vs_f64_mfma_peak"] > 1.0   # the note, not the headline
    assert r["traffic"] == 66.6e6 and r["evals_per_launch"] == 2048   # HBM bytes per launch
    # without a record of this build: the live int8 matrix-core fraction
    monkeypatch.setattr(bench, "load_record", lambda name, key, bid: None)
    r = bench.score_roofline("C3", 64, 2000, 0, 2048, 10, 0.1466, 0.149, "y")
    assert r["bound"] == "mfma" and r["frac"] <= 1.0 and r["traffic"] is None


def test_kernel_tags():
    assert bench.kernel_tag(10) == "i8l" and bench.kernel_tag(8) == "i8o" and bench.kernel_tag(4) == "i8"
    assert bench.kernel_tag(9) == "win2" and bench.kernel_tag(2) == "pipe" and bench.kernel_tag(1) == "factored"
    # fact_kernel 20 is score_i8l_kernel split into a prep-only and a walk-only
    # launch; 15 is the capped lookup-table kernel's round-1 form
    assert bench.kernel_tag(20) == "i8l" and bench.kernel_tag(15) == "win" and bench.kernel_tag(13) == "i8s"
    assert bench.kernel_tag(18) == "i8w" and bench.kernel_tag(3) == "pipe"


@pytest.mark.timeout(180)
def test_cpu_baseline_procs_plumbing():
    r = bench.cpu_baseline_procs("C2", nproc=2, seconds=0.5)
    assert r["cores"] == 2 and r["kind"] == "port" and r["value"] > 0


def test_stream_roofline_is_a_hardware_fraction():
    # the streaming kernel's algorithmic bytes exceed HBM's (the table is
    # Infinity-Cache resident and re-read across the batch): priced against
    # the L2 read rate they give a fraction <= 1, HBM from the PMC record
    bpe = bench.algorithmic_bytes_per_eval(64, 2000, 0, 8)
    r = bench.stream_roofline(128, bpe, 0.2925, {"bytes_per_launch": 3.0e8})
    assert r["bound"] == "l2" and 0.3 < r["frac"] <= 1.0
    assert abs(r["achieved"] - 128 * bpe / 0.2925e-3 / 1e9) < 1e-6
    assert 0.0 < r["secondary"]["hbm"]["frac"] <= 1.0 and r["traffic"] == 3.0e8
    assert "secondary" not in bench.stream_roofline(128, bpe, 0.2925, None)
