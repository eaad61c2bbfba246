"""Turn a rocprofv3 PMC pass (SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA
GRBM_GUI_ACTIVE SQ_WAVES) over bench.py into profiles/valu.json: how busy the
VALU of the score kernel is.

    python tools/make_valu.py <pmc_csv> <key_prefix> [profiles/valu.json]

Units (MI355X_MICROARCH.md, PMC notes): SQ_ACTIVE_INST_VALU counts quad-cycles
summed over waves; GRBM_GUI_ACTIVE is the kernel's GPU-busy cycles summed over
the 8 XCDs.  valu_busy = 4 * SQ_ACTIVE_INST_VALU / (1024 SIMDs * GRBM_GUI_ACTIVE / 8):
the fraction of SIMD cycles in which a VALU instruction issued.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
from nemo.build import KERNEL_TU, build_id, code_id  # noqa: E402  (the record names the build it measured)

TAGS = (("score_window2_kernel", "win2"), ("score_window_kernel", "win"), ("score_i8w_kernel", "i8w"), ("score_i8l_kernel", "i8l"), ("score_i8s_kernel", "i8s"), ("score_i8o_kernel", "i8o"), ("score_i8_kernel", "i8"), ("score_factored_pipe_kernel", "pipe"),
        ("score_factored_kernel", "factored"), ("score_kernel", "stream"))


def main():
    src, prefix = sys.argv[1:3]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "valu.json")
    # per dispatch: counter rows are per XCD / SE instance, summed here
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        for tag, kind in TAGS:
            if tag in name:
                per[(kind, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
                break
    # the first dispatch of each kernel runs cold (code and tables not yet
    # resident: ~2.5x the cycles), so it is dropped when there are others
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    first = {}
    for (kind, disp) in sorted(per):
        first.setdefault(kind, disp)
    for (kind, disp), cnt in per.items():
        if disp == first[kind] and sum(1 for k, _ in per if k == kind) > 1:
            continue
        for c, v in cnt.items():
            agg[kind][c].append(v)
    data = json.load(open(out)) if os.path.exists(out) else {}
    for kind, d in agg.items():
        key = prefix.replace("{kind}", kind)
        # passes of the same kernel merge: counters of earlier passes are kept
        old = data.get(key, {})
        m = {k: v for k, v in old.items() if k.isupper()} if old.get("build_id") == build_id() else {}
        m.update({k: sum(v) / len(v) for k, v in d.items()})
        rec = {k: m[k] for k in sorted(m)}
        if "SQ_ACTIVE_INST_VALU" in m and "GRBM_GUI_ACTIVE" in m:
            simd_cyc = 1024.0 * m["GRBM_GUI_ACTIVE"] / 8.0
            rec["valu_busy"] = 4.0 * m["SQ_ACTIVE_INST_VALU"] / simd_cyc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                rec["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cyc
            if "SQ_VALU_MFMA_COEXEC_CYCLES" in m:
                rec["mfma_coexec_frac"] = m["SQ_VALU_MFMA_COEXEC_CYCLES"] / max(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 1.0), 1.0)
            if "SQ_LDS_IDX_ACTIVE" in m:
                rec["lds_busy"] = m["SQ_LDS_IDX_ACTIVE"] / (256.0 * m["GRBM_GUI_ACTIVE"] / 8.0)
        rec["formula"] = ("valu_busy = 4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); "
                          "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / the same; mfma_coexec_frac = "
                          "SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES (MFMA cycles with a VALU "
                          "issue beside them); lds_busy = SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE / 8)")
        rec["build_id"] = build_id()
        if kind in KERNEL_TU:  # the kernel's own unit: the record holds while it is unchanged
            rec["code_id"] = code_id(KERNEL_TU[kind])
        data[key] = rec
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(data, indent=1))


if __name__ == "__main__":
    main()
