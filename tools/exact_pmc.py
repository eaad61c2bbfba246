"""Per-kernel PMC summary of the exact kernels (tools/gpu_tasks.sh exact_pmc):
VALU issue and LDS occupancy per launch shape from a rocprofv3 --pmc pass.

    python tools/exact_pmc.py gpurun_out/exact_pmc/score/p_counter_collection.csv

valu_busy = 4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), the
bench's definition (bench.py roofline, MI355X_MICROARCH.md's PMC section);
lds_busy = SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM / 8); conflict share =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE."""
import collections
import csv
import re
import sys


def main():
    rows = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(sys.argv[1])):
        m = re.search(r"(exact_\w+|local_opt_exact\w*|score_\w+_kernel)", r.get("Kernel_Name", "")) if "Kernel_Name" in r else None
        name = m.group(1) if m else r.get("Kernel_Name", "kernel")[:40]
        key = (name, int(r["Grid_Size"]), int(r["Workgroup_Size"]))
        rows[key][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for (name, grid, wg), disp in sorted(rows.items()):
        ds = [d for d in disp.values() if "GRBM_GUI_ACTIVE" in d and d["GRBM_GUI_ACTIVE"] > 0]
        if not ds:
            continue
        ds = ds[1:] if len(ds) > 2 else ds   # the first dispatch of a shape runs cold
        g = sum(d["GRBM_GUI_ACTIVE"] for d in ds) / len(ds)
        cyc = g / 8.0
        out = {"launches": len(ds), "grid": grid, "wg": wg, "kernel_cycles": cyc}
        if all("SQ_ACTIVE_INST_VALU" in d for d in ds):
            a = sum(d["SQ_ACTIVE_INST_VALU"] for d in ds) / len(ds)
            out["valu_busy"] = 4 * a / (1024 * cyc)
        if all("SQ_INSTS_VALU" in d for d in ds):
            out["SQ_INSTS_VALU"] = sum(d["SQ_INSTS_VALU"] for d in ds) / len(ds)
        if all("SQ_LDS_IDX_ACTIVE" in d for d in ds):
            li = sum(d["SQ_LDS_IDX_ACTIVE"] for d in ds) / len(ds)
            out["lds_busy"] = li / (256 * cyc)
            if all("SQ_LDS_BANK_CONFLICT" in d for d in ds):
                out["lds_conflict_share"] = sum(d["SQ_LDS_BANK_CONFLICT"] for d in ds) / len(ds) / max(li, 1.0)
        # wave-state split (quad-cycles, summed over waves): parked on a waitcnt /
        # barrier, stalled at issue, issuing
        if all("SQ_WAVE_CYCLES" in d for d in ds):
            wc = sum(d["SQ_WAVE_CYCLES"] for d in ds) / len(ds)
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if all(c in d for d in ds):
                    out[c.lower()[3:] + "_frac"] = sum(d[c] for d in ds) / len(ds) / max(wc, 1.0)
        if all("TCC_HIT_sum" in d and "TCC_MISS_sum" in d for d in ds):
            h = sum(d["TCC_HIT_sum"] for d in ds)
            out["l2_hit_rate"] = h / max(h + sum(d["TCC_MISS_sum"] for d in ds), 1.0)
            out["l2_req_per_launch"] = (h + sum(d["TCC_MISS_sum"] for d in ds)) / len(ds)
        for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
            if all(c in d for d in ds):   # per launch (FETCH / WRITE_SIZE in KB, x2 on gfx950 for bytes)
                out[c] = sum(d[c] for d in ds) / len(ds)
        if all("SQ_WAVES" in d for d in ds):
            out["SQ_WAVES"] = sum(d["SQ_WAVES"] for d in ds) / len(ds)
        print(name, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()})


if __name__ == "__main__":
    main()
