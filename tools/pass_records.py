"""Turn a round pass's gpurun_out directory (tools/gpu_final.sh) into the
committed records: per config the kernel stats, the score kernel's PMC rows
(fetch / write / valu / stalls), the trace summary of the bench's launches,
and profiles/valu.json + profiles/traffic.json entries stamped with this
tree's build id and the kernel unit's code id.

    python tools/pass_records.py gpurun_out/r3h r3h
"""
import csv
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
# sub-directory -> (record key prefix, batch)
CONFIGS = {"c3": ("C3", 2048), "w128": ("W128", 2048), "c5": ("C5", 2048), "stream": ("C3", 128)}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out = os.path.join(REPO, "profiles", "r3")
    for sub, (key, b) in CONFIGS.items():
        d = os.path.join(src, sub)
        if not os.path.isdir(d):
            continue
        shutil.copy(os.path.join(d, "trace", "t_kernel_stats.csv"), os.path.join(out, f"{tag}_{sub}_kernel_stats.csv"))
        for part, pre in (("fetch", "f"), ("write", "w"), ("valu", "v"), ("stalls", "s")):
            p = os.path.join(d, part, f"{pre}_counter_collection.csv")
            if not os.path.exists(p):
                continue
            rows = list(csv.DictReader(open(p)))
            keep = [r for r in rows if "score_" in r["Kernel_Name"]]
            with open(os.path.join(out, f"{tag}_{sub}_pmc_{part}.csv"), "w", newline="") as fh:
                w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(keep)
        summ = subprocess.run([sys.executable, os.path.join(HERE, "trace_filter.py"),
                               os.path.join(d, "trace", "t_kernel_trace.csv")], capture_output=True, text=True,
                              check=True).stdout
        open(os.path.join(out, f"{tag}_{sub}_trace_summary.csv"), "w").write(summ)
        print(sub, summ.strip().splitlines()[-1] if summ.strip() else "")
        prefix = f"{key}:{{kind}}:b{b}"
        subprocess.run([sys.executable, os.path.join(HERE, "make_valu.py"),
                        os.path.join(d, "valu", "v_counter_collection.csv"), prefix], check=True, capture_output=True)
        subprocess.run([sys.executable, os.path.join(HERE, "make_traffic.py"),
                        os.path.join(d, "fetch", "f_counter_collection.csv"),
                        os.path.join(d, "write", "w_counter_collection.csv"), prefix], check=True,
                       capture_output=True)
    bench = os.path.join(src, "bench.log")
    if os.path.exists(bench):
        line = [ln for ln in open(bench) if ln.startswith("{")][-1]
        open(os.path.join(out, f"{tag}_bench.json"), "w").write(line)
    for name in ("pytest_gpu.log", "parity_stats.log"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(out, f"{tag}_{name.replace('.log', '.txt')}"))


if __name__ == "__main__":
    main()
