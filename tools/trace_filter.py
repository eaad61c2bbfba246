"""Per-(kernel, grid) launch durations from a rocprofv3 kernel-trace CSV, so
the bench step's own launches can be compared with bench.py's HIP-event
kernel time (the trace of a bench run also holds the extras' launches).

    python tools/trace_filter.py <kernel_trace.csv> [name-substring ...]
"""
import collections
import csv
import statistics
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2:] or ["score_"]
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if not any(s in name for s in subs):
            continue
        key = (name.split("(")[0], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Workgroup_Size_X"]))
        g[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print("kernel,workgroups,workgroup_size,launches,mean_ms,median_ms,min_ms")
    for (name, wg, ws), v in sorted(g.items()):
        print(f"{name},{wg},{ws},{len(v)},{statistics.mean(v):.6f},{statistics.median(v):.6f},{min(v):.6f}")


if __name__ == "__main__":
    main()
