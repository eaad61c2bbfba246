"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/traffic.json:
HBM-side bytes per launch of the score kernels, corrected as
MI355X_MICROARCH.md prescribes (FETCH_SIZE reads 1/2 of a wide streaming read
on gfx950 -> x2; both counters in KiB -> x1024).

    python tools/make_traffic.py <fetch_csv> <write_csv> <key_prefix> [profiles/traffic.json]
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nem-mcmc-optimization_amd"))
from nemo.build import KERNEL_TU, build_id, code_id  # noqa: E402  (the record names the build it measured)


def per_kernel(path, counter):
    """Mean per dispatch (rows of one dispatch summed), the first (cold)
    dispatch of each kernel dropped when there are others."""
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        for tag, kind in (("score_window2_kernel", "win2"), ("score_window_kernel", "win"),
                          ("score_i8w_kernel", "i8w"), ("score_i8l_kernel", "i8l"), ("score_i8s_kernel", "i8s"), ("score_i8o_kernel", "i8o"),
                          ("score_i8_kernel", "i8"), ("score_factored_pipe_kernel", "pipe"),
                          ("score_factored_kernel", "factored"), ("score_kernel", "stream")):
            if tag in name:
                per[(kind, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
                break
    agg = collections.defaultdict(list)
    for (kind, disp), v in sorted(per.items()):
        agg[kind].append(v)
    return {k: sum(v[1:]) / len(v[1:]) if len(v) > 1 else v[0] for k, v in agg.items()}


def main():
    fetch, write, prefix = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json")
    f = per_kernel(fetch, "FETCH_SIZE")
    w = per_kernel(write, "WRITE_SIZE")
    data = json.load(open(out)) if os.path.exists(out) else {}
    for kind in f:
        key = prefix.replace("{kind}", kind)
        data[key] = {"bytes_per_launch": 2 * 1024 * f[kind] + 1024 * w.get(kind, 0.0),
                     "fetch_size_kib": f[kind], "write_size_kib": w.get(kind, 0.0),
                     "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount) + WRITE_SIZE, KiB",
                     "build_id": build_id()}
        if kind in KERNEL_TU:  # the kernel's own unit: the record holds while it is unchanged
            data[key]["code_id"] = code_id(KERNEL_TU[kind])
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(data, indent=1))


if __name__ == "__main__":
    main()
