"""Summarise rocprofv3 PMC csv passes per kernel: python tools/pmc_summary.py DIR"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/p*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if not any(s in k for s in ("score", "local_opt", "prep")):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print("  %-32s %16.1f" % (c, sum(v) / len(v)))
