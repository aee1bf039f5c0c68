"""Sum rocprofv3 PMC counters per kernel-name substring over a run's passes.
    python tools/pmc_sum.py gpurun_out/TAG vare"""
import collections
import csv
import glob
import sys

root, pat = sys.argv[1], sys.argv[2]
agg, calls = collections.defaultdict(float), collections.Counter()
for f in glob.glob(f"{root}/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            calls[(f, r["Counter_Name"])] += 1
n = max(calls.values()) if calls else 1
for k, v in sorted(agg.items()):
    print(f"{k:24s} {v / n:16.4g}  per call")
