"""Average per-dispatch counters of the kernels matching a substring: python scripts/pmc_report.py DIR SUBSTR"""
import collections
import csv
import glob
import sys

d, sub = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"{d}/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(f"{d}/t/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if sub in r["Name"]:
            print(f"avg duration {float(r['AverageNs']) / 1e3:.1f} us over {r['Calls']} calls: {r['Name'][:120]}")
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v) / len(v):14.4g}")
