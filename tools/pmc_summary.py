"""Average PMC counters per dispatch of each kernel: python tools/pmc_summary.py <tag>"""
import collections
import csv
import glob
import os
import sys

d = os.path.join("gpurun_out", sys.argv[1])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(p)):
        acc[r["Kernel_Name"][:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        # counters arrive per dispatch (summed over dimensions already or per-XCD rows)
        print(f"   {c:24s} mean/dispatch-row {sum(v)/len(v):16.1f}  rows {len(v)}")
