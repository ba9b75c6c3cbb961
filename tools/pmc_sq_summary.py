"""Per-kernel SQ counter totals per dispatch for tools/gpu_pmc_sq.sh runs:
python tools/pmc_sq_summary.py TAG"""
import collections
import csv
import glob
import os
import sys

d = os.path.join("gpurun_out", sys.argv[1])
for sd in sorted(glob.glob(os.path.join(d, "set*"))):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in sorted(glob.glob(os.path.join(sd, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"][:40]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    print(os.path.basename(sd))
    for k, cs in acc.items():
        if "jit" not in k and "tis_" not in k:
            continue
        print("  ", k)
        for c, v in sorted(cs.items()):
            n = max(1, len(disp[(k, c)]))
            print(f"     {c:22s} per-dispatch {v / n:18.1f}")
