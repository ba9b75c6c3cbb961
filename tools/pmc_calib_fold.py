"""Fold tools/gpu_pmc_calib.sh: counted bytes per launch over known bytes
per launch, per access mode and counter (FETCH_SIZE / WRITE_SIZE are KiB,
summed over the XCD rows; the first two launches are warm-up)."""
import collections
import csv
import glob
import json
import os
import sys

out_dir = sys.argv[1]
res = {}
for mode in ("st4", "ld4", "ld16"):
    known = json.load(open(os.path.join(out_dir, f"{mode}.json")))
    row = {"known_bytes": known["bytes_per_launch"], "GBps": known["GBps"]}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        by = collections.defaultdict(float)
        for p in glob.glob(os.path.join(out_dir, mode, c, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                if r["Counter_Name"] == c:
                    by[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        ids = sorted(by)[2:]
        kib = sum(by[i] for i in ids) / max(1, len(ids))
        row[c + "_bytes"] = kib * 1024
        row[c + "_over_known"] = kib * 1024 / known["bytes_per_launch"]
    res[mode] = row
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out_dir, "calib.json"), "w"), indent=1)
