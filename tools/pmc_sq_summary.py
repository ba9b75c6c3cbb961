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
        # derived, per dispatch of the executor kernel
        per = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
        if per.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in per:
            print(f"     VALU lane utilisation (THREAD_CYCLES_VALU / (ACTIVE_INST_VALU * 64)) "
                  f"{per['SQ_THREAD_CYCLES_VALU'] / (per['SQ_ACTIVE_INST_VALU'] * 64):.3f}")
        rec = None
        for log in sorted(glob.glob(os.path.join(sd, "pmc*.log"))):
            for line in open(log):
                if line.startswith("{"):
                    import json

                    rec = json.loads(line)
        if rec and "jit" in k:
            retired = rec["node_instr_per_lane"] * rec["config"]["lanes_per_gpu"]
            print(f"     retired node-instructions per dispatch {retired:.4g} ({rec['config']['workload']})")
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64"):
                if c in per:
                    print(f"     {c} lane-ops per node-instruction {per[c] * 64 / retired:.3f}")
