"""Print the key numbers of a gpu_check.sh run: python tools/summarize.py <tag>"""
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
d = os.path.join("gpurun_out", tag)
for name in ("pytest_gpu.log",):
    p = os.path.join(d, name)
    if os.path.exists(p):
        print(name, open(p).read().strip().splitlines()[-1])
for name in sorted(glob.glob(os.path.join(d, "bench*.log"))):
    for line in open(name):
        if line.startswith("{"):
            r = json.loads(line)
            print(f"{os.path.basename(name):28s} {r['value']/1e9:9.1f} G node-instr/s  kernel {r['kernel_ms_per_step']*1e3:8.1f} us"
                  f"  issue-frac {r['roofline']['frac']:.3f}  hbm-frac {r['roofline_hbm']['frac']:.3f}  {r['config'].get('executor','')}")
for p in glob.glob(os.path.join(d, "prof_*", "*kernel_stats.csv")):
    for row in csv.DictReader(open(p)):
        print(f"  {row['Name'][:60]:60s} calls {row['Calls']:>4s} avg {float(row['AverageNs'])/1e3:9.1f} us")
