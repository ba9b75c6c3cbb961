"""Roofline of the stateful sessions from a
tools/gpu_sessprof.sh run:

    python tools/sess_roofline.py TAG [OUT.json]

Per launch kind (percall: one call per instance per launch; burst: `calls`
sequential calls per instance in one launch), from the probe's JSON line, the
rocprofv3 kernel statistics and the PMC passes:

  * launches per call: which kernels ran per launch (mk_sess_exec and the
    interpreter tis_session, which first imports any call handed off to it
    and otherwise exits at once) and their average durations;
  * algorithmic bytes of mk_sess_exec per launch, per instance:
      state  2 x (4 B superblock + 8 B x live registers)  (loaded once, stored once)
      calls  k x (8 B int64 input + 4 B out + 1 B status + 4 B steps)
      slots  4 B per PUSH and per POP that reach memory (0 here: the compiled
             session keeps the example network's stack entry in a register)
    (program.go:80-92 state kept across calls; master.go:216-219 one input,
    one output per call);
  * HBM bytes from FETCH_SIZE (x2, the gfx950 correction of tools/pmc_profile.py)
    and WRITE_SIZE, and the executed VALU work (SQ_INSTS_VALU x 64);
  * roofline: algorithmic bytes / mk_sess_exec's average duration against
    8 TB/s, and the whole call (every kernel of the launch, host clock)
    against the same bytes."""
import collections
import csv
import glob
import json
import os
import re
import sys

HBM = 8.0e12
tag = sys.argv[1]
root = os.path.join("gpurun_out", tag)


def stats(mode):
    out = {}
    for p in glob.glob(os.path.join(root, mode, "stats", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            out[r["Name"]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return out


def pmc(mode, pas, kernel="mk_sess_exec"):
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(os.path.join(root, mode, pas, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Kernel_Name"].startswith(kernel):
                rows[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    res = {}
    for c, by in rows.items():
        ids = sorted(by)[1:]  # the first launch loads the module and touches the state
        res[c] = sum(by[i] for i in ids) / max(1, len(ids))
    return res


report = {"source": f"gpurun_out/{tag} (tools/gpu_sessprof.sh + tools/sess_roofline.py)"}
for mode in ("percall", "burst"):
    line = json.loads(open(os.path.join(root, f"{mode}.json")).read().splitlines()[-1])
    n, k = line["instances"], line["calls_per_launch"]
    m = re.search(r"state_regs=(\d+)", line["plan"])
    regs = int(m.group(1)) if m else None
    st = stats(mode)
    ex = next((v for name, v in st.items() if name.startswith("mk_sess_exec")), None)
    state_b = 2 * (4 + 8 * (regs or 0))
    call_b = 8 + 4 + 1 + 4
    alg = n * (state_b + k * call_b)
    fetch = pmc(mode, "FETCH_SIZE").get("FETCH_SIZE")
    write = pmc(mode, "WRITE_SIZE").get("WRITE_SIZE")
    sq = pmc(mode, "SQ")
    hbm = (2 * fetch * 1024 + write * 1024) if fetch is not None and write is not None else None
    rec = {
        "instances": n, "calls_per_launch": k, "state_regs": regs,
        "host_us_per_launch": line["us_per_launch"], "host_us_per_call": line["us_per_call"],
        "kernels_per_launch": {name: v for name, v in st.items()},
        "bytes_per_instance": {"state": state_b, "per_call": call_b},
        "algorithmic_bytes_per_launch": alg,
        "hbm_bytes_per_launch": hbm,
        "traffic_over_algorithmic": hbm / alg if hbm else None,
        "valu_lane_ops_per_launch": sq.get("SQ_INSTS_VALU", 0) * 64 or None,
        "plan": line["plan"],
    }
    if ex:
        rec["roofline"] = {"bound": "hbm", "kernel": "mk_sess_exec", "achieved": alg / (ex["avg_us"] * 1e-6) / 1e9,
                           "peak": HBM / 1e9, "unit": "GB/s", "frac": alg / (ex["avg_us"] * 1e-6) / HBM,
                           "traffic": hbm, "launch_us": ex["avg_us"]}
        rec["call_roofline"] = {"frac": alg / (line["us_per_launch"] * 1e-6) / HBM,
                                "model": "the same bytes over the host-clock time of the launch's kernels"}
    report[mode] = rec
out = sys.argv[2] if len(sys.argv) > 2 else None
txt = json.dumps(report, indent=1)
if out:
    open(out, "w").write(txt + "\n")
print(txt)
