#!/usr/bin/env python3
"""Benchmark: simulated TIS node-instructions/sec for the batched /compute path.

One "step" = one pass of the executor over one batch of synthetic /compute
inputs already resident in HBM (BASELINE.json config 2 by default: the
docker-compose example network, 16,777,216 lanes per GPU).  With --gpus N
every rank (one process per GPU) runs its own contiguous shard of global lane
indices -- weak scaling, no data-path collective; RCCL carries only the final
counter reduction and the ordered output gather to rank 0 (`end_to_end`,
timed separately and verified against one launch over every global lane).

Ranks: under torch.distributed.run each process is one rank.  A bare
`python bench.py --gpus N` (N > 1, WORLD_SIZE unset) starts its own N child
ranks first -- fresh processes with the launcher's RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* variables, started before anything loads the executor
or touches a GPU (misaka_net_amd.dist.launch_ranks) -- forwards rank 0's
line and exits non-zero if any rank fails.

Prints ONE JSON line on rank 0 (keys per the driver contract + roofline +
cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _gpus_arg(argv) -> int:
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--gpus", type=int, default=1)
    return p.parse_known_args(argv)[0].gpus


if __name__ == "__main__":
    # importing the package loads no library and touches no GPU (the ctypes
    # binding loads libmisaka_amd.so on first use): the parent stays GPU-free
    from misaka_net_amd import dist as _mkdist

    _n = _gpus_arg(sys.argv[1:])
    if _mkdist.needs_launch(_n, os.environ):
        sys.exit(_mkdist.launch_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], _n))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from misaka_net_amd import _native as N  # noqa: E402

SEED = 0x4D49534B41
METRIC = "simulated TIS node-instructions/sec (whole node) + /compute results/sec at 1/2/4/8 GPU"

# Spec int32 VALU issue: 256 CUs x 4 SIMD x 32 lanes/clk x 2.4 GHz (the FP32
# vector rate of MI355X_MICROARCH.md: 157.3 TFLOP/s = 78.6 T FMA lane-ops/s).
SPEC_LANE_OPS = 256 * 4 * 32 * 2.4e9
K_LANE_OPS = 4  # algorithmic lane-ops per retired node-instruction
HBM_PEAK = 8.0e12
L2_PEAK = 34.5e12  # aggregate XCD L2 bandwidth, MI355X_MICROARCH.md section L2
# LDS (MI355X_MICROARCH.md section LDS): one LDS array per CU, 256 CUs at 2.4 GHz
LDS_CUS, LDS_CLOCK = 256, 2.4e9
# 4-byte stack slots move by ds_write_b32 / ds_read_b32, whose rates the guide
# gives per CU: 64 B/clk for ds_write_b32 (4 cycles per wave-instruction: the
# address and data transfer) and 128 B/clk for ds_read_b32 (2 LDS cycles).  A
# slot is written once (PUSH) and read once (POP): half the LDS-resident
# bytes at each rate.  (Round 3 priced them at 150 TB/s, the guide's
# ds_read_b64/b128 figure: 2-4x too fast for 4-byte slots.)
LDS_WRITE_B32 = 64 * LDS_CUS * LDS_CLOCK  # 39.3 TB/s
LDS_READ_B32 = 128 * LDS_CUS * LDS_CLOCK  # 78.6 TB/s


def lds_slot_seconds(nbytes):
    """Lower bound on the LDS time of `nbytes` of slot traffic, half pushes, half pops."""
    return nbytes / 2 / LDS_WRITE_B32 + nbytes / 2 / LDS_READ_B32

WORKLOADS = {
    # name: (workload, network factory, lanes per GPU, generator kind, mask)
    "c2": ("c2_example_net_16M", mk.networks.example_network, 1 << 24, N.MK_GEN_FULL, 0),
    "c3": ("c3_sample_net_8M_per_gpu", mk.networks.sample_network, 1 << 23, N.MK_GEN_FULL, 0),
    "c4": ("c4_pipeline_d64_1M", lambda: mk.networks.pipeline_network(64), 1 << 20, N.MK_GEN_FULL, 0),
    "c4d256": ("c4_pipeline_d256_512K", lambda: mk.networks.pipeline_network(256), 1 << 19, N.MK_GEN_FULL, 0),
    "c4d1024": ("c4_pipeline_d1024_256K", lambda: mk.networks.pipeline_network(1024), 1 << 18, N.MK_GEN_FULL, 0),
    "c5": ("c5_countdown_4M", mk.networks.countdown_network, 1 << 22, N.MK_GEN_MASKED, 1023),
    # tier census classes (networks.census_classes) whose stack depths follow the
    # data: until r02i tier 2 / tier 1, now dynamic stacks on the native tier
    "t2_dyn_depth": ("t2_dyn_depth_1M", lambda: mk.networks.census_classes()["data_dependent_stack_depth"][0][1],
                     1 << 20, N.MK_GEN_MASKED, 255),
    "t1_two_stacks": ("t1_two_stacks_1M",
                      lambda: mk.networks.census_classes()["two_stacks_independent_depths"][0][1],
                      1 << 20, N.MK_GEN_MASKED, 255),
    # the other two census classes: a JRO dispatch loop (8 arms, x >> 3 rounds) and a 16-node ring
    "t_jro_heavy": ("t_jro_heavy_4M", lambda: mk.networks.census_classes()["jro_heavy"][0][1],
                    1 << 22, N.MK_GEN_MASKED, 1023),
    "t_ring16": ("t_ring16_16M", lambda: mk.networks.census_classes()["sixteen_nodes"][0][1],
                 1 << 24, N.MK_GEN_FULL, 0),
}
# Stack-node traffic per lane (PUSH + POP, 4 bytes each), part of the
# algorithmic bytes: the pipeline's 8 nodes each push `depth` values and pop
# them all (networks.pipeline_program); the other networks have no stacks.
# The census classes push x values (dyn_depth: and pop them; two_stacks: x
# onto each of two stacks) for inputs x uniform in 0..255: 2 * 127.5 slot
# accesses per lane in expectation.
STACK_OPS_PER_LANE = {"c4": 2 * 64 * 8, "c4d256": 2 * 256 * 8, "c4d1024": 2 * 1024 * 8,
                      "t2_dyn_depth": 255, "t1_two_stacks": 255}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def usable_cpus():
    """(threads this process may run at once, whole-host CPU count, cgroup
    quota in CPUs or None): the affinity mask bounded by the cgroup quota."""
    host = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = host
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    for var in ("OMP_NUM_THREADS",):  # the box's CPU share, set by the harness
        v = os.environ.get(var)
        if v and v.isdigit() and quota is None:
            quota = int(v)
    return min(aff, quota or aff), host, quota


def cpu_baseline(nodes, gen_kind, mask, seconds=10.0, refstruct_seconds=5.0):
    """CPU baselines on the host cores, bounded samples of the same workload:
    (i) the oracle (oracle/tis_oracle.c, the C port; test infrastructure)
    batch-parallel on every usable core; (ii) the reference-structured
    emulation (oracle/refstruct.py: a thread per node, a fresh loopback gRPC
    call per network hop, program.go:80-92 / 475-566), sequential /compute
    calls as the reference's single master serves them."""
    from oracle import pyoracle

    threads, host, quota = usable_cpus()
    on = pyoracle.OracleNet(nodes)
    n = 4096
    total_lanes = total_steps = 0
    t_total = 0.0
    while t_total < seconds:
        xs = pyoracle.gen_inputs(SEED, n, kind=gen_kind, mask=mask)
        t0 = time.perf_counter()
        _, _, sp = on.compute_batch(xs, threads=threads)
        dt = time.perf_counter() - t0
        t_total += dt
        total_lanes += n
        total_steps += int(sp.sum())
        if dt < seconds / 8:
            n *= 2
    rec = {
        "value": total_steps / t_total,
        "unit": "node-instr/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{total_lanes} lanes of the same workload in {t_total:.1f} s, oracle/tis_oracle.c, {threads} threads "
                  f"(usable CPUs: affinity bounded by the cgroup / box CPU share)",
        "results_per_s": total_lanes / t_total,
        "nproc": host,
        "cpu_quota": quota,
    }
    if refstruct_seconds > 0:
        try:
            from oracle import refstruct

            xs = pyoracle.gen_inputs(SEED, 256, kind=gen_kind, mask=mask)
            ref = on.compute_batch(xs)
            xs = xs[(ref[1] & pyoracle.ST_HAS_OUTPUT) != 0]  # the reference's /compute hangs without an output
            r = refstruct.time_compute(nodes, xs, seconds=refstruct_seconds) if xs.size else None
            if r and r["results"]:
                rec["reference_structured"] = {
                    "value": r["node_instr_per_s"],
                    "unit": "node-instr/s",
                    "results_per_s": r["results_per_s"],
                    "cores": r["threads"],
                    "kind": "emulation",
                    "sample": f"{r['results']} sequential /compute calls in {r['seconds']:.1f} s through "
                              "oracle/refstruct.py: one thread per program node, a fresh insecure loopback gRPC "
                              "channel per network hop (the reference dials per op over TLS), Python threads",
                }
            else:
                rec["reference_structured"] = {"value": None, "note": "no /compute completed within the sample"}
        except Exception as e:  # pragma: no cover - reported, never fatal
            rec["reference_structured"] = {"value": None, "note": f"emulation failed: {e}"}
    return rec


def measured_profile(workload):
    """The committed rocprofv3 PMC summary for this workload
    (profiles/pmc_<workload>.json, tools/gpu_pmc_all.sh + tools/pmc_profile.py), or {}."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f)


def plan_signature(plan):
    """The executor fields a PMC profile must share with a run to describe it:
    same kernel shape, stack slots and generated source (a profile of the
    HBM-slot kernel says nothing about the LDS one, though both retire the
    same instructions)."""
    f = dict(w.split("=", 1) for w in plan.split() if "=" in w)
    # kernel: hash of the generated module source (a new code generator or
    # layout is a new kernel, whose counters the old profile does not hold)
    return f.get("tier"), f.get("shape"), f.get("slots"), f.get("kernel")


def measured_traffic(workload):
    """HBM bytes per executor launch from the committed PMC pass, or None."""
    return measured_profile(workload).get("hbm_bytes_per_launch")


def occupancy_cap(waves_per_simd):
    """Measured VALU issue cap at this many resident waves per SIMD: the best
    rate over independent chains of full-rate int ops in
    profiles/valu_rates.jsonl (tools/probe/valu_rates.hip, MI355X; rows for
    every occupancy 1..8 since round 6).  A fractional occupancy (15 one-wave
    blocks per CU are 3.75 per SIMD) is priced at its whole part, explicitly:
    `measured_at_waves_per_simd`.  None without a match."""
    p = os.path.join(ROOT, "profiles", "valu_rates.jsonl")
    if not waves_per_simd or not os.path.exists(p):
        return None
    rows = [json.loads(line) for line in open(p) if line.strip()]
    rows = [r for r in rows if r["op"] in ("add_u32_vop2", "sub_clamp_vop3")]
    whole = int(waves_per_simd)
    ws = [r["waves_per_simd"] for r in rows if r["waves_per_simd"] <= whole]
    if not ws:
        return None
    w = max(ws)
    best = max((r for r in rows if r["waves_per_simd"] == w), key=lambda r: r["T_lane_ops"])
    return {"waves_per_simd": waves_per_simd, "measured_at_waves_per_simd": w, "cap": best["T_lane_ops"],
            "unit": "Tlane-op/s", "op": best["op"], "chains": best["chains"],
            "source": "profiles/valu_rates.jsonl"}


def valu_peak(stream):
    """Live dependency-free v_add_u32 probe on this GPU (lane-ops/s)."""
    blocks, iters = 256 * 8 * 4, 2000
    mk.valu_probe_device(blocks, 200, stream=stream)  # warm
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops = mk.valu_probe_device(blocks, iters, stream=stream)
    e1.record()
    torch.cuda.synchronize()
    return ops / (e0.elapsed_time(e1) * 1e-3)


def sessions_leg(net, n, calls, stream):
    """Stateful mode (row f2) at scale: n independent instances of the
    network, each keeping its node state between calls (program.go:80-92),
    `calls` sequential /compute calls per instance (mk_session_compute_device
    per call, inputs and results in HBM, one result buffer per call), timed
    with HIP events on the sessions' stream around `reps` back-to-back passes
    (the host clock around the same passes and a final synchronize is
    reported beside it).  The session kernel is the interpreter's round
    structure with the instances' state loaded from and stored back to HBM
    around each call."""
    sess = net.sessions(n)
    # a stream of its own: a session call given the null stream runs on the
    # session's own stream (mk.h), which events on the null stream would not
    # bracket
    stream = torch.cuda.Stream()
    sh = stream.cuda_stream
    x32 = torch.empty(calls * n, dtype=torch.int32, device="cuda")
    mk.generate_inputs_device(calls * n, x32.data_ptr(), seed=SEED, stream=sh)
    torch.cuda.synchronize()
    x = x32.to(torch.int64).view(calls, n)  # call c of instance i takes x[c, i]
    torch.cuda.synchronize()

    def run(burst, reps=0):
        """From the reset state: one pass (its results are returned), then,
        with reps > 0, `reps` more passes back to back, the instances keeping
        their state as sessions do, timed as one span (HIP events on the
        stream; the host clock beside them).  A single pass between two events
        is not timed (one launch between two events is mostly launch
        latency)."""
        out = torch.empty((calls, n), dtype=torch.int32, device="cuda")
        st = torch.empty((calls, n), dtype=torch.uint8, device="cuda")
        sp = torch.empty((calls, n), dtype=torch.int32, device="cuda")

        def one():
            if burst:  # one launch: every instance's `calls` sequential calls
                sess.compute_seq_device(x.data_ptr(), calls, out.data_ptr(), st.data_ptr(), sp.data_ptr(), stream=sh)
            else:
                for c in range(calls):
                    sess.compute_device(x[c].data_ptr(), out[c].data_ptr(), st[c].data_ptr(), sp[c].data_ptr(),
                                        stream=sh)

        sess.reset()
        torch.cuda.synchronize()
        one()
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            res = (out.clone(), st.clone(), sp.clone())
        torch.cuda.synchronize()
        if not reps:
            return res, None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(reps):
            one()
        e1.record(stream)
        torch.cuda.synchronize()
        host = (time.perf_counter() - t0) / reps
        secs = e0.elapsed_time(e1) * 1e-3 / reps
        outs = int(((st & 0x10) != 0).sum())
        total = int(sp.to(torch.int64).sum())
        return res, {"results_per_s": outs / secs, "node_instr_per_s": total / secs,
                     "ms_per_call": secs / calls * 1e3, "host_ms_per_call": host / calls * 1e3, "reps": reps}

    run(False)  # warm-up (module load)
    run(True)
    a, per_call = run(False, reps=10)
    b, burst = run(True, reps=10)
    same = all(torch.equal(u, v) for u, v in zip(a, b))
    plan = sess.plan()
    sess.close()
    # Byte model of the native sessions kernel (mk_sess_exec; VERDICT r03
    # item 6): per instance and launch, the state loaded once and stored once
    # (superblock 4 B + 8 B per live register, mk_session_plan's state_regs),
    # per call the int64 input, int32 out, u8 status and u32 steps
    # (program.go:80-92: state kept across calls; master.go:216-219).  The
    # time is the whole launch's (HIP events on the stream, every kernel of
    # the call), so `frac` is a lower bound on mk_sess_exec's own
    # (tools/sess_roofline.py has the rocprofv3 split,
    # profiles/r04o_sessions_roofline.json).
    m = re.search(r"state_regs=(\d+)", plan)
    roof = None
    if m:
        state_b, call_b = 2 * (4 + 8 * int(m.group(1))), 8 + 4 + 1 + 4
        roof = {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK / 1e9,
                "bytes_per_instance": {"state": state_b, "per_call": call_b},
                "model": "n x (state + calls x per_call) bytes per launch / launch time (HIP events on the "
                         "sessions' stream around back-to-back launches; every kernel of the call)"}
        for key, res, k in (("burst", burst, calls), ("per_call", per_call, 1)):
            t = res["ms_per_call"] * 1e-3 * k  # one launch
            b = n * (state_b + k * call_b)
            roof[key] = {"bytes_per_launch": b, "achieved": b / t / 1e9, "frac": b / t / HBM_PEAK}
        roof["frac"] = roof["burst"]["frac"]
    return {"instances": n, "calls_per_instance": calls, **burst, "per_call": per_call, "roofline": roof,
            "burst_equals_per_call": same, "plan": plan,
            "note": "stateful sessions, inputs resident in HBM: the burst (mk_session_compute_seq_device, "
                    f"{calls} sequential calls per instance in one launch) is the headline; per_call = one "
                    "mk_session_compute_device launch per call; HIP events around the calls (host clock in "
                    "host_ms_per_call); not the value"}


def http_leg(nodes, clients, seconds=5.0):
    """Single-value /compute requests through the HTTP master (stateful, the
    reference's semantics; concurrent requests coalesced into one launch per
    burst): `clients` threads, each with a keep-alive connection, for about
    `seconds`.  Python clients and server: this measures the drop-in surface,
    not the executor."""
    import http.client
    import threading

    from misaka_net_amd.master import MasterNode, make_server

    info = {n.name: {"type": n.kind} for n in nodes if n.kind != "master"}
    progs = {n.name: n.program for n in nodes if n.kind == "program"}
    m = MasterNode(info, progs)
    srv = make_server(m, port=0)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    hdr = {"Content-Type": "application/x-www-form-urlencoded"}
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    c.request("POST", "/run", body="", headers=hdr)
    c.getresponse().read()
    counts = [0] * clients
    errors = [0] * clients
    stop = threading.Event()

    def client(i):
        conn = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
        k = 0
        while not stop.is_set():
            conn.request("POST", "/compute", body=f"value={i * 100003 + k}", headers=hdr)
            r = conn.getresponse()
            r.read()
            if r.status == 200:
                counts[i] += 1
            else:
                errors[i] += 1
            k += 1
        conn.close()

    ts = [threading.Thread(target=client, args=(i,), daemon=True) for i in range(clients)]
    b0, q0 = m.coalescer.batches, m.coalescer.requests
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    time.sleep(seconds)
    stop.set()
    for t in ts:
        t.join(30)
    dt = time.perf_counter() - t0
    srv.shutdown()
    batches, reqs = m.coalescer.batches - b0, m.coalescer.requests - q0
    return {"requests_per_s": sum(counts) / dt, "clients": clients, "errors": sum(errors),
            "launches": batches, "requests_per_launch": reqs / max(1, batches),
            "mode": "stateful (one persistent network instance, mk_session_compute_seq per burst)",
            "note": "Python ThreadingHTTPServer + Python clients in one process; not the value"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--sessions", type=int, default=0, metavar="N",
                    help="also time N stateful instances x 8 sequential /compute calls (row f2; reported as "
                         "sessions, never as value)")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per GPU (default: the config's)")
    ap.add_argument("--gather", action="store_true", help="also time an ordered RCCL gather of outputs to rank 0")
    ap.add_argument("--interp", action="store_true", help="force the tier-1 bytecode interpreter (= --mode interp)")
    ap.add_argument("--mode", default=None, choices=["jit", "tile", "refill", "interp"],
                    help="force an executor mode (default: automatic)")
    ap.add_argument("--gen-inputs", action="store_true",
                    help="diagnostic: generate inputs inside the executor instead of reading them from HBM")
    ap.add_argument("--graph", action="store_true", help="replay the timed launches as one captured HIP graph")
    ap.add_argument("--dist-backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearse the multi-rank path on one GPU, with --dist-backend gloo)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--host-io", action="store_true",
                    help="also time mk_compute_batch on host buffers (int64 in, int32 out + u8 status over PCIe); "
                         "reported as host_io, never as value")
    ap.add_argument("--http", type=int, default=0, metavar="CLIENTS",
                    help="also time single-value /compute requests through the HTTP master with this many "
                         "concurrent keep-alive clients (reported as http, never as value)")
    ap.add_argument("--no-verify-gather", dest="verify_gather", action="store_false",
                    help="N > 1: skip rank 0's check of the gathered outputs against one launch over every "
                         "global lane (on by default)")
    ap.add_argument("--verify-gather", dest="verify_gather", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--refstruct-seconds", type=float, default=5.0,
                    help="sample length of the reference-structured CPU emulation (0: skip)")
    args = ap.parse_args()
    if args.interp:
        args.mode = "interp"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if not args.same_device and world > 1 and local >= torch.cuda.device_count():
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) visible "
                         "(--same-device rehearses N ranks on one GPU)")
    dist = None
    if args.same_device:  # rehearsal of the N-rank path on a one-GPU box
        local = 0
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    name, factory, lanes, gen_kind, mask = WORKLOADS[args.config]
    if args.lanes:
        lanes = args.lanes
    nodes = factory()
    net = mk.Network(nodes)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    # Inputs resident in HBM before the timed region (global lane indices
    # [rank*lanes, (rank+1)*lanes)).
    x = torch.empty(lanes, dtype=torch.int32, device="cuda")
    lo, _ = mk.dist.shard(rank, lanes)
    mk.generate_inputs_device(lanes, x.data_ptr(), seed=SEED, gen_kind=gen_kind, gen_mask=mask,
                              offset=lo, device=dev, stream=sh)
    out = torch.empty(lanes, dtype=torch.int32, device="cuda")
    st = torch.empty(lanes, dtype=torch.uint8, device="cuda")
    stats = torch.zeros(N.MK_STATS_LEN, dtype=torch.int64, device="cuda")

    # count: the launch adds its counters on the device (folded once, below)
    launchers = {
        count: net.device_launcher(lanes, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(),
                                   in_ptr=None if args.gen_inputs else x.data_ptr(), in_kind=N.MK_IN_I32,
                                   seed=SEED, gen_kind=gen_kind, gen_mask=mask, offset=lo, device=dev,
                                   mode=args.mode, defer_stats=count)
        for count in (False, True)
    }

    def step(count, stream_handle=sh):
        launchers[count](stream_handle)

    net.prepare(mode=args.mode, device=dev)  # schedule + native kernel compiled before any timing
    for _ in range(args.warmup):
        step(False)
    net.stats_fold(stats.data_ptr(), device=dev, stream=sh)  # clear anything left on the device
    torch.cuda.synchronize()
    stats.zero_()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # Timed region: K executor launches, each counting its lanes' retired
    # instructions on the device, plus the one fold of those counters.
    graph = None
    if args.graph:
        # the K launches + fold captured once as a HIP graph and replayed below
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            ch = torch.cuda.current_stream().cuda_stream
            for _ in range(args.steps):
                step(True, ch)
            net.stats_fold(stats.data_ptr(), device=dev, stream=ch)
        torch.cuda.synchronize()
        stats.zero_()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    if graph is not None:
        graph.replay()
    else:
        for _ in range(args.steps):
            step(True)
        net.stats_fold(stats.data_ptr(), device=dev, stream=sh)
    e1.record(stream)
    enqueue_s = time.perf_counter() - t0  # host time to issue the timed work
    torch.cuda.synchronize()
    # This rank's time for its K steps ends when its stream drains; the job's
    # time is the max over ranks (below). The closing barrier only keeps the
    # ranks together and is not itself part of any rank's K steps.
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
        torch.cuda.synchronize()
    kernel_s = e0.elapsed_time(e1) * 1e-3  # HIP events on the launch stream

    # Average duration of one executor launch (the dominant kernel) for the
    # roofline: HIP events around K launches on the launch stream.
    k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k0.record(stream)
    for _ in range(args.steps):
        step(False)
    k1.record(stream)
    torch.cuda.synchronize()
    launch_s = k0.elapsed_time(k1) * 1e-3 / args.steps

    peak_meas = None
    if rank == 0:
        try:
            peak_meas = valu_peak(sh)
        except Exception as e:  # pragma: no cover
            log("valu probe failed:", e)
    peak = max(SPEC_LANE_OPS, peak_meas or 0.0)

    # per-rank -> whole job (max time over ranks, summed work)
    t = torch.tensor([wall, kernel_s, launch_s], dtype=torch.float64, device="cuda")
    tot = mk.dist.reduce_counters(stats.clone(), dist)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max, kern_max, launch_max = t.tolist()
    tot = tot.cpu().numpy()
    retired, with_out, finished = int(tot[0]), int(tot[1]), int(tot[2])
    assert finished == lanes * world * args.steps, (finished, lanes, world, args.steps)

    # End to end (N > 1): K steps of launch + ordered gather of the step's
    # int32 outputs and status bytes to rank 0 (RCCL over xGMI, SURVEY.md
    # section 8 row e), timed like the compute-only loop.  Reported beside
    # `value`, which stays the sharded compute (no data-path collective).
    e2e = None
    if dist and (world > 1 or args.gather):
        # each step's outputs and statuses in one packed buffer (one gather
        # per step), two buffers so that step k's gather overlaps step k + 1
        packs = [torch.empty(5 * lanes, dtype=torch.uint8, device="cuda") for _ in range(2)]
        pack_run = []
        for pk in packs:
            o_v, s_v = mk.dist.pack_views(pk, lanes)
            pack_run.append(net.device_launcher(lanes, out_ptr=o_v.data_ptr(), status_ptr=s_v.data_ptr(),
                                                in_ptr=None if args.gen_inputs else x.data_ptr(),
                                                in_kind=N.MK_IN_I32, seed=SEED, gen_kind=gen_kind,
                                                gen_mask=mask, offset=lo, device=dev, mode=args.mode))
        e2e_s, g = mk.dist.timed_gather(lambda b: pack_run[b](sh), packs, dist, args.steps,
                                        sync=torch.cuda.synchronize)
        g_out, g_st = mk.dist.unpack_gathered(g, lanes, world) if rank == 0 else (None, None)
        e2e = {"value": None, "ms_per_step": e2e_s / args.steps * 1e3,
               "gathered_bytes_per_step": 5 * lanes * world, "collectives_per_step": 1,
               "collective": f"ordered gather to rank 0 ({dist.get_backend()}) of one packed buffer per rank "
               "(outputs int32 + status u8), issued async so that it overlaps the next step"}
        if args.verify_gather and rank == 0:
            # the gathered shards == one launch over all world x lanes global lanes
            def full():
                xf = torch.empty(lanes * world, dtype=torch.int32, device="cuda")
                mk.generate_inputs_device(lanes * world, xf.data_ptr(), seed=SEED, gen_kind=gen_kind,
                                          gen_mask=mask, offset=0, device=dev, stream=sh)
                of = torch.empty_like(xf)
                sf = torch.empty(lanes * world, dtype=torch.uint8, device="cuda")
                net.compute_device(lanes * world, out_ptr=of.data_ptr(), status_ptr=sf.data_ptr(),
                                   in_ptr=xf.data_ptr(), device=dev, stream=sh, mode=args.mode)
                torch.cuda.synchronize()
                return of, sf

            e2e["verified"] = mk.dist.verify_gathered(g_out, g_st, full)
            assert e2e["verified"], "gathered outputs differ from a single launch over the global lanes"

    host_io = None
    if args.host_io and rank == 0:
        # the host-buffer boundary (mk_compute_batch): inputs as int64 /compute
        # values in pageable host memory, outputs and statuses copied back
        xh = x.cpu().numpy().astype(np.int64)
        net.compute_batch(xh, steps=False, mode=args.mode)  # warm (allocations)
        reps = max(1, min(args.steps, 5))
        th = time.perf_counter()
        for _ in range(reps):
            net.compute_batch(xh, steps=False, mode=args.mode)
        dt = (time.perf_counter() - th) / reps
        host_io = {
            "ms_per_call": dt * 1e3,
            "node_instr_per_s": retired / (world * args.steps) / dt,
            "results_per_s": with_out / (world * args.steps) / dt,
            "bytes_per_lane": 8 + 4 + 1,
            "note": "pageable host buffers, PCIe-inclusive; not the value",
        }

    value = retired / wall_max
    if e2e is not None:
        e2e["value"] = retired / (e2e["ms_per_step"] * 1e-3 * args.steps)
        e2e["results_per_s"] = with_out / (e2e["ms_per_step"] * 1e-3 * args.steps)
    # ---- roofline of the dominant kernel, per launch -----------------------
    instr_per_launch = retired / world / args.steps
    plan = net.plan(mode=args.mode)
    prof = measured_profile(name) if not args.mode and not args.gen_inputs else {}
    if prof and (abs(prof.get("retired_per_launch", 0) - instr_per_launch) > 0.01 * instr_per_launch or
                 plan_signature(prof.get("executor", "")) != plan_signature(plan)):
        prof = {}  # counters of another lane count / network / kernel: not this launch
    traffic = prof.get("hbm_bytes_per_launch")
    # int32 input read, int32 out + u8 status written, stack slots written and read back
    io_bytes = ((0 if args.gen_inputs else 4) + 4 + 1) * lanes
    slot_bytes = 4 * STACK_OPS_PER_LANE.get(args.config, 0) * lanes
    # the heavy kernel may keep the slots in LDS: then they are no HBM/L2 bytes;
    # split between LDS and HBM, the bytes PMC did not see leave L2 are priced
    # at the LDS peak instead of the L2 one (a lower bound on their time)
    lds_slots = "shape=stream-heavy-lds" in plan
    lds_split = "shape=stream-heavy-split" in plan
    bytes_per_launch = io_bytes + (0 if lds_slots else slot_bytes)
    hbm_achieved = bytes_per_launch / launch_max
    # Lower bound on the launch's memory time: the bytes PMC saw leave the
    # XCDs' L2s at the HBM peak, the algorithmic bytes that never did
    # (stack slots popped back while still in L2) at the L2 peak.
    # Without a matching PMC profile (another lane count), only the streaming
    # I/O is known to cross HBM: the slot bytes are priced at the L2 peak, a
    # lower bound on the memory time, so `frac` stays a bound (<= 1).
    fabric = min(traffic, bytes_per_launch) if traffic else io_bytes
    # Split slots (LDS + HBM + registers): the LDS share is what the LDS
    # instructions moved (PMC SQ_INSTS_LDS x 64 lanes x 4 B, b32-priced);
    # entries kept in registers cost no memory time.  Without a matching
    # profile only the I/O is known to move: a lower bound.
    lds_insts = prof.get("lds", {}).get("SQ_INSTS_LDS") if traffic else None
    if lds_split:
        t_mem = fabric / HBM_PEAK + (lds_slot_seconds(lds_insts * 64 * 4) if lds_insts else 0.0)
    else:
        t_mem = fabric / HBM_PEAK + (bytes_per_launch - fabric) / L2_PEAK
    hbm = {
        "bound": "hbm",
        "achieved": hbm_achieved / 1e9,
        "peak": bytes_per_launch / t_mem / 1e9,
        "unit": "GB/s",
        "frac": t_mem / launch_max,
        "traffic": traffic,
        "bytes_per_lane": bytes_per_launch // lanes,
        "bytes_per_launch": bytes_per_launch,
        "launch_us": launch_max * 1e6,
        "model": ("peak = algorithmic bytes / (PMC fabric bytes / 8 TB/s + LDS bytes of SQ_INSTS_LDS x 256 B, half at "
                  "ds_write_b32's 39.3 TB/s and half at ds_read_b32's 78.6 TB/s; register-held entries free)"
                  if traffic and lds_split else
                  "peak = I/O bytes / 8 TB/s: no PMC profile for this launch, so the LDS / HBM / register split of "
                  "the stack slots is not measured (a lower bound)" if lds_split else
                  "peak = algorithmic bytes / (PMC fabric bytes / 8 TB/s + L2-resident bytes / 34.5 TB/s)"
                  if traffic and bytes_per_launch > fabric * 1.001 else
                  "peak = HBM 8 TB/s; stack slots in LDS (roofline_lds)" if lds_slots else
                  "peak = algorithmic bytes / (I/O bytes / 8 TB/s + stack-slot bytes / 34.5 TB/s): no PMC profile "
                  "for this launch" if not traffic and slot_bytes else "peak = HBM 8 TB/s"),
        "counter_source": prof.get("source"),
    }
    sq = prof.get("sq", {})
    if sq.get("SQ_INSTS_VALU"):
        # executed work from the committed SQ counters: VALU wave-instructions x 64 lanes
        exec_ops = sq["SQ_INSTS_VALU"] * 64
        issue = {
            "bound": "valu",
            "achieved": exec_ops / launch_max / 1e12,
            "peak": peak / 1e12,
            "unit": "Tlane-op/s",
            "frac": exec_ops / launch_max / peak,
            "traffic": traffic,
            "model": "executed VALU lane-ops per launch (PMC SQ_INSTS_VALU x 64) / launch time",
            "valu_lane_ops_per_instr": prof.get("valu_lane_ops_per_instr"),
            "salu_per_instr": prof.get("salu_per_instr"),
            "valu_lane_util": prof.get("valu_lane_util"),
            "k_model_frac": K_LANE_OPS * instr_per_launch / launch_max / peak,
            "peak_spec": SPEC_LANE_OPS / 1e12,
            "peak_measured": None if peak_meas is None else peak_meas / 1e12,
            "launch_us": launch_max * 1e6,
            "counter_source": prof.get("source"),
        }
        # the same executed rate against what a kernel at this occupancy can
        # issue (one wave per SIMD issues a VALU op only
        # every ~8.8 cycles), reproducible from profiles/
        m = re.search(r"waves_per_simd=([\d.]+)", plan)
        occ = occupancy_cap(float(m.group(1)) if m else 0)
        if occ:
            occ["frac"] = issue["achieved"] / occ["cap"]
        issue["occupancy"] = occ
    else:
        # No PMC profile of this kernel: the executed work is unknown.  The
        # frozen k = 4 model is reported beside it,
        # never as the bound: the compiler retires node-instructions for far
        # less than 4 lane-ops each (registers, LDS; C4 d256 would read 2.6).
        achieved = K_LANE_OPS * instr_per_launch / launch_max
        issue = {
            "bound": "valu",
            "achieved": None,
            "peak": peak / 1e12,
            "unit": "Tlane-op/s",
            "frac": None,
            "k_model_frac": achieved / peak,
            "traffic": traffic,
            "model": "no PMC profile for this launch: executed VALU work not measured (k_model_frac: k = 4 "
                     "lane-ops per retired node-instruction, BASELINE.md section 2, not a bound)",
            "k_lane_ops_per_instr": K_LANE_OPS,
            "peak_spec": SPEC_LANE_OPS / 1e12,
            "peak_measured": None if peak_meas is None else peak_meas / 1e12,
            "launch_us": launch_max * 1e6,
        }
    # Stack slots in LDS: the LDS-array cycles the PMC pass counted
    # (SQ_LDS_IDX_ACTIVE, summed over the CUs; MI355X_MICROARCH.md section
    # LDS) per CU against the launch's cycles.  LLVM keeps many LDS-resident
    # slots in registers (a store it can forward to the load), so the count of
    # LDS instructions, not the stack's pushes and pops, is the measure.
    lds = None
    if lds_slots or lds_split:
        lsq = prof.get("lds", {})
        cyc = lsq.get("SQ_LDS_IDX_ACTIVE")
        if cyc:
            per_cu = cyc / LDS_CUS
            lds = {"bound": "lds", "achieved": per_cu / launch_max / 1e9, "peak": LDS_CLOCK / 1e9,
                   "unit": "G LDS-array cycles/s per CU", "frac": per_cu / LDS_CLOCK / launch_max,
                   "traffic": traffic, "lds_wave_instr_per_launch": lsq.get("SQ_INSTS_LDS"),
                   "lds_array_cycles_per_launch": cyc, "bank_conflict_cycles": lsq.get("SQ_LDS_BANK_CONFLICT"),
                   "model": "PMC SQ_LDS_IDX_ACTIVE / 256 CUs / 2.4 GHz per launch (LDS array busy)",
                   "launch_us": launch_max * 1e6, "counter_source": prof.get("source")}
        else:
            lds = {"bound": "lds", "frac": None, "model": "no PMC profile of this kernel: LDS work not measured"}
    # C4: how much of the stack traffic the kernel actually executes (VERDICT
    # r03 item 5).  Slot instructions = LDS wave-instructions + the vector
    # memory instructions beyond the lanes' I/O (one input load, the out and
    # status stores per wave), times 64 lanes, per retired PUSH/POP.  Near 1:
    # every push and pop is a memory operation (d256, d1024); far below 1:
    # the compiler forwarded pushes to pops in registers (d64, straight-line
    # code with static slot indices) -- that config then measures the
    # folded program, not stack traffic.
    stack = None
    if STACK_OPS_PER_LANE.get(args.config) and args.config.startswith("c4"):
        pp = STACK_OPS_PER_LANE[args.config] * lanes
        lsq, ssq = prof.get("lds", {}), prof.get("sq", {})
        stack = {"push_pop_per_launch": pp, "stack_ops_executed_per_push_pop": None,
                 "model": "(SQ_INSTS_LDS + SQ_INSTS_VMEM_RD + SQ_INSTS_VMEM_WR - 3 x waves) x 64 / retired PUSH+POP"}
        if lsq.get("SQ_INSTS_LDS") is not None and ssq.get("SQ_INSTS_VMEM_RD") is not None:
            waves = lanes / 64
            slot_vmem = max(0.0, ssq["SQ_INSTS_VMEM_RD"] + ssq.get("SQ_INSTS_VMEM_WR", 0.0) - 3 * waves)
            stack["stack_ops_executed_per_push_pop"] = (lsq["SQ_INSTS_LDS"] + slot_vmem) * 64 / pp
            stack["counter_source"] = prof.get("source")
    # The dominant kernel's roofline is the tightest bound: the byte stream
    # for short networks (C2, C3), integer issue for long ones, LDS for
    # stacks kept there.
    bounds = [b for b in (hbm, issue, lds) if b and b.get("frac") is not None]
    headline = max(bounds, key=lambda b: b["frac"])
    # What the node-instr/s figure is a count of: the
    # executed VALU lane-ops per retired node-instruction from the matching
    # PMC profile, and whether the compiler folded the program, so that
    # node-instr/s counts the reference's work rather than issued work.
    # Folded: a stack network whose PUSH/POPs mostly never reach a slot (C4
    # d64, d256: pushes forwarded to pops in registers), or a network whose
    # superblock graph is acyclic (the stream shapes: every lane runs a path
    # fixed at compile time, C2 and C3 a few adds and branches, whatever
    # their retired count).  Not folded: the machine shape's loops retire
    # each iteration (C5); C4 d1024 moves 0.94 slot operations per PUSH/POP.
    vpi = prof.get("valu_lane_ops_per_instr") if sq.get("SQ_INSTS_VALU") else None
    spp = stack.get("stack_ops_executed_per_push_pop") if stack else None
    m = re.search(r"\bshape=(\S+)", plan) if "tier=native" in plan else None
    if spp is not None:
        folded, basis = spp < 0.5, f"{spp:.3f} stack-slot operations executed per PUSH/POP (folded below 0.5)"
    elif m:
        folded = m.group(1).startswith("stream")
        basis = f"shape={m.group(1)}: " + ("acyclic superblock graph, a path fixed at compile time" if folded
                                           else "loops that retire each iteration")
    else:
        folded, basis = None, "no stack counters and no native module"
    executed = {"valu_lane_ops_per_node_instr": vpi,
                "compile_folded": folded,
                "folded_basis": basis,
                "bound": headline["bound"],
                "note": "node-instr/s counts retired reference instructions; executed VALU lane-ops per "
                        "node-instruction from the PMC profile of this module (null: no matching profile)"}

    http = None
    if args.http and rank == 0:
        http = http_leg(nodes, args.http, seconds=5.0)
    sessions = None
    if args.sessions and rank == 0:
        with torch.cuda.stream(stream):  # the per-call reductions on the sessions' stream
            sessions = sessions_leg(net, args.sessions, 8, stream)

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # the host-core baseline is an N=1 figure
            cpu = cpu_baseline(nodes, gen_kind, mask, args.cpu_seconds, args.refstruct_seconds)
        rec = {
            "metric": METRIC,
            "value": value,
            "unit": "node-instr/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (splitmix64 int32 /compute inputs, resident in HBM)",
            "config": {
                "workload": name,
                "lanes_per_gpu": lanes,
                "global_lanes": lanes * world,
                "network": args.config,
                "parallelism": f"dp{world} (contiguous lane shards, no data-path collective)",
                "executor": plan,
            },
            "results_per_s": with_out / wall_max,
            "node_instr_per_lane": retired / (lanes * world * args.steps),
            "kernel_ms_per_step": kern_max / args.steps * 1e3,
            "host_enqueue_us_per_step": enqueue_s / args.steps * 1e6,
            "launch": "hip graph replay" if args.graph else "stream launches",
            "executed": executed,
            "roofline": headline,
            "roofline_issue": issue,
            "roofline_hbm": hbm,
            "roofline_lds": lds,
            "cpu_baseline": cpu,
        }
        if stack is not None:
            rec["stack"] = stack
        if e2e is not None:
            rec["end_to_end"] = e2e
        if host_io is not None:
            rec["host_io"] = host_io
        if http is not None:
            rec["http"] = http
        if sessions is not None:
            rec["sessions"] = sessions
        print(json.dumps(rec), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
