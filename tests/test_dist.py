"""world_size-2 gloo run of the sharding / counter-reduction / ordered-gather
path of bench.py (misaka_net_amd.dist) on CPU.  The per-rank compute is the
oracle here (no GPU in CI); on the GPU box the same helpers wrap the HIP
executor with the nccl (RCCL) backend."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import misaka_net_amd as mk

SEED = 0x4D49534B41
LANES = 3000


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import pyoracle as po

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = mk.dist.shard(rank, LANES)
    xs = po.gen_inputs(SEED, hi - lo, offset=lo)
    out, st, sp = po.OracleNet(mk.networks.sample_network()).compute_batch(xs)
    stats = torch.tensor([int(sp.sum()), int(((st & 0x10) != 0).sum()), hi - lo, 0, 0, 0, 0, 0], dtype=torch.int64)
    mk.dist.reduce_counters(stats, dist)
    gathered = mk.dist.gather_outputs(torch.from_numpy(out), dist)
    # bench.py's end-to-end leg, the code an N-GPU run executes: K steps of
    # (fill this rank's packed out + status buffer, one ordered gather of it
    # to rank 0, overlapped with the next step), timed as the max over ranks,
    # then rank 0 checks the gathered batch against one evaluation over all
    # global lanes
    n = hi - lo
    bufs = [torch.zeros(5 * n, dtype=torch.uint8) for _ in range(2)]
    calls = []

    def step(b):
        calls.append(b)
        o_v, s_v = mk.dist.pack_views(bufs[b], n)
        o_v.copy_(torch.from_numpy(out))
        s_v.copy_(torch.from_numpy(st))

    secs, g = mk.dist.timed_gather(step, bufs, dist, 3)
    verified = caught = None
    if rank == 0:
        g_out, g_st = mk.dist.unpack_gathered(g, n, world)

        def full():
            xa = po.gen_inputs(SEED, world * LANES)
            fo, fs, _ = po.OracleNet(mk.networks.sample_network()).compute_batch(xa)
            return torch.from_numpy(fo), torch.from_numpy(fs)

        verified = mk.dist.verify_gathered(g_out, g_st, full)
        wrong = g_out.clone()
        wrong[LANES] ^= 1  # a lane of rank 1's shard: a gather out of order or short would differ too
        caught = not mk.dist.verify_gathered(wrong, g_st, full)
        wrong_st = g_st.clone()
        wrong_st[2 * LANES - 1] ^= 0x10  # the last status byte of rank 1's packed row
        caught = caught and not mk.dist.verify_gathered(g_out, wrong_st, full)
    else:
        assert g is None
    if rank == 0:
        q.put((stats.numpy().tolist(), gathered.numpy().tolist(), secs > 0 and calls == [0, 1, 0], verified, caught))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_reduce_gather():
    from oracle import pyoracle as po

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, _port_holder[0], q)) for r in range(world)]
    for p in procs:
        p.start()
    stats, gathered, timed, verified, caught = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    xs = po.gen_inputs(SEED, world * LANES)
    out, st, sp = po.OracleNet(mk.networks.sample_network()).compute_batch(xs)
    assert gathered == out.tolist()  # ordered: rank order == global lane order
    assert stats[0] == int(sp.sum()) and stats[2] == world * LANES
    assert stats[1] == int(((st & 0x10) != 0).sum())
    assert timed and verified and caught  # misaka_net_amd.dist.timed_gather / verify_gathered (bench.py)


_port_holder = [_port()]


def test_rank_env_construction():
    # the variables torch.distributed.run exports, one set per child; stale
    # launcher variables in the parent's environment never leak through
    base = {"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0", "RANK": "5", "MASTER_PORT": "1"}
    envs = [mk.dist.rank_env(base, 4, r, 29511) for r in range(4)]
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == e["ROLE_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "4" and e["GROUP_RANK"] == "0"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["PATH"] == "/usr/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert base["RANK"] == "5"  # the parent's mapping is not modified
    assert mk.dist.needs_launch(8, {}) and not mk.dist.needs_launch(1, {})
    assert not mk.dist.needs_launch(8, {"WORLD_SIZE": "8"})  # already under a launcher


def test_bench_self_launch_argv(monkeypatch):
    # bench.py's parent: --gpus N read before anything touches a GPU, the
    # children get the same argv (so each parses --gpus N and WORLD_SIZE=N)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    assert bench._gpus_arg(["--gpus", "8", "--steps", "20", "--warmup", "3"]) == 8
    assert bench._gpus_arg(["--steps", "5"]) == 1
    seen = {}

    def fake_launch(argv, world, **kw):
        seen.update(argv=argv, world=world)
        return 0

    monkeypatch.setattr(mk.dist, "launch_ranks", fake_launch)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    import runpy

    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "7"])
    try:
        runpy.run_path(bench.__file__, run_name="__main__")
    except SystemExit as e:
        assert e.code == 0
    assert seen["world"] == 4 and seen["argv"][1:] == [os.path.abspath(bench.__file__), "--gpus", "4", "--steps", "7"]


_CHILD = r"""
import json, os, sys, time
r = int(os.environ["RANK"])
with open(os.path.join(sys.argv[1], f"rank{r}.json"), "w") as f:
    json.dump({k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}, f)
mode = sys.argv[2]
if mode == "fail" and r == 1:
    sys.exit(3)
if mode == "fail":
    time.sleep(120)  # would hang the job if the launcher did not stop it
print(json.dumps({"rank": r}) if r == 0 else "not-on-stdout", flush=True)
"""


def test_launch_ranks_children(tmp_path, capfd):
    import sys

    rc = mk.dist.launch_ranks([sys.executable, "-c", _CHILD, str(tmp_path), "ok"], 3)
    assert rc == 0
    import json

    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] and {e["WORLD_SIZE"] for e in envs} == {"3"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    out, err = capfd.readouterr()
    assert out.strip().splitlines() == ['{"rank": 0}']  # only rank 0 on stdout
    assert err.count("not-on-stdout") == 2


def test_launch_ranks_failure_stops_the_others(tmp_path):
    import sys
    import time

    t0 = time.monotonic()
    rc = mk.dist.launch_ranks([sys.executable, "-c", _CHILD, str(tmp_path), "fail"], 2, grace=5.0)
    assert rc == 3 and time.monotonic() - t0 < 60


def test_split_covers_batch():
    for total in (0, 1, 7, 64, 1000003):
        for world in (1, 2, 3, 8):
            parts = [mk.dist.split(total, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))


def test_bench_reads_only_shipped_profiles():
    """bench.py's occupancy cap reads profiles/valu_rates.jsonl on the GPU
    box; a .gpurunignore pattern that matched it would silently null the
    line's `roofline_issue.occupancy` (round 5: r04n_* matched ./profiles/r0*)."""
    import fnmatch

    import bench
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pats = [ln.strip() for ln in open(os.path.join(root, ".gpurunignore")) if ln.strip()]
    for rel in ("profiles/valu_rates.jsonl",):
        assert os.path.exists(os.path.join(root, rel))
        for p in pats:
            assert not fnmatch.fnmatch("./" + rel, p) and not fnmatch.fnmatch(rel, p.lstrip("./")), (rel, p)
    # round 6: a measured row at every occupancy 1..8,
    # so a line is priced at its own; a fraction at its whole part
    for w in range(1, 9):
        occ = bench.occupancy_cap(w)
        assert occ["measured_at_waves_per_simd"] == w == occ["waves_per_simd"], occ
    assert bench.occupancy_cap(6)["cap"] > 40 and bench.occupancy_cap(1)["cap"] < 30
    occ = bench.occupancy_cap(3.75)
    assert occ["measured_at_waves_per_simd"] == 3 and occ["waves_per_simd"] == 3.75
    assert bench.occupancy_cap(0) is None
