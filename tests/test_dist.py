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
    g = mk.dist.gather_outputs(torch.from_numpy(out), dist)
    # bench.py's end-to-end leg, the code an N-GPU run executes: K steps of
    # (fill this rank's shard, ordered gather of out + status to rank 0),
    # timed as the max over ranks, then rank 0 checks the gathered batch
    # against one evaluation over all global lanes
    o_t, s_t = torch.zeros(hi - lo, dtype=torch.int32), torch.zeros(hi - lo, dtype=torch.uint8)
    calls = []

    def step():
        calls.append(1)
        o_t.copy_(torch.from_numpy(out))
        s_t.copy_(torch.from_numpy(st))

    secs, g_out, g_st = mk.dist.timed_gather(step, o_t, s_t, dist, 3)
    verified = None
    if rank == 0:
        def full():
            xa = po.gen_inputs(SEED, world * LANES)
            fo, fs, _ = po.OracleNet(mk.networks.sample_network()).compute_batch(xa)
            return torch.from_numpy(fo), torch.from_numpy(fs)

        verified = mk.dist.verify_gathered(g_out, g_st, full)
        wrong = g_out.clone()
        wrong[LANES] ^= 1  # a lane of rank 1's shard: a gather out of order or short would differ too
        caught = not mk.dist.verify_gathered(wrong, g_st, full)
    else:
        assert g_out is None and g_st is None
    if rank == 0:
        q.put((stats.numpy().tolist(), g.numpy().tolist(), secs > 0 and len(calls) == 3, verified, caught))
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


def test_split_covers_batch():
    for total in (0, 1, 7, 64, 1000003):
        for world in (1, 2, 3, 8):
            parts = [mk.dist.split(total, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
