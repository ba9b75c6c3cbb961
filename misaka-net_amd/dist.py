"""Multi-GPU plumbing for the batched /compute path (SURVEY.md section 8 row e).

The lane batch shards with no exchange: rank r of W evaluates global lane
indices [r*n, (r+1)*n).  RCCL (torch.distributed "nccl") is used only for the
counter reduction and the optional ordered output gather to rank 0.
"""
from __future__ import annotations


def shard(rank: int, lanes_per_rank: int) -> tuple[int, int]:
    """[lo, hi) global lane indices of `rank` (weak scaling: fixed per-rank size)."""
    return rank * lanes_per_rank, (rank + 1) * lanes_per_rank


def split(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous split of a fixed global batch (strong scaling)."""
    return total * rank // world, total * (rank + 1) // world


def reduce_counters(stats, dist):
    """Sum the per-rank executor counters (uint64[MK_STATS_LEN] as int64)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.SUM)
    return stats


def gather_outputs(out, dist, dst: int = 0):
    """Ordered gather of equal-size per-rank output shards to rank `dst`:
    returns the concatenation in rank (= global lane) order on dst, None elsewhere."""
    import torch

    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return out
    world, rank = dist.get_world_size(), dist.get_rank()
    if out.is_cuda and dist.get_backend() == "gloo":  # gloo gathers host tensors only
        g = gather_outputs(out.cpu(), dist, dst)
        return None if g is None else g.to(out.device)
    if rank == dst:
        buf = torch.empty(world * out.numel(), dtype=out.dtype, device=out.device)
        dist.gather(out, gather_list=list(buf.view(world, -1).unbind(0)), dst=dst)
        return buf
    dist.gather(out, dst=dst)
    return None


def timed_gather(step, out, status, dist, steps: int, sync=None):
    """End-to-end leg of an N-rank run (SURVEY.md section 8 row e): `steps`
    times, run one step (`step()`, the launch that fills this rank's `out`
    int32 and `status` u8 shards) and gather both to rank 0 in global lane
    order.  Returns (seconds, the max over ranks; gathered out; gathered
    status), the gathered tensors on rank 0 and None elsewhere.  `sync`
    waits for the device (torch.cuda.synchronize); None on CPU."""
    import time

    import torch

    sync = sync or (lambda: None)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    g_out = g_st = None
    for _ in range(steps):
        step()
        g_out = gather_outputs(out, dist)
        g_st = gather_outputs(status, dist)
    sync()
    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=out.device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return tt.item(), g_out, g_st


def verify_gathered(g_out, g_st, full) -> bool:
    """Rank 0: the gathered shards equal one evaluation over all global lanes
    (`full()` returns that evaluation's (out, status))."""
    import torch

    of, sf = full()
    return bool(torch.equal(of.to(g_out.device), g_out) and torch.equal(sf.to(g_st.device), g_st))


# ---- self-launch: `python bench.py --gpus N` without torch.distributed.run --
#
# The driver's scaling command is a bare `python3 bench.py --gpus N`.  The
# parent then starts N fresh child processes (one per GPU, the same argv, the
# rendezvous variables torch.distributed.run would set) before it has loaded
# the executor library or touched a GPU, and it never exec()s itself.  The
# functions below use only the standard library, so a launching parent stays
# GPU-free.

LAUNCH_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
              "MASTER_ADDR", "MASTER_PORT")


def needs_launch(gpus: int, environ) -> bool:
    """True when N > 1 ranks were asked for and no launcher started this process."""
    return gpus > 1 and "WORLD_SIZE" not in environ


def free_port(addr: str = "127.0.0.1") -> int:
    import socket

    with socket.socket() as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def rank_env(base, world: int, rank: int, port: int, addr: str = "127.0.0.1") -> dict:
    """Environment of child `rank` of a single-node job of `world` ranks (the
    variables torch.distributed.run exports; LOCAL_RANK selects the GPU)."""
    env = {k: v for k, v in base.items() if k not in LAUNCH_ENV}
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", ROLE_RANK=str(rank), MASTER_ADDR=addr, MASTER_PORT=str(port))
    return env


def launch_ranks(argv, world: int, environ=None, port: int = 0, poll: float = 0.1, grace: float = 15.0,
                 log=None) -> int:
    """Run `argv` as `world` child processes, rank r with rank_env(r), and
    wait for them.  Rank 0's stdout is the parent's (it prints the job's one
    JSON line); the other ranks' stdout goes to the parent's stderr.  If a
    rank fails, the others are terminated (their exact PIDs, SIGTERM then
    SIGKILL after `grace` s) so none is left waiting in a collective.  Returns
    0 when every rank exited 0, else the first failure's code (a signal as
    128 + signo)."""
    import os
    import subprocess
    import sys
    import time

    environ = os.environ if environ is None else environ
    log = log or (lambda *a: print(*a, file=sys.stderr, flush=True))
    port = port or free_port()
    procs = []
    rc = 0
    try:
        for r in range(world):
            out = None if r == 0 else sys.stderr.fileno()
            procs.append(subprocess.Popen(list(argv), env=rank_env(environ, world, r, port), stdout=out))
        live = set(range(world))
        while live:
            for r in sorted(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    log(f"launch: rank {r} exited with {code}; stopping the other ranks")
            if rc:
                break
            time.sleep(poll)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.monotonic() + grace
        for p in procs:
            try:
                p.wait(max(0.0, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc
