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


def pack_views(buf, lanes: int):
    """The int32 outputs and u8 statuses of one rank's step as views of one
    packed buffer (uint8[5 * lanes]: 4 * lanes bytes of outputs, then the
    status bytes), so that a step's results leave the rank in ONE collective.
    The status view starts 4 * lanes bytes in: 4-byte aligned, as the
    executor's vector stores need."""
    import torch

    assert buf.dtype == torch.uint8 and buf.numel() == 5 * lanes
    return buf[: 4 * lanes].view(torch.int32), buf[4 * lanes:]


def unpack_gathered(g, lanes: int, world: int):
    """Rank 0: the (outputs int32[world * lanes], statuses u8[world * lanes])
    in global lane order from the gathered packed rows (pack_views' layout)."""
    import torch

    rows = g.view(world, 5 * lanes)
    out = rows[:, : 4 * lanes].contiguous().view(torch.int32).reshape(-1)
    return out, rows[:, 4 * lanes:].reshape(-1)


def timed_gather(step, bufs, dist, steps: int, sync=None):
    """End-to-end leg of an N-rank run (SURVEY.md section 8 row e): `steps`
    times, run one step (`step(b)`: the launch that fills this rank's packed
    results buffer `bufs[b]`, pack_views' layout) and gather that buffer to
    rank 0 in global lane order: one collective per step.  The buffers
    alternate (b = k % 2) and each gather is issued asynchronously, so the
    gather of step k runs while step k + 1 computes (RCCL's stream waits for
    the step's launch; the launch that rewrites a buffer waits for its
    previous gather).  Returns (seconds, the max over ranks; the gathered
    packed rows of the last step), the rows on rank 0 and None elsewhere.
    `sync` waits for the device (torch.cuda.synchronize); None on CPU."""
    import time

    import torch

    sync = sync or (lambda: None)
    world, rank = dist.get_world_size(), dist.get_rank()
    gloo = dist.get_backend() == "gloo"  # gloo gathers host tensors only
    n = bufs[0].numel()
    rdev = torch.device("cpu") if gloo else bufs[0].device
    recv = [torch.empty(world * n, dtype=torch.uint8, device=rdev) for _ in bufs] if rank == 0 else None
    pending, keep = [None] * len(bufs), [None] * len(bufs)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for k in range(steps):
        b = k % len(bufs)
        if pending[b] is not None:
            pending[b].wait()  # the gather still reading bufs[b]
        step(b)
        src = bufs[b].cpu() if gloo and bufs[b].is_cuda else bufs[b]
        keep[b] = src  # alive until its gather completes
        gl = list(recv[b].view(world, n).unbind(0)) if rank == 0 else None
        pending[b] = dist.gather(src, gather_list=gl, dst=0, async_op=True)
    for w in pending:
        if w is not None:
            w.wait()
    sync()
    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=bufs[0].device if not gloo else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    last = None
    if rank == 0 and steps:
        last = recv[(steps - 1) % len(bufs)].to(bufs[0].device)
    return tt.item(), last


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
