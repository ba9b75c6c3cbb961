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
