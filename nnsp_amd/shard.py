"""Stream shards across GPUs.

Independent 16 kHz streams are the data-parallel axis: the reference keeps all
state per stream (evb/src/nnCntrlClass.c:152-272, one nnCntrlClass per
stream), so rank r of a world of N owns a contiguous range of the global
stream population and nothing is exchanged on the data path.  The only
collective is the max-reduce of the timed region's wall time (and the sum of
the frames processed) in bench.py.

  weak scaling   : every rank owns ``per_rank`` streams, [r*per_rank, (r+1)*per_rank)
  strong scaling : ``total`` streams split as evenly as possible, the first
                   total % N ranks one stream more
"""
from __future__ import annotations


def shard_streams(rank: int, world: int, per_rank: int | None = None,
                  total: int | None = None) -> tuple[int, int]:
    """(first global stream, stream count) of rank's shard."""
    if world < 1 or not 0 <= rank < world or (per_rank is None) == (total is None):
        raise ValueError(f"bad shard: rank {rank} of {world}, per_rank={per_rank}, total={total}")
    if per_rank is not None:
        if per_rank < 1:
            raise ValueError(f"bad shard: {per_rank} streams per rank")
        return rank * per_rank, per_rank
    if total < world:
        raise ValueError(f"bad shard: {total} streams over {world} ranks")
    base, extra = divmod(total, world)
    return rank * base + min(rank, extra), base + (1 if rank < extra else 0)


def dist_env() -> tuple[int, int, int, bool]:
    """(rank, world, local rank, launched by torch.distributed.run).  A
    torchrun launch sets RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR even for
    one process; then the process group is initialised at world size 1 too."""
    import os
    launched = all(k in os.environ for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local, launched


def reduce_run(dist, elapsed: float, frames: int, device=None) -> tuple[float, int]:
    """Max over ranks of the timed wall time and sum over ranks of the frames
    processed (the whole-job throughput is frames / max time).  dist None: one
    process, nothing to reduce."""
    if dist is None:
        return elapsed, frames
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    f = torch.tensor([frames], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(f, op=dist.ReduceOp.SUM)
    return float(t.item()), int(f.item())
