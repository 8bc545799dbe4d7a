"""Stream shards across GPUs.

Independent 16 kHz streams are the data-parallel axis: rank r of a world of
N owns streams [r*S, (r+1)*S) of the synthetic population (weak scaling, S
streams per GPU).  Nothing is exchanged on the data path; the only
collective is the max-reduce of the timed region's wall time in bench.py.
"""
from __future__ import annotations


def shard_streams(rank: int, world: int, per_rank: int) -> tuple[int, int]:
    """(first global stream, stream count) of rank's shard."""
    if world < 1 or not 0 <= rank < world or per_rank < 1:
        raise ValueError(f"bad shard: rank {rank} of {world}, {per_rank} streams per rank")
    return rank * per_rank, per_rank
