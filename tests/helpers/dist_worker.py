"""One rank of the world-size-2 gloo test (tests/test_shard.py), launched by
torch.distributed.run on the CPU.  It runs bench.py's multi-GPU bookkeeping
(dist_env, shard_streams, reduce_run) and the oracle cascade on its own
stream shard, then gathers every rank's per-stream outputs on rank 0, which
writes them (and the reduced timing) to argv[1] as .npz."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from nnsp_amd.nets import get_net  # noqa: E402
from nnsp_amd.shard import dist_env, reduce_run, shard_streams  # noqa: E402
from oracle import OracleCascade, OracleNet, load_wavs, synthetic_pcm  # noqa: E402


def main():
    out, mode, total, T = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rank, world, local, launched = dist_env()
    assert launched and world == 2
    dist.init_process_group("gloo")
    if mode == "weak":
        s0, S = shard_streams(rank, world, per_rank=total // world)
    else:
        s0, S = shard_streams(rank, world, total=total)
    wavs = load_wavs()
    oc = OracleCascade({n: OracleNet(get_net(n, "ref")) for n in ("vad", "kws", "s2i")})
    st = oc.new_states(S)
    ran, det, o3 = [], [], []
    for c in range(2):   # two chunks, state carried
        r, d, o, st = oc.run(synthetic_pcm(S, T, t0=c * T, s0=s0, wavs=wavs), st)
        ran.append(r), det.append(d), o3.append(o)
    ran, det, o3 = (np.concatenate(a, axis=1) for a in (ran, det, o3))
    elapsed, frames = reduce_run(dist, 1.5 + rank, S * 2 * T)
    # gather the shards (the test compares them with one unsharded run)
    sizes = [None] * world
    dist.all_gather_object(sizes, (s0, S))
    parts = [None] * world
    dist.all_gather_object(parts, (ran, det, o3))
    if rank == 0:
        np.savez(out, elapsed=elapsed, frames=frames, sizes=np.array(sizes),
                 ran=np.concatenate([p[0] for p in parts]), det=np.concatenate([p[1] for p in parts]),
                 o3=np.concatenate([p[2] for p in parts]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
