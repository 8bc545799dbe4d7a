"""Multi-GPU readiness without GPUs: stream shards are disjoint
and cover the population in both scaling modes, and a world-size-2 gloo run
of bench.py's bookkeeping (nnsp_amd.shard: dist_env, shard_streams,
reduce_run) over the oracle cascade gives per-stream outputs identical to one
unsharded run -- the reference keeps all state per stream
(evb/src/nnCntrlClass.c:152-272), so sharding streams must not change any
output.  The same property on the GPU engine is tests/test_gpu_shards.py."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from nnsp_amd.nets import get_net
from nnsp_amd.shard import reduce_run, shard_streams
from oracle import OracleCascade, OracleNet, load_wavs, synthetic_pcm


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shards_cover_and_are_disjoint(world):
    for kw in ({"per_rank": 4096}, {"total": 262144}, {"total": 1001}):
        seen = []
        for r in range(world):
            s0, n = shard_streams(r, world, **kw)
            seen += list(range(s0, s0 + n))
        want = world * kw["per_rank"] if "per_rank" in kw else kw["total"]
        assert seen == list(range(want))
        sizes = [shard_streams(r, world, **kw)[1] for r in range(world)]
        assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_streams(2, 2, per_rank=4)
    with pytest.raises(ValueError):
        shard_streams(0, 2, per_rank=4, total=8)


def test_reduce_run_single_process():
    assert reduce_run(None, 1.25, 77) == (1.25, 77)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_gloo_world2_matches_unsharded(tmp_path, mode):
    total, T = 26 if mode == "weak" else 27, 60
    out = str(tmp_path / "r.npz")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "helpers", "dist_worker.py"), out, mode, str(total), str(T)]
    subprocess.run(cmd, check=True, env=env, timeout=300, capture_output=True)
    z = np.load(out)
    S = total if mode == "strong" else (total // 2) * 2
    assert z["sizes"].tolist() == [list(shard_streams(r, 2, **({"total": total} if mode == "strong"
                                                               else {"per_rank": total // 2}))) for r in range(2)]
    assert float(z["elapsed"]) == 2.5 and int(z["frames"]) == S * 2 * T
    oc = OracleCascade({n: OracleNet(get_net(n, "ref")) for n in ("vad", "kws", "s2i")})
    st = oc.new_states(S)
    wavs = load_wavs()
    ref = [oc.run(synthetic_pcm(S, T, t0=c * T, s0=0, wavs=wavs), st)[:3] for c in range(2)]
    for k, name in enumerate(("ran", "det", "o3")):
        np.testing.assert_array_equal(z[name], np.concatenate([r[k] for r in ref], axis=1), err_msg=name)
    assert (z["ran"] != 1).any(), "no stream left VAD: the comparison is vacuous"
