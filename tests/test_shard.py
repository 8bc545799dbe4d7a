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


def _bench_dry_run(args, env=None):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"] + args,
                       env=env, timeout=180, capture_output=True, text=True)
    return r


@pytest.mark.parametrize("gpus,scaling", [(2, "weak"), (2, "strong"), (4, "weak")])
def test_bench_gpus_n_launches_n_ranks(gpus, scaling):
    """``python bench.py --gpus N`` (a plain launch, as the driver may start it)
    runs N ranks under torch.distributed.run itself; --dry-run makes each rank
    report its device and stream shard over gloo without touching a GPU.
    stdout carries exactly one JSON line."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = _bench_dry_run(["--gpus", str(gpus), "--scaling", scaling], env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    plan = __import__("json").loads(lines[0])
    assert plan["n_gpus"] == gpus and plan["launched_by"] == "torch.distributed.run"
    ranks = plan["ranks"]
    assert [p["rank"] for p in ranks] == list(range(gpus))
    assert sorted(p["device"] for p in ranks) == list(range(gpus))
    assert len({p["pid"] for p in ranks}) == gpus, "the ranks must be separate processes"
    covered = []
    for p in ranks:
        assert (p["first_stream"], p["streams"]) == shard_streams(
            p["rank"], gpus, **({"per_rank": 32768} if scaling == "weak" else {"total": 262144}))
        covered += list(range(p["first_stream"], p["first_stream"] + p["streams"]))
    assert len(covered) == len(set(covered)), "shards overlap"
    assert len(covered) == (32768 * gpus if scaling == "weak" else 262144)


def test_bench_n1_plan_and_world_mismatch():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = _bench_dry_run([], env)
    assert r.returncode == 0, r.stderr[-2000:]
    plan = __import__("json").loads(r.stdout)
    assert plan["n_gpus"] == 1 and plan["launched_by"] == "plain process"
    assert plan["ranks"][0]["first_stream"] == 0 and plan["ranks"][0]["streams"] == 32768
    # under torch.distributed.run, a world size that disagrees with --gpus is refused
    env.update(RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = _bench_dry_run(["--gpus", "4"], env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
