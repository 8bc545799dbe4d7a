"""Virtual stream shards on one GPU: K engine objects
over disjoint stream ranges (nnsp_amd.shard.shard_streams, the ranges
bench.py gives the ranks) must produce per-stream outputs byte-identical to
one full-size object -- the multi-GPU partitioning without 8 GPUs."""
import numpy as np
import pytest

from oracle import load_wavs, synthetic_pcm

from nnsp_amd.engine import NNSPBatch, NNSPCascade
from nnsp_amd.nets import ref_net, synth_net
from nnsp_amd.shard import shard_streams

pytestmark = pytest.mark.gpu


def _cascade(data, S, T):
    return NNSPCascade({n: NNSPBatch(data[n], S, T) for n in ("vad", "kws", "s2i")})


@pytest.mark.parametrize("weights", ["ref", "synth"])
def test_cascade_virtual_shards(weights):
    total, K, chunks = 100, 3, [100, 37, 100]
    data = {n: (ref_net(n) if weights == "ref" else synth_net(n)) for n in ("vad", "kws", "s2i")}
    pcm = synthetic_pcm(total, sum(chunks), wavs=load_wavs(), every=2)
    full = _cascade(data, total, 100)
    shards = [(s0, n, _cascade(data, n, 100)) for s0, n in (shard_streams(r, K, total=total) for r in range(K))]
    t0 = 0
    for Tc in chunks:
        ref = full.exec(pcm[:, t0:t0 + Tc])
        for s0, n, eng in shards:
            got = eng.exec(pcm[s0:s0 + n, t0:t0 + Tc])
            for a, b, what in zip(got, ref, ("net_ran", "detected", "outputs3")):
                np.testing.assert_array_equal(a, b[s0:s0 + n], err_msg=f"{what} shard@{s0} chunk@{t0}")
        t0 += Tc
    pos = full.positions()
    for s0, n, eng in shards:
        np.testing.assert_array_equal(eng.positions(), pos[s0:s0 + n])


def test_batch_virtual_shards():
    total, K, T = 90, 4, 50
    data = ref_net("s2i")
    pcm = synthetic_pcm(total, 2 * T, wavs=load_wavs(), every=3)
    full = NNSPBatch(data, total, T)
    shards = [(s0, n, NNSPBatch(data, n, T)) for s0, n in (shard_streams(r, K, total=total) for r in range(K))]
    for c in range(2):
        tr, lg, ft = full.exec(pcm[:, c * T:(c + 1) * T], want_logits=True, want_features=True)
        for s0, n, eng in shards:
            t2, l2, f2 = eng.exec(pcm[s0:s0 + n, c * T:(c + 1) * T], want_logits=True, want_features=True)
            np.testing.assert_array_equal(t2, tr[s0:s0 + n])
            np.testing.assert_array_equal(l2, lg[s0:s0 + n])
            np.testing.assert_array_equal(f2, ft[s0:s0 + n])
