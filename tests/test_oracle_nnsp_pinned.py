"""The oracle's NNSPClass_exec, end to end, against the reference's own
portable build: tests/golden/ref_nnsp_portable.npz holds,
per frame, the return value of the reference's NNSPClass_exec
(nn_speech.c:74-127, ARM_OPTIMIZED=0), normFeatContext[200:240], outputs[3]
and counts_category, and the final LSTM h / c, for the three reference nets
at both accumulator widths over the three test wavs (1000 frames) and eight
synthetic streams (200 frames), each with one NNSPClass_reset mid-stream.
The oracle runs in its portable mode (fe_portable + portable)."""
import ctypes as C

import numpy as np
import pytest

from nnsp_e2e import fixture, streams
from oracle import OracleNet, or_stream

from nnsp_amd.nets import ref_net


@pytest.fixture(scope="module")
def g():
    return fixture()


def run_oracle_frames(orc, pcm, reset_at):
    """frame by frame: trig, ctx slot 5, outputs[3], counts per frame; final h / c."""
    T = len(pcm)
    st = orc.new_states(1)
    tr = np.zeros(T, np.int16)
    ft = np.zeros((T, 40), np.int16)
    o3 = np.zeros((T, 3), np.int16)
    ct = np.zeros((T, 8), np.int16)
    for t in range(T):
        if t == reset_at:
            orc.reset_streams(st, np.ones(1, np.uint8))
        trig, _, feats, st = orc.run(pcm[None, t:t + 1], st)
        s = or_stream.from_buffer(st[0])
        tr[t], ft[t] = trig[0, 0], feats[0, 0]
        o3[t], ct[t] = list(s.outputs), list(s.counts)
    s = or_stream.from_buffer(st[0])
    return tr, ft, o3, ct, np.array(s.h[0]), np.array(s.c[0])


@pytest.mark.parametrize("acc", [64, 32])
@pytest.mark.parametrize("name", ["vad", "kws", "s2i"])
def test_oracle_nnsp_exec_vs_reference_portable_build(g, name, acc):
    data = ref_net(name)
    N = data.spec.sizes[1 + data.spec.types.index(1)] if 1 in data.spec.types else 0
    orc = OracleNet(data, acc32=acc == 32, portable=True, fe_portable=True)
    tag = f"{name}_{acc}"
    for i, (pcm, reset_at, r0) in enumerate(streams(g)):
        T = len(pcm)
        tr, ft, o3, ct, h, c = run_oracle_frames(orc, pcm, reset_at)
        rows = slice(r0, r0 + T)
        np.testing.assert_array_equal(ft, g[f"{name}_feats"][rows], err_msg=f"{tag} stream {i} features")
        np.testing.assert_array_equal(tr, g[f"{tag}_trig"][rows], err_msg=f"{tag} stream {i} NNSPClass_exec return")
        np.testing.assert_array_equal(o3, g[f"{tag}_outputs"][rows], err_msg=f"{tag} stream {i} outputs")
        np.testing.assert_array_equal(ct, g[f"{tag}_counts"][rows], err_msg=f"{tag} stream {i} counts_category")
        np.testing.assert_array_equal(h[:N], g[f"{tag}_h"][i], err_msg=f"{tag} stream {i} final h")
        np.testing.assert_array_equal(c[:N], g[f"{tag}_c"][i], err_msg=f"{tag} stream {i} final c")


def test_fixture_is_not_vacuous(g):
    for name in ("vad", "kws", "s2i"):
        assert (g[f"{name}_64_trig"] != 0).sum() > 50, f"{name} never triggered"
    assert (g["s2i_64_outputs"] != 0).any()
    # the reset lands inside the wav streams and the noise streams
    cfg = g["cfg"]
    assert 0 < cfg[1] < cfg[0] and 0 < cfg[3] < cfg[2] and cfg[1] % 2 == 1 and cfg[3] % 2 == 1
