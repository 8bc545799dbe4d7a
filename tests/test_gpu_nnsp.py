"""GPU parity of the batched engine against the CPU oracle (bit-exact).

Synthetic nets of the exact VAD / Hi-Galaxy KWS / S2I shapes and formats
(evb/src/def_nn*.c), synthetic SplitMix64 PCM plus full-scale bursts; every
per-frame trigger, every NN logit and every front-end feature must match.
"""
import numpy as np
import pytest

from oracle import OracleNet, synthetic_pcm

from nnsp_amd.engine import NNSPBatch
from nnsp_amd.nets import synth_net

pytestmark = pytest.mark.gpu

NETS = ["vad", "kws", "s2i"]


def _pcm(S, T, seed=7):
    pcm = synthetic_pcm(S, T, seed=0x4E4E5350 + seed)
    rng = np.random.default_rng(seed)
    # a few loud / quiet streams to exercise wide dynamic range
    pcm[1::5] = (pcm[1::5].astype(np.int32) * 6).clip(-32768, 32767).astype(np.int16)
    pcm[2::5] //= 64
    pcm[3::7, :, :] = rng.integers(-20000, 20000, pcm[3::7].shape).astype(np.int16)
    return pcm


def _compare(name, acc32, S, chunks, seed=3):
    data = synth_net(name, seed)
    orc = OracleNet(data, acc32=acc32)
    eng = NNSPBatch(data, S, max(chunks), acc32=acc32)
    T = sum(chunks)
    pcm = _pcm(S, T, seed)
    o_trig, o_lg, o_ft, _ = orc.run(pcm)
    t0 = 0
    for Tc in chunks:
        trig, lg, ft = eng.exec(pcm[:, t0:t0 + Tc], want_logits=True, want_features=True)
        np.testing.assert_array_equal(ft, o_ft[:, t0:t0 + Tc], err_msg=f"{name} features chunk@{t0}")
        # every frame: both sides hold 0 on the frames where the NN does not run
        np.testing.assert_array_equal(lg, o_lg[:, t0:t0 + Tc], err_msg=f"{name} logits chunk@{t0}")
        np.testing.assert_array_equal(trig, o_trig[:, t0:t0 + Tc], err_msg=f"{name} trig")
        t0 += Tc
    eng.close()


@pytest.mark.parametrize("name", NETS)
@pytest.mark.parametrize("acc32", [False, True])
@pytest.mark.parametrize("path", ["split", "generic", "fused"])
def test_batch_matches_oracle(name, acc32, path, monkeypatch):
    # split = proj_kernel + recur_kernel compiled for the net's shape (default);
    # generic = the same kernels reading the shape at run time;
    # fused = the general per-step nn_kernel (any fc/lstm stack)
    monkeypatch.delenv("NNSP_FUSED_NN", raising=False)
    monkeypatch.delenv("NNSP_GENERIC_SHAPE", raising=False)
    if path == "fused":
        monkeypatch.setenv("NNSP_FUSED_NN", "1")
    elif path == "generic":
        monkeypatch.setenv("NNSP_GENERIC_SHAPE", "1")
    _compare(name, acc32, S=37, chunks=[24, 7, 1, 10])


@pytest.mark.parametrize("name", NETS)
def test_acc64_int64_kernels(name, monkeypatch):
    # acc64 nets run the int32-accumulator kernels when the host bound proves
    # no overflow (ep32; true for these shapes); NNSP_NO_EP32 forces the
    # int64-epilogue instantiations of proj / recur, which must agree too
    monkeypatch.setenv("NNSP_NO_EP32", "1")
    _compare(name, False, S=37, chunks=[24, 7, 1, 10])


@pytest.mark.parametrize("name", NETS)
def test_many_streams_one_long_chunk(name):
    _compare(name, False, S=600, chunks=[61, 3])


@pytest.mark.parametrize("name", NETS)
def test_reset_mask(name):
    data = synth_net(name, 11)
    S, T = 20, 12
    orc = OracleNet(data)
    eng = NNSPBatch(data, S, T)
    pcm = _pcm(S, 3 * T, 11)
    st = orc.new_states(S)
    mask = (np.arange(S) % 3 == 0).astype(np.uint8)
    for c in range(3):
        blk = pcm[:, c * T:(c + 1) * T]
        o_trig, o_lg, _, st = orc.run(blk, st)
        trig, lg, _ = eng.exec(blk, want_logits=True)
        np.testing.assert_array_equal(trig, o_trig)
        np.testing.assert_array_equal(lg, o_lg)
        orc.reset_streams(st, mask)
        eng.reset(mask)
    eng.close()


@pytest.mark.parametrize("name", NETS)
@pytest.mark.parametrize("tseq", ["1", "3", "4"])
def test_recur_tiles_back_to_back(name, tseq, monkeypatch):
    # several 16-stream tiles per recur workgroup through one pipeline
    # (FastRun.tseq): 75 streams = 5 tiles, so tseq 3 leaves a workgroup of 3
    # tiles and one of 2 (the last one partial); chunks of 40, 9, 2 and 13
    # frames give tiles of 20, 5, 1 and 7 NN steps (and padded 1-step tiles)
    monkeypatch.setenv("NNSP_RECUR_TSEQ", tseq)
    _compare(name, True, S=75, chunks=[40, 9, 2, 13])
