"""Row N4 on the GPU: the reference built with ARM_OPTIMIZED=0
(nnsp_batch_create_ex(..., arm_optimized=0)).

* front end: Frac15 window, fft.c's radix-4 DIF rfft, spec2pspec >> 15
  (spectrogram_module.c:33-77, feature_module.c:58-60);
* net: weights in the portable byte order (affine.c:261-346) and the live
  align shift before the bias (affine.c:311-313; it fires on KWS layer 0,
  qbit_input + qbit_kernel = 14).

Checked bit for bit against the oracle with fe_portable / portable set; that
oracle is pinned to the reference's own portable build
(tests/test_oracle_fe_portable.py, tests/test_oracle_nn_pinned.py).
"""
import numpy as np
import pytest

from oracle import OracleCascade, OracleNet, load_wavs, synthetic_pcm

from nnsp_amd.engine import NNSPBatch, NNSPCascade
from nnsp_amd.nets import ref_net, synth_net

pytestmark = pytest.mark.gpu

WAVS = load_wavs()


def _pcm(S, T, t0=0, every=2):
    return synthetic_pcm(S, T, t0=t0, wavs=WAVS, every=every)


def _full_scale(S, T, seed=3):
    """square waves and clipped noise at the int16 limits: the FFT's largest
    values (the no-saturation bound of nnsp_dev.h's portable FFT)"""
    rng = np.random.default_rng(seed)
    n = np.arange(T * 160)
    out = np.empty((S, T * 160), np.int16)
    for s in range(S):
        if s % 3 == 0:
            per = 2 + s
            out[s] = np.where((n // per) % 2 == 0, 32767, -32768)
        elif s % 3 == 1:
            out[s] = np.clip(rng.normal(0, 30000, T * 160), -32768, 32767).astype(np.int16)
        else:
            out[s] = (32767 * np.sign(np.sin(2 * np.pi * n * (100 + 37 * s) / 16000))).astype(np.int16)
    return out.reshape(S, T, 160)


def _compare(data, acc32, S, chunks, pcm):
    orc = OracleNet(data, acc32=acc32, portable=True, fe_portable=True)
    eng = NNSPBatch(data, S, max(chunks), acc32=acc32, arm_optimized=False)
    o_trig, o_lg, o_ft, _ = orc.run(pcm)
    t0 = 0
    for Tc in chunks:
        trig, lg, ft = eng.exec(pcm[:, t0:t0 + Tc], want_logits=True, want_features=True)
        np.testing.assert_array_equal(ft, o_ft[:, t0:t0 + Tc], err_msg=f"features chunk@{t0}")
        np.testing.assert_array_equal(lg, o_lg[:, t0:t0 + Tc], err_msg=f"logits chunk@{t0}")
        np.testing.assert_array_equal(trig, o_trig[:, t0:t0 + Tc], err_msg=f"trig chunk@{t0}")
        t0 += Tc
    eng.close()
    return o_ft, o_trig


@pytest.mark.parametrize("acc32", [False, True])
@pytest.mark.parametrize("name", ["vad", "kws", "s2i"])
def test_portable_batch_reference_nets(name, acc32):
    S, chunks = 40, [37, 1, 50, 12]
    pcm = _pcm(S, sum(chunks))
    ft, trig = _compare(ref_net(name), acc32, S, chunks, pcm)
    # the switch is live: the shipped build's features differ on the same PCM
    _, _, ft_arm, _ = OracleNet(ref_net(name), acc32=acc32).run(pcm)
    assert (ft != ft_arm).any()
    if name == "vad":
        assert (trig != 0).any(), "VAD never triggered: vacuous"


@pytest.mark.parametrize("name", ["vad", "kws"])
def test_portable_batch_full_scale(name):
    S, chunks = 24, [30, 9]
    _compare(ref_net(name), False, S, chunks, _full_scale(S, sum(chunks)))


def test_portable_batch_synthetic_weights():
    S, chunks = 32, [25, 25]
    for name in ("vad", "s2i"):
        _compare(synth_net(name, 9), False, S, chunks, _pcm(S, sum(chunks), every=3))


@pytest.mark.parametrize("window", [16, 0])
def test_portable_cascade_reference_nets(window):
    S, chunks = 48, [100, 57, 100]
    gnets = {n: NNSPBatch(ref_net(n), S, 100, arm_optimized=False) for n in ("vad", "kws", "s2i")}
    gc = NNSPCascade(gnets)
    gc.set_window(window)
    oc = OracleCascade({n: OracleNet(ref_net(n), portable=True, fe_portable=True) for n in ("vad", "kws", "s2i")})
    pcm = _pcm(S, sum(chunks))
    o_ran, o_det, o_o3, _ = oc.run(pcm)
    t0 = 0
    for Tc in chunks:
        ran, det, o3 = gc.exec(pcm[:, t0:t0 + Tc])
        np.testing.assert_array_equal(ran, o_ran[:, t0:t0 + Tc], err_msg=f"net chunk@{t0}")
        np.testing.assert_array_equal(det, o_det[:, t0:t0 + Tc], err_msg=f"detected chunk@{t0}")
        np.testing.assert_array_equal(o3, o_o3[:, t0:t0 + Tc], err_msg=f"outputs3 chunk@{t0}")
        t0 += Tc
    assert len(np.unique(o_ran)) >= 2, "cascade never switched nets: vacuous"
    gc.close()


def test_portable_and_shipped_nets_cannot_share_a_cascade():
    S = 8
    gnets = {n: NNSPBatch(ref_net(n), S, 16, arm_optimized=(n != "kws")) for n in ("vad", "kws", "s2i")}
    with pytest.raises(Exception, match="nnsp_cascade_create"):
        NNSPCascade(gnets)
