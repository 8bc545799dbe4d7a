"""Row N4: the ARM_OPTIMIZED=0 front end.  The oracle's restatement of the
reference's portable FFT path (oracle/nnsp_oracle.c or_rfft512_portable:
fft.c:27-221, complex.c:14-92, spectrogram_module.c:33-77) is pinned against
the reference's own portable build (oracle/_ref/libnnsp_ref_fe_portable.so,
oracle/build_ref.sh) through tests/golden/ref_fe_portable.npz
(tests/golden/make_golden.py fe_portable), and live when the reference tree
is present."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT, needs_reference
import oracle as O

GOLD = os.path.join(ROOT, "tests", "golden", "ref_fe_portable.npz")


def test_rfft_portable_matches_reference_fixture():
    g = np.load(GOLD)
    for x, y in zip(g["rfft_in"], g["rfft_out"]):
        np.testing.assert_array_equal(O.rfft512_portable(x), y)


def _oracle_features(pcm, mean, stdR, qbit, portable=True):
    L = O.lib()
    c = O.or_cfg()
    c.qbit_out = int(qbit)
    mean = np.ascontiguousarray(mean, np.int32)
    stdR = np.ascontiguousarray(stdR, np.int32)
    c.mean, c.stdR = mean.ctypes.data, stdR.ctypes.data
    c.fe_portable = int(portable)
    st = np.zeros(L.or_sizeof_stream(), np.uint8)
    L.or_fe_reset(C.c_void_p(st.ctypes.data), C.byref(c))
    out = np.zeros((len(pcm), 40), np.int16)
    for t, fr in enumerate(np.ascontiguousarray(pcm, np.int16)):
        L.or_fe_exec(C.c_void_p(st.ctypes.data), C.byref(c), C.c_void_p(fr.ctypes.data))
        out[t] = st[960 + 400:960 + 480].view(np.int16)   # or_stream.ctx[200..239]
    return out


def test_feature_class_portable_matches_reference_fixture():
    g = np.load(GOLD)
    for s in range(len(g["fe_pcm"])):
        got = _oracle_features(g["fe_pcm"][s], g["fe_mean"][s], g["fe_stdR"][s], g["fe_qbit"][s])
        np.testing.assert_array_equal(got, g["fe_feats"][s])


def test_portable_and_shipped_front_ends_differ():
    """the switch is live: the two FFT paths give different features"""
    g = np.load(GOLD)
    a = _oracle_features(g["fe_pcm"][0], g["fe_mean"][0], g["fe_stdR"][0], 8, True)
    b = _oracle_features(g["fe_pcm"][0], g["fe_mean"][0], g["fe_stdR"][0], 8, False)
    assert (a != b).any()


@needs_reference
def test_rfft_portable_live_random():
    so = os.path.join(ROOT, "oracle", "_ref", "libnnsp_ref_fe_portable.so")
    if not os.path.exists(so):
        pytest.skip("oracle/_ref not built")
    R = C.CDLL(so)
    rng = np.random.default_rng(7)
    for amp in (1 << 15, 1 << 13, 1 << 9, 3):
        for _ in range(20):
            x = rng.integers(-amp, amp, 512).astype(np.int32)
            xr, y = x.copy(), np.zeros(1024, np.int32)
            R.rfft(512, C.c_void_p(xr.ctypes.data), C.c_void_p(y.ctypes.data))
            np.testing.assert_array_equal(O.rfft512_portable(x), y[:514])
