"""The CPU oracle against the reference's own outputs.

Fixtures (tests/golden/*.npz) were produced by tests/golden/make_golden.py from
the reference C files compiled here from their own sources (oracle/_ref) and
from the reference's python/nnsp_pack/c_weight_man.py; they run everywhere.
When the partial reference build is present, extra random vectors are checked
live as well.
"""
import ctypes as C
import os

import numpy as np
import pytest

import oracle as O
from conftest import ROOT
from nnsp_amd import nets

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLD, "ref_stages.npz"))


def test_activations(g):
    x = g["act_x"]
    np.testing.assert_array_equal(O.act(1, x), g["act_tanh_fix"])
    np.testing.assert_array_equal(O.act(2, x), g["act_sigmoid_fix"])
    np.testing.assert_array_equal(O.act(0, x), g["act_relu6_fix"])
    np.testing.assert_array_equal(O.act(3, x), x)


def test_log10(g):
    np.testing.assert_array_equal(O.log10(g["log_x"]), g["log_y"])
    # log10_vec with bit_frac_in = 12 adds (15 - 12) * log10(2) in Q15
    np.testing.assert_array_equal(O.log10(g["log_x"][:256]) + 3 * 0x2688, g["log_y_q12"])


def test_spec2pspec_truncating_cast(g):
    for i in range(len(g["pspec_in"])):
        np.testing.assert_array_equal(O.spec2pspec(g["pspec_in"][i]), g["pspec_out"][i])


def test_mel(g):
    for i in range(len(g["mel_in"])):
        np.testing.assert_array_equal(O.mel(g["mel_in"][i]), g["mel_out"][i])


def test_pwr2_ceiling(g):
    L = O.lib()
    np.testing.assert_array_equal([L.or_pwr2(int(v)) for v in g["pwr2_x"]], g["pwr2_y"])
    np.testing.assert_array_equal([L.or_ceiling(int(v)) for v in g["pwr2_x"]], g["ceil_y"])


@pytest.mark.parametrize("kind", ["binary", "s2i"])
def test_post_processing_sequences(g, kind):
    L = O.lib()
    e_in, trig = g[f"post_{kind}_in"], g[f"post_{kind}_trig"]
    nseq = len(g["post_thr"])
    nstep = len(e_in) // nseq
    k = 0
    for q in range(nseq):
        st = O.or_stream()
        st.slides = 1
        cfg = O.or_cfg()
        cfg.nn_id = 0 if kind == "s2i" else 1
        cfg.thresh_prob = int(g["post_thr"][q])
        cfg.th_count = int(g["post_cnt"][q])
        for _ in range(nstep):
            e = e_in[k].copy()
            if kind == "s2i":
                L.or_s2i_post(C.byref(st), C.byref(cfg), O.p(e))
            else:
                L.or_binary_post(C.byref(st), C.byref(cfg), O.p(e))
            assert st.trigger == trig[k], (kind, q, k)
            np.testing.assert_array_equal(e, g[f"post_{kind}_est_out"][k])   # T7 overwrite
            np.testing.assert_array_equal(list(st.counts)[:7], g[f"post_{kind}_counts"][k][:7])
            np.testing.assert_array_equal(list(st.outputs), g[f"post_{kind}_outputs"][k])
            assert st.argmax_last == g[f"post_{kind}_argmax_last"][k]
            k += 1


def test_fe_set_default_keeps_slot5(g):
    L = O.lib()
    for i in range(len(g["fe_qbit"])):
        st = O.or_stream()
        for k in range(240):
            st.ctx[k] = 1111
        cfg = O.or_cfg()
        mean, stdR = g["fe_mean"][i].copy(), g["fe_stdR"][i].copy()
        cfg.mean, cfg.stdR, cfg.qbit_out = mean.ctypes.data, stdR.ctypes.data, int(g["fe_qbit"][i])
        L.or_fe_reset(C.byref(st), C.byref(cfg))
        np.testing.assert_array_equal(np.array(st.ctx[:240]), g["fe_ctx"][i][:240])
        assert all(v == 0 for v in st.buf)


def test_weight_layout():
    lay = np.load(os.path.join(GOLD, "layout.npz"))
    k = 0
    while f"fc_{k}_in" in lay:
        m = lay[f"fc_{k}_in"].astype(np.int64)
        np.testing.assert_array_equal(nets.pack_fc(m), lay[f"fc_{k}_out"])
        np.testing.assert_array_equal(nets.unpack_fc(nets.pack_fc(m), *m.shape), m)
        k += 1
    assert k > 10
    j = 0
    while f"lstm_{j}_wf" in lay:
        np.testing.assert_array_equal(nets.pack_lstm(lay[f"lstm_{j}_wf"].astype(np.int64)), lay[f"lstm_{j}_out_wf"])
        np.testing.assert_array_equal(nets.pack_lstm(lay[f"lstm_{j}_wr"].astype(np.int64)), lay[f"lstm_{j}_out_wr"])
        np.testing.assert_array_equal(nets.pack_lstm_bias(lay[f"lstm_{j}_b"].astype(np.int64)), lay[f"lstm_{j}_out_b"])
        j += 1
    assert j == 4


@pytest.mark.skipif(not os.path.exists(O.REF), reason="partial reference build absent")
def test_live_reference_random_vectors():
    R = C.CDLL(O.REF, mode=os.RTLD_LAZY)
    rng = np.random.default_rng(99)
    x = rng.integers(-(2**31 - 1), 2**31 - 1, 50000).astype(np.int32)
    for kind, name in ((1, "tanh_fix"), (2, "sigmoid_fix"), (0, "relu6_fix")):
        y = np.zeros(len(x), np.int16)
        getattr(R, name)(O.p(y), O.p(x), len(x))
        np.testing.assert_array_equal(O.act(kind, x), y)
    lx = rng.integers(1, 2**31 - 1, 20000).astype(np.int32)
    ly = np.zeros(len(lx), np.int32)
    R.log10_vec(O.p(ly), O.p(lx), len(lx), C.c_int16(15))
    np.testing.assert_array_equal(O.log10(lx), ly)
