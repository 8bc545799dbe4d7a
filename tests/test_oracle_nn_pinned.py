"""The oracle's NN half against the reference's own portable NN build.

tests/golden/ref_nn.npz was written by tests/golden/make_golden.py from
affine.c, affine_acc32b.c, lstm.c, neural_nets.c and activation.c compiled here
with the reference's ARM_OPTIMIZED=0 switch (oracle/build_ref.sh), fed with
weights re-packed into that build's byte order.  That build and the shipped
one share every line after the MAC loop (affine.c:186-253 vs :311-339) except
the align shift, which the shipped build applies to a dead buffer (trap T1):

  * ``portable=True`` -- the oracle with the live align shift -- must equal the
    reference on every case, including KWS layer 0 (qi + qk = 14 with a bias);
  * the shipped-semantics oracle (``portable=False``, what the GPU is checked
    against) must equal it wherever the shift is zero, i.e. every layer with
    qi + qk >= 15 or without bias -- all of VAD and S2I, KWS from layer 1 on.

Pins A17-A21 (NeuralNetClass_exe, fc_8x16, rc_Krows / affine_Krows, lstm_8x16
and their _acc32b twins), both accumulator widths, on the reference's three
nets (their own def_nn*.c tables, tests/golden/ref_nets.npz) and on the N3
shapes (rows not a multiple of 4, odd K, 3 / 7 layers, two LSTMs, 256 wide).
"""
import ctypes as C
import os

import numpy as np
import pytest

import oracle as O
from conftest import ROOT, needs_reference
from nnsp_amd import nets

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def g():
    return np.load(os.path.join(GOLD, "ref_nn.npz"))


def _t1(qk, qb, qi):
    """align shift of affine_Krows with a bias (affine.c:69-72, :311-313) is nonzero"""
    return qi + qk < 15


@pytest.mark.parametrize("acc", [64, 32])
def test_fc_layers(g, acc):
    k = 0
    while f"fc{k}_cfg" in g:
        N, K, qk, qb, qi, act = (int(v) for v in g[f"fc{k}_cfg"])
        w, b, x, y = g[f"fc{k}_w"], g[f"fc{k}_b"], g[f"fc{k}_x"], g[f"fc{k}_y{acc}"]
        for r in range(len(x)):
            got = O.fc(w, b, x[r], qk, qb, qi, act, acc == 32, portable=True)
            np.testing.assert_array_equal(got, y[r], err_msg=f"fc case {k} row {r} (portable)")
            if not _t1(qk, qb, qi):
                got = O.fc(w, b, x[r], qk, qb, qi, act, acc == 32, portable=False)
                np.testing.assert_array_equal(got, y[r], err_msg=f"fc case {k} row {r} (shipped)")
        k += 1
    assert k >= 10


@pytest.mark.parametrize("acc", [64, 32])
def test_lstm_layers(g, acc):
    k = 0
    while f"lstm{k}_cfg" in g:
        N, K, qk, qb, qi, qir = (int(v) for v in g[f"lstm{k}_cfg"])
        w, wr, b, x = g[f"lstm{k}_w"], g[f"lstm{k}_wr"], g[f"lstm{k}_b"], g[f"lstm{k}_x"]
        for portable in (True, False):
            if not portable and _t1(qk, qb, qir):
                continue
            h, c = np.zeros(N, np.int16), np.zeros(N, np.int32)
            for r in range(len(x)):
                y = O.lstm(w, wr, b, x[r], h, c, qk, qb, qi, qir, acc == 32, portable)
                np.testing.assert_array_equal(y, g[f"lstm{k}_y{acc}"][r], err_msg=f"lstm {k} call {r}")
                np.testing.assert_array_equal(h, g[f"lstm{k}_h{acc}"][r])
                np.testing.assert_array_equal(c, g[f"lstm{k}_c{acc}"][r])
        k += 1
    assert k >= 6


def _net_data(g, name):
    if name in nets.ALL_GEN_SPECS:
        spec = nets.ALL_GEN_SPECS[name]
        W = [g[f"net_{name}_W{i}"] for i in range(spec.nl)]
        Wr = [g[f"net_{name}_Wr{i}"] if f"net_{name}_Wr{i}" in g else None for i in range(spec.nl)]
        B = [g[f"net_{name}_B{i}"] for i in range(spec.nl)]
        return nets.NetData(spec, W, Wr, B, np.zeros(40, np.int32), np.zeros(40, np.int32))
    return nets.ref_net(name)


NETS = ["vad", "kws", "s2i"] + list(nets.ALL_GEN_SPECS)


@pytest.mark.parametrize("acc", [64, 32])
@pytest.mark.parametrize("name", NETS)
def test_neural_net_exe(g, name, acc):
    """NeuralNetClass_exe (neural_nets.c:44-168) over 24 consecutive calls, LSTM
    state carried; the final h / c too."""
    data = _net_data(g, name)
    sp = data.spec
    t1 = any(_t1(sp.qk[i], sp.qb[i], sp.qi[i]) for i in range(sp.nl) if sp.types[i] == nets.FC) or any(
        _t1(sp.qk[i], sp.qb[i], sp.qi[i + 1] if i + 1 < sp.nl else 0) for i in range(sp.nl)
        if sp.types[i] == nets.LSTM)
    x, y = g[f"net_{name}_x"], g[f"net_{name}_y{acc}"]
    for portable in (True, False):
        if not portable and t1:
            continue
        on = O.OracleNet(data, acc32=acc == 32, portable=portable)
        st = np.zeros(O.lib().or_sizeof_stream(), np.uint8)
        O.lib().or_nnsp_reset(C.byref(on.net), C.c_void_p(st.ctypes.data), C.byref(on.cfg))
        for r in range(len(x)):
            got = on.forward(x[r], st)[:sp.nout]
            if sp.acts[-1] != nets.LINEAR:
                got = got.view(np.int16)[:sp.nout].astype(np.int32)
            np.testing.assert_array_equal(got, y[r], err_msg=f"{name} acc{acc} portable={portable} call {r}")
        ost = O.or_stream.from_buffer(st)
        lstm_w = [sp.sizes[i + 1] for i in range(sp.nl) if sp.types[i] == nets.LSTM]
        h = np.concatenate([np.array(ost.h[k][:n], np.int16) for k, n in enumerate(lstm_w)] + [np.zeros(0, np.int16)])
        c = np.concatenate([np.array(ost.c[k][:n], np.int32) for k, n in enumerate(lstm_w)] + [np.zeros(0, np.int32)])
        np.testing.assert_array_equal(h, g[f"net_{name}_h{acc}"])
        np.testing.assert_array_equal(c, g[f"net_{name}_c{acc}"])


def test_kws_layer0_is_the_t1_case(g):
    """The shipped KWS differs from the portable build only through T1: the
    shipped-semantics oracle must NOT reproduce the portable outputs there."""
    data = nets.ref_net("kws")
    assert data.spec.qi[0] + data.spec.qk[0] == 14
    on = O.OracleNet(data, portable=False)
    st = np.zeros(O.lib().or_sizeof_stream(), np.uint8)
    O.lib().or_nnsp_reset(C.byref(on.net), C.c_void_p(st.ctypes.data), C.byref(on.cfg))
    x, y = g["net_kws_x"], g["net_kws_y64"]
    diff = sum(not np.array_equal(on.forward(x[r], st)[:2], y[r]) for r in range(len(x)))
    assert diff > 0


def test_acc32_equals_acc64_on_reference_nets(g):
    """the worst-case dot product stays below 2^31 for the three
    nets, so both builds agree (reference outputs, both widths)."""
    for name in ("vad", "kws", "s2i"):
        np.testing.assert_array_equal(g[f"net_{name}_y32"], g[f"net_{name}_y64"])


def test_ref_nets_tables():
    """tests/golden/ref_nets.npz holds def_nn*.c's NeuralNetClass fields
    (evb/src/def_nn1_vad.c:29-110 etc.); the shapes are Appendix A's."""
    for name in ("vad", "kws", "s2i"):
        d = nets.ref_net(name)
        sp, ref = d.spec, nets.SPECS[name]
        assert (sp.sizes, sp.types, sp.qk, sp.qi, sp.qb, sp.acts) == (
            ref.sizes, ref.types, ref.qk, ref.qi, ref.qb, ref.acts)
        Wp, Wrp, Bp = d.packed()
        z = np.load(nets.REF_NETS_NPZ)
        for i in range(sp.nl):   # unpack -> pack is the identity on the shipped bytes
            np.testing.assert_array_equal(Wp[i], z[f"{name}_kernel{i}"])
            np.testing.assert_array_equal(Bp[i], z[f"{name}_bias{i}"])
            if Wrp[i] is not None:
                np.testing.assert_array_equal(Wrp[i], z[f"{name}_kernel_rec{i}"])
        assert d.mean.dtype == np.int32 and d.mean.max() < 0 and 15000 < d.stdR.min()


@needs_reference
def test_live_portable_reference_random_nets():
    """Fresh random FC/LSTM layers through the live portable build (container only)."""
    so = os.path.join(ROOT, "oracle", "_ref", "libnnsp_ref_nn_portable.so")
    if not os.path.exists(so):
        pytest.skip("oracle/_ref not built")
    R = C.CDLL(so)
    i16 = C.c_int16
    rng = np.random.default_rng(4242)
    for trial in range(40):
        N, K = int(rng.integers(1, 70)), int(rng.integers(1, 250))
        qk, qi = int(rng.integers(3, 8)), int(rng.integers(8, 16))
        qb = int(rng.integers(10, 18))
        act = int(rng.integers(0, 4))
        acc32 = bool(trial & 1)
        w = rng.integers(-128, 128, (N, K)).astype(np.int8)
        b = rng.integers(-32768, 32768, N).astype(np.int16)
        x = rng.integers(-4000, 4000, K).astype(np.int16)
        y = np.zeros(2 * N + 2, np.int16)
        fn = R.fc_8x16_acc32b if acc32 else R.fc_8x16
        afn = C.cast(getattr(R, ["relu6_fix", "tanh_fix", "sigmoid_fix", "linear_fix"][act]), C.c_void_p)
        wp = nets.pack_fc_portable(w)   # kept alive across the call
        fn(O.p(y), O.p(wp), None, O.p(b), O.p(x), None, None, i16(N), i16(K), i16(N),
           i16(qk), i16(qb), i16(qi), i16(0), C.c_int(act), afn)
        ref = y.view(np.int32)[:N] if act == nets.LINEAR else y[:N].astype(np.int32)
        np.testing.assert_array_equal(O.fc(w, b, x, qk, qb, qi, act, acc32, portable=True), ref)
