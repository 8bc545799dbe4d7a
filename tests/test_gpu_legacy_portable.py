"""Row N4 through the drop-in API: nnsp_set_arm_optimized(0) makes the legacy
entry points reproduce the reference compiled with ARM_OPTIMIZED=0.  Checked
on the GPU directly against outputs of the reference's OWN portable build
(tests/golden/ref_fe_portable.npz, tests/golden/ref_nn.npz, written by
tests/golden/make_golden.py from oracle/_ref's libnnsp_ref_fe_portable.so /
libnnsp_ref_nn_portable.so):

* rfft (fft.c:27-126), fft (fft.c:128-221, in place), spec2pspec,
  stftModule_analyze (spectrogram_module.c:33-77);
* FeatureClass_execute frame by frame (feature_module.c:47-74);
* fc_8x16 / lstm_8x16 and the _acc32b twins, affine_Krows_8x16 (affine.c:261-346)
  on weights in the portable byte order, and NeuralNetClass_exe over 24
  consecutive calls on the reference's three nets and the N3 shapes;
* NNSPClass_exec against the oracle with the portable front end and net.
"""
import ctypes as C
import os

import numpy as np
import pytest

import oracle as O
from conftest import ROOT
from oracle import OracleNet, load_wavs, synthetic_pcm

from nnsp_amd import _lib, nets
from nnsp_amd.nets import NN_ID, ref_net

pytestmark = pytest.mark.gpu

GOLD = os.path.join(ROOT, "tests", "golden")
_KEEP = []
i16 = C.c_int16
ACTS = {0: "relu6_fix", 1: "tanh_fix", 2: "sigmoid_fix", 3: "linear_fix"}


@pytest.fixture(scope="module", autouse=True)
def portable_build():
    L = _lib.lib()
    assert L.nnsp_get_arm_optimized() == 1
    assert L.nnsp_set_arm_optimized(0) == 0
    assert L.nnsp_get_arm_optimized() == 0
    yield
    L.nnsp_set_arm_optimized(1)


@pytest.fixture(scope="module")
def gfe():
    return np.load(os.path.join(GOLD, "ref_fe_portable.npz"))


@pytest.fixture(scope="module")
def gnn():
    return np.load(os.path.join(GOLD, "ref_nn.npz"))


def _rev8(m):
    return int(f"{m:08b}"[::-1], 2)


def test_rfft_vs_reference(gfe):
    L = _lib.lib()
    for x, y in zip(gfe["rfft_in"], gfe["rfft_out"]):
        xi = np.ascontiguousarray(x, np.int32)
        keep = xi.copy()
        out = np.zeros(514, np.int32)
        L.rfft(512, O.p(xi), O.p(out))
        np.testing.assert_array_equal(out, y)
        np.testing.assert_array_equal(xi, keep)   # rfft leaves its input alone
    assert L.nnsp_legacy_status() == 0


def test_fft_in_place_vs_reference(gfe):
    """fft(8): the reference's rfft output rebuilt from it with fft.c's split
    (restated here in int64 numpy), and the in-place input afterwards."""
    L = _lib.lib()
    tw = np.array([(np.int32(w) << 16 >> 16, np.int32(w) >> 16) for w in nets_dif_rtw()], np.int64)
    for x, y in zip(gfe["rfft_in"][:12], gfe["rfft_out"][:12]):
        xi = np.ascontiguousarray(x, np.int32)
        z = np.zeros(512, np.int32)
        L.fft(8, O.p(xi), O.p(z))
        np.testing.assert_array_equal(xi.reshape(256, 2), z.reshape(256, 2)[[_rev8(m) for m in range(256)]])
        Z = z.reshape(256, 2).astype(np.int64)
        j = (256 - np.arange(256)) & 255
        tr, tim = Z[j, 0], -Z[j, 1]
        er, ei = (Z[:, 0] + tr) >> 1, (Z[:, 1] + tim) >> 1
        orr, oi = (Z[:, 1] - tim) >> 1, (-(Z[:, 0] - tr)) >> 1
        re = ((orr * tw[:, 0] - oi * tw[:, 1]) >> 15) + er
        im = ((orr * tw[:, 1] + oi * tw[:, 0]) >> 15) + ei
        got = np.stack([re, im], 1).reshape(-1)
        np.testing.assert_array_equal(got, y[:512].astype(np.int64))
    assert L.nnsp_legacy_status() == 0


def nets_dif_rtw():
    from nnsp_amd import tables
    return tables.rfft_dif_twiddles()


def test_spec2pspec_and_analyze(gfe):
    L = _lib.lib()
    rng = np.random.default_rng(5)
    x = rng.integers(-(1 << 25), 1 << 25, 514).astype(np.int32)
    y = np.zeros(257, np.int32)
    L.spec2pspec(O.p(y), O.p(x), 257)
    xx = x.astype(np.int64)
    want = ((xx[0::2] ** 2 + xx[1::2] ** 2) >> 15).astype(np.uint64).astype(np.uint32).view(np.int32)
    np.testing.assert_array_equal(y, want)
    # stftModule_analyze: the window (Frac15) of the shifted buffer through rfft
    st = _lib.FeatureClass()
    L.FeatureClass_construct(C.byref(st), None, None, 8)
    stft = C.byref(st.state_stftModule)
    L.stftModule_setDefault(stft)
    buf = np.zeros(480, np.int32)
    win = np.array(nets_window(), np.int32)
    pcm = synthetic_pcm(1, 6, wavs=load_wavs(), every=1)[0]
    for t in range(6):
        y = np.zeros(1024, np.int32)
        fr = np.ascontiguousarray(pcm[t])
        assert L.stftModule_analyze(stft, O.p(fr), O.p(y)) == 0
        buf = np.concatenate([buf[160:], fr.astype(np.int32)])
        xin = np.zeros(512, np.int32)
        xin[:480] = (win * buf) >> 15
        np.testing.assert_array_equal(y[:514], O.rfft512_portable(xin))
        assert not y[514:].any()
    assert L.nnsp_legacy_status() == 0


def nets_window():
    from nnsp_amd import tables
    return tables.stft_window()


def test_feature_class_vs_reference(gfe):
    L = _lib.lib()
    for s in range(len(gfe["fe_pcm"])):
        mean = np.ascontiguousarray(gfe["fe_mean"][s], np.int32)
        stdR = np.ascontiguousarray(gfe["fe_stdR"][s], np.int32)
        _KEEP.extend([mean, stdR])
        fc = _lib.FeatureClass()
        L.FeatureClass_construct(C.byref(fc), O.p(mean), O.p(stdR), int(gfe["fe_qbit"][s]))
        L.FeatureClass_setDefault(C.byref(fc))
        for t, fr in enumerate(gfe["fe_pcm"][s]):
            fr = np.ascontiguousarray(fr, np.int16)
            L.FeatureClass_execute(C.byref(fc), O.p(fr))
            np.testing.assert_array_equal(np.ctypeslib.as_array(fc.normFeatContext)[200:240], gfe["fe_feats"][s, t],
                                          err_msg=f"stream {s} frame {t}")
    assert L.nnsp_legacy_status() == 0


@pytest.mark.parametrize("acc", [64, 32])
def test_fc_and_affine_krows_vs_reference(gnn, acc):
    L = _lib.lib()
    k = 0
    while f"fc{k}_cfg" in gnn:
        N, K, qk, qb, qi, act = (int(v) for v in gnn[f"fc{k}_cfg"])
        w, b, xs, ys = gnn[f"fc{k}_w"], gnn[f"fc{k}_b"], gnn[f"fc{k}_x"], gnn[f"fc{k}_y{acc}"]
        wp = np.ascontiguousarray(nets.pack_fc_portable(w))
        bp = np.ascontiguousarray(b, np.int16)
        _KEEP.extend([wp, bp])
        f = L.fc_8x16_acc32b if acc == 32 else L.fc_8x16
        fa = L.affine_Krows_8x16_acc32b if acc == 32 else L.affine_Krows_8x16
        for r in range(len(xs)):
            x = np.ascontiguousarray(xs[r], np.int16)
            y = np.zeros(N, np.int32 if act == 3 else np.int16)
            assert f(O.p(y), O.p(wp), None, O.p(bp), O.p(x), None, None, i16(N), i16(K), i16(N), i16(qk), i16(qb),
                     i16(qi), i16(0), C.c_int(act), C.c_void_p(_lib.fn_addr(ACTS[act]))) == 0
            np.testing.assert_array_equal(y.astype(np.int32), ys[r], err_msg=f"fc_8x16 case {k} row {r}")
            if r < 2:   # the row-block primitive, group by group (fc_8x16's loop, affine.c:409-490)
                y2 = np.zeros(N, y.dtype)
                po = C.c_void_p(y2.ctypes.data)
                pk = C.c_void_p(wp.ctypes.data)
                pb = C.c_void_p(bp.ctypes.data)
                for g0 in range(0, N, 4):
                    R = min(4, N - g0)
                    acc_buf = np.zeros(4, np.int32 if acc == 32 else np.int64)
                    assert fa(i16(R), C.byref(po), C.byref(pk), C.byref(pb), O.p(x), i16(K), i16(qk), i16(qb),
                              i16(qi), O.p(acc_buf), C.c_int8(1), C.c_void_p(_lib.fn_addr(ACTS[act]))) == 0
                np.testing.assert_array_equal(y2.astype(np.int32), ys[r], err_msg=f"affine_Krows case {k} row {r}")
        k += 1
    assert k >= 10
    assert L.nnsp_legacy_status() == 0


@pytest.mark.parametrize("acc", [64, 32])
def test_lstm_vs_reference(gnn, acc):
    L = _lib.lib()
    k = 0
    while f"lstm{k}_cfg" in gnn:
        N, K, qk, qb, qi, qir = (int(v) for v in gnn[f"lstm{k}_cfg"])
        wp = np.ascontiguousarray(nets.pack_lstm_portable(gnn[f"lstm{k}_w"]))
        wrp = np.ascontiguousarray(nets.pack_lstm_portable(gnn[f"lstm{k}_wr"]))
        bp = np.ascontiguousarray(nets.pack_lstm_bias(gnn[f"lstm{k}_b"]), np.int16)
        _KEEP.extend([wp, wrp, bp])
        h, c = np.zeros(N, np.int16), np.zeros(N, np.int32)
        f = L.lstm_8x16_acc32b if acc == 32 else L.lstm_8x16
        for r, x in enumerate(gnn[f"lstm{k}_x"]):
            x = np.ascontiguousarray(x, np.int16)
            y = np.zeros(N, np.int16)
            assert f(O.p(y), O.p(wp), O.p(wrp), O.p(bp), O.p(x), O.p(h), O.p(c), i16(N), i16(K), i16(N),
                     i16(qk), i16(qb), i16(qi), i16(qir), C.c_int(1), C.c_void_p(_lib.fn_addr("tanh_fix"))) == 0
            np.testing.assert_array_equal(y, gnn[f"lstm{k}_y{acc}"][r], err_msg=f"lstm {k} call {r}")
            np.testing.assert_array_equal(h, gnn[f"lstm{k}_h{acc}"][r])
            np.testing.assert_array_equal(c, gnn[f"lstm{k}_c{acc}"][r])
        k += 1
    assert k >= 6
    assert L.nnsp_legacy_status() == 0


def _net_data(g, name):
    if name in nets.ALL_GEN_SPECS:
        spec = nets.ALL_GEN_SPECS[name]
        W = [g[f"net_{name}_W{i}"] for i in range(spec.nl)]
        Wr = [g[f"net_{name}_Wr{i}"] if f"net_{name}_Wr{i}" in g else None for i in range(spec.nl)]
        B = [g[f"net_{name}_B{i}"] for i in range(spec.nl)]
        return nets.NetData(spec, W, Wr, B, np.zeros(40, np.int32), np.zeros(40, np.int32))
    return ref_net(name)


@pytest.mark.parametrize("acc", [64, 32])
@pytest.mark.parametrize("name", ["vad", "kws", "s2i"] + list(nets.ALL_GEN_SPECS))
def test_neural_net_exe_vs_reference(gnn, name, acc):
    L = _lib.lib()
    data = _net_data(gnn, name)
    sp = data.spec
    h = _lib.NetHandle(data, acc32=acc == 32, arm_optimized=False)
    _KEEP.append(h)
    L.NeuralNetClass_setDefault(C.c_void_p(h.addr))
    for r, x in enumerate(gnn[f"net_{name}_x"]):
        x = np.ascontiguousarray(x, np.int16)
        out = np.zeros(160, np.int32)
        L.NeuralNetClass_exe(C.c_void_p(h.addr), O.p(x), O.p(out), -1)
        got = out[:sp.nout] if sp.acts[-1] == nets.LINEAR else out.view(np.int16)[:sp.nout].astype(np.int32)
        np.testing.assert_array_equal(got, gnn[f"net_{name}_y{acc}"][r], err_msg=f"{name} call {r}")
    assert L.nnsp_legacy_status() == 0


@pytest.mark.parametrize("name", ["vad", "kws"])
def test_nnsp_exec_portable(name):
    data = ref_net(name)
    orc = OracleNet(data, portable=True, fe_portable=True)
    h = _lib.NetHandle(data, arm_optimized=False)
    _KEEP.append(h)
    feat, inst = _lib.FeatureClass(), _lib.NNSPClass()
    thr, cnt = np.array([16383], np.int16), np.array([4], np.int16)
    _KEEP.extend([thr, cnt])
    L = _lib.lib()
    assert L.NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([NN_ID[name]]),
                            O.p(h.mean), O.p(h.stdR), O.p(thr), O.p(cnt)) == 0
    L.NNSPClass_reset(C.byref(inst))
    T = 50
    pcm = synthetic_pcm(1, T, s0=4, t0=300, wavs=load_wavs(), every=4)
    o_trig, _, o_feat, _ = orc.run(pcm)
    for t in range(T):
        frame = np.ascontiguousarray(pcm[0, t])
        assert L.NNSPClass_exec(C.byref(inst), O.p(frame)) == o_trig[0, t], f"frame {t}"
        np.testing.assert_array_equal(np.ctypeslib.as_array(feat.normFeatContext)[200:240], o_feat[0, t])
    assert L.nnsp_legacy_status() == 0


@pytest.fixture(scope="module")
def gfc():
    return np.load(os.path.join(GOLD, "ref_fft_complex.npz"))


@pytest.mark.parametrize("num", [256, 512])
def test_rfft_sizes_vs_reference(gfc, num):
    """rfft(256) and rfft(512) on vectors up to the full int32 range, where
    complex.c's clamps and the split's int32 wraps bind (fft.c:27-126)."""
    L = _lib.lib()
    for x, y in zip(gfc[f"rfft{num}_in"], gfc[f"rfft{num}_out"]):
        xi = np.ascontiguousarray(x, np.int32)
        keep = xi.copy()
        out = np.zeros(num + 2, np.int32)
        L.rfft(num, O.p(xi), O.p(out))
        np.testing.assert_array_equal(out, y)
        np.testing.assert_array_equal(xi, keep)
    assert L.nnsp_legacy_status() == 0


@pytest.mark.parametrize("e", range(9))
def test_fft_every_size_vs_reference(gfc, e):
    """fft(exp_nfft) for 0..8: radix-4 stages (8, 7), the radix-2 stage (7),
    the bit-reversal copy alone (< 7); output and the in-place input."""
    L = _lib.lib()
    for x, y, xa in zip(gfc[f"fft{e}_in"], gfc[f"fft{e}_out"], gfc[f"fft{e}_in_after"]):
        xi = np.ascontiguousarray(x, np.int32).copy()
        out = np.zeros(2 << e, np.int32)
        L.fft(e, O.p(xi), O.p(out))
        np.testing.assert_array_equal(out, y, err_msg=f"fft({e}) output")
        np.testing.assert_array_equal(xi, xa, err_msg=f"fft({e}) input afterwards")
    assert L.nnsp_legacy_status() == 0


def test_fft_rfft_unsupported_sizes_report():
    L = _lib.lib()
    x = np.zeros(2048, np.int32)
    y = np.zeros(2048, np.int32)
    L.rfft(1024, O.p(x), O.p(y))
    assert L.nnsp_legacy_status() == -2   # NNSP_EUNSUPPORTED
    L.nnsp_legacy_clear()
    L.fft(9, O.p(x), O.p(y))
    assert L.nnsp_legacy_status() == -2
    L.nnsp_legacy_clear()


def test_complex_helpers_vs_reference(gfc):
    """complex.c's helpers (the drop-in complex.h), full-range operands."""
    L = _lib.lib()
    a, b, m, w, sh = gfc["cx_a"], gfc["cx_b"], gfc["cx_m"], gfc["cx_w16"], gfc["cx_shift"]
    n = a.shape[1]
    for c in range(len(a)):
        A, B, M, W = (np.ascontiguousarray(v[c]) for v in (a, b, m, w))

        def o():
            return np.zeros((n, 2), np.int32)
        r = o(); L.complex32_copy(O.p(r), O.p(A)); np.testing.assert_array_equal(r[0], gfc["cx_copy"][c])
        r = o(); L.complex32_affine(O.p(r), O.p(M), O.p(A), int(sh[c]), n)
        np.testing.assert_array_equal(r, gfc["cx_affine"][c])
        r = A.copy(); L.complex32_affine(O.p(r), O.p(M), O.p(r), int(sh[c]), n)   # out aliases input
        np.testing.assert_array_equal(r, gfc["cx_affine_alias"][c])
        r = o(); L.complex32_interprod(O.p(r), O.p(A), O.p(B), int(sh[c]), n)
        np.testing.assert_array_equal(r[0], gfc["cx_interprod"][c])
        r = o(); L.complex32_complex16_elmtprod(O.p(r), O.p(A), O.p(W), n)
        np.testing.assert_array_equal(r, gfc["cx_elmtprod"][c])
        r = o(); L.complex32_add(O.p(r), O.p(A), O.p(B)); np.testing.assert_array_equal(r[0], gfc["cx_add"][c])
        r = o(); L.complexArry32_add(O.p(r), O.p(A), O.p(B), n); np.testing.assert_array_equal(r, gfc["cx_arry_add"][c])
        r = o(); L.complex32_neg(O.p(r), O.p(A)); np.testing.assert_array_equal(r[0], gfc["cx_neg"][c])
        Bc = B.copy()
        r = o(); L.complex32_sub(O.p(r), O.p(A), O.p(Bc)); np.testing.assert_array_equal(r[0], gfc["cx_sub"][c])
        np.testing.assert_array_equal(Bc[0], gfc["cx_sub_b"][c])   # b negated in place (complex.c:108-113)
        r = o(); L.complex32_mul(O.p(r), O.p(A), O.p(B)); np.testing.assert_array_equal(r[0], gfc["cx_mul"][c])
        r = o(); L.complex32_init(O.p(r), C.c_int32(int(A[0, 0])), C.c_int32(int(A[0, 1])))
        np.testing.assert_array_equal(r[0], gfc["cx_init"][c])
        r = o(); L.complex32_real2cmplx(O.p(r), C.c_int32(int(B[0, 0])))
        np.testing.assert_array_equal(r[0], gfc["cx_real2cmplx"][c])
        re_, im_ = np.ascontiguousarray(A[:, 0]), np.ascontiguousarray(B[:, 1])
        r = o(); L.complexArry32_real2cmplx(O.p(r), O.p(re_), n)
        np.testing.assert_array_equal(r, gfc["cx_arry_real2cmplx"][c])
        r = o(); L.complexArry32_init(O.p(r), O.p(re_), O.p(im_), n)
        np.testing.assert_array_equal(r, gfc["cx_arry_init"][c])
    assert L.nnsp_legacy_status() == 0
