"""GPU parity on the reference's OWN three nets (evb/src/def_nn1_vad.c,
def_nn2_kws_galaxy.c, def_nn0_s2i.c tables, tests/golden/ref_nets.npz) and on
the N3 net shapes, against the CPU oracle (bit-exact).

Inputs are the bench's mix: SplitMix64 noise plus streams that
replay the reference's python/test_wavs recordings, which make the nets
trigger and the cascade switch.  Per stream and frame: features, the logits
of EVERY frame (0 where the NN does not run), triggers; the cascade's net,
detection and outputs[3].  Also the drop-in entry points on those nets
(NNSPClass_exec per frame, fc_8x16 / lstm_8x16 called directly), the image
cache against tables rewritten in place, and the state export / import.
"""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from oracle import OracleCascade, OracleNet, load_wavs, synthetic_pcm

from nnsp_amd import _lib
from nnsp_amd.engine import NNSPBatch, NNSPCascade
from nnsp_amd.nets import GEN_SPECS, LSTM, NN_ID, get_net, ref_net, synth_net

pytestmark = pytest.mark.gpu

WAVS = load_wavs()
_KEEP = []


def _pcm(S, T, t0=0, every=2, seed=0x4E4E5350):
    return synthetic_pcm(S, T, seed=seed, t0=t0, wavs=WAVS, every=every)


def _batch_compare(data, acc32, S, chunks, pcm):
    orc = OracleNet(data, acc32=acc32)
    eng = NNSPBatch(data, S, max(chunks), acc32=acc32)
    o_trig, o_lg, o_ft, _ = orc.run(pcm)
    t0 = 0
    for Tc in chunks:
        trig, lg, ft = eng.exec(pcm[:, t0:t0 + Tc], want_logits=True, want_features=True)
        np.testing.assert_array_equal(ft, o_ft[:, t0:t0 + Tc], err_msg=f"features chunk@{t0}")
        np.testing.assert_array_equal(lg, o_lg[:, t0:t0 + Tc], err_msg=f"logits (every frame) chunk@{t0}")
        np.testing.assert_array_equal(trig, o_trig[:, t0:t0 + Tc], err_msg=f"trig chunk@{t0}")
        t0 += Tc
    eng.close()
    return o_trig


@pytest.mark.parametrize("acc32", [False, True])
@pytest.mark.parametrize("name", ["vad", "kws", "s2i"])
def test_batch_reference_nets(name, acc32):
    S, chunks = 48, [40, 23, 1, 36, 100]
    pcm = _pcm(S, sum(chunks))
    trig = _batch_compare(ref_net(name), acc32, S, chunks, pcm)
    if name == "vad":
        assert (trig != 0).any(), "VAD never triggered on the recordings: vacuous"


def test_cascade_vad_fused_prefix(monkeypatch):
    """The fused prefix stage (opt-in NNSP_FUSE_PREFIX=2; measured slower than
    the default): in the cascade's one-tile VAD recurrences, VAD's
    FC 240 -> 28 and the LSTM's input projection run inside the recurrence on
    its FC waves, one step ahead, instead of in proj_kernel.  Bit-exact against
    the oracle like the default path."""
    monkeypatch.setenv("NNSP_FUSE_PREFIX", "2")   # read by nnsp_batch_create; 2: refuse rather than fall back
    S, chunks = 64, [100, 100, 57]
    gnets = {n: NNSPBatch(ref_net(n), S, 100) for n in ("vad", "kws", "s2i")}
    gc = NNSPCascade(gnets)
    oc = OracleCascade({n: OracleNet(ref_net(n)) for n in ("vad", "kws", "s2i")})
    st = oc.new_states(S)
    pcm = _pcm(S, sum(chunks), every=1)
    t0 = 0
    for Tc in chunks:
        o_ran, o_det, o_o3, st = oc.run(pcm[:, t0:t0 + Tc], st)
        g_ran, g_det, g_o3 = gc.exec(pcm[:, t0:t0 + Tc])
        np.testing.assert_array_equal(g_ran, o_ran, err_msg=f"net_ran chunk@{t0}")
        np.testing.assert_array_equal(g_det, o_det, err_msg=f"detected chunk@{t0}")
        np.testing.assert_array_equal(g_o3, o_o3, err_msg=f"outputs3 chunk@{t0}")
        t0 += Tc
    gc.close()


@pytest.mark.parametrize("name", list(GEN_SPECS))
def test_batch_n3_shapes(name):
    """Rows not a multiple of 4, odd K, 3 / 7 layers, two LSTMs, a 256-wide FC
    (affine.c:103-184, neural_nets.c:44-168) through the batched engine (split
    generic kernels for one-LSTM nets whose tail fits, the fused kernel else)."""
    S, chunks = 40, [30, 7, 1, 22]
    data = synth_net(name, 5)
    for acc32 in (False, True):
        _batch_compare(data, acc32, S, chunks, _pcm(S, sum(chunks), every=3))


@pytest.mark.parametrize("acc32", [False, True])
@pytest.mark.parametrize("window", [16, 0, 5])
def test_cascade_reference_nets_defaults(acc32, window):
    """nnCntrlClass with the reference's parameters (ParamsNNCntrl.h:8-21:
    thresholds 16383 / 4, look-back 80, timeouts 1000) on its own nets."""
    S, chunks = 64, [100, 100, 57, 100, 43]
    gnets = {n: NNSPBatch(ref_net(n), S, 100, acc32=acc32) for n in ("vad", "kws", "s2i")}
    gc = NNSPCascade(gnets)
    gc.set_window(window)
    oc = OracleCascade({n: OracleNet(ref_net(n), acc32=acc32) for n in ("vad", "kws", "s2i")})
    st = oc.new_states(S)
    pcm = _pcm(S, sum(chunks), every=1)
    t0, switches = 0, 0
    for Tc in chunks:
        o_ran, o_det, o_o3, st = oc.run(pcm[:, t0:t0 + Tc], st)
        g_ran, g_det, g_o3 = gc.exec(pcm[:, t0:t0 + Tc])
        np.testing.assert_array_equal(g_ran, o_ran, err_msg=f"net_ran chunk@{t0}")
        np.testing.assert_array_equal(g_det, o_det, err_msg=f"detected chunk@{t0}")
        np.testing.assert_array_equal(g_o3, o_o3, err_msg=f"outputs3 chunk@{t0}")
        switches += int((np.diff(o_ran.astype(np.int32), axis=1) != 0).sum())
        t0 += Tc
    assert switches > 5, "the cascade hardly switched: vacuous"
    gc.close()


@pytest.mark.parametrize("name", ["vad", "kws", "s2i"])
def test_legacy_nnsp_exec_reference_nets(name):
    """NNSPClass_exec frame by frame (nn_speech.c:74-127) on the reference net
    and a recording: trigger, context slot 5 and outputs[3] per frame."""
    data = ref_net(name)
    orc = OracleNet(data)
    h = _lib.NetHandle(data)
    _KEEP.append(h)
    feat, inst = _lib.FeatureClass(), _lib.NNSPClass()
    thr, cnt = np.array([16383], np.int16), np.array([4], np.int16)
    _KEEP.extend([thr, cnt])
    L = _lib.lib()
    assert L.NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([NN_ID[name]]),
                            O.p(h.mean), O.p(h.stdR), O.p(thr), O.p(cnt)) == 0
    L.NNSPClass_reset(C.byref(inst))
    T = 60
    pcm = synthetic_pcm(1, T, s0=4, t0=300, wavs=WAVS, every=4)   # galaxy.wav
    o_trig, _, o_feat, _ = orc.run(pcm)
    for t in range(T):
        frame = np.ascontiguousarray(pcm[0, t])
        assert L.NNSPClass_exec(C.byref(inst), O.p(frame)) == o_trig[0, t], f"frame {t}"
        np.testing.assert_array_equal(np.ctypeslib.as_array(feat.normFeatContext)[200:240], o_feat[0, t])
    assert L.nnsp_legacy_status() == 0


@pytest.mark.parametrize("acc32", [False, True])
def test_legacy_layer_functions_direct(acc32):
    """fc_8x16 / lstm_8x16 (and _acc32b), the functions def_nn*.c store in
    layer_func[] (affine.c:409-490, lstm.c:15-214), called directly on the
    reference nets' layers and on odd shapes."""
    L = _lib.lib()
    rng = np.random.default_rng(17 + acc32)
    acts = {0: "relu6_fix", 1: "tanh_fix", 2: "sigmoid_fix", 3: "linear_fix"}
    cases = []
    for name in ("vad", "kws", "s2i"):
        d = ref_net(name)
        Wp, Wrp, Bp = d.packed()
        for i in range(d.spec.nl):
            cases.append((d.spec.types[i], d.W[i], d.Wr[i], d.B[i], Wp[i], Wrp[i], Bp[i], d.spec.qk[i],
                          d.spec.qb[i], d.spec.qi[i], d.spec.qi[i + 1] if i + 1 < d.spec.nl else 0, d.spec.acts[i]))
    g = synth_net("odd", 9)
    Wp, Wrp, Bp = g.packed()
    for i in range(g.spec.nl):
        cases.append((g.spec.types[i], g.W[i], g.Wr[i], g.B[i], Wp[i], Wrp[i], Bp[i], g.spec.qk[i], g.spec.qb[i],
                      g.spec.qi[i], g.spec.qi[i + 1] if i + 1 < g.spec.nl else 0, g.spec.acts[i]))
    i16 = C.c_int16
    for typ, W, Wr, B, wp, wrp, bp, qk, qb, qi, qir, act in cases:
        wp = np.ascontiguousarray(wp)
        bp = np.ascontiguousarray(bp, np.int16)
        _KEEP.extend([wp, bp])
        if typ == LSTM:
            N, K = W.shape[0] // 4, W.shape[1]
            wrp = np.ascontiguousarray(wrp)
            _KEEP.append(wrp)
            h, c = np.zeros(N, np.int16), np.zeros(N, np.int32)
            oh, oc = h.copy(), c.copy()
            f = L.lstm_8x16_acc32b if acc32 else L.lstm_8x16
            for _ in range(3):   # h / c carried across calls
                x = rng.integers(-32768, 32768, K).astype(np.int16)
                y = np.zeros(N, np.int16)
                assert f(O.p(y), O.p(wp), O.p(wrp), O.p(bp), O.p(x), O.p(h), O.p(c), i16(N), i16(K), i16(N),
                         i16(qk), i16(qb), i16(qi), i16(qir), C.c_int(1), C.c_void_p(_lib.fn_addr("tanh_fix"))) == 0
                oy = O.lstm(W, Wr, B, x, oh, oc, qk, qb, qi, qir, acc32)
                np.testing.assert_array_equal(y, oy)
                np.testing.assert_array_equal(h, oh)
                np.testing.assert_array_equal(c, oc)
        else:
            N, K = W.shape
            x = rng.integers(-32768, 32768, K).astype(np.int16)
            y = np.zeros(N, np.int32 if act == 3 else np.int16)
            f = L.fc_8x16_acc32b if acc32 else L.fc_8x16
            assert f(O.p(y), O.p(wp), None, O.p(bp), O.p(x), None, None, i16(N), i16(K), i16(N), i16(qk), i16(qb),
                     i16(qi), i16(0), C.c_int(act), C.c_void_p(_lib.fn_addr(acts[act]))) == 0
            np.testing.assert_array_equal(y.astype(np.int32), O.fc(W, B, x, qk, qb, qi, act, acc32))


def test_legacy_tables_rewritten_in_place():
    """the device image follows the tables' bytes -- the same
    NeuralNetClass and buffers, rewritten in place with another net's weights,
    must give that net's outputs."""
    a, b = synth_net("vad", 31), synth_net("vad", 32)
    h = _lib.NetHandle(a)
    _KEEP.append(h)
    L = _lib.lib()
    rng = np.random.default_rng(1)
    x = rng.integers(-4000, 4000, 240).astype(np.int16)
    for data in (a, b, a):
        Wp, Wrp, Bp = data.packed()
        for i in range(data.spec.nl):   # overwrite the handle's buffers in place
            np.copyto(np.ctypeslib.as_array((C.c_int8 * len(Wp[i])).from_address(h.net.pt_kernel[i])),
                      Wp[i].view(np.int8))
            np.copyto(np.ctypeslib.as_array((C.c_int16 * len(Bp[i])).from_address(h.net.pt_bias[i])), Bp[i])
            if Wrp[i] is not None:
                np.copyto(np.ctypeslib.as_array((C.c_int8 * len(Wrp[i])).from_address(h.net.pt_kernel_rec[i])),
                          Wrp[i].view(np.int8))
        L.NeuralNetClass_setDefault(C.c_void_p(h.addr))
        out = np.zeros(64, np.int32)
        L.NeuralNetClass_exe(C.c_void_p(h.addr), O.p(x), O.p(out), -1)
        orc = OracleNet(data)
        st = orc.new_states(1)[0]
        np.testing.assert_array_equal(out[:2], orc.forward(x, st)[:2])


def test_state_export_import_across_chunks():
    """nnsp_batch_get_state / set_state (checkpoint / resume): a second batch
    resumed from the first one's state after chunk 1 gives the same outputs on
    chunk 2, equal to the oracle's."""
    data = ref_net("kws")
    S, T = 24, 40
    pcm = _pcm(S, 2 * T)
    a = NNSPBatch(data, S, T)
    a.exec(pcm[:, :T])
    blob = a.get_state()
    b = NNSPBatch(data, S, T)
    b.set_state(blob)
    np.testing.assert_array_equal(b.get_state(), blob)
    ta, la, _ = a.exec(pcm[:, T:], want_logits=True)
    tb, lb, _ = b.exec(pcm[:, T:], want_logits=True)
    np.testing.assert_array_equal(ta, tb)
    np.testing.assert_array_equal(la, lb)
    o_trig, o_lg, _, _ = OracleNet(data).run(pcm)
    np.testing.assert_array_equal(tb, o_trig[:, T:])
    np.testing.assert_array_equal(lb, o_lg[:, T:])
    ps = b.post_state()
    assert ps.shape == (S, 16)
    a.close()
    b.close()


def test_cascade_rejects_nets_out_of_nnsp_id_order():
    """nets[] is indexed by NNSP_ID (0 s2i, 1 vad, 2 kws)."""
    S = 16
    nets = {n: NNSPBatch(get_net(n, "ref"), S, 8) for n in ("vad", "kws", "s2i")}
    arr = (C.c_void_p * 3)(*[nets[n].h.value for n in ("vad", "kws", "s2i")])   # pipeline order: wrong
    h = C.c_void_p()
    prm = _lib.CascadeParams(80, 1000, 80, 1000)
    sq = np.array([1, 2, 0], np.int8)
    rc = _lib.lib().nnsp_cascade_create(C.byref(h), C.addressof(arr), O.p(sq), 3, C.addressof(prm))
    assert rc != 0 and not h.value


def _spec_like(name, sizes, types, acts, nid=1):
    """A synthetic NetSpec of the given shape (qbits of the VAD net's layers)."""
    from nnsp_amd.nets import NetSpec
    n = len(types)
    return NetSpec(name, sizes, types, [6] * n, [8] + [15] * (n - 1), [14] * n, acts,
                   [(4, 4, 300, 6000)] * n, nid=nid)


def test_n3_beyond_the_reference_limits_is_refused():
    """What the reference cannot run is refused with NNSP_EUNSUPPORTED and a
    message, never truncated: a layer wider than neural_nets.c's 300-element
    buffers (:9-10), a linear layer past 150 int32, and -- for NNSPClass_exec,
    whose static int32_t output[50] holds 50 int32 (nn_speech.c:78) -- a
    51-wide linear output."""
    from nnsp_amd.nets import FC, LINEAR, RELU6, TANH
    cases = [("w301", [240, 301, 2], [FC, FC], [TANH, LINEAR]),
             ("lin151", [240, 151, 2], [FC, FC], [LINEAR, LINEAR]),
             ("out51", [240, 64, 51], [FC, FC], [TANH, LINEAR])]
    for name, sizes, types, acts in cases:
        data = synth_net(_spec_like(name, sizes, types, acts), 3)
        with pytest.raises(RuntimeError, match="nnsp_batch_create") as ei:
            NNSPBatch(data, 16, 8)
        assert "EUNSUPPORTED" in str(ei.value) or "outside" in str(ei.value) or "exceeds" in str(ei.value), ei.value
    # the widest the reference allows is accepted: 300 int16 / 100 int16 output
    ok = synth_net(_spec_like("ok300", [240, 300, 100], [FC, FC], [TANH, RELU6]), 3)
    NNSPBatch(ok, 16, 8).close()


def test_cascade_refuses_nets_without_one_lstm():
    """The batched cascade runs nets of the split path (exactly one LSTM, the
    shape of def_nn*.c); a three-LSTM net is refused with a message (the
    single-net engine runs it, test_batch_n3_shapes)."""
    S = 16
    gnets = {"vad": NNSPBatch(synth_net("lstm3", 3), S, 16), "kws": NNSPBatch(ref_net("kws"), S, 16),
             "s2i": NNSPBatch(ref_net("s2i"), S, 16)}
    with pytest.raises(RuntimeError, match="nnsp_cascade_create") as ei:
        NNSPCascade(gnets)
    assert "one LSTM" in str(ei.value), ei.value
