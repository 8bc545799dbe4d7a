"""GPU parity of the single-stream drop-in API (include/nnsp_api.h, the
reference's ns-nnsp C API) against the CPU oracle, bit for bit.

Every legacy entry point runs the gfx950 kernels on a batch of one
(nnsp_amd/csrc/host/nnsp_legacy.c): the front-end stages (arm_fft_exec,
spec2pspec_arm, melSpecProc, log10_vec), the activations, the row-block
primitives (affine_Krows_8x16*, rc_Krows_8x16*, rc_8x16*, shift_64b/32b),
NeuralNetClass_exe, FeatureClass_execute and NNSPClass_exec per frame.
"""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from oracle import OracleNet, synthetic_pcm

from nnsp_amd import _lib
from nnsp_amd.nets import GEN_SPECS, LSTM, synth_net

pytestmark = pytest.mark.gpu

ACT_FN = {0: "relu6_fix", 1: "tanh_fix", 2: "sigmoid_fix", 3: "linear_fix"}
_KEEP = []   # nets stay alive for the session: their tables' addresses are never reused


def L():
    return _lib.lib()


def vp(a):
    return C.c_void_p(a.ctypes.data)


def fn(name):
    return C.c_void_p(_lib.fn_addr(name))


def test_front_end_stages():
    rng = np.random.default_rng(1)
    L().arm_fft_init()
    for amp in (1 << 12, 1 << 20, 1 << 29):
        x = np.zeros(514, np.int32)
        x[:480] = rng.integers(-amp, amp, 480)
        oy, ox = O.rfft512(x[:512])
        y = np.zeros(1024, np.int32)
        L().arm_fft_exec(vp(y), vp(x))
        np.testing.assert_array_equal(y, oy)
        np.testing.assert_array_equal(x[:512], ox)   # pSrc is transformed in place (CMSIS)
        p = np.zeros(1024, np.int32)
        L().spec2pspec_arm(vp(p), vp(y), 257)
        np.testing.assert_array_equal(p[:257], O.spec2pspec(y))
        m = np.zeros(40, np.int32)
        L().melSpecProc(vp(p), vp(m))
        np.testing.assert_array_equal(m, O.mel(p[:257]))
        lg = np.zeros(40, np.int32)
        L().log10_vec(vp(lg), vp(m), 40, 15)
        np.testing.assert_array_equal(lg, O.log10(m))


def test_spec2pspec_arm_any_length():
    """spec2pspec_arm over vectors longer than one frame's 257 bins (the
    reference loops over len; the device buffer is sized per call)."""
    rng = np.random.default_rng(3)
    for n in (1, 1024, 1025, 5000):
        spec = rng.integers(-2 ** 31 + 1, 2 ** 31, 2 * n).astype(np.int32)   # (no int64 overflow)
        got = np.zeros(n, np.int32)
        L().spec2pspec_arm(vp(got), vp(spec), n)
        ref = ((spec[0::2].astype(np.int64) ** 2 + spec[1::2].astype(np.int64) ** 2) >> 27)
        np.testing.assert_array_equal(got, ref.astype(np.uint64).astype(np.uint32).view(np.int32))


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
def test_activations(kind):
    x = np.concatenate([np.arange(-200000, 200000, 97), [0, 1, -1, 2 ** 31 - 1, -2 ** 31 + 1]]).astype(np.int32)
    y = np.zeros(len(x), np.int32 if kind == 3 else np.int16)
    getattr(L(), ACT_FN[kind])(vp(y), vp(x), len(x))
    np.testing.assert_array_equal(y, O.act(kind, x))


QBITS = [(7, 14, 8), (5, 13, 15), (6, 13, 8), (4, 14, 12), (7, 15, 12)]


@pytest.mark.parametrize("acc32", [False, True])
@pytest.mark.parametrize("R", [1, 2, 3, 4])
def test_affine_krows(R, acc32):
    rng = np.random.default_rng(R + 10 * acc32)
    f = L().affine_Krows_8x16_acc32b if acc32 else L().affine_Krows_8x16
    for K in (240, 27, 2):
        for qk, qb, qi in QBITS:
            for act in (0, 1, 2, 3):
                for bias in (True, False):
                    for is_out in (1, 0):
                        w = rng.integers(-128, 128, R * K).astype(np.int8)
                        b = rng.integers(-9000, 9000, R).astype(np.int16)
                        x = rng.integers(-32768, 32768, K).astype(np.int16)
                        acc = rng.integers(-2 ** 22, 2 ** 22, 4).astype(np.int64)
                        oacc = acc.copy()
                        oout = np.zeros(R, np.int32 if act == 3 else np.int16)
                        O.lib().or_affine_krows(R, vp(w), vp(b) if bias else None, vp(x), K, qk, qb, qi, vp(oacc),
                                                int(acc32), is_out, act, vp(oout))
                        gacc = acc.astype(np.int32) if acc32 else acc.copy()
                        gout = np.zeros(R, oout.dtype)
                        po, pw = C.c_void_p(gout.ctypes.data), C.c_void_p(w.ctypes.data)
                        pb = C.c_void_p(b.ctypes.data if bias else None)
                        assert f(R, C.byref(po), C.byref(pw), C.byref(pb), vp(x), K, qk, qb, qi, vp(gacc),
                                 is_out, fn(ACT_FN[act])) == 0
                        np.testing.assert_array_equal(gacc[:R].astype(np.int64), oacc[:R])
                        if is_out:
                            np.testing.assert_array_equal(gout, oout)
                        assert pw.value == w.ctypes.data + R * K
                        assert (pb.value or 0) == (b.ctypes.data + 2 * R if bias else 0)
                        assert po.value == gout.ctypes.data + (gout.nbytes if is_out else 0)


@pytest.mark.parametrize("acc32", [False, True])
@pytest.mark.parametrize("N", [4, 7, 28, 41, 72])
def test_rc_layer_and_krows(N, acc32):
    rng = np.random.default_rng(N + 100 * acc32)
    for K, Kr in ((28, 28), (240, 72), (9, 5)):
        for qk, qb, qi in QBITS:
            qir = 15
            for act in (1, 2, 3):
                w = rng.integers(-128, 128, N * K).astype(np.int8)
                wr = rng.integers(-128, 128, N * Kr).astype(np.int8)
                b = rng.integers(-9000, 9000, N).astype(np.int16)
                x = rng.integers(-32768, 32768, K).astype(np.int16)
                h = rng.integers(-32768, 32768, Kr).astype(np.int16)
                dt = np.int32 if act == 3 else np.int16
                oout = np.zeros(N, dt)
                O.lib().or_rc_layer(N, vp(w), vp(wr), vp(b), vp(x), vp(h), K, Kr, qk, qb, qi, qir, act, int(acc32),
                                    vp(oout))
                gout = np.zeros(N, dt)
                f = L().rc_8x16_acc32b if acc32 else L().rc_8x16
                assert f(vp(gout), vp(w), vp(wr), vp(b), vp(x), vp(h), N, K, Kr, qk, qb, qi, qir, act,
                         fn(ACT_FN[act])) == 0
                np.testing.assert_array_equal(gout, oout)
                # the same layer through rc_Krows_8x16 one 4-row group at a time
                g2 = np.zeros(N, dt)
                po, pw, pwr, pb = (C.c_void_p(a.ctypes.data) for a in (g2, w, wr, b))
                fk = L().rc_Krows_8x16_acc32b if acc32 else L().rc_Krows_8x16
                for r0 in range(0, N, 4):
                    assert fk(min(4, N - r0), C.byref(po), C.byref(pw), C.byref(pwr), C.byref(pb), vp(x), vp(h), K,
                              Kr, qk, qb, qi, qir, fn(ACT_FN[act])) == 0
                np.testing.assert_array_equal(g2, oout)
                assert pw.value == w.ctypes.data + N * K and pwr.value == wr.ctypes.data + N * Kr
                assert pb.value == b.ctypes.data + 2 * N and po.value == g2.ctypes.data + g2.nbytes


@pytest.mark.parametrize("acc32", [False, True])
def test_shift(acc32):
    rng = np.random.default_rng(5)
    for sh in (-31, -7, -1, 0, 1, 5, 20):
        v = rng.integers(-2 ** 62, 2 ** 62, 300, dtype=np.int64)
        if acc32:
            v = rng.integers(-2 ** 31, 2 ** 31, 300).astype(np.int64)
            if sh < -30:
                continue
        o = v.copy()
        O.lib().or_shift(vp(o), sh, len(o), int(acc32))
        if acc32:
            g = v.astype(np.int32)
            L().shift_32b(vp(g), sh, len(g))
        else:
            g = v.copy()
            L().shift_64b(vp(g), sh, len(g))
        np.testing.assert_array_equal(g.astype(np.int64), o)


@pytest.mark.parametrize("name", ["vad", "kws", "s2i"])
def test_neural_net_exe(name):
    data = synth_net(name, 21)
    orc = OracleNet(data)
    h = _lib.NetHandle(data)
    _KEEP.append(h)
    L().NeuralNetClass_setDefault(C.c_void_p(h.addr))
    st = orc.new_states(1)[0]
    rng = np.random.default_rng(3)
    for _ in range(4):   # the LSTM state carries across calls
        x = rng.integers(-20000, 20000, 240).astype(np.int16)
        out = np.zeros(64, np.int32)
        L().NeuralNetClass_exe(C.c_void_p(h.addr), vp(x), vp(out), -1)
        o = orc.forward(x, st)
        np.testing.assert_array_equal(out[:orc.nout], o[:orc.nout])


@pytest.mark.parametrize("name", ["vad", "s2i"])
def test_nnsp_exec_per_frame(name):
    data = synth_net(name, 8)
    orc = OracleNet(data, thresh_prob=3000, th_count=1)
    h = _lib.NetHandle(data)
    _KEEP.append(h)
    feat = _lib.FeatureClass()
    inst = _lib.NNSPClass()
    thr = np.array([3000], np.int16)
    cnt = np.array([1], np.int16)
    nn_id = {"s2i": 0, "vad": 1, "kws": 2}[name]
    assert L().NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([nn_id]), vp(h.mean),
                              vp(h.stdR), vp(thr), vp(cnt)) == 0
    L().NNSPClass_reset(C.byref(inst))
    T = 14
    pcm = synthetic_pcm(1, T, seed=77)
    o_trig, _, o_feat, _ = orc.run(pcm)
    for t in range(T):
        frame = np.ascontiguousarray(pcm[0, t])
        trig = L().NNSPClass_exec(C.byref(inst), vp(frame))
        assert trig == o_trig[0, t], f"frame {t}"
        ctx5 = np.ctypeslib.as_array(feat.normFeatContext)[200:240]
        np.testing.assert_array_equal(ctx5, o_feat[0, t], err_msg=f"features frame {t}")


def test_nnsp_exec_interleaved_nets():
    """NNSPClass_exec on VAD, KWS and S2I instances in turn, frame by frame
    (ADVICE r5): the three nets' staging layouts differ in size, and the
    drop-in completion word must not be satisfied by another net's bytes left
    from the call before.  Every call is compared with that net's oracle.
    (With the resident workers, the default: three of them live at once.)"""
    _interleaved(0.0)


def _interleaved(pause):
    """test_nnsp_exec_interleaved_nets, pause seconds before every call"""
    import time
    nets = []
    for k, name in enumerate(("s2i", "vad", "kws")):
        data = synth_net(name, 30 + k)
        orc = OracleNet(data, thresh_prob=3000, th_count=1)
        h = _lib.NetHandle(data)
        feat = _lib.FeatureClass()
        inst = _lib.NNSPClass()
        thr = np.array([3000], np.int16)
        cnt = np.array([1], np.int16)
        _KEEP.extend([h, feat, inst, thr, cnt])
        assert L().NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([k]), vp(h.mean),
                                  vp(h.stdR), vp(thr), vp(cnt)) == 0
        L().NNSPClass_reset(C.byref(inst))
        nets.append((name, orc, inst, feat))
    T = 12
    pcm = synthetic_pcm(3, T, seed=91)
    ref = [orc.run(pcm[k:k + 1]) for k, (_, orc, _, _) in enumerate(nets)]
    for t in range(T):
        for k in (2, 0, 1) if t % 2 else (1, 2, 0):   # large and small staging layouts alternate
            name, _, inst, feat = nets[k]
            frame = np.ascontiguousarray(pcm[k, t])
            if pause:
                time.sleep(pause)
            trig = L().NNSPClass_exec(C.byref(inst), vp(frame))
            assert trig == ref[k][0][0, t], f"{name} frame {t}"
            ctx5 = np.ctypeslib.as_array(feat.normFeatContext)[200:240]
            np.testing.assert_array_equal(ctx5, ref[k][2][0, t], err_msg=f"{name} features frame {t}")


def test_nnsp_exec_tables_rewritten_in_place():
    """NNSPClass_exec on tables rewritten in place mid-stream (the reference
    reads them on every call): the library compares their bytes with the
    device image's while the call runs, and runs again a call that ran on the
    old ones.  Frames 0-7 on net a, then a's buffers rewritten with net b's
    weights and frames 8-15 continue the stream: every frame, h and c equal the
    oracle's a then b from the same carried state.  (Not after a reset: the
    reference's FeatureClass_setDefault keeps the last context slot, so a
    reset stream is not a fresh oracle stream.)"""
    from nnsp_amd.nets import NetData
    a, b0 = synth_net("kws", 51), synth_net("kws", 52)
    b = NetData(b0.spec, b0.W, b0.Wr, b0.B, a.mean, a.stdR)   # (the feature normalisation unchanged)
    h = _lib.NetHandle(a)
    feat = _lib.FeatureClass()
    inst = _lib.NNSPClass()
    thr = np.array([3000], np.int16)
    cnt = np.array([1], np.int16)
    _KEEP.extend([h, feat, inst, thr, cnt])
    assert L().NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([1]), vp(h.mean), vp(h.stdR),
                              vp(thr), vp(cnt)) == 0
    L().NNSPClass_reset(C.byref(inst))
    T = 16
    pcm = synthetic_pcm(1, T, seed=57)
    orcs = [OracleNet(d, thresh_prob=3000, th_count=1) for d in (a, b)]
    st = orcs[0].new_states(1)
    N = a.spec.sizes[2]   # (layer 1: the LSTM)
    for t in range(T):
        if t == T // 2:   # overwrite the net's buffers in place
            Wp, Wrp, Bp = b.packed()
            for i in range(b.spec.nl):
                np.copyto(np.ctypeslib.as_array((C.c_int8 * len(Wp[i])).from_address(h.net.pt_kernel[i])),
                          Wp[i].view(np.int8))
                np.copyto(np.ctypeslib.as_array((C.c_int16 * len(Bp[i])).from_address(h.net.pt_bias[i])), Bp[i])
                if Wrp[i] is not None:
                    np.copyto(np.ctypeslib.as_array((C.c_int8 * len(Wrp[i])).from_address(h.net.pt_kernel_rec[i])),
                              Wrp[i].view(np.int8))
        o_trig, _, o_feat, st = orcs[t >= T // 2].run(pcm[:, t:t + 1], st)
        frame = np.ascontiguousarray(pcm[0, t])
        assert L().NNSPClass_exec(C.byref(inst), vp(frame)) == o_trig[0, 0], f"frame {t}"
        np.testing.assert_array_equal(np.ctypeslib.as_array(feat.normFeatContext)[200:240], o_feat[0, 0])
        oh, oc = _oracle_hc(st[0])
        np.testing.assert_array_equal(h.h[1], oh[0, :N], err_msg=f"LSTM h, frame {t}")
        np.testing.assert_array_equal(h.c[1], oc[0, :N], err_msg=f"LSTM c, frame {t}")
    assert L().nnsp_legacy_status() == 0


def _oracle_hc(row):
    """Every LSTM's h / c in the oracle's stream state (or_stream,
    oracle/nnsp_oracle.h: buf[480], ctx[240] int16, then h[10][304] int16 and
    c[10][304] int32, indexed by LSTM count)"""
    h = np.frombuffer(row.tobytes(), np.int16, count=10 * 304, offset=1440).reshape(10, 304)
    c = np.frombuffer(row.tobytes(), np.int32, count=10 * 304, offset=1440 + 6080).reshape(10, 304)
    return h, c


@pytest.mark.parametrize("name", list(GEN_SPECS))
def test_nnsp_exec_generic_nets(name):
    """NNSPClass_exec -- the drop-in kernel: the call out of LDS, one stream's
    epilogues spread over lanes, LSTM row tiles in rounds of four, weights that
    do not fit LDS read from memory -- on shapes past the reference's nets: rows
    not a multiple of 4, two and three LSTMs, 256- and 300-wide layers, mixed
    accumulators, a linear layer inside the stack.  Per frame: the trigger,
    context slot 5 and every LSTM's h / c against the oracle's."""
    data = synth_net(name, 8)
    spec = data.spec
    orc = OracleNet(data, thresh_prob=3000, th_count=1)
    h = _lib.NetHandle(data)
    feat, inst = _lib.FeatureClass(), _lib.NNSPClass()
    thr, cnt = np.array([3000], np.int16), np.array([1], np.int16)
    _KEEP.extend([h, feat, inst, thr, cnt])
    assert L().NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([spec.nn_id]), vp(h.mean),
                              vp(h.stdR), vp(thr), vp(cnt)) == 0
    L().NNSPClass_reset(C.byref(inst))
    T = 9
    pcm = synthetic_pcm(1, T, seed=123)
    st = orc.new_states(1)
    lstm = [i for i, ty in enumerate(spec.types) if ty == LSTM]   # (midlin has none: the trigger only)
    for t in range(T):
        o_trig, _, o_feat, st = orc.run(pcm[:, t:t + 1], st)
        frame = np.ascontiguousarray(pcm[0, t])
        assert L().NNSPClass_exec(C.byref(inst), vp(frame)) == o_trig[0, 0], f"{name} frame {t}"
        np.testing.assert_array_equal(np.ctypeslib.as_array(feat.normFeatContext)[200:240], o_feat[0, 0],
                                      err_msg=f"{name} features frame {t}")
        oh, oc = _oracle_hc(st[0])
        for k, i in enumerate(lstm):
            N = spec.sizes[i + 1]
            np.testing.assert_array_equal(h.h[i], oh[k, :N], err_msg=f"{name} LSTM {i} h, frame {t}")
            np.testing.assert_array_equal(h.c[i], oc[k, :N], err_msg=f"{name} LSTM {i} c, frame {t}")
    assert L().nnsp_legacy_status() == 0


def test_nnsp_exec_memory_path():
    """The drop-in kernel with its operands in device memory (NNSP_DROPIN_LDS=0,
    read once per process: a child process) on the reference-shaped and the
    generic nets, against the oracle as above."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # (as conftest.py: torch first, so that its HIP runtime is the process's;
    # the oracle directory ahead of the repository root)
    code = ("import sys; import torch; sys.path[:0] = ['oracle', '.', 'tests']\n"
            "import test_gpu_legacy as t\n"
            "t.test_nnsp_exec_interleaved_nets()\n"
            "for n in ('odd', 'lstm3', 'wide300'): t.test_nnsp_exec_generic_nets(n)\n"
            "print('ok')\n")
    env = dict(os.environ, NNSP_DROPIN_LDS="0")
    out = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout[-2000:] + out.stderr[-4000:]


def _child(code, **env_add):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import sys; import torch; sys.path[:0] = ['oracle', '.', 'tests']\nimport test_gpu_legacy as t\n" + code
    out = subprocess.run([sys.executable, "-c", code + "\nprint('ok')\n"], cwd=root, env=dict(os.environ, **env_add),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout[-2000:] + out.stderr[-4000:]


def test_nnsp_exec_one_launch_per_call():
    """The drop-in call as one launch each (NNSP_DROPIN_WORKER=0, the
    resident workers off; a child process) against the oracle."""
    _child("t.test_nnsp_exec_interleaved_nets()\nfor n in ('odd', 'lstm3'): t.test_nnsp_exec_generic_nets(n)",
           NNSP_DROPIN_WORKER="0")


def test_nnsp_exec_worker_idle_expiry():
    """Resident workers that leave after 2 ms without a request
    (NNSP_DROPIN_IDLE_MS=2) and calls 3 ms apart: every call finds its worker
    expired or leaving, and is relaunched or run in one launch -- results as
    the oracle's."""
    _child("t._interleaved(0.003)", NNSP_DROPIN_IDLE_MS="2")
