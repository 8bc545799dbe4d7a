#!/usr/bin/env python3
"""Generate the committed golden fixtures from the reference itself.

Container-only (needs /root/reference and oracle/_ref/libnnsp_ref_partial.so,
built by oracle/build_ref.sh from the reference C files that compile here
without stand-ins).  Output: small .npz files of inputs and the reference's
outputs, so the oracle is pinned on every machine (the GPU box has no
reference tree).

  ref_stages.npz   activation.c, fixlog10.c, melSpecProc.c, spectrogram_module.c
                   (spec2pspec_arm), nn_speech.c (compute_pwr2, ceiling,
                   my_argmax, binary_post_proc, s2i_post_proc),
                   feature_module.c (FeatureClass_setDefault)
  layout.npz       python/nnsp_pack/c_weight_man.py (weight byte layout)
  ref_nets.npz     evb/src/def_nn{0_s2i,1_vad,2_kws_galaxy}.c as data: every
                   NeuralNetClass field of net_s2i / net_vad / net_kws_galaxy,
                   the int8 kernels and int16 biases byte for byte (interleaved
                   order), feature_mean / feature_stdR (oracle/_ref/libnnsp_ref_nets.so)
  ref_nn.npz       the reference's portable NN build (ARM_OPTIMIZED=0,
                   oracle/_ref/libnnsp_ref_nn_portable.so) on weights re-packed
                   into its byte order: fc_8x16 / lstm_8x16 / rc_8x16 and their
                   _acc32b twins called directly, and NeuralNetClass_exe over
                   consecutive calls (LSTM state carried) on the three reference
                   nets and on the N3 shapes of nnsp_amd.nets.ALL_GEN_SPECS

  ref_fe_portable.npz  the reference's ARM_OPTIMIZED=0 front end (row N4,
                   oracle/_ref/libnnsp_ref_fe_portable.so): rfft(512) and
                   FeatureClass_execute over consecutive frames

  ref_fft_complex.npz  the reference's portable fft.c / complex.c
                   (oracle/_ref/libnnsp_ref_fe_portable.so): rfft(256) and
                   rfft(512), fft(exp_nfft) for exp_nfft 0..8 (output and the
                   in-place input), on vectors from small to full int32 range
                   (complex.c's clamps bind), and every complex32_* helper

  ref_nnsp_portable.npz  the reference's whole portable path end to end
                   (oracle/_ref/libnnsp_ref_nnsp_portable.so: nn_speech.c over
                   the ARM_OPTIMIZED=0 front end and NN): NNSPClass_init /
                   _reset / _exec on each reference net, acc64 and acc32, over
                   the three test wavs x 1000 frames and 8 synthetic streams x
                   200 frames with one mid-stream NNSPClass_reset; per frame
                   the return value, normFeatContext[200:240], outputs[3] and
                   counts_category, and the final LSTM h / c

  test_wavs.npz    python/test_wavs/{speech,galaxy,galaxy_s2i}.wav samples
                   (16 kHz mono int16, 160000 each): the reference's own test
                   inputs, replayed by every 4th synthetic stream

Usage: make_golden.py [stages] [nets] [nn] [wavs] [fe_portable] [fft_complex] [nnsp]   (default: all)
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libnnsp_ref_partial.so")
REF_NN_SO = os.path.join(ROOT, "oracle", "_ref", "libnnsp_ref_nn_portable.so")
REF_NETS_SO = os.path.join(ROOT, "oracle", "_ref", "libnnsp_ref_nets.so")
REF_FE_PORT_SO = os.path.join(ROOT, "oracle", "_ref", "libnnsp_ref_fe_portable.so")
REF_NNSP_PORT_SO = os.path.join(ROOT, "oracle", "_ref", "libnnsp_ref_nnsp_portable.so")
REF_PY = "/root/reference/python"

from nnsp_amd._lib import FeatureClass, NeuralNetClass, NNSPClass  # noqa: E402  (ABI mirrors)
from nnsp_amd import nets as N  # noqa: E402


def P(a):
    return C.c_void_p(a.ctypes.data)


def act_inputs(rng):
    edges = [0, 1, -1, 511, 512, 513, -512, 1023, 1024, 1535, 1536, 163839, 163840, 163841,
             -163839, -163840, -163841, 2**31 - 1, -(2**31 - 1), 2**30, -(2**30)]
    dense = np.arange(-2048, 2048)
    mid = rng.integers(-200000, 200000, 12000)
    full = rng.integers(-(2**31 - 1), 2**31 - 1, 4000)
    return np.concatenate([edges, dense, mid, full]).astype(np.int32)


def log_inputs(rng):
    p2 = np.array([1 << k for k in range(31)], np.int64)
    near = np.concatenate([p2 - 1, p2, p2 + 1])
    lu = np.exp(rng.uniform(0, np.log(2**31 - 1), 16000)).astype(np.int64)
    x = np.concatenate([[0, 1, 2, 3, 2**31 - 1], near, lu, rng.integers(1, 70000, 3000)])
    return np.clip(x, 0, 2**31 - 1).astype(np.int32)


def stages() -> None:
    R = C.CDLL(REF_SO, mode=os.RTLD_LAZY)
    rng = np.random.default_rng(20261015)
    out = {}

    # ---- activations (activation.c)
    x = act_inputs(rng)
    for name in ("tanh_fix", "sigmoid_fix", "relu6_fix"):
        y = np.zeros(len(x), np.int16)
        getattr(R, name)(P(y), P(x), len(x))
        out[f"act_{name}"] = y
    out["act_x"] = x

    # ---- log10 (fixlog10.c)
    lx = log_inputs(rng)
    ly = np.zeros(len(lx), np.int32)
    for i, v in enumerate(lx):
        o = C.c_int32()
        R.my_log10(C.byref(o), C.c_int32(int(v)))
        ly[i] = o.value
    out["log_x"], out["log_y"] = lx, ly
    ly12 = np.zeros(256, np.int32)
    R.log10_vec(P(ly12), P(np.ascontiguousarray(lx[:256])), 256, C.c_int16(12))
    out["log_y_q12"] = ly12

    # ---- spec2pspec_arm (spectrogram_module.c:79-92), incl. T3 wrap
    specs = rng.integers(-2**20, 2**20, (40, 1024)).astype(np.int32)
    specs[::5] = rng.integers(-2**30, 2**30, (8, 1024)).astype(np.int32)   # wraps
    psp = np.zeros((40, 257), np.int32)
    for i in range(40):
        buf = specs[i].copy()
        R.spec2pspec_arm(P(buf), P(buf), 257)   # in place, as feature_module.c:64
        psp[i] = buf[:257]
    out["pspec_in"], out["pspec_out"] = specs, psp

    # ---- melSpecProc (melSpecProc.c:6-27)
    pin = (rng.integers(0, 2**24, (40, 1024)) >> rng.integers(0, 20, (40, 1))).astype(np.int32)
    pin[0, :] = 2**31 - 1   # saturation path
    mel = np.zeros((40, 40), np.int32)
    for i in range(40):
        R.melSpecProc(P(pin[i]), P(mel[i]))
    out["mel_in"], out["mel_out"] = pin, mel

    # ---- compute_pwr2 / ceiling (nn_speech.c:229-258)
    R.compute_pwr2.restype = C.c_int32
    R.ceiling.restype = C.c_int32
    px = np.concatenate([rng.integers(-2**31 + 1, 0, 3000), rng.integers(-600000, 1, 3000),
                         np.arange(-70000, 1, 7), rng.integers(0, 2**20, 200)]).astype(np.int32)
    out["pwr2_x"] = px
    out["pwr2_y"] = np.array([R.compute_pwr2(C.c_int32(int(v))) for v in px], np.int32)
    out["ceil_y"] = np.array([R.ceiling(C.c_int32(int(v))) for v in px], np.int32)

    # ---- my_argmax (last max wins)
    am_in = rng.integers(-5, 5, (300, 17)).astype(np.int32)
    am = np.zeros(300, np.int16)
    for i in range(300):
        r = C.c_int16()
        R.my_argmax(P(am_in[i]), 17, C.byref(r))
        am[i] = r.value
    out["argmax_in"], out["argmax_out"] = am_in, am

    # ---- binary_post_proc / s2i_post_proc sequences (state carried per sequence)
    def run_post(kind, nseq, nstep, thr, cnt):
        est_in, trig, est_out, counts, outs, amlast = [], [], [], [], [], []
        for q in range(nseq):
            inst = NNSPClass()
            tp, tc = C.c_int16(thr[q]), C.c_int16(cnt[q])
            inst.pt_thresh_prob = C.cast(C.pointer(tp), C.c_void_p)
            inst.pt_th_count_trigger = C.cast(C.pointer(tc), C.c_void_p)
            inst.nn_id = b"\x00" if kind == "s2i" else b"\x01"
            inst.slides = 1
            n = 41 if kind == "s2i" else 2
            base = rng.integers(-40000, 40000, n)
            for st in range(nstep):
                if kind == "s2i":
                    e = (base + rng.integers(-30000, 30000, n)).astype(np.int32)
                    if rng.random() < 0.7:   # persistent winner -> triggers
                        e[int(q % 7)] += 90000
                else:
                    e = rng.integers(-60000, 60000, 2).astype(np.int32)
                    if rng.random() < 0.6:
                        e[1] += 50000
                est_in.append(e.copy())
                t = C.c_int16(-7)
                if kind == "s2i":
                    R.s2i_post_proc(C.byref(inst), P(e), C.byref(t))
                else:
                    R.binary_post_proc(C.byref(inst), P(e), C.byref(t))
                trig.append(t.value)
                est_out.append(e.copy())
                counts.append(list(inst.counts_category))
                outs.append(list(inst.outputs))
                amlast.append(inst.argmax_last)
        return (np.array(est_in, np.int32), np.array(trig, np.int16), np.array(est_out, np.int32),
                np.array(counts, np.int16), np.array(outs, np.int16), np.array(amlast, np.int16))

    thr = [16383, 16383, 8000, 30000, 1000] * 4
    cnt = [4, 4, 2, 1, 6] * 4
    for kind in ("binary", "s2i"):
        e_in, t, e_out, cts, outs, aml = run_post(kind, 20, 60, thr, cnt)
        out[f"post_{kind}_in"], out[f"post_{kind}_trig"] = e_in, t
        out[f"post_{kind}_est_out"], out[f"post_{kind}_counts"] = e_out, cts
        out[f"post_{kind}_outputs"], out[f"post_{kind}_argmax_last"] = outs, aml
    out["post_thr"], out["post_cnt"] = np.array(thr, np.int32), np.array(cnt, np.int32)

    # ---- FeatureClass_setDefault (feature_module.c:26-45): slots 0-4, slot 5 kept (T4)
    fe_means = rng.integers(-120000, -10000, (4, 40)).astype(np.int32)
    fe_stds = rng.integers(12000, 30000, (4, 40)).astype(np.int32)
    fe_q = np.array([8, 8, 10, 6], np.int32)
    fe_ctx = np.zeros((4, 300), np.int16)
    for i in range(4):
        fc = FeatureClass()
        fc.state_stftModule.len_win = 480
        fc.num_context, fc.dim_feat, fc.qbit_output = 6, 40, int(fe_q[i])
        fc.pt_norm_mean = fe_means[i].ctypes.data
        fc.pt_norm_stdR = fe_stds[i].ctypes.data
        for k in range(300):
            fc.normFeatContext[k] = 1111   # stale slot-5 marker
        R.FeatureClass_setDefault(C.byref(fc))
        fe_ctx[i] = np.array(fc.normFeatContext[:], np.int16)
    out["fe_mean"], out["fe_stdR"], out["fe_qbit"], out["fe_ctx"] = fe_means, fe_stds, fe_q, fe_ctx

    np.savez_compressed(os.path.join(HERE, "ref_stages.npz"), **out)

    # ---- weight layout (python/nnsp_pack/c_weight_man.py)
    sys.path.insert(0, REF_PY)
    from nnsp_pack.c_weight_man import c_lstm_weight_man, c_matrix_man

    lay = {}
    k = 0
    for N in (1, 2, 3, 4, 5, 7, 28, 41):
        for K in (1, 2, 3, 9, 240):
            m = rng.integers(-128, 128, (N, K))
            lay[f"fc_{k}_in"] = m.astype(np.int8)
            lay[f"fc_{k}_out"] = c_matrix_man(m).astype(np.int64).astype(np.int8)
            k += 1
    for j, (N, K) in enumerate(((1, 5), (3, 7), (6, 10), (28, 28))):
        wf = rng.integers(-128, 128, (4 * N, K))
        wr = rng.integers(-128, 128, (4 * N, N))
        b = rng.integers(-32768, 32768, 4 * N)
        a, ar, bb = c_lstm_weight_man(wf, wr, b)
        lay[f"lstm_{j}_wf"], lay[f"lstm_{j}_wr"] = wf.astype(np.int8), wr.astype(np.int8)
        lay[f"lstm_{j}_b"] = b.astype(np.int16)
        lay[f"lstm_{j}_out_wf"] = a.astype(np.int64).astype(np.int8)
        lay[f"lstm_{j}_out_wr"] = ar.astype(np.int64).astype(np.int8)
        lay[f"lstm_{j}_out_b"] = bb.astype(np.int64).astype(np.int16)
    np.savez_compressed(os.path.join(HERE, "layout.npz"), **lay)


NET_SYMS = {"vad": ("net_vad", "vad"), "kws": ("net_kws_galaxy", "kws_galaxy"), "s2i": ("net_s2i", "s2i")}


def nets() -> None:
    """The three def_nn*.c nets, every table and field, as data."""
    L = C.CDLL(REF_NETS_SO)
    out = {}
    for name, (sym, suffix) in NET_SYMS.items():
        net = NeuralNetClass.in_dll(L, sym)
        nl = net.numlayers
        out[f"{name}_numlayers"] = np.int32(nl)
        for f in ("size_layer", "net_layer_type", "qbit_kernel", "qbit_input", "qbit_bias", "activation_type"):
            key = "layer_type" if f == "net_layer_type" else f
            out[f"{name}_{key}"] = np.array(list(getattr(net, f)), np.int32)
        for i in range(nl):
            K, Nn = net.size_layer[i], net.size_layer[i + 1]
            lstm = net.net_layer_type[i] == N.LSTM
            rows = 4 * Nn if lstm else Nn
            out[f"{name}_kernel{i}"] = np.ctypeslib.as_array((C.c_int8 * (rows * K)).from_address(net.pt_kernel[i])).copy()
            out[f"{name}_bias{i}"] = np.ctypeslib.as_array((C.c_int16 * rows).from_address(net.pt_bias[i])).copy()
            if lstm:
                out[f"{name}_kernel_rec{i}"] = np.ctypeslib.as_array(
                    (C.c_int8 * (rows * Nn)).from_address(net.pt_kernel_rec[i])).copy()
        for what in ("mean", "stdR"):
            out[f"{name}_{what}"] = np.ctypeslib.as_array((C.c_int32 * 40).in_dll(L, f"feature_{what}_{suffix}")).copy()
    np.savez_compressed(os.path.join(HERE, "ref_nets.npz"), **out)


class PortableNet:
    """A NeuralNetClass over the portable reference build, weights re-packed
    into its byte order (affine.c:291-309), private LSTM h/c."""

    def __init__(self, R, data, acc32):
        spec = data.spec
        Wp, Wrp, Bp = data.packed_portable()
        self.keep, self.h, self.c = [], [], []
        n = NeuralNetClass()
        n.numlayers = spec.nl
        for i, s in enumerate(spec.sizes):
            n.size_layer[i] = s
        acts = {N.RELU6: "relu6_fix", N.TANH: "tanh_fix", N.SIGMOID: "sigmoid_fix", N.LINEAR: "linear_fix"}
        for i, t in enumerate(spec.types):
            n.net_layer_type[i] = t
            n.qbit_kernel[i], n.qbit_input[i], n.qbit_bias[i] = spec.qk[i], spec.qi[i], spec.qb[i]
            n.activation_type[i] = spec.acts[i]
            n.act_func[i] = C.cast(getattr(R, acts[spec.acts[i]]), C.c_void_p).value
            a32 = acc32 or bool(spec.accs and spec.accs[i])   # mixed nets: per-layer layer_func
            fn = ("lstm_8x16" if t == N.LSTM else "fc_8x16") + ("_acc32b" if a32 else "")
            n.layer_func[i] = C.cast(getattr(R, fn), C.c_void_p).value
            w, b = np.ascontiguousarray(Wp[i], np.int8), np.ascontiguousarray(Bp[i], np.int16)
            self.keep += [w, b]
            n.pt_kernel[i], n.pt_bias[i] = w.ctypes.data, b.ctypes.data
            if t == N.LSTM:
                wr = np.ascontiguousarray(Wrp[i], np.int8)
                h = np.zeros(spec.sizes[i + 1], np.int16)
                c = np.zeros(spec.sizes[i + 1], np.int32)
                self.keep.append(wr)
                self.h.append(h)
                self.c.append(c)
                n.pt_kernel_rec[i], n.pt_hstate[i], n.pt_cstate[i] = wr.ctypes.data, h.ctypes.data, c.ctypes.data
        self.net, self.R, self.spec = n, R, spec
        R.NeuralNetClass_setDefault(C.byref(n))

    def exe(self, x):
        out = np.zeros(160, np.int32)
        xx = np.ascontiguousarray(x, np.int16)
        self.R.NeuralNetClass_exe(C.byref(self.net), P(xx), P(out), C.c_int8(-1))
        if self.spec.acts[-1] == N.LINEAR:
            return out[:self.spec.nout].copy()
        return out.view(np.int16)[:self.spec.nout].astype(np.int32)


def nn_inputs(rng, n, K):
    """Layer inputs: feature-like (Q8 normalised log-Mel), wide, full range."""
    a = np.clip(np.round(rng.normal(0, 700, (n, K))), -32768, 32767)
    a[n // 2: 3 * n // 4] = rng.integers(-6000, 6000, (n - n // 2 - (n - 3 * n // 4), K))
    a[3 * n // 4:] = rng.integers(-32768, 32768, (n - 3 * n // 4, K))
    return a.astype(np.int16)


# direct layer calls: (N, K, qk, qb, qi, act); cases with qi + qk < 15 and a
# bias hit the align shift that the shipped build leaves dead (T1)
FC_CASES = [(4, 240, 7, 14, 8, N.TANH), (28, 240, 6, 13, 8, N.TANH), (5, 28, 5, 15, 15, N.RELU6),
            (7, 33, 5, 15, 12, N.RELU6), (2, 28, 7, 15, 12, N.LINEAR), (41, 72, 5, 14, 12, N.LINEAR),
            (3, 9, 6, 18, 12, N.SIGMOID), (1, 1, 7, 9, 10, N.TANH), (6, 7, 4, 12, 15, N.LINEAR),
            (256, 240, 7, 14, 8, N.TANH), (9, 256, 5, 15, 12, N.RELU6), (64, 64, 5, 15, 15, N.RELU6)]
# (N, K, qk, qb, qi, qir): qir != qi exercises rc_Krows' shift of the input half
LSTM_CASES = [(28, 240, 5, 13, 15, 15), (5, 7, 5, 13, 15, 15), (6, 33, 5, 14, 15, 15),
              (1, 3, 6, 14, 15, 15), (7, 28, 5, 13, 15, 13), (4, 12, 4, 12, 15, 17), (72, 72, 5, 14, 15, 15),
              (3, 10, 7, 12, 8, 8)]


def nn() -> None:
    R = C.CDLL(REF_NN_SO)
    R.NeuralNetClass_exe.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int8]
    i16 = C.c_int16
    rng = np.random.default_rng(20261016)
    out = {}
    # ---- fc_8x16 / fc_8x16_acc32b (affine.c:409-490)
    for k, (Nn, K, qk, qb, qi, act) in enumerate(FC_CASES):
        w = rng.integers(-128, 128, (Nn, K)).astype(np.int8)
        if k % 3 == 1:
            w = np.clip(np.round(rng.normal(0, 12, (Nn, K))), -128, 127).astype(np.int8)
        b = rng.integers(-32768, 32768, Nn).astype(np.int16)
        x = nn_inputs(rng, 8, K)
        wp = N.pack_fc_portable(w)
        afn = C.cast(getattr(R, {N.RELU6: "relu6_fix", N.TANH: "tanh_fix", N.SIGMOID: "sigmoid_fix",
                                 N.LINEAR: "linear_fix"}[act]), C.c_void_p)
        for acc32 in (0, 1):
            f = R.fc_8x16_acc32b if acc32 else R.fc_8x16
            ys = np.zeros((8, Nn), np.int32)
            for r in range(8):
                y = np.zeros(2 * Nn + 2, np.int16)
                f(P(y), P(wp), None, P(b), P(x[r]), None, None, i16(Nn), i16(K), i16(Nn), i16(qk), i16(qb),
                  i16(qi), i16(0), C.c_int(act), afn)
                ys[r] = y.view(np.int32)[:Nn] if act == N.LINEAR else y[:Nn]
            out[f"fc{k}_y{32 if acc32 else 64}"] = ys
        out[f"fc{k}_w"], out[f"fc{k}_b"], out[f"fc{k}_x"] = w, b, x
        out[f"fc{k}_cfg"] = np.array([Nn, K, qk, qb, qi, act], np.int32)
    # ---- lstm_8x16 / lstm_8x16_acc32b (lstm.c:15-415), 4 calls carrying h / c
    for k, (Nn, K, qk, qb, qi, qir) in enumerate(LSTM_CASES):
        w = np.clip(np.round(rng.normal(0, 10, (4 * Nn, K))), -128, 127).astype(np.int8)
        wr = np.clip(np.round(rng.normal(0, 14, (4 * Nn, Nn))), -128, 127).astype(np.int8)
        if k % 2:
            w = rng.integers(-128, 128, (4 * Nn, K)).astype(np.int8)
        b = rng.integers(-20000, 20000, 4 * Nn).astype(np.int16)
        x = nn_inputs(rng, 4, K)
        if qi < 15:
            x = (x // 64).astype(np.int16)
        wp, wrp, bp = N.pack_lstm_portable(w), N.pack_lstm_portable(wr), N.pack_lstm_bias(b)
        for acc32 in (0, 1):
            f = R.lstm_8x16_acc32b if acc32 else R.lstm_8x16
            h = np.zeros(Nn, np.int16)
            c = np.zeros(Nn, np.int32)
            ys, hs, cs = np.zeros((4, Nn), np.int16), np.zeros((4, Nn), np.int16), np.zeros((4, Nn), np.int32)
            for r in range(4):
                y = np.zeros(Nn + 4, np.int16)
                f(P(y), P(wp), P(wrp), P(bp), P(x[r]), P(h), P(c), i16(Nn), i16(K), i16(Nn), i16(qk), i16(qb),
                  i16(qi), i16(qir), C.c_int(N.TANH), C.cast(R.tanh_fix, C.c_void_p))
                ys[r], hs[r], cs[r] = y[:Nn], h, c
            tag = 32 if acc32 else 64
            out[f"lstm{k}_y{tag}"], out[f"lstm{k}_h{tag}"], out[f"lstm{k}_c{tag}"] = ys, hs, cs
        out[f"lstm{k}_w"], out[f"lstm{k}_wr"], out[f"lstm{k}_b"], out[f"lstm{k}_x"] = w, wr, b, x
        out[f"lstm{k}_cfg"] = np.array([Nn, K, qk, qb, qi, qir], np.int32)
    # ---- NeuralNetClass_exe over consecutive calls: the reference nets (their
    #      own tables, re-packed) and the N3 shapes (synthetic weights)
    cases = [("vad", N.ref_net("vad")), ("kws", N.ref_net("kws")), ("s2i", N.ref_net("s2i"))]
    cases += [(g, N.synth_net(g, 77)) for g in N.ALL_GEN_SPECS]
    for name, data in cases:
        x = nn_inputs(rng, 24, data.spec.sizes[0])
        out[f"net_{name}_x"] = x
        if name in N.ALL_GEN_SPECS:
            for i in range(data.spec.nl):
                out[f"net_{name}_W{i}"], out[f"net_{name}_B{i}"] = data.W[i], data.B[i]
                if data.Wr[i] is not None:
                    out[f"net_{name}_Wr{i}"] = data.Wr[i]
        for acc32 in (0, 1):
            pn = PortableNet(R, data, acc32)
            ys = np.stack([pn.exe(x[r]) for r in range(len(x))])
            tag = 32 if acc32 else 64
            out[f"net_{name}_y{tag}"] = ys
            out[f"net_{name}_h{tag}"] = np.concatenate(pn.h) if pn.h else np.zeros(0, np.int16)
            out[f"net_{name}_c{tag}"] = np.concatenate(pn.c) if pn.c else np.zeros(0, np.int32)
    np.savez_compressed(os.path.join(HERE, "ref_nn.npz"), **out)


WAVS = ("speech", "galaxy", "galaxy_s2i")


def fe_portable() -> None:
    """ref_fe_portable.npz: the reference's ARM_OPTIMIZED=0 front end (row N4,
    oracle/_ref/libnnsp_ref_fe_portable.so): rfft(512) on Frac15 vectors, and
    FeatureClass_execute over consecutive frames (stftModule buffer and feature
    context carried) on the reference's own test wavs and noise."""
    R = C.CDLL(REF_FE_PORT_SO)
    rng = np.random.default_rng(0x4E34)
    out = {}
    xs = []
    for amp in (1 << 15, 1 << 14, 1 << 10, 64):
        for _ in range(8):
            xs.append(rng.integers(-amp, amp, 512))
    xs.append(np.full(512, 32767))
    xs.append(np.full(512, -32768))
    xs = np.array(xs, np.int32)
    xs[:, 480:] = 0
    ys = np.zeros((len(xs), 514), np.int32)
    for i, x in enumerate(xs):
        xi = x.copy()
        y = np.zeros(1024, np.int32)
        R.rfft(512, P(xi), P(y))
        ys[i] = y[:514]
    out["rfft_in"], out["rfft_out"] = xs, ys
    # FeatureClass_execute (feature_module.c:47-74) on 4 streams x 24 frames
    wz = np.load(os.path.join(HERE, "test_wavs.npz"))
    wav = [wz["speech"], wz["galaxy"]]
    S, T = 4, 24
    pcm = np.zeros((S, T, 160), np.int16)
    pcm[0] = wav[0][16000:16000 + T * 160].reshape(T, 160)
    pcm[1] = wav[1][32000:32000 + T * 160].reshape(T, 160)
    pcm[2] = rng.integers(-32768, 32768, (T, 160))
    pcm[3] = rng.integers(-300, 300, (T, 160))
    means = rng.integers(-120000, -10000, (S, 40)).astype(np.int32)
    stds = rng.integers(12000, 30000, (S, 40)).astype(np.int32)
    qb = np.array([8, 10, 6, 8], np.int32)
    feats = np.zeros((S, T, 40), np.int16)
    for s in range(S):
        fc = FeatureClass()
        R.FeatureClass_construct(C.byref(fc), P(means[s]), P(stds[s]), C.c_int8(int(qb[s])))
        R.FeatureClass_setDefault(C.byref(fc))
        for t in range(T):
            x = np.ascontiguousarray(pcm[s, t])
            R.FeatureClass_execute(C.byref(fc), P(x))
            feats[s, t] = np.array(fc.normFeatContext[200:240], np.int16)
    out["fe_pcm"], out["fe_mean"], out["fe_stdR"], out["fe_qbit"], out["fe_feats"] = pcm, means, stds, qb, feats
    np.savez_compressed(os.path.join(HERE, "ref_fe_portable.npz"), **out)


def fft_complex() -> None:
    """ref_fft_complex.npz: fft.c's rfft / fft at every size its tables serve,
    and complex.c's helpers, from the reference's own portable build."""
    R = C.CDLL(REF_FE_PORT_SO)
    rng = np.random.default_rng(0x0FF7)
    out = {}
    amps = [1 << 15, 1 << 20, 1 << 28, 1 << 31]
    for num in (256, 512):
        xs = np.array([rng.integers(-a, a, num) for a in amps for _ in range(4)], np.int64).astype(np.int32)
        ys = np.zeros((len(xs), num + 2), np.int32)
        for i, x in enumerate(xs):
            xi = x.copy()
            y = np.zeros(1024, np.int32)
            R.rfft(num, P(xi), P(y))
            assert np.array_equal(xi, x)
            ys[i] = y[:num + 2]
        out[f"rfft{num}_in"], out[f"rfft{num}_out"] = xs, ys
    for e in range(9):
        n = 1 << e
        xs = np.array([rng.integers(-a, a, 2 * n) for a in amps for _ in range(3)], np.int64).astype(np.int32)
        ys = np.zeros((len(xs), 2 * n), np.int32)
        xo = np.zeros_like(xs)
        for i, x in enumerate(xs):
            xi = x.copy()
            y = np.zeros(2 * n, np.int32)
            R.fft(e, P(xi), P(y))
            ys[i], xo[i] = y, xi
        out[f"fft{e}_in"], out[f"fft{e}_out"], out[f"fft{e}_in_after"] = xs, ys, xo
    # complex.c helpers: [case][...] int32 pairs
    L = 7
    a = rng.integers(-2**31, 2**31, (12, L, 2)).astype(np.int64).astype(np.int32)
    b = rng.integers(-2**31, 2**31, (12, L, 2)).astype(np.int64).astype(np.int32)
    a[:4] >>= 16
    b[:4] >>= 16
    m = rng.integers(-2**31, 2**31, (12, L, L, 2)).astype(np.int64).astype(np.int32)
    m[:6] >>= 12
    w16 = rng.integers(-2**15, 2**15, (12, L, 2)).astype(np.int16)
    sh = np.array([0, 1, 15, 31, 0, 3, 15, 20, 0, 7, 30, 2], np.int32)
    out["cx_a"], out["cx_b"], out["cx_m"], out["cx_w16"], out["cx_shift"] = a, b, m, w16, sh
    res = {k: [] for k in ("copy", "affine", "affine_alias", "interprod", "elmtprod", "add", "arry_add", "neg", "sub", "sub_b",
                           "mul", "init", "real2cmplx", "arry_real2cmplx", "arry_init")}
    for c in range(12):
        A, B, M, W = (np.ascontiguousarray(v[c]) for v in (a, b, m, w16))
        o = np.zeros((L, 2), np.int32)
        R.complex32_copy(P(o), P(A)); res["copy"].append(o[0].copy())
        o = np.zeros((L, 2), np.int32)
        R.complex32_affine(P(o), P(M), P(A), int(sh[c]), L); res["affine"].append(o.copy())
        o = A.copy()   # out aliasing input: later rows read the rows already written (complex.c:14-31)
        R.complex32_affine(P(o), P(M), P(o), int(sh[c]), L); res["affine_alias"].append(o.copy())
        o = np.zeros((L, 2), np.int32)
        R.complex32_interprod(P(o), P(A), P(B), int(sh[c]), L); res["interprod"].append(o[0].copy())
        o = np.zeros((L, 2), np.int32)
        R.complex32_complex16_elmtprod(P(o), P(A), P(W), L); res["elmtprod"].append(o.copy())
        o = np.zeros((L, 2), np.int32)
        R.complex32_add(P(o), P(A), P(B)); res["add"].append(o[0].copy())
        o = np.zeros((L, 2), np.int32)
        R.complexArry32_add(P(o), P(A), P(B), L); res["arry_add"].append(o.copy())
        o = np.zeros((L, 2), np.int32)
        R.complex32_neg(P(o), P(A)); res["neg"].append(o[0].copy())
        o = np.zeros((L, 2), np.int32)
        Bc = B.copy()
        R.complex32_sub(P(o), P(A), P(Bc)); res["sub"].append(o[0].copy()); res["sub_b"].append(Bc[0].copy())
        o = np.zeros((L, 2), np.int32)
        R.complex32_mul(P(o), P(A), P(B)); res["mul"].append(o[0].copy())
        o = np.zeros((L, 2), np.int32)
        R.complex32_init(P(o), C.c_int32(int(A[0, 0])), C.c_int32(int(A[0, 1]))); res["init"].append(o[0].copy())
        o = np.zeros((L, 2), np.int32)
        R.complex32_real2cmplx(P(o), C.c_int32(int(B[0, 0]))); res["real2cmplx"].append(o[0].copy())
        o = np.zeros((L, 2), np.int32)
        re_ = np.ascontiguousarray(A[:, 0]); im_ = np.ascontiguousarray(B[:, 1])
        R.complexArry32_real2cmplx(P(o), P(re_), L); res["arry_real2cmplx"].append(o.copy())
        o = np.zeros((L, 2), np.int32)
        R.complexArry32_init(P(o), P(re_), P(im_), L); res["arry_init"].append(o.copy())
    for k, v in res.items():
        out[f"cx_{k}"] = np.array(v, np.int32)
    np.savez_compressed(os.path.join(HERE, "ref_fft_complex.npz"), **out)


# end-to-end NNSPClass_exec fixture: streams and where each is reset
NNSP_NOISE = [(4096, 0x4E4E5350), (4096, 17), (30000, 5), (30000, 6), (300, 7), (1200, 8), (12000, 9), (64, 10)]
NNSP_WAV_T, NNSP_WAV_RESET = 1000, 611      # a reset on an odd frame: slides restarts at 1
NNSP_NOISE_T, NNSP_NOISE_RESET = 200, 97


def nnsp_streams():
    """[(pcm [T][160] int16, reset frame)]: the three wavs from sample 0, then
    SplitMix64 streams (oracle.synthetic_pcm, one amplitude and seed each)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import synthetic_pcm
    wz = np.load(os.path.join(HERE, "test_wavs.npz"))
    out = [(wz[w][:NNSP_WAV_T * 160].reshape(NNSP_WAV_T, 160), NNSP_WAV_RESET) for w in WAVS]
    for amp, seed in NNSP_NOISE:
        out.append((synthetic_pcm(1, NNSP_NOISE_T, seed=seed, amp=amp)[0], NNSP_NOISE_RESET))
    return out


def nnsp() -> None:
    """ref_nnsp_portable.npz: NNSPClass_exec (nn_speech.c:74-127) of the
    reference's own portable build, frame by frame."""
    R = C.CDLL(REF_NNSP_PORT_SO)
    R.NNSPClass_exec.restype = C.c_int16
    R.NeuralNetClass_exe.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int8]
    streams = nnsp_streams()
    out = {"noise_cfg": np.array(NNSP_NOISE, np.int64),
           "cfg": np.array([NNSP_WAV_T, NNSP_WAV_RESET, NNSP_NOISE_T, NNSP_NOISE_RESET], np.int32)}
    for name in ("vad", "kws", "s2i"):
        data = N.ref_net(name)
        for acc32 in (0, 1):
            tag = f"{name}_{32 if acc32 else 64}"
            pn = PortableNet(R, data, acc32)
            mean = np.ascontiguousarray(data.mean, np.int32)
            stdR = np.ascontiguousarray(data.stdR, np.int32)
            thr, cnt = C.c_int16(N.THRESH_PROB), C.c_int16(N.THRESH_CNTS)
            trig, feats, outs, counts, hs, cs = [], [], [], [], [], []
            for pcm, reset_at in streams:
                feat, inst = FeatureClass(), NNSPClass()
                assert R.NNSPClass_init(C.byref(inst), C.byref(pn.net), C.byref(feat), C.c_char(bytes([N.NN_ID[name]])),
                                        P(mean), P(stdR), C.byref(thr), C.byref(cnt)) == 0
                R.NNSPClass_reset(C.byref(inst))
                T = len(pcm)
                tr = np.zeros(T, np.int16)
                ft = np.zeros((T, 40), np.int16)
                o3 = np.zeros((T, 3), np.int16)
                ct = np.zeros((T, 8), np.int16)
                for t in range(T):
                    if t == reset_at:
                        R.NNSPClass_reset(C.byref(inst))
                    fr = np.ascontiguousarray(pcm[t], np.int16)
                    tr[t] = R.NNSPClass_exec(C.byref(inst), P(fr))
                    ft[t] = np.array(feat.normFeatContext[200:240], np.int16)
                    o3[t] = list(inst.outputs)
                    ct[t] = list(inst.counts_category)
                trig.append(tr)
                feats.append(ft)
                outs.append(o3)
                counts.append(ct)
                hs.append(np.concatenate(pn.h) if pn.h else np.zeros(0, np.int16))
                cs.append(np.concatenate(pn.c) if pn.c else np.zeros(0, np.int32))
            cat = lambda a: np.concatenate(a, 0)   # noqa: E731  (streams back to back, frames of the wavs first)
            out[f"{tag}_trig"], out[f"{tag}_outputs"], out[f"{tag}_counts"] = cat(trig), cat(outs), cat(counts)
            out[f"{tag}_h"], out[f"{tag}_c"] = np.stack(hs), np.stack(cs)
            if acc32:
                assert np.array_equal(cat(feats), out[f"{name}_feats"])
            else:
                out[f"{name}_feats"] = cat(feats)
    np.savez_compressed(os.path.join(HERE, "ref_nnsp_portable.npz"), **out)


def wavs() -> None:
    import wave
    out = {}
    for name in WAVS:
        with wave.open(os.path.join(REF_PY, "test_wavs", f"{name}.wav")) as w:
            assert (w.getframerate(), w.getnchannels(), w.getsampwidth()) == (16000, 1, 2)
            out[name] = np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.int16)
    np.savez_compressed(os.path.join(HERE, "test_wavs.npz"), **out)


def main() -> None:
    for so in (REF_SO, REF_NN_SO, REF_NETS_SO):
        if not os.path.exists(so):
            sys.exit("build oracle/_ref first (oracle/build_ref.sh)")
    which = sys.argv[1:] or ["stages", "nets", "nn", "wavs", "fe_portable", "fft_complex", "nnsp"]
    for w in which:   # nets before nn: nn re-packs the dumped reference nets
        {"stages": stages, "nets": nets, "nn": nn, "wavs": wavs, "fe_portable": fe_portable, "fft_complex": fft_complex,
         "nnsp": nnsp}[w]()
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
