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
REF_PY = "/root/reference/python"

from nnsp_amd._lib import FeatureClass, NNSPClass  # noqa: E402  (ABI mirrors)


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


def main() -> None:
    if not os.path.exists(REF_SO):
        sys.exit("build oracle/_ref first (oracle/build_ref.sh)")
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
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
