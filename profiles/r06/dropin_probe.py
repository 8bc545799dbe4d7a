#!/usr/bin/env python3
"""Development probe (PROBES build via NNSP_LIB, NNSP_DROPIN_PROBE=1): where a
drop-in NNSPClass_exec call's kernel time goes -- the dropin_kernel's phase
clocks (s_memrealtime, 100 MHz): front end, each NN layer, post-processing,
the results' copy to mapped host memory; beside the call's wall time."""
import ctypes as C
import os
import sys
import time

os.environ["NNSP_DROPIN_PROBE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from nnsp_amd import _lib  # noqa: E402
from nnsp_amd.nets import NN_ID, THRESH_CNTS, THRESH_PROB, get_net  # noqa: E402

L = _lib.lib()
L.nnsp_dropin_probes.argtypes = [C.c_void_p]
z = np.load(os.path.join(ROOT, "tests", "golden", "test_wavs.npz"))
T = 400
pcm = np.ascontiguousarray(z["speech"][:T * 160].reshape(T, 160), np.int16)
for net in ("vad", "kws", "s2i"):
    h = _lib.NetHandle(get_net(net, "ref"))
    thr, cnt = np.array([THRESH_PROB], np.int16), np.array([THRESH_CNTS], np.int16)
    feat, inst = _lib.FeatureClass(), _lib.NNSPClass()
    _lib.check(L.NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([NN_ID[net]]),
                                _lib.ptr(h.mean), _lib.ptr(h.stdR), _lib.ptr(thr), _lib.ptr(cnt)), "init")
    L.NNSPClass_reset(C.byref(inst))
    frames = [np.ascontiguousarray(pcm[t]) for t in range(T)]
    nl = h.net.numlayers
    rec, wall = [], []
    pr = np.zeros(96, np.int64)   # NNSP_PROBE_LONGS
    for t in range(T):
        t0 = time.perf_counter()
        L.NNSPClass_exec(C.byref(inst), _lib.ptr(frames[t]))
        wall.append(time.perf_counter() - t0)
        _lib.check(L.nnsp_dropin_probes(pr.ctypes.data), "probes")
        if t >= 50:
            rec.append(pr.copy())
    r = np.array(rec)
    us = lambda a, b: np.median(r[:, b] - r[:, a]) / 100.0   # noqa: E731
    parts = [f"fe {us(0, 1):5.2f}"]
    if os.environ.get("NNSP_DROPIN_LDS", "1") != "0":   # [13] inputs + tables in, [12] weights staged
        parts += [f"(in+tables {us(0, 13):5.2f}, frame {us(13, 1):5.2f}, staged {us(0, 12):5.2f})"]
    if nl <= 5:   # the NN prologue: [7] first barrier, [8] context staged, [9] context barrier
        parts += [f"(nn prologue: bar {us(1, 7):4.2f} ctx {us(7, 8):4.2f} bar {us(8, 9):4.2f})"]
    parts += [f"L{i} {us(1 + i, 2 + i):5.2f}" for i in range(nl)]
    # [10] / [11]: s_memtime (the shader clock) at the start / the end
    mhz = np.median((r[:, 11] - r[:, 10]) / ((r[:, 15] - r[:, 0]) / 100.0))
    parts += [f"post {us(1 + nl, 14):5.2f}", f"copy-out {us(14, 15):5.2f}", f"kernel {us(0, 15):5.2f}", f"clock {mhz:6.0f} MHz"]
    fine = []
    for i in range(nl):   # FC layers: [16 + 8 i + k] entry, B split, first MFMA tile, epilogue, before the barrier
        o = 16 + 8 * i
        if np.all(r[:, o] > 0):
            # (LSTM: ctx is the h staging, rest the barrier and the h stores)
            fine.append(f"L{i}[ctx {us(1 + i, o):4.2f} b {us(o, o + 1):4.2f} mfma {us(o + 1, o + 2):4.2f} "
                        f"ep {us(o + 2, o + 3):4.2f} rest {us(o + 3, o + 4):4.2f} bar {us(o + 4, 2 + i):4.2f}]")
    hus = lambda a, b: np.median(r[:, 88 + b] - r[:, 88 + a]) / 1000.0   # noqa: E731  (host ns)
    host = (f"host: image {hus(0, 1):4.2f} stage {hus(1, 2):4.2f} launch {hus(2, 3):4.2f} "
            f"wait {hus(3, 4):5.2f} total {hus(0, 4):5.2f}")
    print(f"{net}: {host}")
    print(f"{net}: wall median {np.median(wall[50:]) * 1e6:6.1f} us; kernel phases (us): " + "  ".join(parts))
    print("   " + " ".join(fine))
