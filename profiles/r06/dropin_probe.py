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
    pr = np.zeros(16, np.int64)
    for t in range(T):
        t0 = time.perf_counter()
        L.NNSPClass_exec(C.byref(inst), _lib.ptr(frames[t]))
        wall.append(time.perf_counter() - t0)
        _lib.check(L.nnsp_dropin_probes(pr.ctypes.data), "probes")
        if t >= 50:
            rec.append(pr.copy())
    r = np.array(rec)
    us = lambda a, b: np.median(r[:, b] - r[:, a]) / 100.0   # noqa: E731
    parts = [f"fe {us(0, 1):5.2f}"] + [f"L{i} {us(1 + i, 2 + i):5.2f}" for i in range(nl)]
    parts += [f"post {us(1 + nl, 14):5.2f}", f"copy-out {us(14, 15):5.2f}", f"kernel {us(0, 15):5.2f}"]
    print(f"{net}: wall median {np.median(wall[50:]) * 1e6:6.1f} us; kernel phases (us): " + "  ".join(parts))
