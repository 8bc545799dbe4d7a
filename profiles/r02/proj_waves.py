#!/usr/bin/env python3
"""Development probe: per-wave wall-clock records of proj_kernel and fe_kernel
(NNSP_RECUR_CLOCKS=1, single-net batch): lifetimes, staging cost, tiles per
wave, resident waves over the launch.  usage: proj_waves.py [net] [streams]"""
import ctypes as C
import os
import sys

os.environ["NNSP_RECUR_CLOCKS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nnsp_amd import _lib  # noqa: E402
from nnsp_amd.engine import NNSPBatch  # noqa: E402

net = sys.argv[1] if len(sys.argv) > 1 else "vad"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
T = 100
torch.cuda.set_device(0)
eng = NNSPBatch(net, S, T)
pcm = torch.empty((S, T, 160), dtype=torch.int16, device="cuda")
trig = torch.empty((S, T), dtype=torch.int16, device="cuda")
L = _lib.lib()
L.nnsp_batch_debug_clocks_n.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
L.nnsp_synth_pcm(C.c_void_p(pcm.data_ptr()), S, T, C.c_uint64(1), 0, C.c_int64(0), 4096, C.c_void_p(eng.stream))
for _ in range(3):
    eng.exec_device(pcm.data_ptr(), T, trig.data_ptr())
fe, nn = eng.last_timing()
N = 2048 + 4 * 32768 + 4 * 8192
raw = np.zeros(N, np.int64)
_lib.check(L.nnsp_batch_debug_clocks_n(eng.h, C.c_void_p(raw.ctypes.data), N), "clocks")
print(f"{net} S={S}: fe {fe:.3f} ms nn {nn:.3f} ms (events)")
for name, w in (("fe", raw[2048:2048 + 4 * 32768].reshape(-1, 4)), ("proj", raw[2048 + 4 * 32768:].reshape(-1, 4))):
    w = w[(w[:, 0] > 0) & (w[:, 2] >= w[:, 0])]
    if not len(w):
        continue
    t0 = w[:, 0].min()
    st, sg, en, n = (w[:, 0] - t0) * 10, (w[:, 1] - t0) * 10, (w[:, 2] - t0) * 10, w[:, 3]
    life = en - st
    print(f"  {name}: waves {len(w)} span {(en.max()) / 1e3:.1f} us; lifetime median {np.median(life) / 1e3:.1f} max {life.max() / 1e3:.1f} us;"
          f" staging median {np.median(sg - st) / 1e3:.2f} us; units/wave median {np.median(n):.0f};"
          f" ns/unit median {np.median((en - sg) / np.maximum(n, 1)):.0f}")
    edges = np.linspace(0, en.max(), 21)
    print("    resident waves:", [int(((st <= e) & (en > e)).sum()) for e in edges[:-1]])
