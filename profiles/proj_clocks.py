#!/usr/bin/env python3
"""Development probe: per-phase s_memtime clocks of proj_kernel, wave 0 of
workgroup 0, its first tiles (NNSP_RECUR_CLOCKS=1).  usage: proj_clocks.py NET S T"""
import ctypes as C
import os
import sys

os.environ["NNSP_RECUR_CLOCKS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nnsp_amd import _lib  # noqa: E402
from nnsp_amd.engine import NNSPBatch  # noqa: E402

net = sys.argv[1] if len(sys.argv) > 1 else "s2i"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
T = int(sys.argv[3]) if len(sys.argv) > 3 else 100
torch.cuda.set_device(0)
eng = NNSPBatch(net, S, T)
pcm = torch.empty((S, T, 160), dtype=torch.int16, device="cuda")
trig = torch.empty((S, T), dtype=torch.int16, device="cuda")
L = _lib.lib()
L.nnsp_batch_debug_clocks.argtypes = [C.c_void_p, C.c_void_p]
L.nnsp_synth_pcm(C.c_void_p(pcm.data_ptr()), S, T, C.c_uint64(1), 0, C.c_int64(0), 4096, C.c_void_p(eng.stream))
for _ in range(3):
    eng.exec_device(pcm.data_ptr(), T, trig.data_ptr())
fe, nn = eng.last_timing()
clk = np.zeros(64 * 32, np.int64)   # nnsp_batch_debug_clocks copies 64 x 32 longs
_lib.check(L.nnsp_batch_debug_clocks(eng.h, C.c_void_p(clk.ctypes.data)), "clocks")
p = clk.reshape(-1, 16)[:64, 12:16]   # tile `it` of wave 0: longs 12 + 16 it + phase
n = int((p[:, 3] > 0).sum())
p = p[:n]
d = np.diff(p, axis=1)
tile = np.diff(p[:, 0]) if n > 1 else np.array([0])
print(f"{net} S={S} T={T}: fe {fe:.3f} ms nn {nn:.3f} ms; proj tiles probed {n}")
for k, nm in enumerate(("loads+sync", "fc0", "wx+stores")):
    print(f"  {nm:12s} median {np.median(d[:, k]):7.0f}  max {d[:, k].max():7.0f}")
print(f"  tile-to-tile median {np.median(tile):7.0f}")
