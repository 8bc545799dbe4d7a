#!/usr/bin/env python3
"""Development probe: per-wave wall-clock records of fe_kernel (NNSP_RECUR_CLOCKS=1,
single-net batch).  Prints the spread of wave lifetimes, the table set-up
cost, ns per frame and the number of resident waves over the launch.
usage: fe_waves.py [net] [streams]"""
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
S = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
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
N = 2048 + 4 * 32768
raw = np.zeros(N, np.int64)
_lib.check(L.nnsp_batch_debug_clocks_n(eng.h, C.c_void_p(raw.ctypes.data), N), "clocks")
w = raw[2048:].reshape(-1, 4)
w = w[w[:, 0] > 0]
t0 = w[:, 0].min()
st, tb, en, nf = (w[:, 0] - t0) * 10, (w[:, 1] - t0) * 10, (w[:, 2] - t0) * 10, w[:, 3]   # ns
life = en - st
print(f"{net} S={S}: fe {fe:.3f} ms (events); waves recorded {len(w)}; span {(en.max() - st.min()) / 1e3:.1f} us")
print(f"  wave lifetime us: min {life.min() / 1e3:.1f} median {np.median(life) / 1e3:.1f} max {life.max() / 1e3:.1f}")
print(f"  table set-up us: median {np.median(tb - st) / 1e3:.2f} max {(tb - st).max() / 1e3:.2f}")
pf = (en - tb) / np.maximum(nf, 1)
print(f"  ns per frame per wave: median {np.median(pf):.0f} (p10 {np.percentile(pf, 10):.0f}, p90 {np.percentile(pf, 90):.0f}); frames/wave {np.median(nf):.0f}")
print(f"  start times us: p0 {np.percentile(st, 0) / 1e3:.1f} p25 {np.percentile(st, 25) / 1e3:.1f} p50 {np.percentile(st, 50) / 1e3:.1f} p75 {np.percentile(st, 75) / 1e3:.1f} p100 {st.max() / 1e3:.1f}")
edges = np.linspace(0, en.max(), 41)
res = [int(((st <= e) & (en > e)).sum()) for e in edges[:-1]]
print("  resident waves at 40 instants:", res)
busy = life.sum() / (en.max() * min(6144, len(w)))
print(f"  wave-time / (span x 6144 slots) = {busy:.2f}")
