#!/usr/bin/env python3
"""Development probe: per-phase s_memtime clocks of recur_kernel tile 0
(NNSP_RECUR_CLOCKS=1).  Prints median cycles per phase of a step.

Needs a library built with the probes (make -C nnsp_amd PROBES=1, or
NNSP_LIB=<a build with PROBES=1>): the default build compiles them out."""
import ctypes as C
import os
import sys

os.environ["NNSP_RECUR_CLOCKS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nnsp_amd import _lib  # noqa: E402
from nnsp_amd.engine import NNSPBatch  # noqa: E402

net = sys.argv[1] if len(sys.argv) > 1 else "vad"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
T = 100
torch.cuda.set_device(0)
if len(sys.argv) > 3 and sys.argv[3] == "ref":   # the reference's own tables (ref_nets.npz)
    from nnsp_amd.nets import ref_net  # noqa: E402
    eng = NNSPBatch(ref_net(net), S, T)
else:
    eng = NNSPBatch(net, S, T)
pcm = torch.empty((S, T, 160), dtype=torch.int16, device="cuda")
trig = torch.empty((S, T), dtype=torch.int16, device="cuda")
L = _lib.lib()
L.nnsp_batch_debug_clocks.argtypes = [C.c_void_p, C.c_void_p]
L.nnsp_synth_pcm(C.c_void_p(pcm.data_ptr()), S, T, C.c_uint64(1), 0, C.c_int64(0), 4096, C.c_void_p(eng.stream))
for _ in range(3):
    eng.exec_device(pcm.data_ptr(), T, trig.data_ptr())
fe, nn = eng.last_timing()
raw = np.zeros(2048, np.int64)
_lib.check(L.nnsp_batch_debug_clocks(eng.h, C.c_void_p(raw.ctypes.data)), "clocks")
clk = raw[:1024].reshape(64, 16)
fclk = raw[1024:].reshape(128, 8)[:64]
st = clk[:53]
step = np.diff(st[:, 0])
print(f"{net} S={S}: fe {fe:.3f} ms nn {nn:.3f} ms; iteration cycles median {np.median(step[3:48]):.0f}")
names = ("lstm wave 0", "stage 1 fc", "stage 2 fc", "stage 3 fc", "stage 4 post")
if net == "s2i":   # 4-stage pipeline: the last FC layer and the post-processing on one wave
    names = ("lstm wave 0", "stage 1 fc", "stage 2 fc", "stage 3 fc+post")
for k, nm in enumerate(names):
    d = st[3:50, 2 * k + 1] - st[3:50, 2 * k]
    lag = st[3:50, 2 * k] - st[3:50, 0]
    print(f"  {nm:16s} work median {np.median(d):7.0f}  start lag {np.median(lag):6.0f}")
# proj_kernel wave 0 of workgroup 0 (slots 12-15 per tile: start, union loaded, FC done, x stored)
pj = clk[:, 12:16]
nt = int((pj[:, 0] > 0).sum())
if nt > 2:
    d = np.diff(pj[:nt], axis=1)
    tile = np.diff(pj[:nt, 0])
    print(f"  proj tiles {nt}: per tile median {np.median(tile):.0f} cycles; union {np.median(d[:, 0]):.0f}"
          f"  fc {np.median(d[:, 1]):.0f}  x store {np.median(d[:, 2]):.0f}")
# fe_kernel wave 0 of workgroup 0, per frame: start, window, cFFT, split+power, Mel, log+normalise
nf = int((fclk[:, 0] > 0).sum())
if nf > 2:
    d = np.diff(fclk[:nf, :6], axis=1)
    fr = np.diff(fclk[:nf, 0])
    print(f"  fe frames {nf}: per frame median {np.median(fr):.0f} cycles; window {np.median(d[:, 0]):.0f}"
          f"  cfft {np.median(d[:, 1]):.0f}  split+pspec {np.median(d[:, 2]):.0f}  mel {np.median(d[:, 3]):.0f}"
          f"  log+norm {np.median(d[:, 4]):.0f}")
