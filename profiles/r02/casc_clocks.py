#!/usr/bin/env python3
"""Development probe: per-stage s_memtime clocks of recur_pipe_kernel tile 0 in
the cascade's round 0 (NNSP_RECUR_CLOCKS=1), per net, at the bench's default
configuration (32768 streams, the reference nets, the device wav mix)."""
import ctypes as C
import os
import sys

os.environ["NNSP_RECUR_CLOCKS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nnsp_amd import _lib  # noqa: E402
from nnsp_amd.engine import NNSPBatch, NNSPCascade  # noqa: E402
from nnsp_amd.nets import get_net  # noqa: E402

S, T = int(sys.argv[1]) if len(sys.argv) > 1 else 32768, 100
torch.cuda.set_device(0)
nets = {n: NNSPBatch(get_net(n, "ref"), S, T) for n in ("vad", "kws", "s2i")}
eng = NNSPCascade(nets)
L = _lib.lib()
L.nnsp_batch_debug_clocks.argtypes = [C.c_void_p, C.c_void_p]
wav = np.load(os.path.join(ROOT, "tests", "golden", "test_wavs.npz"))
ws = [wav[k].astype(np.int16) for k in sorted(wav.files)]
Lw = min(len(w) for w in ws)
wd = torch.from_numpy(np.stack([w[:Lw] for w in ws])).cuda()
pcm = torch.empty((S, T, 160), dtype=torch.int16, device="cuda")
ran = torch.empty((S, T), dtype=torch.int8, device="cuda")
det = torch.empty((S, T), dtype=torch.int16, device="cuda")
o3 = torch.empty((S, T, 3), dtype=torch.int16, device="cuda")
for c in range(3):
    _lib.check(L.nnsp_synth_pcm_mix(C.c_void_p(pcm.data_ptr()), S, T, C.c_uint64(1), 0, C.c_int64(c * T), 4096,
                                    C.c_void_p(wd.data_ptr()), len(ws), Lw, 4, C.c_void_p(eng.stream)), "synth")
    eng.exec_device(pcm.data_ptr(), T, ran.data_ptr(), det.data_ptr(), o3.data_ptr())
eng.sync()
for n, b in nets.items():
    raw = np.zeros(2048, np.int64)
    _lib.check(L.nnsp_batch_debug_clocks(b.h, C.c_void_p(raw.ctypes.data)), "clocks")
    clk = raw[:1024].reshape(64, 16)
    valid = (clk[:, 0] > 0).sum()
    st = clk[:valid]
    if valid < 8:
        print(n, "too few iterations", valid)
        continue
    step = np.diff(st[:, 0])
    names = ("lstm wave 0", "stage 1 fc", "stage 2 fc", "stage 3 fc", "stage 4 post")
    if n == "s2i":
        names = ("lstm wave 0", "stage 1 fc", "stage 2 fc", "stage 3 fc+post")
    print(f"{n}: {valid} iterations recorded; iteration cycles median {np.median(step[3:valid - 4]):.0f}")
    for k, nm in enumerate(names):
        d = st[3:valid - 2, 2 * k + 1] - st[3:valid - 2, 2 * k]
        print(f"  {nm:16s} work median {np.median(d):7.0f}")
    lw = raw[1536:2048].reshape(64, 8)[:valid]
    if lw[3:valid - 6, 4].any():
        d = lw[3:valid - 6]
        # probe order in time: 0 (loads + MFMA), 3 (x_half), 4 (load_x), 1 (gates), 2 (stores)
        print(f"  lstm: loads+mfma {np.median(d[:, 0] - st[3:valid - 6, 0]):6.0f}  x_half {np.median(d[:, 3] - d[:, 0]):6.0f}"
              f"  load_x {np.median(d[:, 4] - d[:, 3]):6.0f}  gates {np.median(d[:, 1] - d[:, 4]):6.0f}"
              f"  h/c stores {np.median(d[:, 2] - d[:, 1]):6.0f}  rest {np.median(st[4:valid - 5, 0] - d[:, 2]):6.0f}")
    pw = 2 * (len(names) - 1)   # the post wave's slots: start, end, then +2.. its sub-phases
    sub = st[3:valid - 2, pw:pw + 5]
    if sub[:, 2].any():
        print(f"  post: fc/logits {np.median(sub[:, 2] - sub[:, 0]):6.0f}  post_proc {np.median(sub[:, 3] - sub[:, 2]):6.0f}"
              f"  stores+controller {np.median(sub[:, 4] - sub[:, 3]):6.0f}  to end {np.median(sub[:, 1] - sub[:, 4]):6.0f}")
