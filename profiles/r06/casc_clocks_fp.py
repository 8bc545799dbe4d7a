#!/usr/bin/env python3
"""Development probe (PROBES build, NNSP_LIB): per-stage s_memtime clocks of
recur_pipe_kernel tile 0 in the cascade's round 0, per net, with the fused
VAD prefix stage (NNSP_FUSE_PREFIX=1) or without; the prefix wave's work and
its DMA wait are printed when present (slots 14/15 and 13)."""
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
for n in ("vad",):
    b = nets[n]
    raw = np.zeros(2048, np.int64)
    _lib.check(L.nnsp_batch_debug_clocks(b.h, C.c_void_p(raw.ctypes.data)), "clocks")
    clk = raw[:1024].reshape(64, 16)
    valid = (clk[:, 0] > 0).sum()
    st = clk[:valid]
    step = np.diff(st[:, 0])
    print(f"{n} fuse={os.environ.get('NNSP_FUSE_PREFIX', '0')}: {valid} iterations; iteration cycles median "
          f"{np.median(step[3:valid - 4]):.0f}")
    for k, nm in enumerate(("lstm wave 0", "stage 1 fc", "stage 2 fc", "stage 3 fc", "stage 4 post")):
        d = st[3:valid - 4, 2 * k + 1] - st[3:valid - 4, 2 * k]
        print(f"  {nm:16s} work median {np.median(d):7.0f}")
