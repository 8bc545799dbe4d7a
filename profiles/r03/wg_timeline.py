#!/usr/bin/env python3
"""Development probe: where and when every workgroup / wave of one cascade
chunk ran (NNSP_RECUR_CLOCKS records: fe_kernel per wave, proj_kernel per
wave, recur_pipe_kernel per workgroup of round 0; 100 MHz wall clock; CU from
HW_REG_HW_ID / HW_REG_XCC_ID).  Runs the bench workload (32768 streams,
reference nets, wav mix, look-ahead front end), then prints per kernel the
span and duration spread and a 25 us timeline of how many of each were
resident.  usage: wg_timeline.py [S] [out.npz]"""
import ctypes as C
import os
import sys

os.environ["NNSP_RECUR_CLOCKS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nnsp_amd import _lib  # noqa: E402
from nnsp_amd.engine import NNSPBatch, NNSPCascade  # noqa: E402
from nnsp_amd.nets import ref_net  # noqa: E402
from oracle import load_wavs  # noqa: E402

DCLK_FE, DCLK_PROJ, DCLK_RECUR = 2048, 2048 + 4 * 32768, 2048 + 4 * 32768 + 4 * 8192
LONGS = DCLK_RECUR + 4 * 8192
S = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
T = 100
torch.cuda.set_device(0)
nets = {n: NNSPBatch(ref_net(n), S, T) for n in ("vad", "kws", "s2i")}
eng = NNSPCascade(nets)
wav = torch.from_numpy(load_wavs()).to("cuda")
bufs = []
for i in range(6):
    b = torch.empty((S, T, 160), dtype=torch.int16, device="cuda")
    _lib.check(_lib.lib().nnsp_synth_pcm_mix(b.data_ptr(), S, T, 0x4E4E5350, 0, i * T, 4096, wav.data_ptr(), 3, 160000,
                                             4, eng.stream), "synth")
    bufs.append(b)
ran = torch.empty((S, T), dtype=torch.int8, device="cuda")
det = torch.empty((S, T), dtype=torch.int16, device="cuda")
o3 = torch.empty((S, T, 3), dtype=torch.int16, device="cuda")
L = _lib.lib()
for i in range(5):
    if i == 4:   # the instrumented chunk: records of this chunk only
        eng.sync()
        for b in nets.values():
            _lib.check(L.nnsp_batch_debug_clocks_clear(b.h), "clear")
    eng.exec_device(bufs[i].data_ptr(), T, ran.data_ptr(), det.data_ptr(), o3.data_ptr(), next_ptr=bufs[i + 1].data_ptr(),
                    next_T=T)
eng.sync()
rec = {}
for n, b in nets.items():
    buf = np.zeros(LONGS, np.int64)
    _lib.check(L.nnsp_batch_debug_clocks_n(b.h, C.c_void_p(buf.ctypes.data), LONGS), "clocks")
    rec[n] = buf
out = {}


def rows(buf, off, n):
    r = buf[off:off + 4 * n].reshape(n, 4)
    return r[r[:, 2] > 0]


out["fe"] = rows(rec["vad"], DCLK_FE, 32768)
for n in nets:
    out[f"proj_{n}"] = rows(rec[n], DCLK_PROJ, 8192)
    out[f"recur_{n}"] = rows(rec[n], DCLK_RECUR, 8192)
t0 = min(v[:, 0].min() for v in out.values() if len(v))
print(f"S={S}; times in us from the first record (100 MHz clock)")
for k, v in out.items():
    if not len(v):
        print(f"{k:12s} none")
        continue
    st, en = (v[:, 0] - t0) / 100.0, (v[:, 2] - t0) / 100.0
    d = en - st
    where = v[:, 3] >> 32
    cus = len(np.unique(where >> 3))
    print(f"{k:12s} n={len(v):6d} start {st.min():8.1f}..{st.max():8.1f}  end {en.min():8.1f}..{en.max():8.1f}  "
          f"dur med {np.median(d):7.1f} p90 {np.percentile(d, 90):7.1f} max {d.max():7.1f}  CUs {cus}")
span = max(((v[:, 2] - t0) / 100.0).max() for v in out.values() if len(v))
bins = np.arange(0, span + 25, 25)
print("\n   t(us) " + " ".join(f"{k:>10s}" for k in out))
for b0 in bins:
    cnt = []
    for k, v in out.items():
        if not len(v):
            cnt.append(0)
            continue
        st, en = (v[:, 0] - t0) / 100.0, (v[:, 2] - t0) / 100.0
        cnt.append(int(((st < b0 + 12.5) & (en > b0 + 12.5)).sum()))
    print(f"{b0:8.0f} " + " ".join(f"{c:10d}" for c in cnt))
if len(sys.argv) > 2:
    np.savez_compressed(sys.argv[2], **out)
