"""Diagnostic: the bench-config cascade (tests/test_gpu_benchcfg.py) on chunk 0-1,
printing where the GPU and the oracle disagree (stream, frame, net, values)."""
import os
import sys

import torch  # noqa: F401  (first: its HIP runtime is the one the library uses)
import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from oracle import OracleCascade, OracleNet  # noqa: E402
from test_gpu_benchcfg import _device_chunks, _host_pcm, _sample  # noqa: E402

from nnsp_amd.engine import NNSPBatch, NNSPCascade  # noqa: E402
from nnsp_amd.nets import get_net  # noqa: E402

weights = sys.argv[1] if len(sys.argv) > 1 else "ref"
torch.cuda.set_device(0)
S, T = 32768, 100
eng = NNSPCascade({n: NNSPBatch(get_net(n, weights), S, T) for n in ("vad", "kws", "s2i")})
bufs = _device_chunks(S, T, 2, eng.stream)
ran = torch.empty((S, T), dtype=torch.int8, device="cuda")
det = torch.empty((S, T), dtype=torch.int16, device="cuda")
o3 = torch.empty((S, T, 3), dtype=torch.int16, device="cuda")
pick = _sample(S, 256, 1)
oc = OracleCascade({n: OracleNet(get_net(n, weights)) for n in ("vad", "kws", "s2i")})
st = oc.new_states(len(pick))
bad = 0
for c in range(2):
    eng.exec_device(bufs[c].data_ptr(), T, ran.data_ptr(), det.data_ptr(), o3.data_ptr())
    eng.sync()
    o_ran, o_det, o_o3, st = oc.run(_host_pcm(pick, T, c), st)
    idx = torch.from_numpy(pick).to("cuda")
    g_ran, g_det, g_o3 = ran[idx].cpu().numpy(), det[idx].cpu().numpy(), o3[idx].cpu().numpy()
    print(f"chunk {c} window/stats {eng.last_stats()}")
    for name, g, o in (("ran", g_ran, o_ran), ("det", g_det, o_det), ("o3", g_o3, o_o3)):
        w = np.argwhere(g != o)
        print(f"  {name}: {len(w)} mismatches")
        for k in w[:12]:
            i, t = int(k[0]), int(k[1])
            print(f"    stream {pick[i]} frame {t} gpu {g[tuple(k)]} ref {o[tuple(k)]} net gpu {g_ran[i, t]} ref {o_ran[i, t]}"
                  f" nets around {list(o_ran[i, max(0, t - 3):t + 4])} det around {list(o_det[i, max(0, t - 3):t + 4])}"
                  f" gpu {list(g_det[i, max(0, t - 3):t + 4])}")
        bad += len(w)
eng.close()
print("TOTAL_MISMATCH", bad)
