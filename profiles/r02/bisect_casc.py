"""One small cascade run (two chunks) vs the oracle with the library NNSP_LIB
names; prints OK / MISMATCH, raises on a HIP error (development bisection)."""
import os
import sys

import torch  # noqa: F401  (torch's HIP runtime first)

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
from oracle import OracleCascade, OracleNet, synthetic_pcm  # noqa: E402

from nnsp_amd.engine import NNSPBatch, NNSPCascade  # noqa: E402
from nnsp_amd.nets import synth_net  # noqa: E402

S, chunks = 150, (100, 37)
th = {"vad": (3000, 1), "kws": (8000, 1), "s2i": (12000, 1)}
onets, gnets = {}, {}
for name in ("vad", "kws", "s2i"):
    data = synth_net(name, 1234)
    onets[name] = OracleNet(data, thresh_prob=th[name][0], th_count=th[name][1])
    gnets[name] = NNSPBatch(data, S, max(chunks), thresh_prob=th[name][0], th_count=th[name][1])
oc = OracleCascade(onets, (1, 2, 0), 80, 60, 80, 50)
gc = NNSPCascade(gnets, (1, 2, 0), 80, 60, 80, 50)
print("created", flush=True)
pcm = synthetic_pcm(S, sum(chunks))
st = oc.new_states(S)
t0, ok = 0, True
for Tc in chunks:
    o_ran, o_det, o_o3, st = oc.run(pcm[:, t0:t0 + Tc], st)
    g_ran, g_det, g_o3 = gc.exec(pcm[:, t0:t0 + Tc])
    ok &= bool(np.array_equal(g_ran, o_ran) and np.array_equal(g_det, o_det) and np.array_equal(g_o3, o_o3))
    print("chunk", Tc, "ok" if ok else "mismatch", flush=True)
    t0 += Tc
gc.close()
print("OK" if ok else "MISMATCH")
