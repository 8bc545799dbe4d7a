"""Development: first mismatches of the fused-control cascade vs the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "oracle"))
sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
from test_gpu_cascade import _build, _pcm, TH
S, chunks = 150, [100]
oc, gc, _ = _build(TH["lively"], S, 100, False, (1, 2, 0), 80, 60, 80, 50)
gc.set_window(int(sys.argv[1]) if len(sys.argv) > 1 else 32)
pcm = _pcm(S, 100, 11)
st = oc.new_states(S)
o_ran, o_det, o_o3, st = oc.run(pcm, st)
g_ran, g_det, g_o3 = gc.exec(pcm)
bad = np.argwhere(g_ran != o_ran)
print("mismatches", len(bad), "rounds", gc.last_stats())
for s in sorted(set(bad[:, 0]))[:6]:
    t = bad[bad[:, 0] == s][0, 1]
    lo = max(0, t - 6)
    print("stream", s, "first bad frame", t)
    print("  oracle ran", o_ran[s, lo:t + 6], "det", o_det[s, lo:t + 6])
    print("  gpu    ran", g_ran[s, lo:t + 6], "det", g_det[s, lo:t + 6])
