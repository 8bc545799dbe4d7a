"""Parity of the exact timed pipeline.

bench.py's default cascade line times consecutive 100-frame chunks at 32 768
streams, each call with the next chunk's look-ahead front end (``next_ptr``)
and no host synchronisation between calls.  This test builds the engine with
bench.py's own ``make_engine`` and drives it with bench.py's own
``chunk_step``, for the bench's warm-up (2) plus 4 timed chunks.  That covers
  * a full rotation of the cascade's PCM history buffers (hist[k mod 3]) and
    both parities of the chunk-counter blocks at bench size;
  * a look-ahead front end whose rings the next call reads.
Every chunk gets its own output buffers; after the last chunk, >= 256 sampled
streams plus the first and last four are compared with the oracle on every
chunk (reference: evb/src/PcmBufClass.c:30-85, evb/src/nnCntrlClass.c:152-272).
"""
import numpy as np
import pytest
import torch

from oracle import OracleCascade, OracleNet, load_wavs, synthetic_pcm

from bench import AMP, SEED, chunk_step, make_engine
from nnsp_amd import _lib
from nnsp_amd.nets import get_net

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("weights", ["ref", "synth"])
def test_bench_loop_verbatim(weights):
    torch.cuda.set_device(0)
    S, T, W, K = 32768, 100, 2, 4
    n = W + K
    eng = make_engine("cascade", S, T, False, weights, -1)   # bench defaults: window automatic
    wav = torch.from_numpy(load_wavs()).to("cuda")
    bufs = [torch.empty((S, T, 160), dtype=torch.int16, device="cuda") for _ in range(n + 1)]
    for i, b in enumerate(bufs):
        _lib.check(_lib.lib().nnsp_synth_pcm_mix(b.data_ptr(), S, T, SEED, 0, i * T, AMP, wav.data_ptr(), 3, 160000,
                                                 4, eng.stream), "synth_pcm")
    outs = [(torch.full((S, T), -7, dtype=torch.int8, device="cuda"),
             torch.full((S, T), -7, dtype=torch.int16, device="cuda"),
             torch.full((S, T, 3), -7, dtype=torch.int16, device="cuda")) for _ in range(n)]
    eng.sync()
    torch.cuda.synchronize()
    for i in range(n):   # bench.py's warm-up and timed loop: no host wait between chunks
        ran, trig, out3 = outs[i]
        chunk_step(eng, True, T, bufs[i], bufs[i + 1], ran, trig, out3)
    eng.sync()
    torch.cuda.synchronize()
    rng = np.random.default_rng(5)
    pick = np.unique(np.concatenate([[0, 1, 2, 3, S - 4, S - 3, S - 2, S - 1], rng.choice(S, 256, replace=False)]))
    oc = OracleCascade({nm: OracleNet(get_net(nm, weights)) for nm in ("vad", "kws", "s2i")})
    st = oc.new_states(len(pick))
    wavs = load_wavs()
    idx = torch.from_numpy(pick).to("cuda")
    switched = 0
    for c in range(n):
        pcm = np.concatenate([synthetic_pcm(1, T, SEED, t0=c * T, s0=int(s), amp=AMP, wavs=wavs) for s in pick])
        o_ran, o_det, o_o3, st = oc.run(pcm, st)
        ran, trig, out3 = (t[idx].cpu().numpy() for t in outs[c])
        np.testing.assert_array_equal(ran, o_ran, err_msg=f"net_ran, chunk {c}")
        np.testing.assert_array_equal(trig, o_det, err_msg=f"detected, chunk {c}")
        np.testing.assert_array_equal(out3, o_o3, err_msg=f"outputs3, chunk {c}")
        switched += int((o_ran[:, 1:] != o_ran[:, :-1]).sum())
    assert switched > 0, "no net switch in the sample: the comparison would not cover the controller"
    eng.close()
