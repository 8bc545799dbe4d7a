"""Cascade parity past 2^32 ring elements.

The shared front end writes three normalised rings of S * ring * 40 int16
(ring = look-back + 1 + 2 T).  At the strong-scaling shard of SURVEY.md
§8(d) config 5 on one GPU (262 144 streams, here with T = 200 chunks) and at
65 536 streams with T = 1000 (the survey's timed chunk length) the element
offsets pass 2^32: with 32-bit offsets the second and third rings and the
high streams of the first were written over other rows without a fault.
Each case runs two chunks through exec_device with the look-ahead front end
(the steady-state path bench.py times), then compares 256 sampled streams
plus the first and last four with the oracle, which regenerates just those
streams (the device input is counter-based per stream).  Reference
semantics: evb/src/nnCntrlClass.c:152-272, PcmBufClass.c:30-85.
"""
import numpy as np
import pytest
import torch

from oracle import OracleCascade, OracleNet, load_wavs, synthetic_pcm

from nnsp_amd import _lib
from nnsp_amd.engine import NNSPBatch, NNSPCascade
from nnsp_amd.nets import LOOKBACK, get_net

pytestmark = pytest.mark.gpu

SEED, AMP = 0x4E4E5350, 4096


def _sample(S, k, seed):
    rng = np.random.default_rng(seed)
    # half of the sample from the streams whose ring rows pass 2^32 elements
    ring_hi = S - S // 4
    pick = np.concatenate([[0, 1, 2, 3, S - 4, S - 3, S - 2, S - 1], rng.choice(S, k // 2, replace=False),
                           rng.integers(ring_hi, S, k // 2)])
    return np.unique(pick)


def _host_pcm(streams, T, chunk, wavs):
    return np.concatenate([synthetic_pcm(1, T, SEED, t0=chunk * T, s0=int(s), amp=AMP, wavs=wavs) for s in streams])


@pytest.mark.parametrize("S,T", [(262144, 200), (65536, 1000)])
def test_cascade_past_32bit_ring_offsets(S, T):
    ring = LOOKBACK + 1 + 2 * T
    assert 3 * S * ring * 40 > 2 ** 32   # the case this test exists for
    torch.cuda.set_device(0)
    eng = NNSPCascade({n: NNSPBatch(get_net(n, "ref"), S, T) for n in ("vad", "kws", "s2i")})
    wav = torch.from_numpy(load_wavs()).to("cuda")
    bufs = []
    for i in range(2):
        b = torch.empty((S, T, 160), dtype=torch.int16, device="cuda")
        _lib.check(_lib.lib().nnsp_synth_pcm_mix(b.data_ptr(), S, T, SEED, 0, i * T, AMP, wav.data_ptr(), 3, 160000,
                                                 4, eng.stream), "synth")
        bufs.append(b)
    ran = torch.empty((S, T), dtype=torch.int8, device="cuda")
    det = torch.empty((S, T), dtype=torch.int16, device="cuda")
    o3 = torch.empty((S, T, 3), dtype=torch.int16, device="cuda")
    pick = _sample(S, 256, S)
    idx = torch.from_numpy(pick).to("cuda")
    wavs = load_wavs()
    oc = OracleCascade({n: OracleNet(get_net(n, "ref")) for n in ("vad", "kws", "s2i")})
    st = oc.new_states(len(pick))
    try:
        for c in range(2):
            nxt = bufs[c + 1].data_ptr() if c + 1 < len(bufs) else None
            eng.exec_device(bufs[c].data_ptr(), T, ran.data_ptr(), det.data_ptr(), o3.data_ptr(), nxt, T)
            eng.sync()
            o_ran, o_det, o_o3, st = oc.run(_host_pcm(pick, T, c, wavs), st)
            np.testing.assert_array_equal(ran[idx].cpu().numpy(), o_ran, err_msg=f"net_ran chunk {c}")
            np.testing.assert_array_equal(det[idx].cpu().numpy(), o_det, err_msg=f"detected chunk {c}")
            np.testing.assert_array_equal(o3[idx].cpu().numpy(), o_o3, err_msg=f"outputs3 chunk {c}")
        # every stream's sequence position is a valid one (no stray writes into CascState)
        pos = eng.positions()
        assert pos.min() >= 0 and pos.max() <= 2
    finally:
        eng.close()
        for b in eng.nets.values():
            b.close()
        del bufs, ran, det, o3
        torch.cuda.empty_cache()

