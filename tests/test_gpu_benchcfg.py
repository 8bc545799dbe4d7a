"""Parity at the benchmarked configuration.

bench.py's default workload -- the cascade with every library default (window
16, ParamsNNCntrl.h:8-21 thresholds 16383 / 4, look-back 80, timeouts 1000)
at 32768 streams, the reference's nets, the device-generated input mix -- is
run for two 100-frame chunks exactly as the bench runs it (device buffers,
exec_device), then 256+ sampled streams are compared with the oracle, which
regenerates just those streams (the input is counter-based: stream s of the
population depends on s only).  Also one net at configs[1]'s 8192 streams.
Frame indices above 2^21 per launch exercise the kernels' 32-bit indexing.
"""
import numpy as np
import pytest
import torch

from oracle import OracleCascade, OracleNet, load_wavs, synthetic_pcm

from nnsp_amd import _lib
from nnsp_amd.engine import NNSPBatch, NNSPCascade
from nnsp_amd.nets import get_net

pytestmark = pytest.mark.gpu

SEED, AMP = 0x4E4E5350, 4096


def _device_chunks(S, T, n, stream):
    wav = torch.from_numpy(load_wavs()).to("cuda")
    bufs = []
    for i in range(n):
        b = torch.empty((S, T, 160), dtype=torch.int16, device="cuda")
        _lib.check(_lib.lib().nnsp_synth_pcm_mix(b.data_ptr(), S, T, SEED, 0, i * T, AMP, wav.data_ptr(), 3, 160000,
                                                 4, stream), "synth")
        bufs.append(b)
    return bufs


def _sample(S, k, seed):
    rng = np.random.default_rng(seed)
    pick = np.concatenate([[0, 1, 2, 3, S - 4, S - 3, S - 2, S - 1], rng.choice(S, k, replace=False)])
    return np.unique(pick)


def _host_pcm(streams, T, chunk):
    wavs = load_wavs()
    return np.concatenate([synthetic_pcm(1, T, SEED, t0=chunk * T, s0=int(s), amp=AMP, wavs=wavs) for s in streams])


@pytest.mark.parametrize("weights", ["ref", "synth"])
def test_cascade_bench_config(weights):
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
    for c in range(2):
        eng.exec_device(bufs[c].data_ptr(), T, ran.data_ptr(), det.data_ptr(), o3.data_ptr())
        eng.sync()
        o_ran, o_det, o_o3, st = oc.run(_host_pcm(pick, T, c), st)
        idx = torch.from_numpy(pick).to("cuda")
        np.testing.assert_array_equal(ran[idx].cpu().numpy(), o_ran, err_msg=f"net_ran chunk {c}")
        np.testing.assert_array_equal(det[idx].cpu().numpy(), o_det, err_msg=f"detected chunk {c}")
        np.testing.assert_array_equal(o3[idx].cpu().numpy(), o_o3, err_msg=f"outputs3 chunk {c}")
    np.testing.assert_array_equal(eng.positions()[pick], st[:, 100 * 160 * 2 + 4:100 * 160 * 2 + 6].copy()
                                  .view(np.int16)[:, 0].astype(np.int8))
    eng.close()


def test_single_net_bench_config():
    torch.cuda.set_device(0)
    S, T = 8192, 100
    data = get_net("vad", "ref")
    eng = NNSPBatch(data, S, T)
    bufs = _device_chunks(S, T, 2, eng.stream)
    trig = torch.empty((S, T), dtype=torch.int16, device="cuda")
    lg = torch.empty((S, T, 2), dtype=torch.int32, device="cuda")
    pick = _sample(S, 256, 2)
    orc = OracleNet(data)
    st = orc.new_states(len(pick))
    for c in range(2):
        eng.exec_device(bufs[c].data_ptr(), T, trig.data_ptr(), lg.data_ptr())
        eng.sync()
        o_trig, o_lg, _, st = orc.run(_host_pcm(pick, T, c), st)
        idx = torch.from_numpy(pick).to("cuda")
        np.testing.assert_array_equal(trig[idx].cpu().numpy(), o_trig)
        np.testing.assert_array_equal(lg[idx].cpu().numpy(), o_lg)
    eng.close()
