"""Parity at BASELINE.json configs[1..3] sizes and full-scale front-end inputs
through the shipped (ARM_OPTIMIZED) build.

* configs[1..3]: one reference net (def_nn1_vad.c, def_nn2_kws_galaxy.c,
  def_nn0_s2i.c) at 8192 streams, two 100-frame chunks from the bench's
  device-generated input mix, exactly as ``bench.py --net NAME`` runs them
  (device buffers, exec_device); 256+ sampled streams are regenerated on the
  host and run through the oracle.  configs[3] is "32b vs 64b accum
  bit-parity": S2I runs with fc_8x16/lstm_8x16 (acc64) and with the _acc32b
  twins (def_nn0_s2i.c:68-84 selects one of them at compile time), and the two
  GPU runs must agree on every stream and frame, as well as with the oracle.
* full scale: +-32767 square waves of several periods, DC steps and clipped
  N(0, 30000) noise take spec2pspec_arm's ">> 27" truncating cast
  (spectrogram_module.c:86-90, trap T3) to 0.95 * 2^31 and melSpecProc's
  64-bit sums (melSpecProc.c:23-24) to their largest values, through every
  front-end mode of the shipped kernel:
  the batch mode (features compared per frame), the cascade's shared mode and
  its cold mode (the frames right after a net's reset; low thresholds make the
  nets switch often).
"""
import numpy as np
import pytest
import torch

from oracle import OracleCascade, OracleNet, load_wavs, spec2pspec, synthetic_pcm

from nnsp_amd import _lib
from nnsp_amd.engine import NNSPBatch, NNSPCascade
from nnsp_amd.nets import get_net, ref_net

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


def _run_config(name, acc32, S=8192, T=100, chunks=2):
    """configs[k] as bench.py --net runs it; returns (trig, logits) of every
    stream and chunk on the host, after checking the sample against the oracle."""
    torch.cuda.set_device(0)
    data = get_net(name, "ref")
    eng = NNSPBatch(data, S, T, acc32=acc32)
    bufs = _device_chunks(S, T, chunks, eng.stream)
    nout = eng.nout
    trig = torch.empty((S, T), dtype=torch.int16, device="cuda")
    lg = torch.empty((S, T, nout), dtype=torch.int32, device="cuda")
    pick = _sample(S, 256, 11 + acc32)
    orc = OracleNet(data, acc32=acc32)
    st = orc.new_states(len(pick))
    all_trig, all_lg = [], []
    idx = torch.from_numpy(pick).to("cuda")
    for c in range(chunks):
        eng.exec_device(bufs[c].data_ptr(), T, trig.data_ptr(), lg.data_ptr())
        eng.sync()
        o_trig, o_lg, _, st = orc.run(_host_pcm(pick, T, c), st)
        np.testing.assert_array_equal(trig[idx].cpu().numpy(), o_trig, err_msg=f"{name} trig chunk {c}")
        # every frame: the logits are 0 on frames where the NN does not run
        np.testing.assert_array_equal(lg[idx].cpu().numpy(), o_lg, err_msg=f"{name} logits chunk {c}")
        all_trig.append(trig.cpu().numpy())
        all_lg.append(lg.cpu().numpy())
    eng.close()
    tr, lgs = np.concatenate(all_trig, 1), np.concatenate(all_lg, 1)
    assert (lgs != 0).any(axis=-1).mean() > 0.45, "the NN ran on too few frames: vacuous"
    return tr, lgs


def test_config2_kws_8192_streams():
    _run_config("kws", acc32=False)


def test_config3_s2i_8192_streams_acc32_equals_acc64():
    t64, l64 = _run_config("s2i", acc32=False)
    t32, l32 = _run_config("s2i", acc32=True)
    # configs[3]: 32b vs 64b accumulator bit-parity on every stream and frame
    np.testing.assert_array_equal(t32, t64)
    np.testing.assert_array_equal(l32, l64)


def test_config1_vad_8192_streams_acc32_equals_acc64():
    t64, l64 = _run_config("vad", acc32=False)
    t32, l32 = _run_config("vad", acc32=True)
    np.testing.assert_array_equal(t32, t64)
    np.testing.assert_array_equal(l32, l64)


# ---------------------------------------------------------------- full scale
def _full_scale(S, T, seed=5):
    """Per stream one of: +-32767 square wave (period 2..~600 samples), DC
    steps between +-32767 / 0 / -32768, clipped N(0, 30000) noise, a
    full-scale square wave in the middle of silence."""
    rng = np.random.default_rng(seed)
    n = np.arange(T * 160)
    out = np.zeros((S, T * 160), np.int16)
    periods = [2, 3, 4, 8, 16, 32, 64, 100, 160, 320, 512, 640]
    for s in range(S):
        k = s % 4
        if k == 0:
            per = periods[(s // 4) % len(periods)]
            out[s] = np.where((n // (per // 2 if per > 2 else 1)) % 2 == 0, 32767, -32768)
        elif k == 1:
            lv = np.array([32767, 0, -32768, 32767, -32768, 0, 16384])
            step = 160 * (3 + (s // 4) % 7)
            out[s] = lv[(n // step) % len(lv)]
        elif k == 2:
            out[s] = np.clip(rng.normal(0, 30000, T * 160), -32768, 32767).astype(np.int16)
        else:
            sq = np.where((n // (7 + s % 13)) % 2 == 0, 32767, -32768)
            out[s] = np.where((n // 4000) % 2 == 1, sq, 0)
    return out.reshape(S, T, 160)


def test_full_scale_inputs_reach_the_overflow_regions():
    """Vacuity guard (oracle only, no GPU work): the inputs above take
    spec2pspec_arm's (re^2 + im^2) >> 27 to within 10 % of 2^31.  A full-scale
    DC step is the largest bin int16 PCM can make (|X[k]| <= 32768 * sum|win|),
    0.95 * 2^31, so T3's truncating-cast wrap and melSpecProc's int32 clamp
    cannot bind through the front end; they are pinned on direct inputs in
    tests/test_oracle_pinned.py and tests/test_gpu_legacy.py."""
    from oracle import mel, rfft512
    from nnsp_amd.tables import stft_window
    pcm = _full_scale(48, 30)
    w = stft_window().astype(np.int64)
    big = 0
    for s in range(48):
        buf = np.zeros(480, np.int16)
        for t in range(30):
            buf = np.concatenate([buf[160:], pcm[s, t]])
            x = np.zeros(512, np.int64)
            x[:480] = w * buf                       # Q15 x Q15 -> Q30, no shift (spectrogram_module.c:104-110)
            y, _ = rfft512(x.astype(np.int32))
            re = np.abs(y[0::2].astype(np.int64)).astype(np.uint64)
            im = np.abs(y[1::2].astype(np.int64)).astype(np.uint64)
            p = (re * re + im * im) >> np.uint64(27)
            big = max(big, int(p.max()))
            assert int(p.max()) < 2 ** 31
            assert np.abs(mel(spec2pspec(y)).astype(np.int64)).max() < 2 ** 31 - 1
    assert big > 0.9 * 2 ** 31, f"pspec never got near 2^31 ({big / 2 ** 31:.3f})"


@pytest.mark.parametrize("name", ["vad", "kws", "s2i"])
def test_full_scale_batch_mode(name):
    S, chunks = 48, [40, 9, 31]
    pcm = _full_scale(S, sum(chunks))
    data = ref_net(name)
    orc = OracleNet(data)
    eng = NNSPBatch(data, S, max(chunks))
    o_trig, o_lg, o_ft, _ = orc.run(pcm)
    t0 = 0
    for Tc in chunks:
        trig, lg, ft = eng.exec(pcm[:, t0:t0 + Tc], want_logits=True, want_features=True)
        np.testing.assert_array_equal(ft, o_ft[:, t0:t0 + Tc], err_msg=f"{name} features chunk@{t0}")
        np.testing.assert_array_equal(lg, o_lg[:, t0:t0 + Tc], err_msg=f"{name} logits chunk@{t0}")
        np.testing.assert_array_equal(trig, o_trig[:, t0:t0 + Tc], err_msg=f"{name} trig chunk@{t0}")
        t0 += Tc
    eng.close()


@pytest.mark.parametrize("weights,window", [("synth", -1), ("synth", 8), ("ref", -1)])
def test_full_scale_cascade_shared_and_cold(weights, window):
    """The cascade's shared and cold front ends on full-scale input.  With the
    reference nets the full-scale input makes VAD and KWS alternate (KWS never
    triggers, so S2I never runs); the seeded synthetic nets of the same shapes
    run all three nets."""
    S, chunks = 64, [100, 37, 100]
    th = {"vad": (3000, 1), "kws": (6000, 1), "s2i": (9000, 1)}   # low thresholds: frequent resets
    pcm = _full_scale(S, sum(chunks), seed=9)
    gnets = {n: NNSPBatch(get_net(n, weights), S, 100, thresh_prob=th[n][0], th_count=th[n][1]) for n in th}
    gc = NNSPCascade(gnets, (1, 2, 0), 20, 15, 30, 12)
    gc.set_window(window)
    oc = OracleCascade({n: OracleNet(get_net(n, weights), thresh_prob=th[n][0], th_count=th[n][1]) for n in th},
                       (1, 2, 0), 20, 15, 30, 12)
    o_ran, o_det, o_o3, _ = oc.run(pcm)
    t0 = 0
    for Tc in chunks:
        ran, det, o3 = gc.exec(pcm[:, t0:t0 + Tc])
        np.testing.assert_array_equal(ran, o_ran[:, t0:t0 + Tc], err_msg=f"net chunk@{t0}")
        np.testing.assert_array_equal(det, o_det[:, t0:t0 + Tc], err_msg=f"detected chunk@{t0}")
        np.testing.assert_array_equal(o3, o_o3[:, t0:t0 + Tc], err_msg=f"outputs3 chunk@{t0}")
        t0 += Tc
    gc.close()
    # the cold mode ran: the nets switched many times (every switch resets the
    # departing net; its next segment starts with cold frames)
    want = {0, 1, 2} if weights == "synth" else {1, 2}
    assert want <= set(np.unique(o_ran).tolist()), "nets did not switch: vacuous"
    switches = (np.diff(o_ran.astype(np.int16), axis=1) != 0).sum()
    assert switches > S, f"only {switches} net switches: the cold front end barely ran"
