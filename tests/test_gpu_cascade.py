"""GPU parity of the batched VAD -> KWS -> S2I cascade (nnCntrlClass,
evb/src/nnCntrlClass.c:152-272) against the CPU oracle's or_run_cascade.

Per stream and frame: the net that ran, its trigger and NNSPClass.outputs must
match bit-exactly, across chunk boundaries (the speculative per-round segments
are cut at each switch), with look-back into earlier chunks, timeouts and
partial resets (nnCntrlClass_reset keeps the sequence position).
"""
import ctypes as C

import numpy as np
import pytest

from oracle import OracleCascade, OracleNet, lib, load_wavs, synthetic_pcm

from nnsp_amd.engine import NNSPBatch, NNSPCascade
from nnsp_amd.nets import synth_net

pytestmark = pytest.mark.gpu

POS_OFF = 100 * 160 * 2 + 4   # or_cascade.pos_seq (nnsp_oracle.h: ring, idx_set, idx_latest)

# (thresh_prob, th_count) per net: low enough that every stage triggers
TH = {"lively": {"vad": (3000, 1), "kws": (8000, 1), "s2i": (12000, 1)},
      "slow": {"vad": (8000, 1), "kws": (16383, 2), "s2i": (16383, 2)}}


def _pcm(S, T, seed):
    pcm = synthetic_pcm(S, T, seed=0x4E4E5350 + seed)
    rng = np.random.default_rng(seed)
    pcm[1::4] = (pcm[1::4].astype(np.int32) * 5).clip(-32768, 32767).astype(np.int16)
    pcm[2::6] //= 32
    quiet = rng.integers(0, T, S // 3)
    for s, t in zip(range(0, S, 3), quiet):   # silence gaps
        pcm[s, t:t + 40] = 0
    return pcm


def _build(th, S, Tmax, acc32, seq, lb_s2i, to_s2i, lb_kws, to_kws):
    onets, gnets = {}, {}
    for name in ("vad", "kws", "s2i"):
        data = synth_net(name, 1234)
        thr, cnt = th[name]
        onets[name] = OracleNet(data, acc32=acc32, thresh_prob=thr, th_count=cnt)
        gnets[name] = NNSPBatch(data, S, Tmax, acc32=acc32, thresh_prob=thr, th_count=cnt)
    oc = OracleCascade(onets, seq, lb_s2i, to_s2i, lb_kws, to_kws)
    gc = NNSPCascade(gnets, seq, lb_s2i, to_s2i, lb_kws, to_kws)
    return oc, gc, gnets


def _check(oc, gc, pcm, chunks, reset_at=None, reset_mask=None):
    S = pcm.shape[0]
    st = oc.new_states(S)
    t0 = 0
    switches = 0
    for i, Tc in enumerate(chunks):
        if reset_at is not None and i == reset_at:
            gc.reset(reset_mask)
            for s in np.nonzero(reset_mask)[0]:   # nnCntrlClass_reset: position kept
                pos = st[s, POS_OFF:POS_OFF + 2].copy()
                lib().or_cascade_reset(C.c_void_p(st[s].ctypes.data), C.byref(oc.cfg))
                st[s, POS_OFF:POS_OFF + 2] = pos
        seg = pcm[:, t0:t0 + Tc]
        o_ran, o_det, o_o3, st = oc.run(seg, st)
        g_ran, g_det, g_o3 = gc.exec(seg)
        np.testing.assert_array_equal(g_ran, o_ran, err_msg=f"net_ran chunk@{t0}")
        np.testing.assert_array_equal(g_det, o_det, err_msg=f"detected chunk@{t0}")
        np.testing.assert_array_equal(g_o3, o_o3, err_msg=f"outputs3 chunk@{t0}")
        switches += int((np.diff(o_ran.astype(np.int32), axis=1) != 0).sum())
        t0 += Tc
    pos = st[:, POS_OFF:POS_OFF + 2].copy().view(np.int16)[:, 0]
    np.testing.assert_array_equal(gc.positions(), pos.astype(np.int8))
    return switches


@pytest.mark.parametrize("th", ["lively", "slow"])
@pytest.mark.parametrize("acc32", [False, True])
@pytest.mark.parametrize("window", [32, 12, 0])
def test_cascade_matches_oracle(th, acc32, window):
    S, chunks = 150, [100, 37, 1, 63]
    oc, gc, _ = _build(TH[th], S, max(chunks), acc32, (1, 2, 0), 80, 60, 80, 50)
    gc.set_window(window)
    sw = _check(oc, gc, _pcm(S, sum(chunks), 11), chunks)
    assert sw > 50, "cascade never switched nets: test is vacuous"
    r, frames, _ = gc.last_stats()
    assert r >= 1 and frames >= S * chunks[-1]


@pytest.mark.parametrize("th", ["lively", "slow"])
def test_cascade_control_kernel(th, monkeypatch):
    # the controller as its own kernel per round (casc_control_kernel) instead
    # of fused into the nets' recur kernels: same results
    monkeypatch.setenv("NNSP_CASCADE_CONTROL_KERNEL", "1")
    S, chunks = 150, [100, 37, 1, 63]
    oc, gc, _ = _build(TH[th], S, max(chunks), False, (1, 2, 0), 80, 60, 80, 50)
    gc.set_window(12)
    assert _check(oc, gc, _pcm(S, sum(chunks), 12), chunks) > 50


KNOB_VALUE = {"NNSP_CASCADE_WINDOW": "7", "NNSP_FE_SCHED": "0", "NNSP_FE_GUIDE": "6,8"}


@pytest.mark.parametrize("knob", ["NNSP_CASCADE_SERIAL", "NNSP_CASCADE_DEBUG", "NNSP_CASCADE_TIMING",
                                  "NNSP_CASCADE_WINDOW", "NNSP_RECUR_CLOCKS", "NNSP_FE_SCHED", "NNSP_FE_GUIDE",
                                  "NNSP_EARLY_RETURN"])
def test_cascade_development_knobs_keep_results(knob, monkeypatch):
    """The library's remaining environment switches are development aids --
    every net on one stream (SERIAL), a synchronisation after every launch
    (DEBUG), per-round event timing (TIMING), a fixed round window (WINDOW),
    the s_memtime probes of the NN and front-end kernels (RECUR_CLOCKS), the
    shared front end's frame schedule (FE_SCHED: equal ranges; FE_GUIDE:
    another guided split), the early return (EARLY_RETURN): none may change a
    result."""
    monkeypatch.setenv(knob, KNOB_VALUE.get(knob, "1"))
    S, chunks = 90, [100, 37, 1, 63]
    oc, gc, _ = _build(TH["lively"], S, max(chunks), False, (1, 2, 0), 80, 60, 80, 50)
    assert _check(oc, gc, _pcm(S, sum(chunks), 13), chunks) > 30


@pytest.mark.parametrize("S", [1, 3, 17])
def test_cascade_tiny_grids(S):
    """Fewer frames than front-end waves (most waves of the guided schedule get
    an empty range), 1- and 2-frame chunks, a single stream."""
    chunks = [5, 1, 2, 9, 40]
    oc, gc, _ = _build(TH["lively"], S, max(chunks), False, (1, 2, 0), 3, 7, 2, 5)
    _check(oc, gc, _pcm(S, sum(chunks), 21 + S), chunks)


@pytest.mark.parametrize("ctl", ["fused", "kernel"])
def test_cascade_short_lookback_timeouts_and_order(ctl, monkeypatch):
    # odd look-backs, tiny timeouts (counter wrap), a different sequence order
    if ctl == "kernel":
        monkeypatch.setenv("NNSP_CASCADE_CONTROL_KERNEL", "1")
    S, chunks = 70, [30, 30, 17, 50]
    oc, gc, _ = _build(TH["slow"], S, 50, False, (1, 0, 2), 17, 7, 3, 5)
    gc.set_window(5)
    sw = _check(oc, gc, _pcm(S, sum(chunks), 5), chunks)
    assert sw > 50


def test_cascade_partial_reset():
    S, chunks = 64, [40, 40, 40]
    oc, gc, _ = _build(TH["lively"], S, 40, False, (1, 2, 0), 80, 60, 80, 50)
    gc.set_window(1)
    mask = np.zeros(S, np.uint8)
    mask[::3] = 1
    _check(oc, gc, _pcm(S, sum(chunks), 9), chunks, reset_at=2, reset_mask=mask)


@pytest.mark.parametrize("weights", ["synth", "ref"])
def test_cascade_lookahead_front_end(weights):
    """nnsp_cascade_exec_device_ahead: the next chunk's shared front end runs
    overlapped with this chunk's nets; results equal the oracle's, also when a
    call receives a different chunk than the one announced (the look-ahead is
    dropped and recomputed), after a partial reset, and with short chunks
    (look-ahead off below look-back + 1 frames)."""
    import torch

    from nnsp_amd.nets import get_net
    from oracle import load_wavs

    torch.cuda.set_device(0)
    S, Tm = 96, 100
    chunks = [100, 100, 90, 100, 30, 100, 100]
    announce = [1, 1, -1, 1, 1, 1, 1]   # -1: announce a different buffer than the next call gets
    th = TH["lively"] if weights == "synth" else {n: (16383, 4) for n in ("vad", "kws", "s2i")}
    onets, gnets = {}, {}
    for name in ("vad", "kws", "s2i"):
        data = get_net(name, weights)
        onets[name] = OracleNet(data, thresh_prob=th[name][0], th_count=th[name][1])
        gnets[name] = NNSPBatch(data, S, Tm, thresh_prob=th[name][0], th_count=th[name][1])
    oc = OracleCascade(onets)
    gc = NNSPCascade(gnets)
    pcm = synthetic_pcm(S, sum(chunks), wavs=load_wavs(), every=1 if weights == "ref" else 4)
    st = oc.new_states(S)
    bufs, t0 = [], 0
    for Tc in chunks:
        bufs.append(torch.from_numpy(np.ascontiguousarray(pcm[:, t0:t0 + Tc])).to("cuda"))
        t0 += Tc
    decoy = torch.zeros_like(bufs[0])
    ran = torch.empty((S, Tm), dtype=torch.int8, device="cuda")
    det = torch.empty((S, Tm), dtype=torch.int16, device="cuda")
    o3 = torch.empty((S, Tm, 3), dtype=torch.int16, device="cuda")
    t0 = 0
    for i, Tc in enumerate(chunks):
        if i == 5:   # partial nnCntrlClass_reset: position kept
            mask = (np.arange(S) % 4 == 1).astype(np.uint8)
            gc.reset(mask)
            for s in np.nonzero(mask)[0]:
                pos = st[s, POS_OFF:POS_OFF + 2].copy()
                lib().or_cascade_reset(C.c_void_p(st[s].ctypes.data), C.byref(oc.cfg))
                st[s, POS_OFF:POS_OFF + 2] = pos
        nxt = None
        if i + 1 < len(chunks):
            nxt = bufs[i + 1] if announce[i] > 0 else decoy
        gc.exec_device(bufs[i].data_ptr(), Tc, ran.data_ptr(), det.data_ptr(), o3.data_ptr(),
                       next_ptr=nxt.data_ptr() if nxt is not None else None,
                       next_T=chunks[i + 1] if nxt is not None else 0)
        gc.sync()
        o_ran, o_det, o_o3, st = oc.run(pcm[:, t0:t0 + Tc], st)
        # outputs are [S][T] of this call's T (the buffers hold Tm frames per stream)
        g_ran = ran.view(-1)[:S * Tc].view(S, Tc).cpu().numpy()
        g_det = det.view(-1)[:S * Tc].view(S, Tc).cpu().numpy()
        g_o3 = o3.view(-1)[:S * Tc * 3].view(S, Tc, 3).cpu().numpy()
        np.testing.assert_array_equal(g_ran, o_ran, err_msg=f"net_ran chunk {i}")
        np.testing.assert_array_equal(g_det, o_det, err_msg=f"detected chunk {i}")
        np.testing.assert_array_equal(g_o3, o_o3, err_msg=f"outputs3 chunk {i}")
        t0 += Tc
    gc.close()


def test_stats_right_after_exec_device():
    """The statistics getters may be called right after an asynchronous
    exec_device, with the chunk's tail work still queued (no sync): they must
    return, not report a not-ready event (bench.py reads them that way), and
    the per-net frame counts must add up to the chunk's frames at least."""
    import torch
    from nnsp_amd.nets import ref_net
    S, T = 256, 100
    gnets = {n: NNSPBatch(ref_net(n), S, T) for n in ("vad", "kws", "s2i")}
    gc = NNSPCascade(gnets)
    pcm = torch.from_numpy(synthetic_pcm(S, 3 * T, wavs=load_wavs(), every=2)).cuda()
    ran = torch.empty((S, T), dtype=torch.int8, device="cuda")
    for i in range(3):
        chunk = pcm[:, i * T:(i + 1) * T].contiguous()
        gc.exec_device(chunk.data_ptr(), T, ran.data_ptr())
        rounds, frames, ms = gc.last_stats()
        assert rounds >= 1 and frames >= S * T and ms > 0
        assert gc.fe_stats() >= 0
        for n in ("vad", "kws", "s2i"):
            gc.net_stats(n)
    gc.sync()
    gc.close()


@pytest.mark.parametrize("tseq", ["2", "3"])
@pytest.mark.parametrize("window", [0, 16])
def test_cascade_recur_tiles_back_to_back(tseq, window, monkeypatch):
    """Several recur tiles per workgroup through one pipeline (the default for
    short windows): at a tile boundary the next tile's LSTM state, the finished
    tile's state (zero for a stream whose net was reset), its feature context
    and the controller's bookkeeping all change hands mid-pipeline."""
    monkeypatch.setenv("NNSP_RECUR_TSEQ", tseq)
    S, chunks = 150, [100, 37, 1, 63]
    oc, gc, _ = _build(TH["lively"], S, max(chunks), True, (1, 2, 0), 80, 60, 80, 50)
    gc.set_window(window)
    assert _check(oc, gc, _pcm(S, sum(chunks), 21), chunks) > 50
