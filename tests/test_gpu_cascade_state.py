"""Cascade stream-state export / import (nnsp_cascade_get_state / set_state,
include/nnsp_cascade.h).

A stream's blob holds what the reference keeps per stream between frames: its
nnCntrlClass (position, timeout counters; evb/src/nnCntrlClass.h:35-45), the
PcmBufClass look-back frames (PcmBufClass.c:30-85), and the three
NNSPClass / FeatureClass / NeuralNetClass states.  Checked here:
  * resume: state taken mid-stream from one cascade and put into a fresh one
    continues with outputs identical to the oracle run without interruption --
    also when the source cascade had already run the next chunk's look-ahead
    front end;
  * re-sharding: streams run as two half-size shards and moved into one
    full-size cascade (and back) change no output;
  * get(set(x)) == x, and blobs of a cascade with other look-backs are refused.
"""
import numpy as np
import pytest
import torch

from oracle import OracleCascade, OracleNet

from nnsp_amd import _lib
from nnsp_amd.engine import NNSPBatch, NNSPCascade
from nnsp_amd.nets import synth_net

from test_gpu_cascade import TH, _pcm

pytestmark = pytest.mark.gpu

SEQ, LB_S2I, TO_S2I, LB_KWS, TO_KWS = (1, 2, 0), 37, 60, 80, 50
CHUNKS = [100, 90, 85]   # >= the look-back + 1: the look-ahead front end runs


def _gpu(S, Tmax=100, lb_s2i=LB_S2I):
    th = TH["lively"]
    nets = {n: NNSPBatch(synth_net(n, 1234), S, Tmax, thresh_prob=th[n][0], th_count=th[n][1])
            for n in ("vad", "kws", "s2i")}
    return NNSPCascade(nets, SEQ, lb_s2i, TO_S2I, LB_KWS, TO_KWS)


def _oracle_runs(pcm):
    th = TH["lively"]
    oc = OracleCascade({n: OracleNet(synth_net(n, 1234), thresh_prob=th[n][0], th_count=th[n][1])
                        for n in ("vad", "kws", "s2i")}, SEQ, LB_S2I, TO_S2I, LB_KWS, TO_KWS)
    st = oc.new_states(pcm.shape[0])
    out, t0 = [], 0
    for T in CHUNKS:
        r = oc.run(pcm[:, t0:t0 + T], st)
        st = r[3]
        out.append(r[:3])
        t0 += T
    return out


def _same(got, want, what):
    for g, w, name in zip(got, want, ("net_ran", "detected", "outputs3")):
        np.testing.assert_array_equal(g, w, err_msg=f"{what}: {name}")


@pytest.mark.parametrize("lookahead", [False, True])
def test_cascade_state_resume(lookahead):
    torch.cuda.set_device(0)
    S = 96
    pcm = _pcm(S, sum(CHUNKS), 21)
    want = _oracle_runs(pcm)
    a = _gpu(S)
    _same(a.exec(pcm[:, :100]), want[0], "chunk 0")
    c1, c2 = pcm[:, 100:190], pcm[:, 190:275]
    if lookahead:   # chunk 1 on device buffers with chunk 2's front end run ahead
        d1 = torch.from_numpy(np.ascontiguousarray(c1)).cuda()
        d2 = torch.from_numpy(np.ascontiguousarray(c2)).cuda()
        ran = torch.empty((S, 90), dtype=torch.int8, device="cuda")
        det = torch.empty((S, 90), dtype=torch.int16, device="cuda")
        o3 = torch.empty((S, 90, 3), dtype=torch.int16, device="cuda")
        a.exec_device(d1.data_ptr(), 90, ran.data_ptr(), det.data_ptr(), o3.data_ptr(), next_ptr=d2.data_ptr(),
                      next_T=85)
        a.sync()
        _same((ran.cpu().numpy(), det.cpu().numpy(), o3.cpu().numpy()), want[1], "chunk 1")
    else:
        _same(a.exec(c1), want[1], "chunk 1")
    blob = a.get_state()
    assert blob.shape == (S, _lib.lib().nnsp_cascade_state_bytes(a.h))
    hdr = blob[:, :4].copy().view(np.uint32)[:, 0]
    assert (hdr == 0x3153434E).all()
    b = _gpu(S)
    b.set_state(blob)
    np.testing.assert_array_equal(b.get_state(), blob)
    _same(b.exec(c2), want[2], "chunk 2 after resume")
    if lookahead:   # the source keeps its own look-ahead: get_state does not disturb it
        ran = torch.empty((S, 85), dtype=torch.int8, device="cuda")
        det = torch.empty((S, 85), dtype=torch.int16, device="cuda")
        o3 = torch.empty((S, 85, 3), dtype=torch.int16, device="cuda")
        a.exec_device(d2.data_ptr(), 85, ran.data_ptr(), det.data_ptr(), o3.data_ptr())
        a.sync()
        _same((ran.cpu().numpy(), det.cpu().numpy(), o3.cpu().numpy()), want[2], "chunk 2, source")
    else:
        _same(a.exec(c2), want[2], "chunk 2, source")
    assert (want[2][0] != want[2][0][:, :1]).any(), "no net switch in chunk 2: the test would be vacuous"
    a.close()
    b.close()


def test_cascade_state_reshard():
    torch.cuda.set_device(0)
    S, h = 96, 48
    pcm = _pcm(S, sum(CHUNKS), 22)
    want = _oracle_runs(pcm)
    # two shards of 48 streams for chunks 0-1
    shards = [_gpu(h), _gpu(h)]
    for i, sh in enumerate(shards):
        t0 = 0
        for c, T in enumerate(CHUNKS[:2]):
            _same(sh.exec(pcm[i * h:(i + 1) * h, t0:t0 + T]), [w[i * h:(i + 1) * h] for w in want[c]],
                  f"shard {i} chunk {c}")
            t0 += T
    # -> one cascade of 96 streams for chunk 2
    one = _gpu(S)
    for i, sh in enumerate(shards):
        one.set_state(sh.get_state(), first=i * h)
    _same(one.exec(pcm[:, 190:275]), want[2], "chunk 2 after 2 -> 1 shards")
    # and back: streams 48..95 of a full run moved into a half-size cascade
    full = _gpu(S)
    _same(full.exec(pcm[:, :100]), want[0], "full chunk 0")
    _same(full.exec(pcm[:, 100:190]), want[1], "full chunk 1")
    half = _gpu(h)
    half.set_state(full.get_state(first=h, count=h))
    _same(half.exec(pcm[h:, 190:275]), [w[h:] for w in want[2]], "chunk 2 after 1 -> 2 shards")
    # a blob of a cascade with other look-backs (another history length) is
    # refused: by the wrapper (its shape) and by the library itself (header)
    other = _gpu(h, lb_s2i=90)
    foreign = full.get_state(first=0, count=h)
    with pytest.raises(ValueError):
        other.set_state(foreign)
    assert _lib.lib().nnsp_cascade_set_state(other.h, _lib.ptr(foreign), 0, 1) == _lib.NNSP_EINVAL
    # a blob whose nets differ (header signature) or whose size field differs is
    # refused even at the right size (foreign net state imported silently)
    mine = half.get_state()
    for off, what in ((24, "nets_sig"), (20, "state_bytes"), (6, "version")):
        bad = mine.copy()
        bad[0, off] ^= 0x5A
        assert _lib.lib().nnsp_cascade_set_state(half.h, _lib.ptr(bad), 0, h) == _lib.NNSP_EINVAL, what
    half.set_state(mine)
    np.testing.assert_array_equal(half.get_state(), mine)
    for x in shards + [one, full, half, other]:
        x.close()
