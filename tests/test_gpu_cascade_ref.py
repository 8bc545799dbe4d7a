"""Cascade stream state in the reference's own per-stream objects
(nnsp_cascade_set_state_ref / get_state_ref, include/nnsp_cascade.h;
VERDICT r5 next #6).

A single-stream reference application keeps, per stream, one nnCntrlClass
(evb/src/nnCntrlClass.h:35-45), its PcmBufClass voice buffer
(PcmBufClass.c:10-85) and three NNSPClass with their FeatureClass and
NeuralNetClass (ns-nnsp/includes-api/nn_speech.h:12-25, feature_module.h:7-18).
The oracle's per-stream cascade state (or_cascade, oracle/nnsp_oracle.h) holds
exactly those fields, so it stands in for the reference session here:
  * forward: the oracle runs two chunks; its state goes through the
    reference objects into a fresh GPU cascade, which continues the third
    chunk bit-exactly like the oracle run without interruption;
  * reverse: the GPU runs two chunks; its state comes out into reference
    objects, from which the oracle continues the third chunk bit-exactly;
  * round trip: get_state_ref -> set_state_ref into another cascade gives the
    same state blob (the look-back features, which the reference does not
    keep, are recomputed on the device from the voice buffer);
  * at the largest look-back (99, the voice buffer's limit) the oldest frame
    of the current net's STFT buffer lies past the voice buffer.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import OracleCascade, OracleNet, lib as olib

from nnsp_amd import _lib
from nnsp_amd.engine import NNSPBatch, NNSPCascade, RefStream
from nnsp_amd.nets import synth_net

from test_gpu_cascade import TH, _pcm

pytestmark = pytest.mark.gpu

SEQ, TO_S2I, TO_KWS = (1, 2, 0), 60, 50
CHUNKS = [100, 90, 85]
NAMES = ("s2i", "vad", "kws")   # NNSP_ID order

OR_STREAM = np.dtype([("buf", "<i2", 480), ("ctx", "<i2", 240), ("h", "<i2", (10, 304)), ("c", "<i4", (10, 304)),
                      ("slides", "<i2"), ("trigger", "<i2"), ("argmax_last", "<i2"), ("pad0", "<i2"),
                      ("counts", "<i2", 8), ("outputs", "<i2", 3), ("pad1", "<i2")])
OR_CASCADE = np.dtype([("ring", "<i2", (100, 160)), ("idx_set", "<i2"), ("idx_latest", "<i2"), ("pos_seq", "<i2"),
                       ("pad", "<i2"), ("cnt_kws", "<u2"), ("cnt_s2i", "<u2"), ("nnsp", OR_STREAM, 3)])


def _setup(lb_s2i, lb_kws):
    th = TH["lively"]
    data = {n: synth_net(n, 1234) for n in NAMES}
    oc = OracleCascade({n: OracleNet(data[n], thresh_prob=th[n][0], th_count=th[n][1]) for n in NAMES}, SEQ,
                       lb_s2i, TO_S2I, lb_kws, TO_KWS)
    handles = [_lib.NetHandle(data[n]) for n in NAMES]

    def gpu(S):
        nets = {n: NNSPBatch(data[n], S, 100, thresh_prob=th[n][0], th_count=th[n][1]) for n in NAMES}
        return NNSPCascade(nets, SEQ, lb_s2i, TO_S2I, lb_kws, TO_KWS)
    return oc, handles, gpu


def _or_view(states):
    assert OR_CASCADE.itemsize == olib().or_sizeof_cascade()
    return states.view(OR_CASCADE).reshape(-1)


def _lstm_layer(ref, n):
    (i,) = list(ref.h[n])   # the reference nets have one LSTM layer
    return i


def _oracle_to_ref(st, ref):
    """or_cascade (one stream) -> the reference objects: the same fields."""
    ref.pcm[:] = st["ring"]
    ref.pcmbuf.idx_set, ref.pcmbuf.idx_data_latest = int(st["idx_set"]), int(st["idx_latest"])
    ref.cntrl.current_pos_seq = int(st["pos_seq"])
    ref.cntrl.cnt_timeout_kws, ref.cntrl.cnt_timeout_s2i = int(st["cnt_kws"]), int(st["cnt_s2i"])
    for n in range(3):
        o, q, fe = st["nnsp"][n], ref.nnsp[n], ref.feat[n]
        np.ctypeslib.as_array(fe.state_stftModule.dataBuffer)[:480] = o["buf"]
        np.ctypeslib.as_array(fe.normFeatContext)[:240] = o["ctx"]
        i = _lstm_layer(ref, n)
        N = len(ref.h[n][i])
        ref.h[n][i][:] = o["h"][0][:N]
        ref.c[n][i][:] = o["c"][0][:N]
        q.slides, q.trigger, q.argmax_last = int(o["slides"]), int(o["trigger"]), int(o["argmax_last"])
        for k in range(8):
            q.counts_category[k] = int(o["counts"][k])
        for k in range(3):
            q.outputs[k] = int(o["outputs"][k])


def _ref_to_oracle(ref, st):
    """the reference objects -> or_cascade (one stream)."""
    st["ring"] = ref.pcm
    st["idx_set"], st["idx_latest"] = ref.pcmbuf.idx_set, ref.pcmbuf.idx_data_latest
    st["pos_seq"] = ref.cntrl.current_pos_seq
    st["cnt_kws"], st["cnt_s2i"] = ref.cntrl.cnt_timeout_kws, ref.cntrl.cnt_timeout_s2i
    for n in range(3):
        o, q, fe = st["nnsp"][n], ref.nnsp[n], ref.feat[n]
        o["buf"] = np.ctypeslib.as_array(fe.state_stftModule.dataBuffer)[:480]
        o["ctx"] = np.ctypeslib.as_array(fe.normFeatContext)[:240]
        i = _lstm_layer(ref, n)
        N = len(ref.h[n][i])
        o["h"][0][:N] = ref.h[n][i]
        o["c"][0][:N] = ref.c[n][i]
        o["slides"], o["trigger"], o["argmax_last"] = q.slides, q.trigger, q.argmax_last
        o["counts"] = list(q.counts_category)
        o["outputs"] = list(q.outputs)


def _same(got, want, what):
    for g, w, name in zip(got, want, ("net_ran", "detected", "outputs3")):
        np.testing.assert_array_equal(g, w, err_msg=f"{what}: {name}")


def _oracle_chunks(oc, pcm):
    st = oc.new_states(pcm.shape[0])
    outs, states, t0 = [], [], 0
    for T in CHUNKS:
        r = oc.run(pcm[:, t0:t0 + T], st)
        st = r[3]
        outs.append(r[:3])
        states.append(st.copy())
        t0 += T
    return outs, states


@pytest.mark.parametrize("lb_s2i,lb_kws", [(37, 80), (99, 12)])
def test_cascade_state_ref_both_ways(lb_s2i, lb_kws):
    torch.cuda.set_device(0)
    S = 64
    pcm = _pcm(S, sum(CHUNKS), 31 + lb_s2i)
    oc, handles, gpu = _setup(lb_s2i, lb_kws)
    want, ostates = _oracle_chunks(oc, pcm)
    c1 = pcm[:, 100:190]
    c2 = pcm[:, 190:275]
    # ---- forward: the oracle's state after chunk 1 -> reference objects -> GPU
    refs = [RefStream(handles, SEQ) for _ in range(S)]
    ov = _or_view(ostates[1].copy())
    for s in range(S):
        _oracle_to_ref(ov[s], refs[s])
    b = gpu(S)
    b.set_state_ref(refs)
    _same(b.exec(c2), want[2], "GPU chunk 2 from the reference objects")
    # ---- reverse: the GPU's state after chunk 1 -> reference objects -> oracle
    a = gpu(S)
    _same(a.exec(pcm[:, :100]), want[0], "GPU chunk 0")
    _same(a.exec(c1), want[1], "GPU chunk 1")
    blob = a.get_state()
    fresh = blob[:, 16].astype(np.int8)
    pos = blob[:, 8].astype(np.int8)
    cur = np.array(SEQ)[pos]
    # the streams cover every STFT-buffer case of the current net
    assert {0, 1, 2} <= set(fresh.tolist()), np.bincount(fresh)
    assert {0, 1, 2} <= set(cur.tolist()), np.bincount(cur)
    back = [RefStream(handles, SEQ) for _ in range(S)]
    a.get_state_ref(back)
    st = oc.new_states(S)
    sv = _or_view(st)
    for s in range(S):
        _ref_to_oracle(back[s], sv[s])
    sv = sv.copy()   # (the run below advances st)
    r = oc.run(c2, st)
    _same(r[:3], want[2], "oracle chunk 2 from the GPU's reference objects")
    # the reference objects from the GPU hold what the oracle holds where the
    # reference reads them again: the controller, the voice buffer's look-back
    # frames, each net's context slots 1..5, LSTM state and post-processing
    H = max(lb_s2i, lb_kws) + 2
    ov1 = _or_view(ostates[1])
    for s in range(S):
        o, g = ov1[s], sv[s]
        assert (o["pos_seq"], o["cnt_kws"], o["cnt_s2i"]) == (g["pos_seq"], g["cnt_kws"], g["cnt_s2i"])
        oi = [(int(o["idx_latest"]) - j) % 100 for j in range(min(H, 100))]
        gi = [(int(g["idx_latest"]) - j) % 100 for j in range(min(H, 100))]
        np.testing.assert_array_equal(o["ring"][oi], g["ring"][gi])
        for n in range(3):
            for f in ("h", "c", "slides", "trigger", "argmax_last", "counts", "outputs"):
                np.testing.assert_array_equal(o["nnsp"][n][f], g["nnsp"][n][f], err_msg=f"stream {s} net {n} {f}")
            np.testing.assert_array_equal(o["nnsp"][n]["ctx"][40:], g["nnsp"][n]["ctx"][40:])
            np.testing.assert_array_equal(o["nnsp"][n]["buf"][160:], g["nnsp"][n]["buf"][160:],
                                          err_msg=f"stream {s} net {n} STFT buffer")
    # ---- round trip through the reference objects: the same blob, look-back
    #      features recomputed on the device included
    c = gpu(S)
    c.set_state_ref(back)
    got = c.get_state()
    if H > 100:
        # frame -H lies past the 100-frame voice buffer: the reference objects
        # hold it only as the STFT buffer of a current net at look-back H - 2
        # (ran >= 2 frames); elsewhere it is never read again, nor is the
        # look-back feature of frame -(H-2) that the device recomputes from it
        keep = (cur == 0) & (fresh == 2) & (lb_s2i == H - 2) | (cur == 2) & (fresh == 2) & (lb_kws == H - 2)
        look = 32 + H * 320 + 640
        for x in (got, blob):
            x[~keep, 32:32 + 320] = 0
            for n in range(3):
                x[~keep, look + n * (H - 2) * 80:look + n * (H - 2) * 80 + 80] = 0
        assert keep.any()
    bad = np.argwhere(got != blob)
    assert not len(bad), [(int(i), int(o), int(got[i, o]), int(blob[i, o]), int(fresh[i]), int(cur[i])) for i, o in bad[:20]]
    _same(c.exec(c2), want[2], "GPU chunk 2 after the round trip")
    for x in (a, b, c):
        x.close()


def test_cascade_state_ref_refuses_foreign_objects():
    torch.cuda.set_device(0)
    oc, handles, gpu = _setup(37, 80)
    a = gpu(4)
    refs = [RefStream(handles, SEQ) for _ in range(4)]
    a.get_state_ref(refs)   # a fresh cascade: every net reset, position 0
    a.set_state_ref(refs)
    L = _lib.lib()

    def code(rs):
        arr = (_lib.RefStreamC * len(rs))(*[r.c_struct() for r in rs])
        return L.nnsp_cascade_set_state_ref(a.h, 0, len(rs), C.addressof(arr))
    assert code(refs) == 0
    bad = RefStream(handles, (1, 2))   # another sequence length
    assert code([bad]) == _lib.NNSP_EINVAL
    bad = RefStream(handles, SEQ)
    bad.cntrl.current_pos_seq = 3       # past the sequence
    assert code([bad]) == _lib.NNSP_EINVAL
    bad = RefStream(handles, SEQ)
    bad.nnsp[2].nn_id = b"\x00"         # an NNSPClass of another NNSP_ID
    assert code([bad]) == _lib.NNSP_EINVAL
    bad = RefStream(handles, SEQ)
    np.ctypeslib.as_array(bad.feat[2].state_stftModule.dataBuffer)[300] = 7   # KWS not current, not reset
    assert code([bad]) == _lib.NNSP_EINVAL
    bad = RefStream(handles, SEQ)
    np.ctypeslib.as_array(bad.feat[1].state_stftModule.dataBuffer)[170] = 7   # VAD's buffer not the voice buffer's
    assert code([bad]) == _lib.NNSP_EINVAL
    bad = RefStream([handles[1], handles[1], handles[2]], SEQ)   # S2I's slot holds VAD's net (LSTM width)
    bad.nnsp[0].nn_id = b"\x00"
    assert code([bad]) == _lib.NNSP_EINVAL
    a.close()
