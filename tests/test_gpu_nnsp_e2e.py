"""NNSPClass_exec end to end on the GPU against the reference's OWN portable
build (tests/golden/ref_nnsp_portable.npz, written by
make_golden.py nnsp from oracle/_ref/libnnsp_ref_nnsp_portable.so =
nn_speech.c + the ARM_OPTIMIZED=0 front end and NN).  No oracle in between:

* the batched engine built for the portable reference
  (nnsp_batch_create_ex(..., arm_optimized = 0)) over ragged chunks whose
  boundaries include the mid-stream reset: per frame the NNSPClass_exec
  return and normFeatContext[200:240]; outputs[3] and counts_category at every
  chunk end; the final LSTM h / c (nnsp_batch_get_state); then a run of
  one-frame chunks for outputs[3] / counts_category on every frame;
* the drop-in NNSPClass_init / _reset / _exec (nnsp_set_arm_optimized(0)),
  frame by frame: return, features, outputs[3], counts_category, final h / c.

The three reference nets, acc64 and acc32, three wavs x 1000 frames and eight
synthetic streams x 200 frames."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from nnsp_e2e import fixture, groups, streams

from nnsp_amd import _lib
from nnsp_amd.engine import NNSPBatch
from nnsp_amd.nets import NN_ID, ref_net

pytestmark = pytest.mark.gpu

NAMES = ["vad", "kws", "s2i"]
CHUNKS = {1000: [100, 311, 200, 1, 88, 300], 200: [50, 47, 3, 100]}   # boundaries at the resets (611, 97)


@pytest.fixture(scope="module")
def g():
    return fixture()


def _lstm_width(data):
    sp = data.spec
    return sp.sizes[1 + sp.types.index(1)] if 1 in sp.types else 0


def _state_hc(eng, N):
    st = eng.get_state()
    h = st[:, 1040:1040 + 256].copy().view(np.int16)[:, :N]
    c = st[:, 1296:1296 + 512].copy().view(np.int32)[:, :N]
    return h, c


@pytest.mark.parametrize("acc", [64, 32])
@pytest.mark.parametrize("name", NAMES)
def test_portable_batch_vs_reference_nnsp_exec(g, name, acc):
    data = ref_net(name)
    N = _lstm_width(data)
    tag = f"{name}_{acc}"
    for gi, (pcm, reset_at, rows) in enumerate(groups(g)):
        S, T, _ = pcm.shape
        eng = NNSPBatch(data, S, max(CHUNKS[T]), acc32=acc == 32, arm_optimized=False)
        assert _lib.lib().nnsp_batch_state_bytes(eng.h) == 1040 + 768 + 32
        t0 = 0
        for Tc in CHUNKS[T]:
            if t0 == reset_at:
                eng.reset()
            trig, _, ft = eng.exec(pcm[:, t0:t0 + Tc], want_features=True)
            r = rows[:, t0:t0 + Tc]
            np.testing.assert_array_equal(ft, g[f"{name}_feats"][r], err_msg=f"{tag} group {gi} features @{t0}")
            np.testing.assert_array_equal(trig, g[f"{tag}_trig"][r], err_msg=f"{tag} group {gi} return @{t0}")
            ps = eng.post_state()
            last = rows[:, t0 + Tc - 1]
            np.testing.assert_array_equal(ps[:, 12:15], g[f"{tag}_outputs"][last], err_msg=f"{tag} outputs @{t0}")
            np.testing.assert_array_equal(ps[:, 4:12], g[f"{tag}_counts"][last], err_msg=f"{tag} counts @{t0}")
            t0 += Tc
        h, c = _state_hc(eng, N)
        first = 0 if gi == 0 else 3
        np.testing.assert_array_equal(h, g[f"{tag}_h"][first:first + S], err_msg=f"{tag} final h")
        np.testing.assert_array_equal(c, g[f"{tag}_c"][first:first + S], err_msg=f"{tag} final c")
        eng.close()
        # one-frame chunks: outputs[3] and counts_category on every frame
        eng = NNSPBatch(data, S, 1, acc32=acc == 32, arm_optimized=False)
        for t in range(T):
            if t == reset_at:
                eng.reset()
            trig, _, _ = eng.exec(pcm[:, t:t + 1])
            ps = eng.post_state()
            np.testing.assert_array_equal(trig[:, 0], g[f"{tag}_trig"][rows[:, t]])
            np.testing.assert_array_equal(ps[:, 12:15], g[f"{tag}_outputs"][rows[:, t]], err_msg=f"{tag} outputs @{t}")
            np.testing.assert_array_equal(ps[:, 4:12], g[f"{tag}_counts"][rows[:, t]], err_msg=f"{tag} counts @{t}")
        eng.close()


@pytest.fixture(scope="module")
def portable_dropin():
    L = _lib.lib()
    assert L.nnsp_set_arm_optimized(0) == 0
    yield L
    L.nnsp_set_arm_optimized(1)


_KEEP = []


@pytest.mark.parametrize("acc", [64, 32])
@pytest.mark.parametrize("name", NAMES)
def test_dropin_nnsp_exec_vs_reference_nnsp_exec(g, portable_dropin, name, acc):
    L = portable_dropin
    data = ref_net(name)
    N = _lstm_width(data)
    tag = f"{name}_{acc}"
    h = _lib.NetHandle(data, acc32=acc == 32, arm_optimized=False)
    thr, cnt = np.array([16383], np.int16), np.array([4], np.int16)
    _KEEP.extend([h, thr, cnt])
    lstm = data.spec.types.index(1)
    for i, (pcm, reset_at, r0) in enumerate(streams(g)):
        feat, inst = _lib.FeatureClass(), _lib.NNSPClass()
        assert L.NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([NN_ID[name]]),
                                O.p(h.mean), O.p(h.stdR), O.p(thr), O.p(cnt)) == 0
        L.NNSPClass_reset(C.byref(inst))
        for t in range(len(pcm)):
            if t == reset_at:
                L.NNSPClass_reset(C.byref(inst))
            fr = np.ascontiguousarray(pcm[t], np.int16)
            got = L.NNSPClass_exec(C.byref(inst), O.p(fr))
            assert got == g[f"{tag}_trig"][r0 + t], f"{tag} stream {i} frame {t}"
            np.testing.assert_array_equal(np.ctypeslib.as_array(feat.normFeatContext)[200:240],
                                          g[f"{name}_feats"][r0 + t], err_msg=f"{tag} stream {i} frame {t}")
            assert list(inst.outputs) == list(g[f"{tag}_outputs"][r0 + t]), f"{tag} stream {i} frame {t}"
            assert list(inst.counts_category) == list(g[f"{tag}_counts"][r0 + t]), f"{tag} stream {i} frame {t}"
        np.testing.assert_array_equal(h.h[lstm][:N], g[f"{tag}_h"][i], err_msg=f"{tag} stream {i} final h")
        np.testing.assert_array_equal(h.c[lstm][:N], g[f"{tag}_c"][i], err_msg=f"{tag} stream {i} final c")
    assert L.nnsp_legacy_status() == 0
