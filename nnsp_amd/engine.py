"""Python host mirror of the batched C-ABI (include/nnsp_batch.h).

``NNSPBatch`` is the multi-stream counterpart of the reference's
``NNSPClass_init`` / ``NNSPClass_reset`` / ``NNSPClass_exec``
(ns-nnsp/src/nn_speech.c:23-127): S streams share one net, each keeps its own
front-end, LSTM and post-processing state on the GPU, and every call advances
all streams by a chunk of T frames.  Host arrays are numpy; device buffers can
be passed as raw pointers (e.g. ``torch.Tensor.data_ptr()``) to
``exec_device``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .nets import LOOKBACK, NN_ID, THRESH_CNTS, THRESH_PROB, TIMEOUT, NetData, synth_net


class NNSPBatch:
    def __init__(self, net: NetData | str, n_streams: int, max_frames: int, acc32: bool = False,
                 thresh_prob: int = THRESH_PROB, th_count: int = THRESH_CNTS, seed: int = 1234,
                 arm_optimized: bool = True):
        """arm_optimized=False: the reference built with ARM_OPTIMIZED=0 (row N4):
        portable front end and weight byte order (nnsp_batch_create_ex)."""
        if isinstance(net, str):
            net = synth_net(net, seed)
        self.data = net
        self.handle = _lib.NetHandle(net, acc32=acc32, arm_optimized=arm_optimized)
        self.S, self.Tmax = n_streams, max_frames
        self.nn_id = net.spec.nn_id
        L = _lib.lib()
        h = C.c_void_p()
        _lib.check(L.nnsp_batch_create_ex(C.byref(h), self.handle.addr, self.nn_id,
                                          _lib.ptr(self.handle.mean), _lib.ptr(self.handle.stdR),
                                          thresh_prob, th_count, n_streams, max_frames, int(bool(arm_optimized))),
                   "nnsp_batch_create_ex")
        self.h = h
        self.nout = L.nnsp_batch_nout(h)

    def close(self) -> None:
        if getattr(self, "h", None):
            _lib.lib().nnsp_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, mask: np.ndarray | None = None) -> None:
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        _lib.check(_lib.lib().nnsp_batch_reset(self.h, _lib.ptr(m)), "nnsp_batch_reset")

    def exec(self, pcm: np.ndarray, want_logits: bool = False, want_features: bool = False):
        """pcm [S][T][160] int16 -> (trig [S][T], logits [S][T][nout] | None, feats | None)."""
        pcm = np.ascontiguousarray(pcm, np.int16)
        S, T, F = pcm.shape
        assert S == self.S and F == 160 and 1 <= T <= self.Tmax
        trig = np.zeros((S, T), np.int16)
        logits = np.zeros((S, T, self.nout), np.int32) if want_logits else None
        feats = np.zeros((S, T, 40), np.int16) if want_features else None
        _lib.check(_lib.lib().nnsp_batch_exec(self.h, _lib.ptr(pcm), T, _lib.ptr(trig),
                                              _lib.ptr(logits), _lib.ptr(feats)), "nnsp_batch_exec")
        return trig, logits, feats

    def exec_device(self, pcm_ptr: int, T: int, trig_ptr: int | None = None,
                    logits_ptr: int | None = None) -> None:
        _lib.check(_lib.lib().nnsp_batch_exec_device(self.h, pcm_ptr, T, trig_ptr, logits_ptr),
                   "nnsp_batch_exec_device")

    def sync(self) -> None:
        _lib.check(_lib.lib().nnsp_batch_sync(self.h), "nnsp_batch_sync")

    @property
    def stream(self) -> int:
        return _lib.lib().nnsp_batch_stream(self.h)

    def last_timing(self) -> tuple[float, float]:
        fe, nn = C.c_float(), C.c_float()
        _lib.check(_lib.lib().nnsp_batch_last_timing(self.h, C.byref(fe), C.byref(nn)), "timing")
        return fe.value, nn.value

    def post_state(self) -> np.ndarray:
        out = (_lib.PostState * self.S)()
        _lib.check(_lib.lib().nnsp_batch_post_state(self.h, C.addressof(out)), "post_state")
        return np.frombuffer(out, dtype=np.int16).reshape(self.S, 16).copy()

    def get_state(self) -> np.ndarray:
        per = _lib.lib().nnsp_batch_state_bytes(self.h)
        buf = np.zeros((self.S, per), np.uint8)
        _lib.check(_lib.lib().nnsp_batch_get_state(self.h, _lib.ptr(buf), 0, self.S), "get_state")
        return buf

    def set_state(self, buf: np.ndarray) -> None:
        per = _lib.lib().nnsp_batch_state_bytes(self.h)
        if buf.ndim != 2 or buf.shape != (self.S, per):
            raise ValueError(f"set_state: blobs of shape {buf.shape}, this batch takes ({self.S}, {per})")
        buf = np.ascontiguousarray(buf, np.uint8)
        _lib.check(_lib.lib().nnsp_batch_set_state(self.h, _lib.ptr(buf), 0, self.S), "set_state")


class NNSPCascade:
    """Batched nnCntrlClass (evb/src/nnCntrlClass.c:57-272): three NNSPBatch
    objects (s2i, vad, kws; same stream count) driven by the VAD -> KWS -> S2I
    sequence controller.  ``seq`` lists NNSP_IDs per position (default
    vad, kws, s2i as in the reference's main)."""

    def __init__(self, nets: dict, seq=(1, 2, 0), lookback_s2i: int = LOOKBACK,
                 timeout_s2i: int = TIMEOUT, lookback_kws: int = LOOKBACK, timeout_kws: int = TIMEOUT):
        self.nets = nets   # keep the batches alive
        order = [nets["s2i"], nets["vad"], nets["kws"]]
        self.S, self.Tmax = order[0].S, min(b.Tmax for b in order)
        arr = (C.c_void_p * 3)(*[b.h.value for b in order])
        sq = np.ascontiguousarray(seq, np.int8)
        prm = _lib.CascadeParams(lookback_s2i, timeout_s2i, lookback_kws, timeout_kws)
        h = C.c_void_p()
        _lib.check(_lib.lib().nnsp_cascade_create(C.byref(h), C.addressof(arr), _lib.ptr(sq), len(sq),
                                                  C.addressof(prm)), "nnsp_cascade_create")
        self.h = h

    def close(self) -> None:
        if getattr(self, "h", None):
            _lib.lib().nnsp_cascade_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, mask: np.ndarray | None = None) -> None:
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        _lib.check(_lib.lib().nnsp_cascade_reset(self.h, _lib.ptr(m)), "nnsp_cascade_reset")

    def exec(self, pcm: np.ndarray):
        """pcm [S][T][160] -> net_ran [S][T] int8, detected [S][T] int16, outputs3 [S][T][3]."""
        pcm = np.ascontiguousarray(pcm, np.int16)
        S, T, F = pcm.shape
        assert S == self.S and F == 160 and 1 <= T <= self.Tmax
        ran = np.zeros((S, T), np.int8)
        det = np.zeros((S, T), np.int16)
        o3 = np.zeros((S, T, 3), np.int16)
        _lib.check(_lib.lib().nnsp_cascade_exec(self.h, _lib.ptr(pcm), T, _lib.ptr(ran), _lib.ptr(det),
                                                _lib.ptr(o3)), "nnsp_cascade_exec")
        return ran, det, o3

    def exec_device(self, pcm_ptr: int, T: int, ran_ptr=None, det_ptr=None, o3_ptr=None,
                    next_ptr: int | None = None, next_T: int = 0) -> None:
        """Device buffers; next_ptr: the chunk the next call will get (its front
        end then runs ahead, overlapped with this chunk's nets)."""
        _lib.check(_lib.lib().nnsp_cascade_exec_device_ahead(self.h, pcm_ptr, T, next_ptr, next_T if next_ptr else 0,
                                                             ran_ptr, det_ptr, o3_ptr), "nnsp_cascade_exec_device")

    def sync(self) -> None:
        _lib.check(_lib.lib().nnsp_cascade_sync(self.h), "nnsp_cascade_sync")

    def set_window(self, frames: int) -> None:
        """Frames per stream and round (0: to the chunk end; -1: automatic)."""
        _lib.check(_lib.lib().nnsp_cascade_set_window(self.h, frames), "nnsp_cascade_set_window")

    def window(self) -> tuple[int, bool, int]:
        """(window of the next chunk, automatic?, net-switch cuts in the last chunk)"""
        w, a, n = C.c_int(), C.c_int(), C.c_int()
        _lib.check(_lib.lib().nnsp_cascade_get_window(self.h, C.byref(w), C.byref(a), C.byref(n)), "get_window")
        return w.value, bool(a.value), n.value

    def set_serial(self, on: bool) -> None:
        """The nets' work of a round one after another on one stream (instrumentation)."""
        _lib.check(_lib.lib().nnsp_cascade_set_serial(self.h, int(on)), "nnsp_cascade_set_serial")

    def set_timing(self, on: bool) -> None:
        """Per-round, per-net device timing for net_stats (off by default)."""
        _lib.check(_lib.lib().nnsp_cascade_set_timing(self.h, int(on)), "nnsp_cascade_set_timing")

    @property
    def stream(self) -> int:
        return _lib.lib().nnsp_cascade_stream(self.h)

    def last_stats(self) -> tuple[int, int, float]:
        r, f, ms = C.c_int(), C.c_longlong(), C.c_float()
        _lib.check(_lib.lib().nnsp_cascade_last_stats(self.h, C.byref(r), C.byref(f), C.byref(ms)), "stats")
        return r.value, f.value, ms.value

    def totals(self) -> dict:
        """Running totals since create / totals_reset (nnsp_cascade_totals)."""
        ch, r, f = C.c_longlong(), C.c_longlong(), C.c_longlong()
        fe, cm = C.c_double(), C.c_double()
        _lib.check(_lib.lib().nnsp_cascade_totals(self.h, C.byref(ch), C.byref(r), C.byref(f), C.byref(fe),
                                                  C.byref(cm)), "totals")
        return {"chunks": ch.value, "rounds": r.value, "frames_run": f.value, "fe_ms": fe.value,
                "chunk_ms": cm.value}

    def totals_reset(self) -> None:
        _lib.check(_lib.lib().nnsp_cascade_totals_reset(self.h), "totals_reset")

    def net_stats(self, name: str) -> tuple[int, float, float, int]:
        """(frames scheduled, fe ms, nn ms, launches) of one net in the last chunk."""
        f, fe, nn, n = C.c_longlong(), C.c_float(), C.c_float(), C.c_int()
        _lib.check(_lib.lib().nnsp_cascade_last_net_stats(self.h, NN_ID[name], C.byref(f), C.byref(fe),
                                                          C.byref(nn), C.byref(n)), "net_stats")
        return f.value, fe.value, nn.value, n.value

    def fe_stats(self) -> float:
        """Device ms of the shared front end (log-Mel of every frame) in the last chunk."""
        ms = C.c_float()
        _lib.check(_lib.lib().nnsp_cascade_last_fe_stats(self.h, C.byref(ms)), "fe_stats")
        return ms.value

    def round_stats(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Last chunk, [round][net id]: streams listed, cold-FE ms, NN ms (ms only with timing on)."""
        lists = np.zeros((32, 3), np.int32)
        fe = np.zeros((32, 3), np.float32)
        nn = np.zeros((32, 3), np.float32)
        n = _lib.lib().nnsp_cascade_last_rounds(self.h, 32, _lib.ptr(lists), _lib.ptr(fe), _lib.ptr(nn))
        if n < 0:
            _lib.check(n, "nnsp_cascade_last_rounds")
        return lists[:n], fe[:n], nn[:n]

    def get_state(self, first: int = 0, count: int | None = None) -> np.ndarray:
        """Per-stream state blobs [count][state_bytes] (include/nnsp_cascade.h:
        header, PCM history, STFT tail, look-back features, 3 net states)."""
        count = self.S - first if count is None else count
        per = _lib.lib().nnsp_cascade_state_bytes(self.h)
        buf = np.zeros((count, per), np.uint8)
        _lib.check(_lib.lib().nnsp_cascade_get_state(self.h, _lib.ptr(buf), first, count), "nnsp_cascade_get_state")
        return buf

    def set_state(self, buf: np.ndarray, first: int = 0) -> None:
        per = _lib.lib().nnsp_cascade_state_bytes(self.h)
        if buf.ndim != 2 or buf.shape[1] != per or first < 0 or first + buf.shape[0] > self.S:
            raise ValueError(f"set_state: blobs of shape {buf.shape} at stream {first}; this cascade takes "
                             f"[<= {self.S - first}][{per}]")
        buf = np.ascontiguousarray(buf, np.uint8)
        _lib.check(_lib.lib().nnsp_cascade_set_state(self.h, _lib.ptr(buf), first, buf.shape[0]),
                   "nnsp_cascade_set_state")

    def set_state_ref(self, refs: list, first: int = 0) -> None:
        """Streams first.. take the state held by the reference objects of
        each RefStream (nnsp_cascade_set_state_ref)."""
        arr = (_lib.RefStreamC * len(refs))(*[r.c_struct() for r in refs])
        _lib.check(_lib.lib().nnsp_cascade_set_state_ref(self.h, first, len(refs), C.addressof(arr)),
                   "nnsp_cascade_set_state_ref")

    def get_state_ref(self, refs: list, first: int = 0) -> None:
        """The state of streams first.. into each RefStream's reference objects
        (nnsp_cascade_get_state_ref)."""
        arr = (_lib.RefStreamC * len(refs))(*[r.c_struct() for r in refs])
        _lib.check(_lib.lib().nnsp_cascade_get_state_ref(self.h, first, len(refs), C.addressof(arr)),
                   "nnsp_cascade_get_state_ref")

    def positions(self) -> np.ndarray:
        pos = np.zeros(self.S, np.int8)
        _lib.check(_lib.lib().nnsp_cascade_positions(self.h, _lib.ptr(pos)), "positions")
        return pos


def device_info() -> dict:
    cu, clk = C.c_int(), C.c_int()
    arch = C.create_string_buffer(64)
    _lib.check(_lib.lib().nnsp_device_info(C.byref(cu), C.byref(clk), arch, 64), "device_info")
    return {"compute_units": cu.value, "clock_khz": clk.value, "arch": arch.value.decode()}


class RefStream:
    """One stream's state in the reference's own per-stream objects, as a
    single-stream reference application holds them: an nnCntrlClass, its
    PcmBufClass (num_frs x 160 voice buffer) and, by NNSP_ID, an NNSPClass
    with its FeatureClass and NeuralNetClass (the LSTM state in this stream's
    own h / c arrays).  ``handles``: _lib.NetHandle per NNSP_ID (s2i, vad,
    kws), whose layer tables the NeuralNetClass copies share."""

    def __init__(self, handles: list, seq=(1, 2, 0), num_frs: int = 100):
        self.seq = np.ascontiguousarray(seq, np.int8)
        self.cntrl = _lib.RefCntrl()
        self.cntrl.pt_seq_cntrl = self.seq.ctypes.data
        self.cntrl.len_seq_cntrl = len(seq)
        self.pcm = np.zeros((num_frs, 160), np.int16)
        self.pcmbuf = _lib.RefPcmBuf(self.pcm.ctypes.data, 0, num_frs - 1, num_frs, 160)
        self.feat = [_lib.FeatureClass() for _ in range(3)]
        self.net, self.h, self.c, self.nnsp = [], [], [], []
        for n, hd in enumerate(handles):
            net = _lib.NeuralNetClass.from_buffer_copy(hd.net)
            hs, cs = {}, {}
            for i in range(net.numlayers):
                if net.net_layer_type[i] == 1:   # lstm
                    N = net.size_layer[i + 1]
                    hs[i], cs[i] = np.zeros(N, np.int16), np.zeros(N, np.int32)
                    net.pt_hstate[i], net.pt_cstate[i] = hs[i].ctypes.data, cs[i].ctypes.data
            q = _lib.NNSPClass()
            q.nn_id = bytes([n])
            q.pt_net = C.addressof(net)
            q.pt_feat = C.addressof(self.feat[n])
            self.net.append(net)
            self.h.append(hs)
            self.c.append(cs)
            self.nnsp.append(q)

    def c_struct(self) -> "_lib.RefStreamC":
        r = _lib.RefStreamC()
        r.cntrl = C.addressof(self.cntrl)
        r.pcmbuf = C.addressof(self.pcmbuf)
        for n in range(3):
            r.nnsp[n] = C.addressof(self.nnsp[n])
        return r
