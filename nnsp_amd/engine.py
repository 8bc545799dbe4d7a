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
from .nets import NN_ID, THRESH_CNTS, THRESH_PROB, NetData, synth_net


class NNSPBatch:
    def __init__(self, net: NetData | str, n_streams: int, max_frames: int, acc32: bool = False,
                 thresh_prob: int = THRESH_PROB, th_count: int = THRESH_CNTS, seed: int = 1234):
        if isinstance(net, str):
            net = synth_net(net, seed)
        self.data = net
        self.handle = _lib.NetHandle(net, acc32=acc32)
        self.S, self.Tmax = n_streams, max_frames
        self.nn_id = NN_ID[net.spec.name]
        L = _lib.lib()
        h = C.c_void_p()
        _lib.check(L.nnsp_batch_create(C.byref(h), self.handle.addr, self.nn_id,
                                       _lib.ptr(self.handle.mean), _lib.ptr(self.handle.stdR),
                                       thresh_prob, th_count, n_streams, max_frames),
                   "nnsp_batch_create")
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
        buf = np.ascontiguousarray(buf, np.uint8)
        _lib.check(_lib.lib().nnsp_batch_set_state(self.h, _lib.ptr(buf), 0, self.S), "set_state")


def device_info() -> dict:
    cu, clk = C.c_int(), C.c_int()
    arch = C.create_string_buffer(64)
    _lib.check(_lib.lib().nnsp_device_info(C.byref(cu), C.byref(clk), arch, 64), "device_info")
    return {"compute_units": cu.value, "clock_khz": clk.value, "arch": arch.value.decode()}
