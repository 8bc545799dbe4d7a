"""ctypes view of libnnsp_mi355x.so (the C-ABI of include/nnsp_api.h and
include/nnsp_batch.h).

The library is built in-tree (``nnsp_amd/libnnsp_mi355x.so``, see
``__graft_entry__.build``).  Loading fails loudly when it is missing: there is
no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NNSP_LIB: another in-tree build of the same library (development A/B runs)
LIB_PATH = os.environ.get("NNSP_LIB") or os.path.join(HERE, "libnnsp_mi355x.so")

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


class NeuralNetClass(C.Structure):
    """ABI mirror of NeuralNetClass (reference neural_nets.h:15-32)."""
    _fields_ = [
        ("numlayers", C.c_int8),
        ("size_layer", C.c_int16 * 11),
        ("net_layer_type", C.c_int * 10),
        ("qbit_kernel", C.c_int8 * 10),
        ("qbit_input", C.c_int8 * 10),
        ("qbit_bias", C.c_int8 * 10),
        ("activation_type", C.c_int * 10),
        ("pt_cstate", C.c_void_p * 10),
        ("pt_hstate", C.c_void_p * 10),
        ("act_func", C.c_void_p * 10),
        ("layer_func", C.c_void_p * 10),
        ("pt_kernel", C.c_void_p * 10),
        ("pt_bias", C.c_void_p * 10),
        ("pt_kernel_rec", C.c_void_p * 10),
    ]


class stftModule(C.Structure):
    _fields_ = [("len_win", C.c_int16), ("hop", C.c_int16), ("len_fft", C.c_int16),
                ("dataBuffer", C.c_int16 * 512), ("window", C.c_void_p)]


class FeatureClass(C.Structure):
    _fields_ = [("state_stftModule", stftModule), ("feature", C.c_int32 * 50),
                ("normFeatContext", C.c_int16 * 300), ("num_context", C.c_int16),
                ("dim_feat", C.c_int16), ("pt_norm_mean", C.c_void_p),
                ("pt_norm_stdR", C.c_void_p), ("qbit_output", C.c_int8)]


class NNSPClass(C.Structure):
    _fields_ = [("nn_id", C.c_char), ("pt_net", C.c_void_p), ("pt_feat", C.c_void_p),
                ("slides", C.c_int8), ("trigger", C.c_int16), ("pt_thresh_prob", C.c_void_p),
                ("counts_category", C.c_int16 * 8), ("pt_th_count_trigger", C.c_void_p),
                ("num_dnsmpl", C.c_int16), ("outputs", C.c_int16 * 3), ("argmax_last", C.c_int16)]


class CascadeParams(C.Structure):
    """nnsp_cascade_params (include/nnsp_cascade.h), ParamCntrlClass subset."""
    _fields_ = [("frs_vbufBk_s2i", C.c_int16), ("thresh_timeout_s2i", C.c_int16),
                ("frs_vbufBk_kws", C.c_int16), ("thresh_timeout_kws", C.c_int16)]


class RefParams(C.Structure):
    """nnsp_ref_params: ABI mirror of ParamCntrlClass (evb/src/nnCntrlClass.h:11-31)."""
    _fields_ = [(n, C.c_int16) for n in (
        "thresh_prob_vad", "thresh_cnts_vad", "frs_vbufBk_s2i", "thresh_timeout_s2i", "thresh_prob_s2i",
        "thresh_cnts_s2i", "frs_vbufBk_kws", "thresh_timeout_kws", "thresh_prob_kws", "thresh_cnts_kws")]


class RefCntrl(C.Structure):
    """nnsp_ref_cntrl: ABI mirror of nnCntrlClass (evb/src/nnCntrlClass.h:35-45)."""
    _fields_ = [("pt_seq_cntrl", C.c_void_p), ("len_seq_cntrl", C.c_int8), ("current_pos_seq", C.c_int8),
                ("pt_nnsp_arry", C.c_void_p), ("Params", RefParams), ("cnt_timeout_kws", C.c_uint16),
                ("cnt_timeout_s2i", C.c_uint16), ("cnt_voice_frames_detected", C.c_uint16),
                ("cnt_voice_frames_not_detected", C.c_uint16)]


class RefPcmBuf(C.Structure):
    """nnsp_ref_pcmbuf: ABI mirror of PcmBufClass (evb/src/PcmBufClass.h:9-16)."""
    _fields_ = [("pcm_buffer", C.c_void_p), ("idx_set", C.c_int16), ("idx_data_latest", C.c_int16),
                ("num_frs", C.c_int16), ("smpls_fr", C.c_int16)]


class RefStreamC(C.Structure):
    """nnsp_ref_stream (include/nnsp_cascade.h)."""
    _fields_ = [("cntrl", C.c_void_p), ("pcmbuf", C.c_void_p), ("nnsp", C.c_void_p * 3)]


class PostState(C.Structure):
    _fields_ = [("slides", C.c_int16), ("trigger", C.c_int16), ("argmax_last", C.c_int16),
                ("pad0", C.c_int16), ("counts_category", C.c_int16 * 8),
                ("outputs", C.c_int16 * 3), ("pad1", C.c_int16)]


P = C.c_void_p
I = C.c_int
# error codes (include/nnsp_batch.h)
NNSP_EINVAL, NNSP_EUNSUPPORTED, NNSP_ENOMEM = -1, -2, -3


def _declare(L: C.CDLL) -> None:
    sig = {
        "nnsp_batch_create": (I, [C.POINTER(P), P, I, P, P, C.c_int16, C.c_int16, I, I]),
        "nnsp_batch_create_ex": (I, [C.POINTER(P), P, I, P, P, C.c_int16, C.c_int16, I, I, I]),
        "nnsp_batch_destroy": (None, [P]),
        "nnsp_batch_reset": (I, [P, P]),
        "nnsp_batch_exec": (I, [P, P, I, P, P, P]),
        "nnsp_batch_exec_device": (I, [P, P, I, P, P]),
        "nnsp_batch_sync": (I, [P]),
        "nnsp_batch_stream": (P, [P]),
        "nnsp_batch_streams": (I, [P]),
        "nnsp_batch_nout": (I, [P]),
        "nnsp_batch_features_device": (P, [P]),
        "nnsp_batch_last_timing": (I, [P, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
        "nnsp_batch_post_state": (I, [P, P]),
        "nnsp_batch_state_bytes": (C.c_size_t, [P]),
        "nnsp_batch_get_state": (I, [P, P, I, I]),
        "nnsp_batch_set_state": (I, [P, P, I, I]),
        "nnsp_cascade_create": (I, [C.POINTER(P), P, P, I, P]),
        "nnsp_cascade_destroy": (None, [P]),
        "nnsp_cascade_reset": (I, [P, P]),
        "nnsp_cascade_exec": (I, [P, P, I, P, P, P]),
        "nnsp_cascade_exec_device": (I, [P, P, I, P, P, P]),
        "nnsp_cascade_exec_device_ahead": (I, [P, P, I, P, I, P, P, P]),
        "nnsp_cascade_sync": (I, [P]),
        "nnsp_cascade_set_window": (I, [P, I]),
        "nnsp_cascade_set_timing": (I, [P, I]),
        "nnsp_cascade_set_serial": (I, [P, I]),
        "nnsp_cascade_get_window": (I, [P, C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
        "nnsp_cascade_stream": (P, [P]),
        "nnsp_cascade_last_stats": (I, [P, C.POINTER(I), C.POINTER(C.c_longlong), C.POINTER(C.c_float)]),
        "nnsp_cascade_positions": (I, [P, P]),
        "nnsp_cascade_state_bytes": (C.c_size_t, [P]),
        "nnsp_cascade_totals": (I, [P, P, P, P, P, P]),
        "nnsp_cascade_totals_reset": (I, [P]),
        "nnsp_cascade_get_state": (I, [P, P, I, I]),
        "nnsp_cascade_set_state": (I, [P, P, I, I]),
        "nnsp_cascade_set_state_ref": (I, [P, I, I, P]),
        "nnsp_cascade_get_state_ref": (I, [P, I, I, P]),
        "nnsp_cascade_last_rounds": (I, [P, I, P, P, P]),
        "nnsp_cascade_last_fe_stats": (I, [P, C.POINTER(C.c_float)]),
        "nnsp_cascade_last_net_stats": (I, [P, I, C.POINTER(C.c_longlong), C.POINTER(C.c_float),
                                            C.POINTER(C.c_float), C.POINTER(I)]),
        "nnsp_synth_pcm": (I, [P, I, I, C.c_uint64, I, C.c_int64, I, P]),
        "nnsp_synth_pcm_mix": (I, [P, I, I, C.c_uint64, I, C.c_int64, I, P, I, I, I, P]),
        "nnsp_device_count": (I, [C.POINTER(I)]),
        "nnsp_set_device": (I, [I]),
        "nnsp_device_info": (I, [C.POINTER(I), C.POINTER(I), C.c_char_p, I]),
        "nnsp_strerror": (C.c_char_p, [I]),
        "NNSPClass_init": (I, [P, P, P, C.c_char, P, P, P, P]),
        "NNSPClass_reset": (I, [P]),
        "NNSPClass_exec": (C.c_int16, [P, P]),
        "NeuralNetClass_exe": (None, [P, P, P, C.c_int8]),
        "NeuralNetClass_setDefault": (None, [P]),
        "FeatureClass_construct": (None, [P, P, P, C.c_int8]),
        "FeatureClass_setDefault": (None, [P]),
        "FeatureClass_execute": (None, [P, P]),
        "arm_fft_exec": (None, [P, P]),
        "spec2pspec_arm": (None, [P, P, I]),
        "melSpecProc": (None, [P, P]),
        "log10_vec": (None, [P, P, C.c_int32, C.c_int16]),
        "my_log10": (None, [P, C.c_int32]),
        "norm_oneTwo": (None, [C.c_int32, P, P]),
        "compute_pwr2": (C.c_int32, [C.c_int32]),
        "ceiling": (C.c_int32, [C.c_int32]),
        "my_argmax": (None, [P, I, P]),
        "binary_post_proc": (None, [P, P, P]),
        "s2i_post_proc": (None, [P, P, P]),
        "tanh_fix": (P, [P, P, I]),
        "sigmoid_fix": (P, [P, P, I]),
        "relu6_fix": (P, [P, P, I]),
        "linear_fix": (P, [P, P, I]),
        "affine_Krows_8x16": (I, [C.c_int16, C.POINTER(P), C.POINTER(P), C.POINTER(P), P, C.c_int16, C.c_int16,
                                  C.c_int16, C.c_int16, P, C.c_int8, P]),
        "affine_Krows_8x16_acc32b": (I, [C.c_int16, C.POINTER(P), C.POINTER(P), C.POINTER(P), P, C.c_int16,
                                         C.c_int16, C.c_int16, C.c_int16, P, C.c_int8, P]),
        "rc_Krows_8x16": (I, [C.c_int16, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P), P, P, C.c_int16,
                              C.c_int16, C.c_int16, C.c_int16, C.c_int16, C.c_int16, P]),
        "rc_Krows_8x16_acc32b": (I, [C.c_int16, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P), P, P,
                                     C.c_int16, C.c_int16, C.c_int16, C.c_int16, C.c_int16, C.c_int16, P]),
        "rc_8x16": (I, [P, P, P, P, P, P, C.c_int16, C.c_int16, C.c_int16, C.c_int16, C.c_int16, C.c_int16,
                        C.c_int16, I, P]),
        "rc_8x16_acc32b": (I, [P, P, P, P, P, P, C.c_int16, C.c_int16, C.c_int16, C.c_int16, C.c_int16,
                               C.c_int16, C.c_int16, I, P]),
        "shift_64b": (None, [P, C.c_int8, I]),
        "shift_32b": (None, [P, C.c_int8, I]),
        "arm_fft_init": (None, []),
        # the ARM_OPTIMIZED=0 build (row N4)
        "nnsp_set_arm_optimized": (I, [I]),
        "nnsp_get_arm_optimized": (I, []),
        "rfft": (None, [I, P, P]),
        "fft": (None, [I, P, P]),
        "spec2pspec": (None, [P, P, I]),
        "stftModule_analyze": (I, [P, P, P]),
        "stftModule_setDefault": (I, [P]),
    }
    for name, (res, args) in sig.items():
        try:
            f = getattr(L, name)
        except AttributeError:
            # NNSP_LIB (development A/B against an older in-tree build): symbols
            # added since are absent there (has() says so); the shipped library
            # must export every one
            if os.environ.get("NNSP_LIB"):
                continue
            raise
        f.restype = res
        f.argtypes = args


def has(name: str) -> bool:
    """The loaded library exports `name` (False only for an older NNSP_LIB build)."""
    return hasattr(lib(), name)


def check(code: int, what: str = "") -> None:
    if code != 0:
        msg = lib().nnsp_strerror(code)
        raise RuntimeError(f"{what}: libnnsp_mi355x error {code}: {msg.decode() if msg else ''}")


def fn_addr(name: str) -> int:
    return C.cast(getattr(lib(), name), C.c_void_p).value


def ptr(a: np.ndarray | None) -> int | None:
    return None if a is None else a.ctypes.data


class NetHandle:
    """A NeuralNetClass built from nnsp_amd.nets.NetData, holding every buffer
    it points to (packed weights exactly as a def_nn*.c file holds them)."""

    def __init__(self, data, acc32: bool = False, arm_optimized: bool = True):
        from .nets import LSTM, LINEAR
        spec = data.spec
        # the byte order the reference build reads (ARM_OPTIMIZED 1: interleaved; 0: portable)
        Wp, Wrp, Bp = data.packed() if arm_optimized else data.packed_portable()
        self.data = data
        self.keep = []
        n = NeuralNetClass()
        n.numlayers = spec.nl
        for i, s in enumerate(spec.sizes):
            n.size_layer[i] = s
        names = {0: "relu6_fix", 1: "tanh_fix", 2: "sigmoid_fix", 3: "linear_fix"}
        self.h, self.c = [None] * spec.nl, [None] * spec.nl
        for i, t in enumerate(spec.types):
            a32 = acc32 or bool(spec.accs and spec.accs[i])   # per-layer layer_func (mixed nets)
            n.net_layer_type[i] = t
            n.qbit_kernel[i] = spec.qk[i]
            n.qbit_input[i] = spec.qi[i]
            n.qbit_bias[i] = spec.qb[i]
            n.activation_type[i] = {0: 0, 1: 1, 2: 2, 3: 3}[spec.acts[i]]
            n.act_func[i] = fn_addr(names[spec.acts[i]])
            if t == LSTM:
                lf = "lstm_8x16_acc32b" if a32 else "lstm_8x16"
                N = spec.sizes[i + 1]
                self.h[i] = np.zeros(N, np.int16)
                self.c[i] = np.zeros(N, np.int32)
                n.pt_hstate[i] = ptr(self.h[i])
                n.pt_cstate[i] = ptr(self.c[i])
            else:
                lf = "fc_8x16_acc32b" if a32 else "fc_8x16"
            n.layer_func[i] = fn_addr(lf)
            w = np.ascontiguousarray(Wp[i]).view(np.int8)
            b = np.ascontiguousarray(Bp[i]).astype(np.int16)
            self.keep += [w, b]
            n.pt_kernel[i] = ptr(w)
            n.pt_bias[i] = ptr(b)
            if Wrp[i] is not None:
                wr = np.ascontiguousarray(Wrp[i]).view(np.int8)
                self.keep.append(wr)
                n.pt_kernel_rec[i] = ptr(wr)
        self.net = n
        self.mean = np.ascontiguousarray(data.mean, np.int32)
        self.stdR = np.ascontiguousarray(data.stdR, np.int32)
        del LINEAR

    @property
    def addr(self) -> int:
        return C.addressof(self.net)
