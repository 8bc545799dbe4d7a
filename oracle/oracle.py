"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU oracle (liboracle.so,
a scalar restatement of the reference path; see nnsp_oracle.h for what is
pinned and how).  Imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NNSP_ORACLE_LIB: another build of nnsp_oracle.c (bench.py's cpu_baseline
# compiles one with -march=native on the host it runs on)
LIB = os.environ.get("NNSP_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
REF = os.path.join(HERE, "_ref", "libnnsp_ref_partial.so")

MAXL = 10
MAX_LSTM, MAX_WIDTH = 10, 304   # nnsp_oracle.h OR_MAX_LSTM / OR_MAX_WIDTH


class or_net(C.Structure):
    _fields_ = [("nl", C.c_int32), ("size", C.c_int32 * (MAXL + 1)), ("type", C.c_int32 * MAXL),
                ("qk", C.c_int32 * MAXL), ("qi", C.c_int32 * MAXL), ("qb", C.c_int32 * MAXL),
                ("act", C.c_int32 * MAXL), ("acc32", C.c_int32), ("W", C.c_void_p * MAXL),
                ("Wr", C.c_void_p * MAXL), ("B", C.c_void_p * MAXL), ("portable", C.c_int32),
                ("acc32_layer", C.c_int32 * MAXL)]


class or_cfg(C.Structure):
    _fields_ = [("nn_id", C.c_int32), ("thresh_prob", C.c_int32), ("th_count", C.c_int32),
                ("qbit_out", C.c_int32), ("mean", C.c_void_p), ("stdR", C.c_void_p),
                ("fe_portable", C.c_int32)]


class or_cascade_cfg(C.Structure):
    _fields_ = [("net", C.c_void_p * 3), ("cfg", or_cfg * 3), ("seq", C.c_int32 * 3),
                ("len_seq", C.c_int32), ("lookback_kws", C.c_int32), ("lookback_s2i", C.c_int32),
                ("timeout_kws", C.c_int32), ("timeout_s2i", C.c_int32)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "liboracle.so"], cwd=HERE)
        _lib = C.CDLL(LIB)
        _lib.or_log10.restype = C.c_int32
        _lib.or_log10.argtypes = [C.c_int32]
        _lib.or_pwr2.restype = C.c_int32
        _lib.or_pwr2.argtypes = [C.c_int32]
        _lib.or_ceiling.restype = C.c_int32
        _lib.or_ceiling.argtypes = [C.c_int32]
        _lib.or_nnsp_exec.restype = C.c_int16
        _lib.or_cascade_exec.restype = C.c_int32
        _lib.or_sizeof_stream.restype = C.c_int32
        _lib.or_sizeof_cascade.restype = C.c_int32
    return _lib


def p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


class OracleNet:
    """or_net + or_cfg built from nnsp_amd.nets.NetData (packed byte layout)."""

    def __init__(self, data, acc32: bool = False, thresh_prob: int = 32767 >> 1, th_count: int = 4,
                 portable: bool = False, fe_portable: bool = False):
        spec = data.spec
        Wp, Wrp, Bp = data.packed()
        self.keep = []
        n = or_net()
        n.nl = spec.nl
        for i, s in enumerate(spec.sizes):
            n.size[i] = s
        for i in range(spec.nl):
            n.type[i] = spec.types[i]
            n.qk[i], n.qi[i], n.qb[i] = spec.qk[i], spec.qi[i], spec.qb[i]
            n.act[i] = spec.acts[i]
            w = np.ascontiguousarray(Wp[i]).view(np.int8)
            b = np.ascontiguousarray(Bp[i], np.int16)
            self.keep += [w, b]
            n.W[i] = w.ctypes.data
            n.B[i] = b.ctypes.data
            if Wrp[i] is not None:
                wr = np.ascontiguousarray(Wrp[i]).view(np.int8)
                self.keep.append(wr)
                n.Wr[i] = wr.ctypes.data
        n.acc32 = int(acc32)
        for i, a in enumerate(spec.accs or []):   # mixed fc_8x16 / _acc32b layers (NetSpec.accs)
            n.acc32_layer[i] = int(a)
        n.portable = int(portable)   # the ARM_OPTIMIZED=0 build's live align shift (pinning only)
        self.net = n
        self.mean = np.ascontiguousarray(data.mean, np.int32)
        self.stdR = np.ascontiguousarray(data.stdR, np.int32)
        c = or_cfg()
        c.nn_id = spec.nn_id
        c.thresh_prob = thresh_prob
        c.th_count = th_count
        c.qbit_out = spec.qi[0]
        c.mean = self.mean.ctypes.data
        c.stdR = self.stdR.ctypes.data
        c.fe_portable = int(fe_portable)   # the ARM_OPTIMIZED=0 build's front end (row N4)
        self.cfg = c
        self.nout = spec.nout

    def new_states(self, S: int) -> np.ndarray:
        L = lib()
        st = np.zeros((S, L.or_sizeof_stream()), np.uint8)
        for s in range(S):
            L.or_nnsp_reset(C.byref(self.net), C.c_void_p(st[s].ctypes.data), C.byref(self.cfg))
        return st

    def run(self, pcm: np.ndarray, states: np.ndarray | None = None, want_logits=True,
            want_feats=True):
        """pcm [S][T][160] -> trig [S][T], logits [S][T][nout] (0 on non-NN frames), feats."""
        pcm = np.ascontiguousarray(pcm, np.int16)
        S, T, _ = pcm.shape
        if states is None:
            states = self.new_states(S)
        trig = np.zeros((S, T), np.int16)
        logits = np.zeros((S, T, self.nout), np.int32) if want_logits else None
        feats = np.zeros((S, T, 40), np.int16) if want_feats else None
        lib().or_run_streams(C.byref(self.net), C.byref(self.cfg), p(states), S, T, p(pcm),
                             p(trig), p(logits), p(feats))
        return trig, logits, feats, states

    def reset_streams(self, states: np.ndarray, mask) -> None:
        for s in np.nonzero(mask)[0]:
            lib().or_nnsp_reset(C.byref(self.net), C.c_void_p(states[s].ctypes.data), C.byref(self.cfg))

    def forward(self, x240: np.ndarray, state: np.ndarray, n_layers: int = -1) -> np.ndarray:
        out = np.zeros(160, np.int32)
        x = np.ascontiguousarray(x240, np.int16)
        lib().or_net_forward(C.byref(self.net), C.c_void_p(state.ctypes.data), p(x), p(out), n_layers)
        return out


class OracleCascade:
    """or_cascade (nnCntrlClass restatement) over S streams; nets by nn id."""

    def __init__(self, nets: dict, seq=(1, 2, 0), lookback_s2i=80, timeout_s2i=1000,
                 lookback_kws=80, timeout_kws=1000):
        self.nets = nets
        c = or_cascade_cfg()
        for i, name in enumerate(("s2i", "vad", "kws")):
            c.net[i] = C.addressof(nets[name].net)
            c.cfg[i] = nets[name].cfg
        for i, v in enumerate(seq):
            c.seq[i] = v
        c.len_seq = len(seq)
        c.lookback_kws, c.lookback_s2i = lookback_kws, lookback_s2i
        c.timeout_kws, c.timeout_s2i = timeout_kws, timeout_s2i
        self.cfg = c
        self.st = None

    def new_states(self, S: int) -> np.ndarray:
        st = np.zeros((S, lib().or_sizeof_cascade()), np.uint8)
        for s in range(S):
            lib().or_cascade_reset(C.c_void_p(st[s].ctypes.data), C.byref(self.cfg))
        return st

    def run(self, pcm: np.ndarray, states: np.ndarray | None = None):
        """pcm [S][T][160] -> net_ran [S][T] int8, detected [S][T], outputs3 [S][T][3], states."""
        pcm = np.ascontiguousarray(pcm, np.int16)
        S, T, _ = pcm.shape
        if states is None:
            states = self.new_states(S)
        ran = np.zeros((S, T), np.int8)
        det = np.zeros((S, T), np.int16)
        o3 = np.zeros((S, T, 3), np.int16)
        lib().or_run_cascade(C.byref(self.cfg), p(states), S, T, p(pcm), p(ran), p(det), p(o3))
        return ran, det, o3, states


def fc(w: np.ndarray, b: np.ndarray, x: np.ndarray, qk: int, qb: int, qi: int, act: int, acc32: bool,
       portable: bool = False) -> np.ndarray:
    """fc_8x16(_acc32b) on natural W[N][K] (packed here in the shipped order)."""
    from nnsp_amd.nets import LINEAR, pack_fc
    N, K = w.shape
    wp = np.ascontiguousarray(pack_fc(w))
    bb = None if b is None else np.ascontiguousarray(b, np.int16)
    xx = np.ascontiguousarray(x, np.int16)
    y = np.zeros(N, np.int32 if act == LINEAR else np.int16)
    lib().or_fc(N, p(wp), p(bb), p(xx), K, qk, qb, qi, act, int(acc32), int(portable), p(y))
    return y.astype(np.int32)


def lstm(w, wr, b, x, h, c, qk, qb, qi, qir, acc32: bool, portable: bool = False) -> np.ndarray:
    """lstm_8x16(_acc32b) on natural gate-major W[4N][K]; h (int16[N]) and c
    (int32[N]) are updated in place."""
    from nnsp_amd.nets import pack_lstm, pack_lstm_bias
    N, K = w.shape[0] // 4, w.shape[1]
    wp, wrp = np.ascontiguousarray(pack_lstm(w)), np.ascontiguousarray(pack_lstm(wr))
    bp = np.ascontiguousarray(pack_lstm_bias(b))
    xx = np.ascontiguousarray(x, np.int16)
    y = np.zeros(N, np.int16)
    lib().or_lstm(N, p(wp), p(wrp), p(bp), p(xx), p(h), p(c), K, qk, qb, qi, qir, int(acc32), int(portable), p(y))
    return y


def rfft512(x: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    x = np.ascontiguousarray(x, np.int32).copy()
    xi = np.zeros(514, np.int32)
    xi[:512] = x
    y = np.zeros(1024, np.int32)
    lib().or_rfft512(p(xi), p(y))
    return y, xi[:512]


def rfft512_portable(x: np.ndarray) -> np.ndarray:
    """The ARM_OPTIMIZED=0 build's rfft(512): 512 Frac15 int32 -> 257 complex (514 int32)."""
    xi = np.ascontiguousarray(x, np.int32)
    y = np.zeros(514, np.int32)
    lib().or_rfft512_portable(p(xi), p(y))
    return y


def synthetic_pcm(S: int, T: int, seed: int = 0x4E4E5350, t0: int = 0, s0: int = 0,
                  amp: int = 4096, wavs: np.ndarray | None = None, every: int = 4) -> np.ndarray:
    """SplitMix64(seed, stream, sample) -> int16 in [-amp, amp-1];
    with wavs ([n_wavs][len] int16): stream g = s0 + s with g % every == 0
    replays wav (g // every) % n_wavs cyclically from offset (g * 1601) % len
    (nnsp_synth_pcm_mix on the device)."""
    s = (np.arange(S, dtype=np.uint64) + np.uint64(s0))[:, None]
    n = (np.arange(T * 160, dtype=np.uint64) + np.uint64(t0 * 160))[None, :]
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + s * np.uint64(0x9E3779B97F4A7C15) + n * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    v = ((z % np.uint64(2 * amp)).astype(np.int64) - amp).astype(np.int16)
    if wavs is not None:
        L = wavs.shape[1]
        g = np.arange(S, dtype=np.int64) + s0
        for i in np.nonzero(g % every == 0)[0]:
            w = wavs[(g[i] // every) % len(wavs)]
            v[i] = w[(g[i] * 1601 % L + t0 * 160 + np.arange(T * 160, dtype=np.int64)) % L]
    return v.reshape(S, T, 160)


def load_wavs() -> np.ndarray:
    """python/test_wavs/{speech,galaxy,galaxy_s2i}.wav as [3][160000] int16
    (committed as tests/golden/test_wavs.npz)."""
    z = np.load(os.path.join(os.path.dirname(HERE), "tests", "golden", "test_wavs.npz"))
    return np.stack([z[k] for k in ("speech", "galaxy", "galaxy_s2i")])


class or_stream(C.Structure):
    _fields_ = [("buf", C.c_int16 * 480), ("ctx", C.c_int16 * 240), ("h", (C.c_int16 * MAX_WIDTH) * MAX_LSTM),
                ("c", (C.c_int32 * MAX_WIDTH) * MAX_LSTM), ("slides", C.c_int16), ("trigger", C.c_int16),
                ("argmax_last", C.c_int16), ("pad0", C.c_int16), ("counts", C.c_int16 * 8),
                ("outputs", C.c_int16 * 3), ("pad1", C.c_int16)]


def act(kind: int, x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.int32)
    y = np.zeros(len(x), np.int32 if kind == 3 else np.int16)
    lib().or_act(kind, p(x), p(y), len(x))
    return y


def log10(x: np.ndarray) -> np.ndarray:
    return np.array([lib().or_log10(int(v)) for v in np.asarray(x, np.int64)], np.int32)


def spec2pspec(spec1024: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(spec1024, np.int32)
    y = np.zeros(257, np.int32)
    lib().or_spec2pspec(p(y), p(x), 257)
    return y


def mel(pspec: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(pspec, np.int32)
    y = np.zeros(40, np.int32)
    lib().or_mel(p(x), p(y))
    return y
