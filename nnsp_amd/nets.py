"""Net descriptions, synthetic weights and the ns-nnsp weight byte layout.

The three reference nets share one topology (python/nn_arch/def_*_nn_arch.txt,
exported by python/c_code_table_converter.py): conv1d(k=6 frames, stride 2) as
an FC over the 6x40 context -> LSTM -> FC -> FC -> FC.  Their shapes and
fixed-point formats are the ``NeuralNetClass`` initialisers of
evb/src/def_nn1_vad.c:29-110, def_nn2_kws_galaxy.c:29-111, def_nn0_s2i.c:29-110.

Weights: ``ref_net`` loads the reference's own tables (def_nn*.c, dumped as
data into tests/golden/ref_nets.npz); ``synth_net`` draws seeded synthetic
weights of exactly those shapes and formats, with per-layer spreads that match
the shipped tables (int8 std 3-30, int16 bias std 2e3-1.2e4) -- the reference's
tables are themselves random (reference README.md:67, :111).

Byte layout (``pack_fc`` / ``pack_lstm``): the CMSIS-NN interleaved order the
shipped ARM path walks (ns-nnsp/src/affine.c:80-149; producer
python/nnsp_pack/c_weight_man.py:23-124, checked byte-for-byte by
tests/test_layout.py when the reference is present).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

FC, LSTM = 0, 1
RELU6, TANH, SIGMOID, LINEAR = 0, 1, 2, 3
NN_ID = {"s2i": 0, "vad": 1, "kws": 2}


@dataclass
class NetSpec:
    name: str
    sizes: list[int]
    types: list[int]
    qk: list[int]
    qi: list[int]
    qb: list[int]
    acts: list[int]
    # synthetic-weight spreads per layer: (std of W, std of Wrec, bias mean, bias std)
    spread: list[tuple] = field(default_factory=list)
    nid: int | None = None   # NNSP_ID of a net not named vad/kws/s2i (post-processing kind)
    accs: list[int] | None = None   # per layer 1: fc_8x16_acc32b / lstm_8x16_acc32b (mixed nets)

    @property
    def nl(self) -> int:
        return len(self.types)

    @property
    def nout(self) -> int:
        return self.sizes[-1]

    @property
    def nn_id(self) -> int:
        return self.nid if self.nid is not None else NN_ID[self.name]


SPECS = {
    # evb/src/def_nn1_vad.c:31-41
    "vad": NetSpec("vad", [240, 28, 28, 28, 28, 2], [FC, LSTM, FC, FC, FC],
                   [7, 5, 5, 5, 7], [8, 15, 15, 12, 12], [14, 13, 15, 15, 15],
                   [TANH, TANH, RELU6, RELU6, LINEAR],
                   [(14, 0, 1700, 10000), (7, 15, 500, 8300), (12, 0, -2800, 8300),
                    (19, 0, 5000, 4300), (30, 0, 0, 7000)]),
    # evb/src/def_nn2_kws_galaxy.c:31-41
    "kws": NetSpec("kws", [240, 64, 64, 64, 64, 2], [FC, LSTM, FC, FC, FC],
                   [6, 5, 5, 5, 7], [8, 15, 15, 12, 12], [13, 14, 15, 15, 15],
                   [TANH, TANH, RELU6, RELU6, LINEAR],
                   [(14, 0, 400, 7300), (5, 12.5, 4600, 10000), (11, 0, 2900, 5500),
                    (10, 0, 2200, 8500), (19, 0, 0, 2000)]),
    # evb/src/def_nn0_s2i.c:31-41
    "s2i": NetSpec("s2i", [240, 72, 72, 72, 72, 41], [FC, LSTM, FC, FC, FC],
                   [7, 5, 4, 4, 5], [8, 15, 15, 12, 12], [14, 14, 14, 14, 14],
                   [TANH, TANH, RELU6, RELU6, LINEAR],
                   [(12.6, 0, -800, 7300), (2.8, 9.6, 4800, 8000), (5.2, 0, -3000, 6000),
                    (11.3, 0, 2800, 6400), (12.9, 0, -11000, 12000)]),
}

# Cascade / post-processing parameters, evb/src/ParamsNNCntrl.h:8-21
THRESH_PROB = 32767 >> 1
THRESH_CNTS = 4
LOOKBACK = 80
TIMEOUT = 1000


# --------------------------------------------------------------------------
# byte layout
# --------------------------------------------------------------------------
def _pack_block(m: np.ndarray) -> list[np.ndarray]:
    """One affine_Krows block of R<=4 rows over K columns (affine.c:74-184)."""
    R, K = m.shape
    out = []
    for p in range(K // 2):
        c0, c1 = m[:, 2 * p], m[:, 2 * p + 1]
        if R == 4:
            out.append(np.array([c0[0], c0[1], c1[0], c1[1], c0[2], c0[3], c1[2], c1[3]]))
        elif R == 3:
            out.append(np.array([c0[0], c0[1], c1[0], c1[1], c0[2], c1[2]]))
        elif R == 2:
            out.append(np.array([c0[0], c0[1], c1[0], c1[1]]))
        else:
            out.append(np.array([c0[0], c1[0]]))
    if K % 2:
        out.append(m[:, K - 1].copy())
    return out


def pack_fc(w: np.ndarray) -> np.ndarray:
    """Natural W[N][K] int8 -> interleaved byte stream."""
    N = w.shape[0]
    parts = []
    for r0 in range(0, N, 4):
        parts += _pack_block(w[r0:r0 + 4])
    return np.concatenate(parts).astype(np.int8)


def unpack_fc(blob: np.ndarray, N: int, K: int) -> np.ndarray:
    """Inverse of pack_fc (via the packed order of element indices)."""
    ids = _pack_index(N, K)
    out = np.zeros(N * K, dtype=np.int8)
    out[ids] = np.asarray(blob, dtype=np.int8)[: N * K]
    return out.reshape(N, K)


def _pack_index(N: int, K: int) -> np.ndarray:
    ar = np.arange(N * K).reshape(N, K)
    parts = []
    for r0 in range(0, N, 4):
        parts += _pack_block(ar[r0:r0 + 4])
    return np.concatenate(parts)


def pack_lstm(w: np.ndarray, dtype=np.int8) -> np.ndarray:
    """Natural gate-major W[4N][K] (rows: i block, j block, f block, o block;
    python/c_code_table_converter.py:64-73 order) -> per-4-unit-group
    [i rows][j rows][f rows][o rows] interleaved stream (c_weight_man.py:61-92)."""
    N = w.shape[0] // 4
    g = [w[k * N:(k + 1) * N] for k in range(4)]
    parts = []
    for u0 in range(0, N, 4):
        for k in range(4):
            parts += _pack_block(g[k][u0:u0 + 4])
    return np.concatenate(parts).astype(dtype)


def pack_lstm_bias(b: np.ndarray, dtype=np.int16) -> np.ndarray:
    N = b.shape[0] // 4
    g = [b[k * N:(k + 1) * N] for k in range(4)]
    parts = []
    for u0 in range(0, N, 4):
        for k in range(4):
            parts.append(g[k][u0:u0 + 4])
    return np.concatenate(parts).astype(dtype)


def unpack_lstm(blob: np.ndarray, N: int, K: int) -> np.ndarray:
    """Inverse of pack_lstm: interleaved stream -> natural gate-major W[4N][K]."""
    ids = pack_lstm(np.arange(4 * N * K).reshape(4 * N, K).astype(np.int64), dtype=np.int64)
    out = np.zeros(4 * N * K, dtype=np.int8)
    out[ids] = np.asarray(blob, dtype=np.int8)[: 4 * N * K]
    return out.reshape(4 * N, K)


def unpack_lstm_bias(blob: np.ndarray, N: int) -> np.ndarray:
    ids = pack_lstm_bias(np.arange(4 * N), dtype=np.int64)
    out = np.zeros(4 * N, dtype=np.int16)
    out[ids] = np.asarray(blob, dtype=np.int16)[: 4 * N]
    return out


# --------------------------------------------------------------------------
# the reference's portable (ARM_OPTIMIZED=0) byte order, affine.c:291-309:
# per row block (4 rows, remainder last), per column pair, per row, the pair's
# two bytes; the odd-column tail one byte per row.  Only the oracle's pinning
# fixtures use it (tests/golden/make_golden.py feeds the reference's portable
# build with it); the shipped tables are in the interleaved order above.
# --------------------------------------------------------------------------
def _pack_block_portable(m: np.ndarray) -> list[np.ndarray]:
    R, K = m.shape
    out = [m[:, 2 * p:2 * p + 2].reshape(-1).copy() for p in range(K // 2)]
    if K % 2:
        out.append(m[:, K - 1].copy())
    return out


def pack_fc_portable(w: np.ndarray) -> np.ndarray:
    parts = []
    for r0 in range(0, w.shape[0], 4):
        parts += _pack_block_portable(w[r0:r0 + 4])
    return np.concatenate(parts).astype(np.int8)


def pack_lstm_portable(w: np.ndarray) -> np.ndarray:
    N = w.shape[0] // 4
    g = [w[k * N:(k + 1) * N] for k in range(4)]
    parts = []
    for u0 in range(0, N, 4):
        for k in range(4):
            parts += _pack_block_portable(g[k][u0:u0 + 4])
    return np.concatenate(parts).astype(np.int8)


# --------------------------------------------------------------------------
# synthetic nets
# --------------------------------------------------------------------------
@dataclass
class NetData:
    spec: NetSpec
    W: list            # natural int8 matrices (W[N][K]; LSTM: [4N][K] gate-major i,j,f,o)
    Wr: list           # LSTM recurrent [4N][N] or None
    B: list            # natural int16 biases (LSTM: [4N] gate-major)
    mean: np.ndarray   # int32[40]
    stdR: np.ndarray   # int32[40]

    def packed(self):
        """Byte streams exactly as a def_nn*.c file holds them."""
        Wp, Wrp, Bp = [], [], []
        for i, t in enumerate(self.spec.types):
            if t == LSTM:
                Wp.append(pack_lstm(self.W[i]))
                Wrp.append(pack_lstm(self.Wr[i]))
                Bp.append(pack_lstm_bias(self.B[i]))
            else:
                Wp.append(pack_fc(self.W[i]))
                Wrp.append(None)
                Bp.append(self.B[i].astype(np.int16))
        return Wp, Wrp, Bp

    def packed_portable(self):
        """Byte streams in the reference's ARM_OPTIMIZED=0 order (biases as packed())."""
        Wp, Wrp, Bp = [], [], []
        for i, t in enumerate(self.spec.types):
            if t == LSTM:
                Wp.append(pack_lstm_portable(self.W[i]))
                Wrp.append(pack_lstm_portable(self.Wr[i]))
                Bp.append(pack_lstm_bias(self.B[i]))
            else:
                Wp.append(pack_fc_portable(self.W[i]))
                Wrp.append(None)
                Bp.append(self.B[i].astype(np.int16))
        return Wp, Wrp, Bp

    @classmethod
    def from_packed(cls, spec: NetSpec, Wp, Wrp, Bp, mean, stdR) -> "NetData":
        """A net from the byte streams a def_nn*.c file holds (interleaved order)."""
        W, Wr, B = [], [], []
        for i, t in enumerate(spec.types):
            K, N = spec.sizes[i], spec.sizes[i + 1]
            if t == LSTM:
                W.append(unpack_lstm(Wp[i], N, K))
                Wr.append(unpack_lstm(Wrp[i], N, N))
                B.append(unpack_lstm_bias(Bp[i], N))
            else:
                W.append(unpack_fc(Wp[i], N, K))
                Wr.append(None)
                B.append(np.asarray(Bp[i], np.int16)[:N].copy())
        return cls(spec, W, Wr, B, np.asarray(mean, np.int32).copy(), np.asarray(stdR, np.int32).copy())


# The reference's own three nets: the tables of evb/src/def_nn0_s2i.c,
# def_nn1_vad.c and def_nn2_kws_galaxy.c (weights, biases, feature mean/stdR,
# every NeuralNetClass field), dumped as data by tests/golden/make_golden.py
# from those files compiled here; the GPU box has no reference tree.
REF_NETS_NPZ = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                            "ref_nets.npz")


def ref_net(name: str, path: str | None = None) -> NetData:
    """NetData of the reference's def_nn*.c net ``name`` ("vad", "kws", "s2i")."""
    z = np.load(path or REF_NETS_NPZ, allow_pickle=False)
    nl = int(z[f"{name}_numlayers"])
    spec = NetSpec(name, [int(v) for v in z[f"{name}_size_layer"][:nl + 1]],
                   [int(v) for v in z[f"{name}_layer_type"][:nl]], [int(v) for v in z[f"{name}_qbit_kernel"][:nl]],
                   [int(v) for v in z[f"{name}_qbit_input"][:nl]], [int(v) for v in z[f"{name}_qbit_bias"][:nl]],
                   [int(v) for v in z[f"{name}_activation_type"][:nl]])
    Wp = [z[f"{name}_kernel{i}"] for i in range(nl)]
    Wrp = [z[f"{name}_kernel_rec{i}"] if f"{name}_kernel_rec{i}" in z else None for i in range(nl)]
    Bp = [z[f"{name}_bias{i}"] for i in range(nl)]
    return NetData.from_packed(spec, Wp, Wrp, Bp, z[f"{name}_mean"], z[f"{name}_stdR"])


def get_net(name: str, weights: str = "ref", seed: int = 1234) -> NetData:
    """weights "ref": the reference's def_nn*.c tables; "synth": seeded synthetic."""
    if weights == "ref":
        return ref_net(name)
    if weights == "synth":
        return synth_net(name, seed)
    raise ValueError(f"weights must be 'ref' or 'synth', not {weights!r}")


# Net shapes beyond the three reference nets: any FC/LSTM
# stack of <= 10 layers the NeuralNetClass struct can describe -- rows not a
# multiple of 4 (affine.c:103-149), odd K (:157-184), 3 and 7 layers, two
# LSTM layers, a 256-wide FC layer.  Post-processing kind by nid.
GEN_SPECS = {
    "gen3": NetSpec("gen3", [240, 30, 21, 2], [FC, LSTM, FC], [7, 5, 6], [8, 15, 13], [14, 13, 15],
                    [TANH, TANH, LINEAR], [(12, 0, 500, 6000), (6, 12, 300, 7000), (20, 0, 0, 6000)], nid=1),
    "odd": NetSpec("odd", [240, 33, 21, 7, 2], [FC, LSTM, FC, FC], [7, 5, 5, 7], [8, 15, 15, 12],
                   [14, 13, 15, 15], [TANH, TANH, RELU6, LINEAR],
                   [(12, 0, 500, 6000), (6, 12, 300, 7000), (15, 0, 2000, 5000), (25, 0, 0, 6000)], nid=2),
    "lstm2": NetSpec("lstm2", [240, 64, 48, 36, 20, 12, 41, 41], [FC, LSTM, LSTM, FC, FC, FC, FC],
                     [7, 5, 5, 5, 5, 6, 5], [8, 15, 15, 15, 12, 12, 12], [14, 13, 13, 15, 15, 15, 14],
                     [TANH, TANH, TANH, RELU6, RELU6, RELU6, LINEAR],
                     [(12, 0, 500, 6000), (5, 10, 300, 7000), (6, 10, 300, 7000), (12, 0, 2000, 5000),
                      (14, 0, 2000, 5000), (16, 0, 2000, 5000), (12, 0, -8000, 9000)], nid=0),
    "wide": NetSpec("wide", [240, 256, 28, 256, 2], [FC, LSTM, FC, FC], [7, 5, 5, 7], [8, 15, 15, 12],
                    [14, 13, 15, 15], [TANH, TANH, RELU6, LINEAR],
                    [(10, 0, 500, 6000), (3, 12, 300, 7000), (15, 0, 2000, 5000), (8, 0, 0, 6000)], nid=1),
    # the reference's own limits (neural_nets.c:9-10: 300-element activation
    # buffers): a 300-wide FC, a 300-wide LSTM (K = 300), then 300 -> 41
    "wide300": NetSpec("wide300", [240, 300, 300, 300, 41], [FC, LSTM, FC, FC], [7, 6, 5, 6], [8, 15, 15, 12],
                       [14, 14, 15, 14], [TANH, TANH, RELU6, LINEAR],
                       [(8, 0, 500, 6000), (1.5, 2, 300, 7000), (4, 0, 2000, 5000), (5, 0, -8000, 9000)], nid=0),
    # three LSTM layers, the first straight on the 240-wide context
    "lstm3": NetSpec("lstm3", [240, 96, 64, 40, 2], [LSTM, LSTM, LSTM, FC], [5, 5, 5, 7], [8, 15, 15, 15],
                     [13, 13, 13, 15], [TANH, TANH, TANH, LINEAR],
                     [(4, 6, 300, 7000), (5, 8, 300, 7000), (6, 9, 300, 7000), (20, 0, 0, 6000)], nid=1),
    # fc_8x16 and fc_8x16_acc32b / lstm_8x16 layers mixed in one net (per-layer layer_func)
    "mixacc": NetSpec("mixacc", [240, 28, 28, 28, 28, 2], [FC, LSTM, FC, FC, FC],
                      [7, 5, 5, 5, 7], [8, 15, 15, 12, 12], [14, 13, 15, 15, 15],
                      [TANH, TANH, RELU6, RELU6, LINEAR],
                      [(14, 0, 1700, 10000), (7, 15, 500, 8300), (12, 0, -2800, 8300),
                       (19, 0, 5000, 4300), (30, 0, 0, 7000)], nid=1, accs=[1, 0, 1, 0, 1]),
    # a linear layer inside the stack: its int32 outputs sit in the int16
    # buffer, and the next layer reads size_layer int16 of them (neural_nets.c:131-149)
    "midlin": NetSpec("midlin", [240, 48, 64, 2], [FC, FC, FC], [7, 5, 7], [8, 15, 12], [14, 15, 15],
                      [LINEAR, RELU6, LINEAR], [(6, 0, 500, 6000), (3, 0, 2000, 5000), (20, 0, 0, 6000)], nid=2),
}

# Shapes only NeuralNetClass_exe takes (not NNSPClass_exec: its context is 240
# wide and its static int32_t output[50], nn_speech.c:78, holds 50 int32 or
# 100 int16): a 300-wide input, the widest linear layer (150 int32), a
# 300-wide int16 output.
DIRECT_SPECS = {
    "direct300": NetSpec("direct300", [300, 300, 150], [LSTM, FC], [5, 6], [12, 15], [13, 14], [TANH, LINEAR],
                         [(2, 2, 300, 7000), (4, 0, -2000, 9000)], nid=1),
    "int16out": NetSpec("int16out", [300, 200, 300], [FC, FC], [6, 6], [12, 15], [14, 15], [TANH, RELU6],
                        [(5, 0, 500, 6000), (6, 0, 2000, 5000)], nid=1),
}
ALL_GEN_SPECS = {**GEN_SPECS, **DIRECT_SPECS}


def synth_net(name: str | NetSpec, seed: int = 1234) -> NetData:
    spec = name if isinstance(name, NetSpec) else (SPECS.get(name) or ALL_GEN_SPECS[name])
    rng = np.random.default_rng([seed, spec.nn_id] + ([] if spec.name in SPECS else [len(spec.types)]))

    def i8(shape, std):
        return np.clip(np.round(rng.normal(0.0, std, shape)), -128, 127).astype(np.int8)

    def i16(n, mean, std):
        return np.clip(np.round(rng.normal(mean, std, n)), -32768, 32767).astype(np.int16)

    W, Wr, B = [], [], []
    for i, t in enumerate(spec.types):
        K, N = spec.sizes[i], spec.sizes[i + 1]
        sw, swr, bm, bs = spec.spread[i]
        if t == LSTM:
            W.append(i8((4 * N, K), sw))
            Wr.append(i8((4 * N, N), swr))
            B.append(i16(4 * N, bm, bs))
        else:
            W.append(i8((N, K), sw))
            Wr.append(None)
            B.append(i16(N, bm, bs))
    # feature statistics in the ranges of the shipped tables (def_nn*.c:8-9)
    mean = np.sort(rng.uniform(-110000, -25000, 40)).astype(np.int32)[::-1].copy()
    stdR = rng.uniform(16500, 24500, 40).astype(np.int32)
    return NetData(spec, W, Wr, B, mean, stdR)
