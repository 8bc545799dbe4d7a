"""Constant-table generator for the ns-nnsp hot path.

Every constant table the fixed-point path needs is regenerated here from a
closed-form rule; nothing is copied from the reference.  Each rule was pinned
against the reference's own table bytes in the build container (see
tests/test_tables.py, which re-checks all of them whenever /root/reference is
present):

=========================  ==========================================  ==========================================
table                      reference location                          rule (exact, all entries)
=========================  ==========================================  ==========================================
stft window (480 x i16)    ns-nnsp/src/window_stft_coef.c:6            floor(sqrt(hop/win*(1-cos(2*pi*n/win)))*2^15)
                           (generator python/nnsp_pack/gen_stft_win.py:14-19)
mel banks (534 x i16)      ns-nnsp/src/melSpec_coeff.c:5               packed [start,end,coef...] per bank,
                           (generator python/nnsp_pack/mel.py:10-50)   coef = floor(tri * 2^15)
log10 interp (256 x i16)   ns-nnsp/src/fixlog10.c:6                    [floor(ln(1+k/128)*2^15), min(floor(2^15/(1+k/128)),32767)]
tanh interp (384 x i16)    ns-nnsp/src/activation.c:5                  c=(512+1024k)/2^15: [floor(tanh c*2^15), floor((1-tanh^2 c)*2^15)]
cfft twiddles (384 x q31)  CMSIS-DSP 1.10.0 twiddleCoef_256_q31         floor(x*2^31 + 0.05), x = cos/sin(2*pi*i/256)
                           (binary only: evb/libs/libCMSISDSP.a)
rfft split A/B (q31)       CMSIS-DSP 1.10.0 realCoefAQ31/realCoefBQ31   round(0.5*(1-+sin t)*2^31), round(-+0.5*cos t*2^31)
bit reversal               CMSIS-DSP armBitRevIndexTable_fixed_256      8-bit bit reversal of the 256 complex slots
=========================  ==========================================  ==========================================

The twiddle rule ("floor(x*2^31 + 0.05)") is empirical: it is the rule that
reproduces all 384 words of the shipped ``twiddleCoef_256_q31`` data section
(plain round() misses 171 words, plain floor() 18).

``write_header`` emits ``nnsp_amd/csrc/gen/nnsp_tables.h`` used by both the
HIP kernels / host library and the test oracle.
"""
from __future__ import annotations

import math
import os

import numpy as np

WIN_LEN = 480      # LEN_STFT_WIN_COEFF, ambiq_nnsp_const.h:4
HOP = 160          # LEN_STFT_HOP, ambiq_nnsp_const.h:5
FFT_LEN = 512      # LEN_FFT_NNSP, ambiq_nnsp_const.h:3
N_MEL = 40         # NUM_MELBANKS, ambiq_nnsp_const.h:6
FS = 16000         # SAMPLING_RATE, ambiq_nnsp_const.h:9


def stft_window() -> np.ndarray:
    n = np.arange(WIN_LEN)
    w = np.sqrt(HOP / WIN_LEN * (1.0 - np.cos(2.0 * np.pi / WIN_LEN * n)))
    return np.minimum(np.floor(w * 2 ** 15), 32767).astype(np.int16)


def mel_bank_packed() -> np.ndarray:
    hi = 2595.0 * np.log10(1.0 + (FS / 2) / 700.0)
    mel_pts = np.linspace(0.0, hi, N_MEL + 2)
    hz = 700.0 * (10.0 ** (mel_pts / 2595.0) - 1.0)
    edge = np.floor((FFT_LEN + 1) * hz / FS)
    out: list[int] = []
    for b in range(1, N_MEL + 1):
        lo, mid, up = edge[b - 1], edge[b], edge[b + 1]
        tri = np.zeros(FFT_LEN // 2 + 1)
        for k in range(int(lo), int(mid)):
            tri[k] = (k - lo) / (mid - lo)
        for k in range(int(mid), int(up)):
            tri[k] = (up - k) / (up - mid)
        out += [int(lo) + 1, int(up) - 1]
        for k in range(int(lo) + 1, int(up)):
            out.append(int(min(max(math.floor(tri[k] * 2 ** 15), -32768), 32767)))
    return np.asarray(out, dtype=np.int16)


def log_interp() -> np.ndarray:
    k = np.arange(128)
    val = np.floor(np.log(1.0 + k / 128.0) * 2 ** 15)
    slope = np.minimum(np.floor(2 ** 15 / (1.0 + k / 128.0)), 32767)
    return np.stack([val, slope], 1).reshape(-1).astype(np.int16)


def tanh_interp() -> np.ndarray:
    k = np.arange(192)
    c = (512.0 + 1024.0 * k) / 2 ** 15
    t = np.tanh(c)
    val = np.floor(t * 2 ** 15)
    der = np.floor((1.0 - t * t) * 2 ** 15)
    return np.minimum(np.stack([val, der], 1).reshape(-1), 32767).astype(np.int16)


def tanh_interp_shifted() -> np.ndarray:
    """The tanh (value, slope) table re-indexed for the split NN kernels'
    branch-light lookup (nnsp_dev.h tanh_q15s): entry k' = (|x| + 512) >> 10
    (k' - 1 is activation.c's segment), so the offset inside the segment is
    (|x| + 512) & 1023 with no clamp of the index from below.  Entry 0 covers
    |x| < 512, where the reference's segment 0 evaluates to |x| - 1
    (511 + floor((|x| - 512) * 32760 / 2^15)): (-512, 32767) gives the same.
    Entries 193..255 keep the 8-bit index in bounds past |x| >= 5 * 2^15, where
    the result is 32767 regardless (tests/test_tables.py checks all of it)."""
    t = tanh_interp().astype(np.int64).reshape(-1, 2)
    pad = np.tile([[32767, 0]], (256 - 1 - len(t), 1))
    return np.concatenate([[[-512, 32767]], t, pad]).reshape(-1).astype(np.int16)


ACT_ENTRIES = 322   # half-segments j = (|x| + 512) >> 9 <= 321 after the clamp


def act_affine_table() -> np.ndarray:
    """tanh_fix / sigmoid_fix (activation.c:31-83) as one multiply-add per
    lookup (nnsp_dev.h act_q15): int32 [ACT_ENTRIES][4] = (A_pos, b_pos, A_neg,
    b_neg) per half-segment j = bb >> 9 of bb = |x| + 512, with bb clamped to
    164352 (|x| >= 5 * 2^15 lands on j = 321, dx = 0: activation.c's saturation
    to 32767 -- with 1024-wide entries it would fall mid-entry) and
    dx = bb & 511.  Entry j is half (j & 1) of tanh_interp_shifted's entry
    j >> 1: A = val << 15 + (j & 1) * 512 * slope, b = slope, so
    z = A + dx * b is the reference's val * 2^15 + dx1024 * slope exactly.
      tanh:    z >> 15 (arithmetic).  Negative x takes the negated result,
               -floor(z / 2^15) = floor((32767 - z) / 2^15): A_neg = 32767 - A,
               b_neg = -b.  Entry 0 (|x| < 512) starts at A = -2^24 + 512, which
               gives |x| - 1 for |x| >= 1 and 0 at x = 0 -- activation.c's
               max(., 0) -- so the result needs no clamp.
      sigmoid: 16384 + (tanh(w) >> 1) of the pre-shifted input w is
               (z + 2^30) >>> 16 with the same z (nested floors; the sum is
               non-negative and below 2^32), for either sign.
    tests/test_tables.py checks both against activation.c's definitions."""
    t = tanh_interp_shifted().astype(np.int64).reshape(-1, 2)
    j = np.arange(ACT_ENTRIES)
    k = j >> 1
    val, b = t[k, 0], t[k, 1].copy()
    A = (val << 15) + (j & 1) * 512 * b
    A[0] = -(1 << 24) + 512
    A[1] = -(1 << 24) + 512 + 512 * 32767
    sat = j >= 321
    A[sat] = 32767 << 15
    b[sat] = 0
    out = np.stack([A, b, 32767 - A, -b], 1)
    return (out & 0xFFFFFFFF).astype(np.uint32).view(np.int32)


def cfft256_twiddles() -> np.ndarray:
    i = np.arange(192)
    v = np.stack([np.cos(2 * np.pi * i / 256), np.sin(2 * np.pi * i / 256)], 1).reshape(-1) * 2.0 ** 31
    return np.clip(np.floor(v + 0.05), -2 ** 31, 2 ** 31 - 1).astype(np.int32)


def rfft_split_full(n: int = 4096) -> tuple[np.ndarray, np.ndarray]:
    """Full CMSIS realCoefAQ31 / realCoefBQ31 (n complex entries each)."""
    i = np.arange(n)
    th = 2 * np.pi * i / (2 * n)

    def q31(x):
        return np.clip(np.round(x * 2.0 ** 31), -2 ** 31, 2 ** 31 - 1).astype(np.int64)

    a = np.stack([q31(0.5 * (1 - np.sin(th))), q31(-0.5 * np.cos(th))], 1).reshape(-1)
    b = np.stack([q31(0.5 * (1 + np.sin(th))), q31(0.5 * np.cos(th))], 1).reshape(-1)
    return a.astype(np.int32), b.astype(np.int32)


def rfft512_split_coefs() -> np.ndarray:
    """The (A_re, A_im, B_re) triple the 512-point split uses for bins k=0..255.

    arm_rfft_init_q31(512) sets twidCoefRModifier = 8192/512 = 16, so bin k
    reads realCoefAQ31[2*16*k], [2*16*k+1] and realCoefBQ31[2*16*k].
    """
    a, b = rfft_split_full()
    k = np.arange(256)
    return np.stack([a[32 * k], a[32 * k + 1], b[32 * k]], 1).astype(np.int32)


def mel_segments(max_len: int = 11, lanes: int = 64) -> np.ndarray:
    """Work split of the 40-bank Mel sum over the 64 lanes of a wave.

    Each row = (bank, first bin, n coefficients <= max_len, offset of the first
    coefficient in the packed table); banks wider than max_len are cut into
    near-equal segments.  Rows past the last segment have n = 0.  The kernel
    adds the int64 partial sums of a bank's segments in segment order, which
    equals the reference's sequential sum (integer addition)."""
    t = mel_bank_packed().astype(np.int64)
    segs, off = [], 0
    for b in range(N_MEL):
        st, en = int(t[off]), int(t[off + 1])
        n = en - st + 1
        k = -(-n // max_len)
        base, extra = divmod(n, k)
        j, c = st, off + 2
        for i in range(k):
            m = base + (1 if i < extra else 0)
            segs.append((b, j, m, c))
            j += m
            c += m
        off += 2 + n
    assert len(segs) <= lanes, len(segs)
    segs += [(N_MEL, 0, 0, 0)] * (lanes - len(segs))
    return np.asarray(segs, dtype=np.int32)


def _cplx16_words(th: np.ndarray) -> np.ndarray:
    """exp(-j th) as the portable build's COMPLEX16 words (imag << 16 | real):
    real = min(floor(2^15 cos), 2^15 - 1), imag = floor(-2^15 sin) (matches
    twiddle_fft_dif.c word for word, tests/test_tables.py)."""
    re_ = np.minimum(np.floor(32768.0 * np.cos(th)), 32767).astype(np.int64)
    im = np.floor(-32768.0 * np.sin(th)).astype(np.int64)
    w = ((im & 0xFFFF) << 16) | (re_ & 0xFFFF)
    return np.where(w >= 2 ** 31, w - 2 ** 32, w).astype(np.int32)


def dif_twiddles() -> np.ndarray:
    """fft_tw_coeff (twiddle_fft_dif.c, ARM_OPTIMIZED=0): per radix-4 index k
    in 0..63 the four twiddles [W^0, W^2k, W^k, W^3k] of the DIF butterfly's
    output slots, W = exp(-j 2 pi / 256)."""
    k = np.arange(64)
    return _cplx16_words(np.stack([0 * k, 2 * k, k, 3 * k], 1).reshape(-1) * 2 * np.pi / 256)


def rfft_dif_twiddles() -> np.ndarray:
    """rfft_tw_coeff (twiddle_fft_dif.c): exp(-j 2 pi i / 512), i in 0..255."""
    return _cplx16_words(np.arange(256) * 2 * np.pi / 512)


def bitrev8() -> np.ndarray:
    return np.array([int(f"{i:08b}"[::-1], 2) for i in range(256)], dtype=np.int32)


def _c_array(ctype: str, name: str, vals, per_line: int = 12) -> str:
    vals = [int(v) for v in np.asarray(vals).reshape(-1)]
    lines = []
    for i in range(0, len(vals), per_line):
        lines.append("    " + ", ".join(str(v) for v in vals[i:i + per_line]) + ",")
    return (f"static const {ctype} {name}[{len(vals)}] __attribute__((aligned(16))) = {{\n"
            + "\n".join(lines) + "\n};\n")


def header_text() -> str:
    mel = mel_bank_packed()
    parts = [
        "/* GENERATED by nnsp_amd/tables.py -- do not edit.\n"
        " * Closed-form regenerations of the ns-nnsp / CMSIS-DSP constant tables;\n"
        " * exactness vs the reference is checked by tests/test_tables.py. */\n",
        "#ifndef NNSP_GEN_TABLES_H\n#define NNSP_GEN_TABLES_H\n#include <stdint.h>\n",
        f"#define NNSP_TBL_MEL_LEN {len(mel)}\n",
        _c_array("int16_t", "nnsp_tbl_window", stft_window()),
        _c_array("int16_t", "nnsp_tbl_mel", mel),
        _c_array("int16_t", "nnsp_tbl_log", log_interp()),
        _c_array("int16_t", "nnsp_tbl_tanh", tanh_interp()),
        _c_array("int16_t", "nnsp_tbl_tanh1", tanh_interp_shifted()),
        _c_array("int32_t", "nnsp_tbl_act", act_affine_table(), 8),
        _c_array("int32_t", "nnsp_tbl_tw256", cfft256_twiddles(), 6),
        _c_array("int32_t", "nnsp_tbl_split", rfft512_split_coefs(), 6),
        _c_array("int32_t", "nnsp_tbl_melseg", mel_segments(), 4),
        _c_array("int32_t", "nnsp_tbl_dif_tw", dif_twiddles(), 8),
        _c_array("int32_t", "nnsp_tbl_dif_rtw", rfft_dif_twiddles(), 8),
        _c_array("int16_t", "nnsp_tbl_bitrev8", bitrev8()),
        "#endif\n",
    ]
    return "\n".join(parts)


def export_text() -> str:
    """C file exporting the tables under the reference library's symbol names
    (window_stft_coef.c:3-6, melSpec_coeff.c:3-5, fixlog10.c:6, activation.c:5)."""
    def arr(ctype, name, vals):
        return _c_array(ctype, name, vals).replace("static const ", "").replace(f"{ctype} {name}", f"{ctype} {name}")
    mel = mel_bank_packed()
    return "\n".join([
        "/* GENERATED by nnsp_amd/tables.py -- do not edit. */",
        "#include <stdint.h>",
        f"const int16_t len_stft_win_coeff = {WIN_LEN};",
        f"const int16_t hop = {HOP};",
        f"const int16_t num_mfltrBank = {N_MEL};",
        arr("const int16_t", "stft_win_coeff", stft_window()),
        arr("const int16_t", "mfltrBank_coeff", mel),
        arr("const int16_t", "log_tayler_coeff", log_interp()),
        arr("int16_t", "coeffs_tanh", tanh_interp()),
        # the ARM_OPTIMIZED=0 build's FFT tables (twiddle_fft_dif.c:8-77)
        arr("const int32_t", "fft_tw_coeff", dif_twiddles()),
        arr("const int32_t", "rfft_tw_coeff", rfft_dif_twiddles()),
        arr("const int16_t", "br_coeff", bitrev8()),
    ])


def write_header(path: str | None = None) -> str:
    if path is None:
        path = os.path.join(os.path.dirname(__file__), "csrc", "gen", "nnsp_tables.h")
    for p, text in ((path, header_text()),
                    (os.path.join(os.path.dirname(path), "nnsp_tables_export.c"), export_text())):
        old = open(p).read() if os.path.exists(p) else None
        if old != text:
            os.makedirs(os.path.dirname(p), exist_ok=True)
            with open(p, "w") as f:
                f.write(text)
    return path


if __name__ == "__main__":
    print(write_header())
