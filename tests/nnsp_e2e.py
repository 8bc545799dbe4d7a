"""Shared by the end-to-end NNSPClass_exec parity tests: the streams of
tests/golden/ref_nnsp_portable.npz (written by make_golden.py nnsp from the
reference's own ARM_OPTIMIZED=0 build of nn_speech.c + front end + NN) and the
fixture's per-stream slices.  Everything here is test infrastructure."""
import os

import numpy as np

from conftest import ROOT
from oracle import synthetic_pcm

GOLD = os.path.join(ROOT, "tests", "golden", "ref_nnsp_portable.npz")
WAVS = ("speech", "galaxy", "galaxy_s2i")


def fixture():
    return np.load(GOLD)


def streams(g):
    """[(pcm [T][160] int16, reset frame, first row in the fixture)], the
    same order and inputs as make_golden.nnsp_streams()."""
    wav_t, wav_r, noise_t, noise_r = (int(v) for v in g["cfg"])
    wz = np.load(os.path.join(ROOT, "tests", "golden", "test_wavs.npz"))
    out, row = [], 0
    for w in WAVS:
        out.append((wz[w][:wav_t * 160].reshape(wav_t, 160), wav_r, row))
        row += wav_t
    for amp, seed in g["noise_cfg"]:
        out.append((synthetic_pcm(1, noise_t, seed=int(seed), amp=int(amp))[0], noise_r, row))
        row += noise_t
    return out


def groups(g):
    """The streams as two equal-length groups (the wavs, the noise) for the
    batched engine: (pcm [S][T][160], reset frame, fixture rows [S][T])."""
    st = streams(g)
    out = []
    for sel in (st[:3], st[3:]):
        pcm = np.stack([s[0] for s in sel])
        T = pcm.shape[1]
        rows = np.stack([np.arange(s[2], s[2] + T) for s in sel])
        out.append((pcm, sel[0][1], rows))
    return out
