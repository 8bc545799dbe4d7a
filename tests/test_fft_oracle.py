"""The CMSIS arm_rfft_q31 restatement against a float DFT (scale 2^-9).

CMSIS-DSP 1.10.0 ships here only as a Cortex-M binary (never executed), so the
restated butterflies / rounding cannot be compared to the shipped code bit for
bit; this test pins the transform's mathematics (size, scaling, sign, bin
order, conjugate-symmetric upper half) to within the fixed-point error of its
guard-bit scheme."""
import numpy as np
import pytest

import oracle as O
from nnsp_amd.tables import stft_window


@pytest.mark.parametrize("amp", [1, 100, 4096, 20000, 32767])
def test_rfft_vs_float_dft(amp):
    rng = np.random.default_rng(amp)
    w = stft_window().astype(np.int64)
    for _ in range(20):
        pcm = rng.integers(-amp, amp + 1, 480)
        x = np.zeros(512, np.int64)
        x[:480] = w * pcm
        y, _ = O.rfft512(x.astype(np.int32))
        ref = np.fft.fft(x.astype(np.float64)) / 512.0
        got = y[0::2] + 1j * y[1::2]
        assert np.abs(got - ref).max() < 16.0
        # bins 257..511 are the conjugates of 255..1 (arm_split_rfft_q31 pOut2)
        np.testing.assert_array_equal(y[2 * 257::2], y[2 * 255:0:-2][:255])
        np.testing.assert_array_equal(y[2 * 257 + 1::2], -y[2 * 255 + 1:1:-2][:255])


def test_rfft_dc_and_impulse():
    x = np.zeros(512, np.int32)
    x[0] = 1 << 28
    y, _ = O.rfft512(x)
    # an impulse has a flat spectrum of 2^28 / 512 = 2^19 (within guard-bit error)
    assert np.abs(y[0::2][:257] - (1 << 19)).max() <= 16
    assert np.abs(y[1::2][:257]).max() <= 16
