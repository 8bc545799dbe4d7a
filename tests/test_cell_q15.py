"""The range check of nnsp_dev.h's cell_q15 (recur_pipe_kernel's LSTM cell
update, lstm.c's sat32((i*g + f*c) >> 15)) restated in numpy and checked
against the plain 64-bit saturating form over the operand extremes: the
kernel tests the high word only (x >> 15 fits int32 iff x >> 46 is 0 or -1,
for |x| < 2^47) and takes the low word from a funnel shift."""
import numpy as np


def _sat32_ref(x):
    return np.clip(x >> 15, -2**31, 2**31 - 1)


def _cell_q15(x):
    hi = (x >> 32).astype(np.int64)            # the high word, arithmetic
    y = ((x >> 15) & 0xFFFFFFFF).astype(np.int64)
    y = np.where(y >= 2**31, y - 2**32, y)     # alignbit(hi, lo, 15) as int32
    fits = (((hi >> 14) + 1) & 0xFFFFFFFF) < 2
    sat = np.where(hi < 0, -2**31, 2**31 - 1)
    return np.where(fits, y, sat)


def test_cell_q15_matches_sat32_at_the_extremes():
    g = np.array([-32768, -32767, -16384, -1, 0, 1, 16384, 32767], np.int64)
    c = np.array([-2**31, -2**31 + 1, -2**30, -65536, -32768, -1, 0, 1, 32767, 65536, 2**30,
                  2**31 - 2, 2**31 - 1], np.int64)
    a, b, f, cc = np.meshgrid(g, g, g, c, indexing="ij")
    x = a * b + f * cc
    np.testing.assert_array_equal(_cell_q15(x.ravel()), _sat32_ref(x.ravel()))


def test_cell_q15_matches_sat32_random():
    rng = np.random.default_rng(7)
    n = 1 << 20
    a, b, f = (rng.integers(-32768, 32768, n) for _ in range(3))
    cc = rng.integers(-2**31, 2**31, n)
    x = a * b + f * cc
    np.testing.assert_array_equal(_cell_q15(x), _sat32_ref(x))


def test_sat32_shr15_any_int64():
    """nnsp_dev.h's sat32_shr15 (the same check, used on the front end's Mel
    sums) holds over the whole int64 range, not only the cell's |x| < 2^47."""
    rng = np.random.default_rng(11)
    edges = np.array([-2**63, -2**63 + 1, -2**46 - 1, -2**46, -2**46 + 1, -1, 0, 1, 2**46 - 1, 2**46,
                      2**46 + 1, 2**63 - 1], np.int64)
    x = np.concatenate([edges, rng.integers(-2**63, 2**63 - 1, 1 << 20, dtype=np.int64),
                        rng.integers(-2**48, 2**48, 1 << 20, dtype=np.int64)])
    np.testing.assert_array_equal(_cell_q15(x), _sat32_ref(x))


def test_cell_without_saturation_for_lstm_gate_ranges():
    """cell_q15_gates (nnsp_dev.h, recur_pipe_kernel): for the gates' own
    ranges -- i, f in [0, 32767] (sigmoid_fix) and g in [-32767, 32767]
    (tanh_fix) -- and any int32 cell state, lstm.c's sat32((i*g + f*c) >> 15)
    never saturates, so the plain shift equals it."""
    i = np.array([0, 1, 16384, 32766, 32767], np.int64)
    g = np.array([-32767, -32766, -1, 0, 1, 32766, 32767], np.int64)
    c = np.array([-2**31, -2**31 + 1, -2**30, -1, 0, 1, 2**30, 2**31 - 2, 2**31 - 1], np.int64)
    a, b, f, cc = np.meshgrid(i, g, i, c, indexing="ij")
    x = (a * b + f * cc).ravel()
    assert (x >> 15).max() <= 2147450878 and (x >> 15).min() >= -2147450879
    np.testing.assert_array_equal(x >> 15, _sat32_ref(x))
    rng = np.random.default_rng(3)
    n = 1 << 20
    a, f = rng.integers(0, 32768, n), rng.integers(0, 32768, n)
    b, cc = rng.integers(-32767, 32768, n), rng.integers(-2**31, 2**31, n)
    x = a * b + f * cc
    np.testing.assert_array_equal(x >> 15, _sat32_ref(x))
