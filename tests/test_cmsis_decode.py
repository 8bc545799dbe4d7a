"""Row N1: the oracle's CMSIS rFFT restatement (oracle/nnsp_oracle.c:29-170,
nnsp_amd/csrc/kernels/nnsp_dev.h bfly4 / split_bin) against a static decode of
the shipped evb/libs/libCMSISDSP.a -- the archive is read as bytes by
oracle/tools/cmsis_decode.py, never executed.  The decode's instruction counts
are committed as tests/golden/cmsis_decode.json; when the reference tree is
present the decode is re-run and must reproduce the fixture.

What the counts pin (hand-read from the decoded stream of arm_split_rfft_q31
as well, e.g. `mov.w r3,#0x80000000; smlal r3,r0,r12,r1` = a rounded product,
and `negs; sbc.w; adds.w #0x80000000; adc.w #0` = a rounded subtract):
  * arm_radix4_butterfly_q31 multiplies with SMULL only and never adds the low
    words (no SMLAL, ADC, SBC): each twiddle product is its truncated high word,
    (a * b) >> 32 -- the restatement's mulhi;
  * its immediate shifts include asr #4 (the first stage's guard bits), asr #2
    (the sums of the later stages), asr #1 and lsl #1 (the rotated outputs);
  * arm_split_rfft_q31 rounds every product on its own: 8 products per loop
    body, each with the 2^31 rounding constant and a carry into the high word
    -- rnd_add / rnd_sub, SMMLAR / SMMLSR semantics (none.h:185-194);
  * the split's only arithmetic shift is asr #1 (DC and Nyquist, (p0 +- p1) >> 1).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "cmsis_decode.json")
ARCHIVE = "/root/reference/evb/libs/libCMSISDSP.a"


def fixture():
    with open(FIX) as f:
        return json.load(f)["functions"]


def test_butterfly_products_truncated_high_word():
    b = fixture()["arm_radix4_butterfly_q31"]
    assert b["smull"] >= 24            # 12 products per butterfly, first and middle stages
    assert b["smlal"] == 0 and b["adc"] == 0 and b["sbc"] == 0
    assert b["smmul"] == b["smmulr"] == b["smmla"] == b["smmlar"] == 0
    assert b["imm_2p31"] == 0          # no rounding constant anywhere in the butterflies


def test_butterfly_guard_bit_shifts():
    sh = fixture()["arm_radix4_butterfly_q31"]["shifts"]
    for k in ("asr#4", "asr#2", "asr#1", "lsl#1"):
        assert sh.get(k, 0) > 0, k
    assert not any(k.startswith("asr#") and k not in ("asr#1", "asr#2", "asr#4") for k in sh)


def test_split_rounds_each_product():
    s = fixture()["arm_split_rfft_q31"]
    products = s["smull"] + s["smlal"]
    assert products == 16              # two loop bodies x 8 products (4 per output, re and im)
    assert s["imm_2p31"] == products   # one rounding constant per product
    assert s["adc"] > 0 and s["sbc"] > 0
    assert set(k for k in s["shifts"] if k.startswith("asr")) == {"asr#1"}


def test_inverse_paths_mirror_forward():
    f = fixture()
    assert f["arm_radix4_butterfly_inverse_q31"]["smull"] == f["arm_radix4_butterfly_q31"]["smull"]
    assert f["arm_radix4_butterfly_inverse_q31"]["shifts"] == f["arm_radix4_butterfly_q31"]["shifts"]


@pytest.mark.skipif(not os.path.exists(ARCHIVE), reason="reference tree absent (GPU box)")
def test_decode_reproduces_fixture():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "tools", "cmsis_decode.py"), ARCHIVE],
                         check=True, capture_output=True, text=True).stdout
    assert json.loads(out)["functions"] == fixture()
