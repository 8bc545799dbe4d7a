import os
import sys

import pytest

# torch first: its bundled HIP runtime is then the one every test process
# uses (the product library resolves libamdhip64 to it); initialising the HIP
# runtime through libnnsp_mi355x.so first leaves torch without GPUs.
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def have_reference() -> bool:
    return os.path.isdir(os.path.join(REFERENCE, "ns-nnsp"))


needs_reference = pytest.mark.skipif(not have_reference(), reason="reference tree not present")
