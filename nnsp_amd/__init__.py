"""nnsp_amd -- MI355X-native ns-nnsp per-frame inference (front end + 8x16
fixed-point NN), bit-exact with the reference C library.

The product is ``libnnsp_mi355x.so`` (hand-written gfx950 kernels + a C host
library exporting the reference's NNSPClass / FeatureClass / NeuralNetClass C
API and a batched multi-stream API).  This package is its Python host mirror.
"""
from .nets import SPECS, NetData, NetSpec, synth_net  # noqa: F401

__all__ = ["SPECS", "NetData", "NetSpec", "synth_net", "NNSPBatch"]


def __getattr__(name):
    if name == "NNSPBatch":
        from .engine import NNSPBatch
        return NNSPBatch
    raise AttributeError(name)
