"""Row N4, host side (no GPU): nnsp_batch_create_ex(arm_optimized=0) refuses,
before touching the device, a layer whose live align shift (affine.c:311-313)
the engine's bias-then-shift epilogue cannot reproduce exactly -- here KWS
layer 0 (qbit_input + qbit_kernel = 14) with qbit_bias raised above 14."""
import ctypes as C
import dataclasses

from nnsp_amd import _lib
from nnsp_amd.nets import ref_net


def _create(data, arm_optimized):
    h = _lib.NetHandle(data, arm_optimized=bool(arm_optimized))
    b = C.c_void_p()
    rc = _lib.lib().nnsp_batch_create_ex(C.byref(b), h.addr, data.spec.nn_id, _lib.ptr(h.mean), _lib.ptr(h.stdR),
                                         16383, 4, 4, 4, arm_optimized)
    return rc, _lib.lib().nnsp_strerror(rc).decode()


def test_portable_align_not_representable_is_refused():
    d = ref_net("kws")
    d2 = dataclasses.replace(d, spec=dataclasses.replace(d.spec, qb=[15] + list(d.spec.qb[1:])))
    rc, msg = _create(d2, 0)
    assert rc == -2 and "portable align shift" in msg, msg


def test_arm_optimized_flag_validated():
    rc, msg = _create(ref_net("vad"), 2)
    assert rc == -1 and "arm_optimized" in msg, msg
