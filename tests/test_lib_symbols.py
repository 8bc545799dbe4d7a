"""libnnsp_mi355x.so loads on a machine without a GPU and exports every
function and table declared in include/*.h (no compute calls here)."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT
from nnsp_amd import _lib


def _declared_functions():
    names = set()
    for h in ("nnsp_api.h", "nnsp_batch.h", "nnsp_cascade.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"typedef[^;]*;", "", text, flags=re.S)
        text = re.sub(r"#define[^\n]*", "", text)
        for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", text):
            n = m.group(1)
            if n not in ("if", "while", "sizeof", "MAX", "MIN"):
                names.add(n)
    return names


def test_every_declared_symbol_is_exported():
    L = _lib.lib()
    names = _declared_functions()
    assert len(names) > 50
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing


def test_tables_exported():
    L = _lib.lib()
    for sym, n in (("stft_win_coeff", 480), ("mfltrBank_coeff", 534), ("log_tayler_coeff", 256),
                   ("coeffs_tanh", 384)):
        arr = (C.c_int16 * n).in_dll(L, sym)
        assert any(arr)
    assert C.c_int16.in_dll(L, "len_stft_win_coeff").value == 480
    assert C.c_int16.in_dll(L, "hop").value == 160
    assert C.c_int16.in_dll(L, "num_mfltrBank").value == 40


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "neural_nets.h"
#include "nn_speech.h"
#include "feature_module.h"
#define O(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f))
int main(void) {
    printf("NeuralNetClass %zu\nNNSPClass %zu\nFeatureClass %zu\nstftModule %zu\n",
           sizeof(NeuralNetClass), sizeof(NNSPClass), sizeof(FeatureClass), sizeof(stftModule));
    O(NeuralNetClass, size_layer); O(NeuralNetClass, net_layer_type); O(NeuralNetClass, qbit_kernel);
    O(NeuralNetClass, activation_type); O(NeuralNetClass, pt_cstate); O(NeuralNetClass, act_func);
    O(NeuralNetClass, layer_func); O(NeuralNetClass, pt_kernel_rec);
    O(NNSPClass, pt_net); O(NNSPClass, slides); O(NNSPClass, trigger); O(NNSPClass, counts_category);
    O(NNSPClass, pt_th_count_trigger); O(NNSPClass, outputs); O(NNSPClass, argmax_last);
    O(FeatureClass, feature); O(FeatureClass, normFeatContext); O(FeatureClass, pt_norm_mean);
    O(FeatureClass, qbit_output); O(stftModule, dataBuffer); O(stftModule, window);
    return 0;
}
"""


def _layout(include_dir):
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "p.c")
        open(src, "w").write(PROBE)
        exe = os.path.join(d, "p")
        subprocess.check_call(["gcc", "-I", include_dir, src, "-o", exe])
        return dict(l.rsplit(" ", 1) for l in subprocess.check_output([exe]).decode().split("\n") if l)


def _ctypes_layout():
    out = {"NeuralNetClass": C.sizeof(_lib.NeuralNetClass), "NNSPClass": C.sizeof(_lib.NNSPClass),
           "FeatureClass": C.sizeof(_lib.FeatureClass), "stftModule": C.sizeof(_lib.stftModule)}
    for T in (_lib.NeuralNetClass, _lib.NNSPClass, _lib.FeatureClass, _lib.stftModule):
        for f, *_ in T._fields_:
            out[f"{T.__name__}.{f}"] = getattr(T, f).offset
    return {k: str(v) for k, v in out.items()}


def test_struct_abi_matches_headers():
    mine = _layout(os.path.join(ROOT, "include"))
    ct = _ctypes_layout()
    for k, v in mine.items():
        assert ct[k] == v, (k, v, ct[k])


@pytest.mark.skipif(not os.path.isdir("/root/reference/ns-nnsp"), reason="reference absent")
def test_struct_abi_matches_reference_headers():
    assert _layout(os.path.join(ROOT, "include")) == _layout("/root/reference/ns-nnsp/includes-api")


CNTRL_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include <stdint.h>
#ifdef MINE
#include "nnsp_cascade.h"
#define CNTRL nnsp_ref_cntrl
#define PCMBUF nnsp_ref_pcmbuf
#define PARAMS nnsp_ref_params
#else
#include "nnCntrlClass.h"
#include "PcmBufClass.h"
#define CNTRL nnCntrlClass
#define PCMBUF PcmBufClass
#define PARAMS ParamCntrlClass
#endif
#define O(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f))
int main(void) {
    printf("cntrl %zu\npcmbuf %zu\nparams %zu\n", sizeof(CNTRL), sizeof(PCMBUF), sizeof(PARAMS));
    O(CNTRL, pt_seq_cntrl); O(CNTRL, len_seq_cntrl); O(CNTRL, current_pos_seq); O(CNTRL, pt_nnsp_arry);
    O(CNTRL, Params); O(CNTRL, cnt_timeout_kws); O(CNTRL, cnt_timeout_s2i); O(CNTRL, cnt_voice_frames_detected);
    O(CNTRL, cnt_voice_frames_not_detected);
    O(PARAMS, thresh_prob_vad); O(PARAMS, frs_vbufBk_s2i); O(PARAMS, thresh_timeout_s2i); O(PARAMS, frs_vbufBk_kws);
    O(PARAMS, thresh_timeout_kws); O(PARAMS, thresh_cnts_kws);
    O(PCMBUF, pcm_buffer); O(PCMBUF, idx_set); O(PCMBUF, idx_data_latest); O(PCMBUF, num_frs); O(PCMBUF, smpls_fr);
    return 0;
}
"""


def _cntrl_layout(mine: bool):
    import subprocess
    import tempfile
    inc = os.path.join(ROOT, "include") if mine else "/root/reference/evb/src"
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "p.c")
        open(src, "w").write(CNTRL_PROBE)
        exe = os.path.join(d, "p")
        subprocess.check_call(["gcc"] + (["-DMINE"] if mine else []) + ["-I", inc, src, "-o", exe])
        out = subprocess.check_output([exe]).decode().split("\n")
    return dict(l.rsplit(" ", 1) for l in out if l)


def test_ref_stream_mirrors_match_ctypes():
    """nnsp_ref_cntrl / nnsp_ref_pcmbuf / nnsp_ref_params (include/nnsp_cascade.h)
    against the ctypes mirrors the Python bindings pass."""
    mine = _cntrl_layout(True)
    assert mine["cntrl"] == str(C.sizeof(_lib.RefCntrl)) and mine["pcmbuf"] == str(C.sizeof(_lib.RefPcmBuf))
    assert mine["params"] == str(C.sizeof(_lib.RefParams))
    for k, v in mine.items():
        if "." in k:
            T, f = k.split(".")
            cls = {"CNTRL": _lib.RefCntrl, "PCMBUF": _lib.RefPcmBuf, "PARAMS": _lib.RefParams}[T]
            assert str(getattr(cls, f).offset) == v, (k, v)


@pytest.mark.skipif(not os.path.isdir("/root/reference/evb/src"), reason="reference absent")
def test_ref_stream_mirrors_match_reference_headers():
    """The mirrors are ABI-identical to the reference's own nnCntrlClass,
    ParamCntrlClass and PcmBufClass (evb/src/nnCntrlClass.h:11-45,
    PcmBufClass.h:9-16), so an application passes pointers to its objects."""
    assert _cntrl_layout(True) == _cntrl_layout(False)


@pytest.mark.skipif(not os.path.isdir("/root/reference/evb/src"), reason="reference absent")
@pytest.mark.parametrize("acc32", [False, True])
def test_reference_def_nets_compile_and_link_unchanged(tmp_path, acc32):
    """The reference's evb/src/def_nn{0_s2i,1_vad,2_kws_galaxy}.c compile
    unchanged against include/ and link against libnnsp_mi355x.so (the drop-in
    claim); their layer_func / act_func entries resolve to this
    library's fc_8x16 / lstm_8x16 (or the _acc32b twins under DEF_ACC32BIT_OPT,
    evb/Makefile:30-32) and activations, and their tables equal the committed
    tests/golden/ref_nets.npz dump."""
    import subprocess

    import numpy as np

    from nnsp_amd import nets

    src = "/root/reference/evb/src"
    so = str(tmp_path / "libdefnets.so")
    cmd = ["gcc", "-O1", "-fPIC", "-shared", "-I", os.path.join(ROOT, "include")]
    cmd += ["-DDEF_ACC32BIT_OPT"] if acc32 else []
    cmd += [os.path.join(src, f) for f in ("def_nn0_s2i.c", "def_nn1_vad.c", "def_nn2_kws_galaxy.c")]
    cmd += ["-L", os.path.dirname(_lib.LIB_PATH), "-lnnsp_mi355x", "-Wl,-rpath," + os.path.dirname(_lib.LIB_PATH),
            "-Wl,-z,defs", "-Wl,--allow-shlib-undefined", "-o", so]
    subprocess.check_call(cmd)
    L = _lib.lib()
    D = C.CDLL(so)
    z = np.load(nets.REF_NETS_NPZ)
    for name, sym in (("vad", "net_vad"), ("kws", "net_kws_galaxy"), ("s2i", "net_s2i")):
        n = _lib.NeuralNetClass.in_dll(D, sym)
        for i in range(n.numlayers):
            lstm = n.net_layer_type[i] == nets.LSTM
            want = ("lstm_8x16" if lstm else "fc_8x16") + ("_acc32b" if acc32 else "")
            assert n.layer_func[i] == _lib.fn_addr(want), (name, i)
            act = ["relu6_fix", "tanh_fix", "sigmoid_fix", "linear_fix"][n.activation_type[i]]
            assert n.act_func[i] == _lib.fn_addr(act), (name, i)
            K, N = n.size_layer[i], n.size_layer[i + 1]
            rows = 4 * N if lstm else N
            kern = np.ctypeslib.as_array((C.c_int8 * (rows * K)).from_address(n.pt_kernel[i]))
            np.testing.assert_array_equal(kern, z[f"{name}_kernel{i}"])


PORTABLE_APP = r"""
#include <stdint.h>
#include "fft.h"
#include "complex.h"
#include "spectrogram_module.h"
/* a portable (ARM_OPTIMIZED=0) caller of the reference's fft.h / complex.h
 * API: compiles against include/ and links; nothing is run (no GPU here) */
int use(int32_t *x, void *y)
{
    COMPLEX32 a = {1, 2}, b = {3, 4}, o;
    COMPLEX16 w = {5, 6};
    rfft(512, x, y);
    fft(7, x, y);
    complex32_add(&o, &a, &b);
    complex32_sub(&o, &a, &b);
    complex32_mul(&o, &a, &b);
    complex32_complex16_elmtprod(&o, &a, &w, 1);
    complex32_interprod(&o, &a, &b, 0, 1);
    complexArry32_print(&o, 1);
    spec2pspec((int32_t *)y, x, 257);
    return o.real;
}
"""


def test_portable_fft_complex_headers_compile_and_link(tmp_path):
    """include/fft.h and include/complex.h stand in for ns-nnsp/includes-api's
    (fft.h:4-5, complex.h): a portable application compiles and links."""
    import subprocess
    src = tmp_path / "app.c"
    src.write_text(PORTABLE_APP)
    so = str(tmp_path / "libapp.so")
    subprocess.check_call(["gcc", "-Wall", "-Werror", "-fPIC", "-shared", "-I", os.path.join(ROOT, "include"), str(src),
                           "-L", os.path.dirname(_lib.LIB_PATH), "-lnnsp_mi355x", "-Wl,-z,defs",
                           "-Wl,--allow-shlib-undefined", "-o", so])


@pytest.mark.skipif(not os.path.isdir("/root/reference/ns-nnsp"), reason="reference absent")
def test_complex_types_match_reference_header(tmp_path):
    import subprocess
    probe = ('#include <stdio.h>\n#include <stddef.h>\n#include "complex.h"\nint main(void){printf("%zu %zu %zu %zu\\n",'
             ' sizeof(COMPLEX32), offsetof(COMPLEX32, imag), sizeof(COMPLEX16), offsetof(COMPLEX16, imag));}\n')
    (tmp_path / "p.c").write_text(probe)
    outs = []
    for inc in (os.path.join(ROOT, "include"), "/root/reference/ns-nnsp/includes-api"):
        exe = str(tmp_path / "p")
        subprocess.check_call(["gcc", "-I", inc, str(tmp_path / "p.c"), "-o", exe])
        outs.append(subprocess.check_output([exe]))
    assert outs[0] == outs[1] == b"8 4 4 2\n"
