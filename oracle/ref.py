"""TEST INFRASTRUCTURE ONLY: ctypes bindings of oracle/_ref/libdlq_ref.so.

That library is the reference DlQuantization C++ itself, compiled in place from
/root/reference by oracle/build_ref.sh (plus the extern "C" shim oracle/ref_shim.cpp).
It exists only where /root/reference exists (the build container); tests that need it
skip elsewhere. Used to generate tests/golden and to pin the C restatement.
"""
import ctypes
import os
import subprocess

import numpy as np

from oracle.oracle import Encoding, PDF_SIZE, _f32, _fp

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_ref", "libdlq_ref.so")
_REF_ROOT = os.environ.get("AIMET_REFERENCE", "/root/reference")


def available() -> bool:
    return os.path.exists(_LIB_PATH) or os.path.isdir(os.path.join(_REF_ROOT, "ModelOptimizations"))


def build():
    subprocess.run(["bash", os.path.join(_HERE, "build_ref.sh")], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        i64 = ctypes.c_int64
        pe = ctypes.POINTER(Encoding)
        L.ref_qdq_per_tensor.argtypes = [fp, fp, i64, ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.ref_quantize_per_tensor.argtypes = [fp, fp, i64, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                              ctypes.c_int]
        L.ref_fill_encoding_info.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, pe]
        L.ref_qdq_per_channel.argtypes = [fp, fp, i64, i64, i64, fp, fp, fp, fp]
        L.ref_get_computed_encodings.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_int, pe]
        L.ref_partial_encoding.argtypes = [ctypes.c_int, pe, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.ref_get_min.restype = ctypes.c_float
        L.ref_get_min.argtypes = [fp, i64]
        L.ref_get_max.restype = ctypes.c_float
        L.ref_get_max.argtypes = [fp, i64]
        L.ref_analyzer_create.restype = ctypes.c_void_p
        L.ref_analyzer_create.argtypes = [ctypes.c_int]
        L.ref_analyzer_destroy.argtypes = [ctypes.c_void_p]
        L.ref_analyzer_update.argtypes = [ctypes.c_void_p, fp, i64]
        L.ref_analyzer_compute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           pe]
        L.ref_analyzer_set_percentile.argtypes = [ctypes.c_void_p, ctypes.c_float]
        L.ref_analyzer_histogram.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double)]
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.ref_qdq_broadcast.argtypes = [fp, fp, i64, i64, i64p, i64p, fp, fp, fp, fp]
        L.ref_tpp_create.restype = ctypes.c_void_p
        L.ref_tpp_destroy.argtypes = [ctypes.c_void_p]
        L.ref_tpp_update.argtypes = [ctypes.c_void_p, fp, i64]
        L.ref_tpp_get.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


def qdq_per_tensor(x, enc_min, enc_max, bw):
    x = _f32(x)
    out = np.empty_like(x)
    lib().ref_qdq_per_tensor(_fp(x), _fp(out), x.size, float(enc_min), float(enc_max), int(bw))
    return out


def quantize_per_tensor(x, enc_min, enc_max, bw, shift_to_signed):
    x = _f32(x)
    out = np.empty_like(x)
    lib().ref_quantize_per_tensor(_fp(x), _fp(out), x.size, float(enc_min), float(enc_max), int(bw),
                                  int(bool(shift_to_signed)))
    return out


def fill_encoding_info(bw, mn, mx) -> Encoding:
    e = Encoding()
    lib().ref_fill_encoding_info(int(bw), float(mn), float(mx), ctypes.byref(e))
    return e


def qdq_per_channel(x, C, K, table):
    x = _f32(x)
    t = np.array(table, dtype=np.float32, copy=True)
    out = np.empty_like(x)
    lib().ref_qdq_per_channel(_fp(x), _fp(out), int(C), x.size, int(K), _fp(t[0]), _fp(t[1]), _fp(t[2]), _fp(t[3]))
    return out


def get_computed_encodings(bw, mn, mx, sym=False, strict=False, unsign=False) -> Encoding:
    e = Encoding()
    lib().ref_get_computed_encodings(int(bw), float(mn), float(mx), int(sym), int(strict), int(unsign),
                                     ctypes.byref(e))
    return e


def partial_encoding(bw, enc: Encoding, sym=False, unsign=False, strict=False) -> Encoding:
    e = Encoding(*enc.as_tuple())
    if lib().ref_partial_encoding(int(bw), ctypes.byref(e), int(sym), int(unsign), int(strict)) != 0:
        raise RuntimeError("Cannot determine how to compute partial encoding")
    return e


def qdq_broadcast(x, input_strides, encoding_strides, emin, emax, edelta, eoffset):
    x = _f32(x)
    out = np.empty_like(x)
    ist = np.ascontiguousarray(input_strides, dtype=np.int64)
    est = np.ascontiguousarray(encoding_strides, dtype=np.int64)
    arrs = [_f32(a) for a in (emin, emax, edelta, eoffset)]
    P = ctypes.POINTER(ctypes.c_int64)
    lib().ref_qdq_broadcast(_fp(x), _fp(out), x.size, len(ist), ist.ctypes.data_as(P), est.ctypes.data_as(P),
                            *[_fp(a) for a in arrs])
    return out


def get_min(x):
    x = _f32(x)
    return lib().ref_get_min(_fp(x), x.size)


def get_max(x):
    x = _f32(x)
    return lib().ref_get_max(_fp(x), x.size)


class Analyzer:
    def __init__(self, scheme):
        self._p = lib().ref_analyzer_create(int(scheme))
        self.scheme = scheme

    def __del__(self):
        if getattr(self, "_p", None) and _lib is not None:
            _lib.ref_analyzer_destroy(self._p)
            self._p = None

    def update(self, x):
        x = _f32(x)
        lib().ref_analyzer_update(self._p, _fp(x), x.size)

    def set_percentile(self, p):
        lib().ref_analyzer_set_percentile(self._p, float(p))

    def compute(self, bw, sym=False, strict=False, unsign=False) -> Encoding:
        e = Encoding()
        lib().ref_analyzer_compute(self._p, int(bw), int(sym), int(strict), int(unsign), ctypes.byref(e))
        return e

    def histogram(self):
        if self.scheme == 5:
            # EntropyEncodingAnalyzer::getStatsHistogram (EntropyEncodingAnalyzer.cpp:56-78) builds a
            # 1024-entry PDF next to a ~513-entry xLeft (assert) -- never called on this path
            raise NotImplementedError("getStatsHistogram is not defined for the entropy analyzer")
        xl = np.zeros(PDF_SIZE, dtype=np.float64)
        pdf = np.zeros(PDF_SIZE, dtype=np.float64)
        n = lib().ref_analyzer_histogram(self._p, xl.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                         pdf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        return xl[:n], pdf[:n]


class TensorProfilingParams:
    """The entropy analyzer's histogram state updated by the reference updateTensorHistogram_cpu."""

    def __init__(self):
        self._p = lib().ref_tpp_create()

    def __del__(self):
        if getattr(self, "_p", None) and _lib is not None:
            _lib.ref_tpp_destroy(self._p)
            self._p = None

    def update(self, x):
        x = _f32(x)
        lib().ref_tpp_update(self._p, _fp(x), x.size)

    def state(self):
        mn, mx, it = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        h = np.zeros(PDF_SIZE, dtype=np.float64)
        n = lib().ref_tpp_get(self._p, ctypes.byref(mn), ctypes.byref(mx),
                              h.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(it))
        return dict(has_hist=int(n != 0), min=mn.value, max=mx.value, hist=h, iterations=it.value)
