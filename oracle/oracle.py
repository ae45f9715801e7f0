"""TEST INFRASTRUCTURE ONLY: ctypes bindings of oracle/liboracle.so (dlq_oracle.c).

Mirrors the reference CPU DlQuantization arithmetic; see dlq_oracle.c for file:line
citations. Never imported by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
PDF_SIZE = 512

QUANTIZATION_TF, QUANTIZATION_TF_ENHANCED, QUANTIZATION_RANGE_LEARNING, QUANTIZATION_PERCENTILE, \
    QUANTIZATION_MSE, QUANTIZATION_ENTROPY = range(6)


class Encoding(ctypes.Structure):
    _fields_ = [("min", ctypes.c_double), ("max", ctypes.c_double), ("delta", ctypes.c_double),
                ("offset", ctypes.c_double), ("bw", ctypes.c_int)]

    def as_tuple(self):
        return (self.min, self.max, self.delta, self.offset, self.bw)

    def __repr__(self):
        return "Encoding(min=%r, max=%r, delta=%r, offset=%r, bw=%d)" % self.as_tuple()


def build():
    """Compile liboracle.so (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or \
                os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "dlq_oracle.c")):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        dp = ctypes.POINTER(ctypes.c_double)
        i64 = ctypes.c_int64
        L.orc_get_computed_encodings.restype = Encoding
        L.orc_get_computed_encodings.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                                 ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_fill_encoding_info.restype = Encoding
        L.orc_fill_encoding_info.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double]
        L.orc_min_max_from_delta_offset.argtypes = [ctypes.c_int, ctypes.POINTER(Encoding), ctypes.c_int,
                                                    ctypes.c_int, ctypes.c_int]
        L.orc_delta_offset_from_min_max.argtypes = L.orc_min_max_from_delta_offset.argtypes
        L.orc_qdq_per_tensor.argtypes = [fp, fp, i64, ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.orc_quantize_per_tensor.argtypes = [fp, fp, i64, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                              ctypes.c_int]
        L.orc_per_channel_table.argtypes = [ctypes.POINTER(Encoding), i64, fp]
        L.orc_qdq_per_channel.argtypes = [fp, fp, i64, i64, i64, fp]
        L.orc_qdq_per_tensor_omp.argtypes = [fp, fp, i64, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                             ctypes.c_int]
        L.orc_qdq_per_channel_omp.argtypes = [fp, fp, i64, i64, i64, fp, ctypes.c_int]
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.orc_qdq_broadcast.argtypes = [fp, fp, i64, i64, i64p, i64p, fp, fp, fp, fp]
        L.orc_permute.argtypes = [fp, fp, i64, i64, i64p, i64p]
        L.orc_ste_backward.argtypes = [fp, fp, fp, i64, i64, i64, fp, fp]
        L.orc_get_min.restype = ctypes.c_float
        L.orc_get_min.argtypes = [fp, i64]
        L.orc_get_max.restype = ctypes.c_float
        L.orc_get_max.argtypes = [fp, i64]
        L.orc_analyzer_size.restype = ctypes.c_size_t
        L.orc_analyzer_init.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_analyzer_set_percentile.argtypes = [ctypes.c_void_p, ctypes.c_float]
        L.orc_analyzer_update.argtypes = [ctypes.c_void_p, fp, i64]
        L.orc_analyzer_compute.restype = Encoding
        L.orc_analyzer_compute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_analyzer_histogram.argtypes = [ctypes.c_void_p, dp, dp]
        L.orc_analyzer_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), dp, dp,
                                         ctypes.POINTER(ctypes.c_int), fp, dp, ctypes.POINTER(ctypes.c_int)]
        L.orc_analyzer_fold_minmax.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float]
        L.orc_analyzer_pdf.restype = ctypes.c_void_p
        L.orc_analyzer_pdf.argtypes = [ctypes.c_void_p]
        L.orc_update_pdf_from_counts.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), i64]
        L.orc_initialize_pdf.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_int]
        L.orc_get_histogram.argtypes = [fp, i64, ctypes.POINTER(ctypes.c_uint32), ctypes.c_float, ctypes.c_float,
                                        ctypes.c_int]
        _lib = L
    return _lib


def _f32(x):
    return np.ascontiguousarray(x, dtype=np.float32)


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def get_computed_encodings(bw, mn, mx, sym=False, strict=False, unsign=False) -> Encoding:
    return lib().orc_get_computed_encodings(int(bw), float(mn), float(mx), int(sym), int(strict), int(unsign))


def fill_encoding_info(bw, mn, mx) -> Encoding:
    return lib().orc_fill_encoding_info(int(bw), float(mn), float(mx))


def partial_encoding(bw, enc: Encoding, sym=False, unsign=False, strict=False):
    e = Encoding(*enc.as_tuple())
    if e.min == 0 and e.max == 0:
        rc = lib().orc_min_max_from_delta_offset(int(bw), ctypes.byref(e), int(sym), int(unsign), int(strict))
    elif e.delta == 0:
        rc = lib().orc_delta_offset_from_min_max(int(bw), ctypes.byref(e), int(sym), int(unsign), int(strict))
    else:
        rc = -1
    if rc != 0:
        raise RuntimeError("Cannot determine how to compute partial encoding")
    return e


def qdq_per_tensor(x, enc_min, enc_max, bw):
    x = _f32(x)
    out = np.empty_like(x)
    lib().orc_qdq_per_tensor(_fp(x), _fp(out), x.size, float(enc_min), float(enc_max), int(bw))
    return out


def quantize_per_tensor(x, enc_min, enc_max, bw, shift_to_signed):
    x = _f32(x)
    out = np.empty_like(x)
    lib().orc_quantize_per_tensor(_fp(x), _fp(out), x.size, float(enc_min), float(enc_max), int(bw),
                                  int(bool(shift_to_signed)))
    return out


def per_channel_table(encs):
    """encs: list of (min, max, delta, offset, bw) -> float32 [4, C] (min, max, delta, offset)."""
    C = len(encs)
    arr = (Encoding * C)(*[Encoding(*map(float, e[:4]), int(e[4])) for e in encs])
    table = np.empty((4, C), dtype=np.float32)
    lib().orc_per_channel_table(arr, C, _fp(table))
    return table


def qdq_per_tensor_omp(x, enc_min, enc_max, bw, threads):
    x = _f32(x)
    out = np.empty_like(x)
    lib().orc_qdq_per_tensor_omp(_fp(x), _fp(out), x.size, float(enc_min), float(enc_max), int(bw), int(threads))
    return out


def qdq_per_channel_omp(x, C, K, table, threads):
    x = _f32(x)
    out = np.empty_like(x)
    table = _f32(table)
    lib().orc_qdq_per_channel_omp(_fp(x), _fp(out), int(C), x.size, int(K), _fp(table), int(threads))
    return out


def openmp_enabled():
    return bool(lib().orc_openmp_enabled())


def qdq_per_channel(x, C, K, table):
    x = _f32(x)
    out = np.empty_like(x)
    table = _f32(table)
    lib().orc_qdq_per_channel(_fp(x), _fp(out), int(C), x.size, int(K), _fp(table))
    return out


def ste_backward(x, g, mins, maxs, C=1, K=1):
    x, g = _f32(x), _f32(g)
    mins, maxs = _f32(np.atleast_1d(mins)), _f32(np.atleast_1d(maxs))
    out = np.empty_like(x)
    lib().orc_ste_backward(_fp(x), _fp(g), _fp(out), x.size, int(C), int(K), _fp(mins), _fp(maxs))
    return out


def _i64a(v):
    a = np.ascontiguousarray(v, dtype=np.int64)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def qdq_broadcast(x, input_strides, encoding_strides, emin, emax, edelta, eoffset):
    """trim_functions.cpp:633-660 quantizeDequantizeBroadcastCpu (float encoding arrays, used as given)."""
    x = _f32(x)
    out = np.empty_like(x)
    ist, ip = _i64a(input_strides)
    est, ep = _i64a(encoding_strides)
    arrs = [_f32(a) for a in (emin, emax, edelta, eoffset)]
    lib().orc_qdq_broadcast(_fp(x), _fp(out), x.size, len(ist), ip, ep, *[_fp(a) for a in arrs])
    return out


def permute(x, input_strides, output_strides):
    """QuantizeDequantizeUtils.cpp:64-95 permuteTensorCPU."""
    x = _f32(x)
    out = np.empty_like(x)
    ist, ip = _i64a(input_strides)
    ost, op = _i64a(output_strides)
    lib().orc_permute(_fp(x), _fp(out), x.size, len(ist), ip, op)
    return out


def _row_major(shape):
    st, s = [], 1
    for d in reversed(shape):
        st.append(s)
        s *= d
    return st[::-1]


def broadcast_shape_info(input_shape, channel_axis, block_axis, block_size):
    """QuantizeDequantizeUtils.cpp:100-170 BroadcastShapeInfo (+ hasContiguousBlocks)."""
    tshape, eshape = [], []
    for i, d in enumerate(input_shape):
        if i == channel_axis:
            tshape.append(d)
            eshape.append(d)
        elif i == block_axis:
            if d % block_size != 0:
                raise RuntimeError("Block dimension is not evenly divisible by block size.")
            tshape += [d // block_size, block_size]
            eshape += [d // block_size, 1]
        else:
            tshape.append(d)
            eshape.append(1)
    estr = [0 if (e == 1 and t != 1) else s for e, t, s in zip(eshape, tshape, _row_major(eshape))]
    contiguous, prev = True, False
    for t, e in zip(tshape, eshape):
        if prev and t == e:
            contiguous = False
        prev = t != e
    return dict(num_dims=len(tshape), tensor_shape=tshape, encoding_shape=eshape, tensor_strides=_row_major(tshape),
                encoding_strides=estr, num_elements=int(np.prod(input_shape)) if len(input_shape) else 1,
                num_encodings=int(np.prod(eshape)) if eshape else 1, contiguous_blocks=contiguous)


def block_layout_strides(info):
    """copyToContiguousBlockLayout's output strides (QuantizeDequantizeUtils.cpp:173-203)."""
    nd, es, ts = info["num_dims"], info["encoding_strides"], info["tensor_shape"]
    order = [i for i in range(nd) if es[i] != 0] + [i for i in range(nd) if es[i] == 0]
    ost = [0] * nd
    ost[order[-1]] = 1
    for i in range(nd - 2, -1, -1):
        ost[order[i]] = ost[order[i + 1]] * ts[order[i + 1]]
    return ost


def copy_to_contiguous_block_layout(x, info):
    return permute(x, info["tensor_strides"], block_layout_strides(info))


def qdq_fp16(x):
    """quantizeDequantizeFp16Cpu (AimetOpUtils.cpp:61-67): float -> half (RNE) -> float."""
    with np.errstate(over="ignore"):
        return _f32(x).astype(np.float16).astype(np.float32)


def get_min(x):
    x = _f32(x)
    return lib().orc_get_min(_fp(x), x.size)


def get_max(x):
    x = _f32(x)
    return lib().orc_get_max(_fp(x), x.size)


def histogram(x, bucket_size, pdf_offset, is_signed=True):
    x = _f32(x)
    h = np.zeros(PDF_SIZE, dtype=np.uint32)
    lib().orc_get_histogram(_fp(x), x.size, h.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                            float(bucket_size), float(pdf_offset), int(is_signed))
    return h


class _Tpp(ctypes.Structure):
    """orc_tpp (TensorProfilingParams, math_functions.hpp:71-77)."""
    _fields_ = [("min", ctypes.c_double), ("max", ctypes.c_double), ("hist", ctypes.c_double * PDF_SIZE),
                ("has_hist", ctypes.c_int), ("iterations", ctypes.c_int)]


class Analyzer:
    """IQuantizationEncodingAnalyzer<float> restated (TF, TF-E, percentile, MSE, entropy)."""

    def __init__(self, scheme):
        L = lib()
        self._buf = ctypes.create_string_buffer(L.orc_analyzer_size())
        if L.orc_analyzer_init(self._buf, int(scheme)) != 0:
            raise ValueError("scheme %d not restated in the oracle" % scheme)
        self.scheme = scheme

    def update(self, x):
        x = _f32(x)
        lib().orc_analyzer_update(self._buf, _fp(x), x.size)

    def update_from_counts(self, counts, n):
        """PDF update from histogram counts summed elsewhere (sharded calibration)."""
        c = np.ascontiguousarray(counts, dtype=np.uint64)
        pdf = lib().orc_analyzer_pdf(self._buf)
        lib().orc_update_pdf_from_counts(pdf, c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), int(n))

    def set_percentile(self, p):
        lib().orc_analyzer_set_percentile(self._buf, float(p))

    def fold_minmax(self, mn, mx):
        """Apply an exchanged batch min/max; True when a histogram update must follow."""
        return bool(lib().orc_analyzer_fold_minmax(self._buf, float(mn), float(mx)))

    def compute(self, bw, sym=False, strict=False, unsign=False) -> Encoding:
        return lib().orc_analyzer_compute(self._buf, int(bw), int(sym), int(strict), int(unsign))

    def stats(self):
        """Reduced statistics: dict(stats_updated, acc_min, acc_max, initialized, hist_min, bucket_size,
        iterations, pdf)."""
        su, ini, it = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        amin, amax, bs = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        hm = ctypes.c_float()
        lib().orc_analyzer_stats(self._buf, ctypes.byref(su), ctypes.byref(amin), ctypes.byref(amax),
                                 ctypes.byref(ini), ctypes.byref(hm), ctypes.byref(bs), ctypes.byref(it))
        _, pdf = self.histogram()
        return dict(stats_updated=su.value, acc_min=amin.value, acc_max=amax.value, initialized=ini.value,
                    hist_min=hm.value, bucket_size=bs.value, iterations=it.value,
                    pdf=pdf if ini.value else np.zeros(PDF_SIZE))

    def entropy_state(self):
        """TensorProfilingParams of the entropy analyzer: dict(has_hist, min, max, hist, iterations)."""
        L = lib()
        L.orc_analyzer_tpp.restype = ctypes.POINTER(_Tpp)
        t = L.orc_analyzer_tpp(self._buf).contents
        return dict(has_hist=t.has_hist, min=t.min, max=t.max, hist=np.array(t.hist[:], dtype=np.float64),
                    iterations=t.iterations)

    def histogram(self):
        xl = np.zeros(PDF_SIZE, dtype=np.float64)
        pdf = np.zeros(PDF_SIZE, dtype=np.float64)
        n = lib().orc_analyzer_histogram(self._buf, xl.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                         pdf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        return xl[:n], pdf[:n]
