"""CPU tests of the product library: it loads, exports every symbol include/aimet_amd.h declares,
and its HOST-side encoding math (the part of the path that runs on the CPU in the reference too)
is bit-exact against the golden vectors. No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, analyzer_case

import aimet_amd
from aimet_amd import _native
from aimet_amd._native import TfEncodingC
from oracle import oracle as O

HEADER = os.path.join(REPO, "include", "aimet_amd.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(aimet_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_exports_header_symbols():
    lib = aimet_amd.native_library()
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), "libaimet_amd.so does not export %s" % s
    # the Python binding covers every declared entry point, and nothing else
    assert sorted(_native.EXPORTED_SYMBOLS) == syms
    assert lib.aimet_version().decode().startswith("aimet_amd")


def test_library_has_gfx950_code_object():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def _enc(fn, *args):
    out = TfEncodingC()
    _native.call(fn, *args, out)
    return (out.min, out.max, out.delta, out.offset, out.bw)


def test_host_computed_encodings_golden(golden_core):
    for inp, want in zip(golden_core["gce_in"], golden_core["gce_out"]):
        bw, mn, mx, sym, strict, un = inp
        got = _enc("aimet_get_computed_encodings", int(bw), mn, mx, int(sym), int(strict), int(un))
        np.testing.assert_array_equal(np.array(got[:4]), want[:4])
        assert got[4] == int(want[4])


def test_host_fill_encoding_info_golden(golden_core):
    for enc, want in zip(golden_core["pt_enc"], golden_core["pt_fill"]):
        got = _enc("aimet_fill_encoding_info", int(enc[2]), enc[0], enc[1])
        assert got[:4] == tuple(want[:4])


def test_host_partial_encoding_vs_oracle():
    rng = np.random.default_rng(3)
    for _ in range(200):
        bw = int(rng.choice([4, 8, 16]))
        sym, unsign, strict = (int(v) for v in rng.integers(0, 2, 3))
        if rng.uniform() < 0.5:
            e = O.Encoding(0.0, 0.0, float(rng.uniform(1e-4, 0.1)), float(-rng.integers(0, 2 ** bw)), bw)
        else:
            lo, hi = sorted(rng.uniform(-5, 5, 2))
            e = O.Encoding(lo, hi, 0.0, 0.0, bw)
        want = O.partial_encoding(bw, e, sym, unsign, strict).as_tuple()
        # argument order of the C-ABI: (bw, enc, use_symmetric, use_unsigned_symmetric, use_strict_symmetric)
        c = TfEncodingC(*e.as_tuple())
        _native.call("aimet_compute_partial_encoding", bw, ctypes.byref(c), sym, unsign, strict)
        assert (c.min, c.max, c.delta, c.offset, c.bw) == want
    with pytest.raises(RuntimeError):
        c = TfEncodingC(1.0, 2.0, 0.1, 3.0, 8)
        _native.call("aimet_compute_partial_encoding", 8, ctypes.byref(c), 0, 0, 0)


def test_host_analyzer_math_golden(golden_analyzers):
    """Reduced statistics (as the HIP path keeps them in HBM) -> encodings, bit-exact vs the reference."""
    n = int(golden_analyzers["count"])
    for i in range(n):
        c = analyzer_case(golden_analyzers, i)
        a = O.Analyzer(c["scheme"])
        for b in c["batches"]:
            a.update(b)
        st = a.stats()
        if c["scheme"] != O.QUANTIZATION_TF and st["initialized"]:
            # the (hist_min, bucket_size) parametrisation reproduces xLeft exactly
            xl = np.float64(st["hist_min"]) + np.arange(512, dtype=np.float64) * st["bucket_size"]
            np.testing.assert_array_equal(xl, c["xleft"])
            np.testing.assert_array_equal(st["pdf"], c["pdf"])
        pdf = np.ascontiguousarray(st["pdf"], dtype=np.float64)
        for (bw, sym, strict, un), want in c["encs"].items():
            if c["scheme"] == O.QUANTIZATION_TF:
                got = _enc("aimet_encoding_from_minmax", st["acc_min"], st["acc_max"], bw, sym, strict, un)
            else:
                got = _enc("aimet_encoding_from_histogram", c["scheme"], st["initialized"], st["stats_updated"],
                           st["hist_min"], st["bucket_size"], pdf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                           c["percentile"], bw, sym, strict, un)
            assert got == tuple(want[:4]) + (int(want[4]),), (i, c["scheme"], bw, sym, strict, un, got, want)


def test_kernel_entry_points_reject_host_memory():
    """No CPU path: a host pointer is refused loudly, never computed on the CPU."""
    x = np.ones(16, np.float32)
    y = np.zeros(16, np.float32)
    enc = TfEncodingC(-1.0, 1.0, 0.0, 0.0, 8)
    rc = aimet_amd.native_library().aimet_qdq_per_tensor(x.ctypes.data, y.ctypes.data, 16, ctypes.byref(enc), 0, 0,
                                                        None)
    assert rc != 0
    assert np.all(y == 0)


def test_python_layer_refuses_cpu_tensors():
    import torch
    from aimet_amd.libpymo import TfEncoding
    q = aimet_amd.AimetTensorQuantizer(aimet_amd.QuantizationMode.QUANTIZATION_TF)
    enc = TfEncoding()
    enc.min, enc.max, enc.bw = -1.0, 1.0, 8
    with pytest.raises(RuntimeError):
        q.quantizeDequantize(torch.ones(4), enc, aimet_amd.RoundingMode.ROUND_NEAREST, False)
    with pytest.raises(RuntimeError):
        q.updateStats(torch.ones(4), False)


def test_libpymo_surface():
    from aimet_amd import libpymo
    e = libpymo.TfEncoding()
    assert e.to_tuple() == (0.0, 0.0, 0.0, 0.0, 0)
    v = libpymo.TfEncoding._version
    e.min = -1
    assert libpymo.TfEncoding._version == v + 1 and isinstance(e.min, float)
    assert libpymo.QUANTIZATION_TF_ENHANCED == 1 and libpymo.ROUND_STOCHASTIC == 1
    assert libpymo.QuantizationMode.QUANTIZATION_MSE == 4
    with pytest.raises(NotImplementedError):
        libpymo.GetSVDInstance()
    enc = libpymo.getComputedEncodings(8, -1.0, 2.0, False, False, False)
    assert enc.to_tuple() == O.get_computed_encodings(8, -1.0, 2.0).as_tuple()


def test_host_tfe_search_vs_oracle_sparse_and_extreme():
    """The TF-Enhanced search over prepared bins (tfe_core.hpp, shared with the device kernel:
    empty bins skipped when the range is bounded) == the oracle's full loops, on sparse PDFs,
    ranges near FLT_MAX (no skipping), constant and one-sided data, every flag set and width."""
    rng = np.random.default_rng(17)
    cases = []
    for k in (3, 40, 700):
        cases.append(rng.standard_normal(k) * rng.uniform(0.01, 5) + rng.uniform(-2, 2))
    cases.append(np.abs(rng.standard_normal(100)) * 3)
    cases.append(np.full(50, 2.5))
    cases.append(rng.standard_normal(200) * 3e36)
    cases.append(rng.standard_normal(200) * 2e29)
    cases.append(np.concatenate([rng.standard_normal(100), [1e5]]))
    for x in cases:
        a = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
        a.update(x.astype(np.float32))
        st = a.stats()
        pdf = np.ascontiguousarray(st["pdf"], dtype=np.float64)
        for bw in (4, 8, 16):
            for fl in [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 1)]:
                got = _enc("aimet_encoding_from_histogram", O.QUANTIZATION_TF_ENHANCED, st["initialized"],
                           st["stats_updated"], st["hist_min"], st["bucket_size"],
                           pdf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 100.0, bw, *fl)
                assert got == a.compute(bw, *fl).as_tuple(), (x[:3], bw, fl)
