"""Entropy analyzer (QUANTIZATION_ENTROPY).

Reference: EntropyEncodingAnalyzer.cpp:80-435 over updateTensorHistogram_cpu /
rescaleHistogram (math_functions.cpp:470-641). The reference GPU build copies every tensor to the
host for this analyzer (math_functions.cpp:449-456); here min/max, the range widening, the
512-bin histogram and the KL search (entropy_search.hip, near-ties re-checked with glibc's log on
the host) run on the device.

CPU tests pin the oracle (oracle/dlq_oracle.c) to golden vectors of the reference C++ itself
(tests/golden/golden_entropy.npz, make_golden.py) and to the property KATs of
TestEntropyEncodingAnalyzer.cpp, and check the product's host KL search through the C-ABI.
GPU tests run the device statistics and searches through AimetTensorQuantizer: bit-exact state and
encodings.
"""
import ctypes

import numpy as np
import pytest

from conftest import entropy_case, gpu_available
from oracle import oracle as O

FLAGS = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 1), (0, 1, 0)]   # (symmetric, strict, unsigned)
ENTROPY = O.QUANTIZATION_ENTROPY


def _cases(en):
    return [entropy_case(en, i) for i in range(int(en["count"]))]


def _assert_state(st, want, ctx):
    assert st["has_hist"] == want["has_hist"], ctx
    assert (st["min"], st["max"], st["iterations"]) == (want["min"], want["max"], want["iterations"]), ctx
    np.testing.assert_array_equal(st["hist"], want["hist"], err_msg=str(ctx))


# ---- CPU: oracle vs the reference ---------------------------------------------------------------
def test_oracle_entropy_golden(golden_entropy):
    for i, c in enumerate(_cases(golden_entropy)):
        a = O.Analyzer(ENTROPY)
        for b in c["batches"]:
            a.update(b)
        _assert_state(a.entropy_state(), c["tpp"], i)
        for (bw, sym, strict, un), want in c["encs"].items():
            assert a.compute(bw, sym, strict, un).as_tuple() == want, (i, bw, sym, strict, un)


def test_oracle_entropy_kat(golden_entropy):
    """TestEntropyEncodingAnalyzer.cpp:56-296 (N(2, 2) from std::mt19937(1), 100000 samples)."""
    x = golden_entropy["kat_x"]
    mean, std = 2.0, 2.0
    a = O.Analyzer(ENTROPY)
    a.update(x)
    for fl, want in zip(FLAGS, golden_entropy["kat_enc_vals"]):
        assert a.compute(8, *fl).as_tuple() == tuple(want[:4]) + (int(want[4]),)
    e = a.compute(8, False, False, False)                                  # Asymmetric
    assert mean - 6 * std < e.min < mean - 2 * std and mean + 2 * std < e.max < mean + 6 * std
    amax = float(max(abs(x.max()), abs(x.min())))
    e = a.compute(8, True, False, False)                                   # Symmetric
    assert -amax < e.min and e.max < amax and e.offset == -128 and e.bw == 8
    np.testing.assert_allclose(e.delta, (e.max - e.min) / 255, rtol=1e-6)
    np.testing.assert_allclose(e.offset, e.min / e.delta, rtol=1e-6)
    e = a.compute(8, True, True, False)                                    # StrictSymmetric
    assert -amax < e.min and e.max < amax and e.offset == -127 and e.min == -e.max
    np.testing.assert_allclose(e.delta, (e.max - e.min) / 254, rtol=1e-6)
    u = O.Analyzer(ENTROPY)                                                # SymmetricUnsigned
    xu = np.maximum(x, np.float32(0))
    u.update(xu)
    e = u.compute(8, True, False, True)
    assert e.min == 0 and e.max <= float(xu.max())
    np.testing.assert_allclose(e.delta, (e.max - e.min) / 255, rtol=1e-6)
    for v, lo_ok in ((4.0, lambda e: e.min <= 0 and e.max >= 3.9),       # AllSameValuesAsymmetric
                     (-5.0, lambda e: e.min <= -4.99992 and e.max >= 0)):
        s = O.Analyzer(ENTROPY)
        s.update(np.full(100, v, np.float32))
        assert lo_ok(s.compute(8, False, False, False))
    z = O.Analyzer(ENTROPY)                                                # AllZeroesAsymmetric
    z.update(np.zeros(6000, np.float32))
    e = z.compute(8, False, False, False)
    assert abs(e.min - -1.00392) < 1e-4 and abs(e.max - 0.996078) < 1e-4 and e.offset == -128 and e.bw == 8


@pytest.mark.ref
def test_oracle_entropy_vs_compiled_reference_random():
    """Randomized cross-check against the reference C++ compiled in place (build container only)."""
    from oracle import ref as R
    if not R.available():
        pytest.skip("reference not present")
    rng = np.random.default_rng(23)
    for t in range(60):
        a, r = O.Analyzer(ENTROPY), R.Analyzer(ENTROPY)
        for _ in range(int(rng.integers(1, 5))):
            n = int(rng.integers(1, 4000))
            kind = int(rng.integers(0, 5))
            if kind == 0:
                x = rng.normal(rng.uniform(-3, 3), rng.uniform(0.01, 5), n)
            elif kind == 1:
                x = rng.uniform(0, rng.uniform(0.1, 10), n)
            elif kind == 2:
                x = -rng.exponential(rng.uniform(0.1, 3), n)
            elif kind == 3:
                x = np.zeros(n)
            else:
                x = rng.laplace(0, 1, n) * rng.uniform(0.5, 20)
            x = x.astype(np.float32)
            a.update(x)
            r.update(x)
        bw = 8 if t % 4 else int(rng.integers(4, 16))
        for fl in FLAGS:
            assert a.compute(bw, *fl).as_tuple() == r.compute(bw, *fl).as_tuple(), (t, bw, fl)


# ---- CPU: the product's host KL search ----------------------------------------------------------
def _host_encoding(st, bw, sym, strict, un, stats_updated=1):
    from aimet_amd import _native
    from aimet_amd._native import TfEncodingC
    h = np.ascontiguousarray(st["hist"], dtype=np.float64)
    out = TfEncodingC()
    _native.call("aimet_encoding_from_entropy_histogram", int(st["has_hist"]), stats_updated, st["min"], st["max"],
                 h.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), bw, sym, strict, un, out)
    return (out.min, out.max, out.delta, out.offset, out.bw)


def test_host_entropy_encoding_golden(golden_entropy):
    for i, c in enumerate(_cases(golden_entropy)):
        for (bw, sym, strict, un), want in c["encs"].items():
            assert _host_encoding(c["tpp"], bw, sym, strict, un) == want, (i, bw, sym, strict, un)
    empty = dict(has_hist=0, min=0.0, max=0.0, hist=np.zeros(512))
    for fl in FLAGS:
        z = O.Analyzer(ENTROPY)
        z.update(np.zeros(10, np.float32))   # stats updated, histogram never initialised
        assert _host_encoding(empty, 8, *fl) == z.compute(8, *fl).as_tuple()
        assert _host_encoding(empty, 8, *fl, stats_updated=0) == (0.0, 0.0, 0.0, 0.0, 0)


def _random_entropy_analyzers(seed, count):
    """Oracle analyzers fed 1-4 random batches each (normal / uniform / one-sided / zero / Laplace)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(count):
        a = O.Analyzer(ENTROPY)
        batches = []
        for _ in range(int(rng.integers(1, 5))):
            n = int(rng.integers(1, 4000))
            kind = int(rng.integers(0, 5))
            if kind == 0:
                x = rng.normal(rng.uniform(-3, 3), rng.uniform(0.01, 5), n)
            elif kind == 1:
                x = rng.uniform(0, rng.uniform(0.1, 10), n)
            elif kind == 2:
                x = -rng.exponential(rng.uniform(0.1, 3), n)
            elif kind == 3:
                x = np.zeros(n)
            else:
                x = rng.laplace(0, 1, n) * rng.uniform(0.5, 20)
            x = x.astype(np.float32)
            a.update(x)
            batches.append(x)
        out.append((a, batches))
    return out


def test_host_entropy_encoding_random():
    """The product's KL search (entropy_kl.hpp, streamed windows) vs the oracle's array form."""
    for t, (a, _) in enumerate(_random_entropy_analyzers(31, 40)):
        st = a.entropy_state()
        for fl in FLAGS:
            assert _host_encoding(st, 8, *fl) == a.compute(8, *fl).as_tuple(), (t, fl)


# ---- GPU: device statistics ---------------------------------------------------------------------
gpu = pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")


def _enc_tuple(e):
    return (e.min, e.max, e.delta, e.offset, e.bw)


@pytest.mark.gpu
@gpu
def test_entropy_device_stats_golden(golden_entropy):
    import torch
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    for i, c in enumerate(_cases(golden_entropy)):
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY)
        for b in c["batches"]:
            q.updateStats(torch.from_numpy(b).cuda(), True)
        _assert_state(q.entropy_state(), c["tpp"], i)
        for (bw, sym, strict, un), want in c["encs"].items():
            e, valid = q.getEncoding(bw, bool(sym), bool(strict), bool(un))
            assert valid and _enc_tuple(e) == want, (i, bw, sym, strict, un)


@pytest.mark.gpu
@gpu
def test_entropy_device_kat(golden_entropy):
    import torch
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY)
    q.updateStats(torch.from_numpy(golden_entropy["kat_x"]).cuda(), True)
    for fl, want in zip(FLAGS, golden_entropy["kat_enc_vals"]):
        e, valid = q.getEncoding(8, *(bool(v) for v in fl))
        assert valid and _enc_tuple(e) == tuple(want[:4]) + (int(want[4]),)


@pytest.mark.gpu
@gpu
def test_entropy_per_channel_vs_oracle():
    """One analyzer per channel (AimetTensorQuantizer.cpp:209-315): every channel bit-exact vs an
    oracle analyzer fed that channel's slice of each batch."""
    import torch
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    rng = np.random.default_rng(5)
    outer, C, K = 3, 7, 130
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY, num_channels=C)
    ref = [O.Analyzer(ENTROPY) for _ in range(C)]
    for k in range(4):
        x = (rng.standard_normal((outer, C, K)) * rng.uniform(0.1, 3, (1, C, 1)) * (1 + k)).astype(np.float32)
        x[:, 2, :] = 0                    # an all-zero channel: never initialised
        if k == 1:
            x[:, 4, :] = 0.5              # constant batch on one channel
        q.updateStatsPerChannel(torch.from_numpy(x).cuda(), 1, True)
        for c in range(C):
            ref[c].update(np.ascontiguousarray(x[:, c, :]).ravel())
    for c in range(C):
        _assert_state(q.entropy_state(c), ref[c].entropy_state(), c)
    for fl in FLAGS:
        encs, valid = q.getEncoding(8, *(bool(v) for v in fl))
        assert valid
        for c in range(C):
            assert _enc_tuple(encs[c]) == ref[c].compute(8, *fl).as_tuple(), (c, fl)


@pytest.mark.gpu
@gpu
def test_entropy_many_and_phased_equal_single():
    """updateStatsMany (one launch per phase for all quantizers) and the phased, exchange-ready path
    (aimet_amd.distributed, world 1) give the same statistics as per-quantizer updateStats."""
    import torch
    from aimet_amd import distributed as D
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    rng = np.random.default_rng(8)
    sizes = [1, 37, 4096, 300001, 2 * 131072 + 3]
    mk = lambda: [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY) for _ in sizes]  # noqa: E731
    single, many, phased = mk(), mk(), mk()
    ex = None
    for k in range(3):
        xs = [torch.from_numpy((rng.standard_normal(n) * (1 + k) * rng.uniform(0.1, 4)).astype(np.float32)).cuda()
              for n in sizes]
        if k == 0:
            xs[1].zero_()
        for q, x in zip(single, xs):
            q.updateStats(x, True)
        AimetTensorQuantizer.updateStatsMany(many, xs)
        ex = D.sharded_update_stats(phased, xs, exchange=ex, fused=False)
    for i in range(len(sizes)):
        want = single[i].entropy_state()
        _assert_state(many[i].entropy_state(), want, ("many", i))
        _assert_state(phased[i].entropy_state(), want, ("phased", i))
    got = AimetTensorQuantizer.getEncodings(many, 8, False, False, False)
    for q, (e, valid) in zip(single, got):
        assert valid and _enc_tuple(e) == _enc_tuple(q.getEncoding(8, False, False, False)[0])


@pytest.mark.gpu
@gpu
def test_entropy_binning_at_bin_edges_large():
    """Values exactly on bin edges (integer quotients: the reciprocal binning falls back to the
    IEEE division), signed zeros and NaN (counted in the last bin, as the reference), over a
    tensor large enough for the multi-workgroup histogram path."""
    import torch
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    rng = np.random.default_rng(9)
    n = (1 << 22) + 5
    x = (rng.integers(-256, 257, n).astype(np.float32) / np.float32(256))   # k / 256: binWidth = 1/256
    x[:3] = [-1.0, 1.0, -0.0]
    x[10:20] = np.nan
    x[20:40] = rng.standard_normal(20).astype(np.float32)
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY)
    a = O.Analyzer(ENTROPY)
    for b in (x, x[: n // 3] * np.float32(1.5)):
        q.updateStats(torch.from_numpy(np.ascontiguousarray(b)).cuda(), True)
        a.update(b)
    _assert_state(q.entropy_state(), a.entropy_state(), "edges")
    for fl in FLAGS:
        assert _enc_tuple(q.getEncoding(8, *(bool(v) for v in fl))[0]) == a.compute(8, *fl).as_tuple()


@pytest.mark.gpu
@gpu
def test_entropy_device_kl_search_random():
    """The device KL search (entropy_search.hip) over 40 random statistics sequences, all flag
    combinations, through the batched getEncodings (one launch for every quantizer) and the
    per-quantizer getEncoding: bit-exact vs the oracle's glibc search."""
    import torch
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    cases = _random_entropy_analyzers(47, 40)
    qs = []
    for a, batches in cases:
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY)
        for x in batches:
            q.updateStats(torch.from_numpy(x).cuda(), True)
        qs.append(q)
    for fl in FLAGS:
        batched = AimetTensorQuantizer.getEncodings(qs, 8, *(bool(v) for v in fl))
        for t, ((a, _), q, (e, valid)) in enumerate(zip(cases, qs, batched)):
            want = a.compute(8, *fl).as_tuple()
            assert valid and _enc_tuple(e) == want, (t, fl)
            e1, _ = q.getEncoding(8, *(bool(v) for v in fl))
            assert _enc_tuple(e1) == want, (t, fl)


@pytest.mark.gpu
@gpu
def test_entropy_device_kl_search_per_channel_many():
    """Per-channel entropy statistics of 3 weights (one workgroup per channel) and their KL
    searches in one launch: every channel bit-exact vs an oracle analyzer of its slice."""
    import torch
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    rng = np.random.default_rng(12)
    shapes = [(64, 27), (128, 576), (32, 2048)]
    ws = [(rng.standard_normal(s) * rng.uniform(0.01, 0.2, (s[0], 1))).astype(np.float32) for s in shapes]
    ws[1][5] = 0                                      # an all-zero channel
    ws[2][:, ::3] = np.abs(ws[2][:, ::3])             # skewed channels
    # degenerate histograms (equal divergences: near-ties the host search finishes) among channels
    # the device finishes, so that one quantizer mixes both (its flagged rows read back alone)
    ws[0][3] = 0.5
    ws[0][10] = np.where(np.arange(27) % 2 == 0, 0.25, -0.25).astype(np.float32)
    ws[1][17] = np.float32(1e-3)
    qs = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY, num_channels=s[0]) for s in shapes]
    AimetTensorQuantizer.updateStatsPerChannelMany(qs, [torch.from_numpy(w).cuda() for w in ws])
    torch.cuda.synchronize()
    for fl in ((1, 0, 0), (0, 0, 0), (1, 1, 0)):
        res = AimetTensorQuantizer.getEncodings(qs, 8, *(bool(v) for v in fl))
        for w, (encs, valid) in zip(ws, res):
            assert valid
            for c in sorted(set(range(0, w.shape[0], 7)) | {3, 5, 10, 17}):
                a = O.Analyzer(ENTROPY)
                a.update(w[c])
                assert _enc_tuple(encs[c]) == a.compute(8, *fl).as_tuple(), (w.shape, c, fl)
