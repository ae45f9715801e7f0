"""Parity of the HIP path (through the C-ABI) with the reference: golden vectors of the reference
C++ (bit-exact), the reference test-suites' KATs, the CPU oracle on seeded inputs, and at full
size size-independent properties. Needs an MI355X."""
import ctypes
import os

import numpy as np
import pytest
import torch

from conftest import analyzer_case, bits, gpu_available, per_channel_case
from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

from aimet_amd import AimetTensorQuantizer  # noqa: E402
from aimet_amd.libpymo import QuantizationMode, RoundingMode, TfEncoding  # noqa: E402

DEV = "cuda"
# learned-grid range gradients: error bound in units of 2^-24 x (sum of |terms|) of the float64 sum
LG_BOUND_C = 2.0   # range-gradient bar in units of 2^-24 x the sum of |terms| (fixed: part of the test)
NEAREST = RoundingMode.ROUND_NEAREST
FLAGS = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 1)]


def enc_of(mn, mx, bw, delta=0.0, offset=0.0):
    e = TfEncoding()
    e.min, e.max, e.bw, e.delta, e.offset = mn, mx, bw, delta, offset
    return e


def gpu(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(DEV)


def host(t):
    return t.detach().cpu().numpy()


# ------------------------------------------------------------------------------------------
# QDQ / quantize-only
# ------------------------------------------------------------------------------------------
def test_kat_qdq(kat):
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
    for name in ("qdq_sanity", "qdq_gated_min", "qdq_gated_equal", "qdq_gated_max"):
        k = kat[name]
        y = host(q.quantizeDequantize(gpu(k["x"]), enc_of(k["min"], k["max"], k["bw"]), NEAREST, True))
        np.testing.assert_array_max_ulp(y, np.array(k["expected"], np.float32), maxulp=4)
        np.testing.assert_array_equal(bits(y), bits(O.qdq_per_tensor(k["x"], k["min"], k["max"], k["bw"])))
    for name in ("quantize_unsigned", "quantize_signed"):
        k = kat[name]
        y = host(q.quantize(gpu(k["x"]), enc_of(k["min"], k["max"], k["bw"]), NEAREST, True, k["shift"]))
        np.testing.assert_array_equal(y, np.array(k["expected"], np.float32))


def test_golden_qdq_per_tensor_bit_exact(golden_core):
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
    for i, (x, e) in enumerate(zip(golden_core["pt_x"], golden_core["pt_enc"])):
        enc = enc_of(e[0], e[1], int(e[2]))
        xd = gpu(x)
        np.testing.assert_array_equal(bits(host(q.quantizeDequantize(xd, enc, NEAREST, True))),
                                      bits(golden_core["pt_qdq"][i]), err_msg="case %d" % i)
        np.testing.assert_array_equal(bits(host(q.quantize(xd, enc, NEAREST, True, False))),
                                      bits(golden_core["pt_q_unsigned"][i]))
        np.testing.assert_array_equal(bits(host(q.quantize(xd, enc, NEAREST, True, True))),
                                      bits(golden_core["pt_q_signed"][i]))
        # unaligned / ragged views take the scalar path: same bits
        y = host(q.quantizeDequantize(xd[1:], enc, NEAREST, True))
        np.testing.assert_array_equal(bits(y), bits(golden_core["pt_qdq"][i][1:]))


def test_golden_qdq_per_channel_bit_exact(golden_core):
    for i in range(int(golden_core["pc_count"])):
        c = per_channel_case(golden_core, i)
        encs = [enc_of(*e[:2], int(e[4]), e[2], e[3]) for e in c["encs"]]
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
        table = q.channelTable(encs, torch.device(DEV))
        np.testing.assert_array_equal(bits(host(table)), bits(c["table"]))
        N = c["x"].size
        y = q.quantizeDequantizePerChannel(gpu(c["x"]), encs, c["C"], N, c["K"], NEAREST, True)
        np.testing.assert_array_equal(bits(host(y)), bits(c["y"]), err_msg="case %d" % i)


def test_kat_per_channel(kat):
    for name in ("per_channel_symmetric", "per_channel_asymmetric"):
        k = kat[name]
        x = np.array(k["x"], np.float32)
        encs = [enc_of(e[0], e[1], int(e[4]), e[2], e[3]) for e in k["encodings"]]
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
        y = host(q.quantizeDequantizePerChannel(gpu(x), encs, 4, x.size, x.shape[1], NEAREST, True))
        np.testing.assert_allclose(y, np.array(k["expected"], np.float32), atol=k["atol"])


@pytest.mark.parametrize("shape,axis", [((64, 3, 7, 7), 0), ((256, 64, 3, 3), 0), ((32, 16, 3, 3), 1),
                                        ((1000, 2048), 0), ((7, 5, 3), 2)])
def test_per_channel_vs_oracle_random(shape, axis):
    rng = np.random.default_rng(hash(shape) % 1000)
    x = (rng.standard_normal(shape) * 0.1).astype(np.float32)
    C = shape[axis]
    encs = []
    for c in range(C):
        lo, hi = sorted(rng.uniform(-0.3, 0.3, 2))
        encs.append(enc_of(lo, hi, 8))
    from aimet_amd.tensor_quantizer import per_channel_view, qdq_per_channel_table
    outer, C_, K = per_channel_view(shape, axis)
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
    table = q.channelTable(encs, torch.device(DEV))
    y = host(qdq_per_channel_table(gpu(x), table, outer, C_, K))
    otab = O.per_channel_table([e.to_tuple() for e in encs])
    want = O.qdq_per_channel(x.ravel(), C_, K, otab).reshape(shape)
    np.testing.assert_array_equal(bits(y), bits(want))


def test_qdq_full_size_bit_exact_and_properties():
    """ResNet-50 bs256 conv1 output size (256x64x112x112 = 205M elements): bit-exact vs the
    oracle, idempotent, on the quantization grid."""
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(256, 64, 112, 112, device=DEV, generator=g) * 2.0
    enc = enc_of(-3.1, 5.7, 8)
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
    y = q.quantizeDequantize(x, enc, NEAREST, True)
    want = O.qdq_per_tensor(host(x).ravel(), enc.min, enc.max, 8)
    np.testing.assert_array_equal(bits(host(y).ravel()), bits(want))
    y2 = q.quantizeDequantize(y, enc, NEAREST, True)
    assert torch.equal(y, y2)
    codes = q.quantize(x, enc, NEAREST, True, False)
    assert float(codes.min()) >= 0 and float(codes.max()) <= 255
    assert torch.equal(codes, torch.round(codes))


def test_stochastic_rounding_is_unbiased():
    x = torch.full((1 << 22,), 0.3, device=DEV)
    enc = enc_of(-1.0, 1.0, 8)
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
    e = O.fill_encoding_info(8, -1.0, 1.0)
    y = q.quantizeDequantize(x, enc, RoundingMode.ROUND_STOCHASTIC, True)
    lo = np.float32(e.delta) * (np.floor(np.float32(0.3) / np.float32(e.delta) - np.float32(e.offset)) +
                                np.float32(e.offset))
    vals = torch.unique(y).cpu().numpy()
    assert len(vals) == 2 and abs(vals[0] - lo) < 1e-6
    assert abs(float(y.mean()) - 0.3) < 2e-4


# ------------------------------------------------------------------------------------------
# statistics + encodings
# ------------------------------------------------------------------------------------------
def test_golden_analyzers_bit_exact(golden_analyzers):
    n = int(golden_analyzers["count"])
    for i in range(n):
        c = analyzer_case(golden_analyzers, i)
        q = AimetTensorQuantizer(QuantizationMode(c["scheme"]))
        if c["scheme"] == QuantizationMode.QUANTIZATION_PERCENTILE:
            q.setPercentileValue(c["percentile"])
        for b in c["batches"]:
            q.updateStats(gpu(b), True)
        for (bw, sym, strict, un), want in c["encs"].items():
            got, valid = q.getEncoding(bw, sym, strict, un)
            assert valid
            assert got.to_tuple() == tuple(want[:4]) + (int(want[4]),), (i, c["scheme"], bw, sym, strict, un)
        if c["scheme"] != QuantizationMode.QUANTIZATION_TF:
            h = q.getStatsHistogram()
            if len(c["xleft"]):
                np.testing.assert_array_equal(np.array([t[0] for t in h]), c["xleft"])
                np.testing.assert_array_equal(np.array([t[1] for t in h]), c["pdf"])


def test_kat_tfe(kat, golden_torch):
    k = kat["tfe_normal"]
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
    q.updateStats(gpu(golden_torch["tfe_kat_x"]), True)
    e, valid = q.getEncoding(8, False, False, False)
    assert valid and e.to_tuple() == tuple(k["ref_encoding"])
    y = host(q.quantizeDequantize(gpu(np.full(8, 5.0)), e, NEAREST, True))
    assert float(y[0]) == k["ref_qdq5"]
    z = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
    z.updateStats(torch.zeros(6000, device=DEV), True)
    e, _ = z.getEncoding(8, False, False, False)
    kz = kat["tfe_all_zero"]
    assert abs(e.min - kz["expected_min"]) < kz["tol"] and e.offset == kz["expected_offset"]


def test_invalid_without_stats():
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
    _, valid = q.getEncoding(8, False, False, False)
    assert not valid
    q.updateStats(torch.randn(100, device=DEV), True)
    q.resetEncodingStats()
    _, valid = q.getEncoding(8, False, False, False)
    assert not valid


@pytest.mark.parametrize("scheme", [QuantizationMode.QUANTIZATION_TF, QuantizationMode.QUANTIZATION_TF_ENHANCED,
                                    QuantizationMode.QUANTIZATION_PERCENTILE, QuantizationMode.QUANTIZATION_MSE])
@pytest.mark.parametrize("shape,axis", [((64, 3, 7, 7), 0), ((96, 32, 3, 3), 0), ((16, 24, 3, 3), 1),
                                        ((40, 130), 0)])
def test_per_channel_stats_vs_per_channel_oracle(scheme, shape, axis):
    """One batched launch == C independent reference analyzers over select(axis, c).contiguous()."""
    rng = np.random.default_rng(7)
    C = shape[axis]
    q = AimetTensorQuantizer(scheme, num_channels=C)
    if scheme == QuantizationMode.QUANTIZATION_PERCENTILE:
        q.setPercentileValue(99.5)
    orcs = [O.Analyzer(int(scheme)) for _ in range(C)]
    for batch in range(2):
        x = (rng.standard_normal(shape) * rng.uniform(0.01, 2)).astype(np.float32)
        x[(slice(None),) * axis + (1,)] = 0.0          # one all-zero channel
        if batch == 1:
            x = np.maximum(x, 0)
        q.updateStatsPerChannel(gpu(x), axis, True)
        for c in range(C):
            orcs[c].update(np.ascontiguousarray(np.take(x, c, axis=axis)))
        if scheme == QuantizationMode.QUANTIZATION_PERCENTILE:
            for o in orcs:
                o.set_percentile(99.5)
    for fl in FLAGS[:2] if scheme == QuantizationMode.QUANTIZATION_MSE else FLAGS:
        encs, valid = q.getEncoding(8, *fl)
        assert valid
        for c in range(C):
            assert encs[c].to_tuple() == orcs[c].compute(8, *fl).as_tuple(), (c, fl)


@pytest.mark.parametrize("scheme,C,bws", [(QuantizationMode.QUANTIZATION_TF_ENHANCED, 600, (4, 8, 16)),
                                          (QuantizationMode.QUANTIZATION_TF_ENHANCED, 200, (4, 8, 16)),
                                          (QuantizationMode.QUANTIZATION_MSE, 160, (8, 4))])
def test_device_search_many_channels(scheme, C, bws):
    """Device encoding searches (tfe_search.hip: one workgroup per channel, or below 512 channels
    each channel's candidates split over one-wave workgroups merged by the last to finish;
    mse_search.hip: channel x candidate-slice grid) == the oracle's host searches, for channels of
    varied shape, every flag set and several bit-widths."""
    rng = np.random.default_rng(21)
    K = 96
    scale = rng.uniform(1e-3, 30, (C, 1))
    shift = rng.uniform(-3, 3, (C, 1))
    x = rng.standard_t(3, (C, K)) * scale + shift * scale
    x[5] = 0.0
    x[7] = np.abs(x[7])
    x[9, :] = 2.5                                   # constant channel
    x[11] = rng.standard_normal(K) * 3e36           # range near FLT_MAX: every bin visited
    x[13, :3] = 7.0                                 # nearly empty PDF
    x[13, 3:] = 0.0
    x = x.astype(np.float32)
    q = AimetTensorQuantizer(scheme, num_channels=C)
    q.updateStatsPerChannel(gpu(x), 0, True)
    orcs = []
    for c in range(C):
        o = O.Analyzer(int(scheme))
        o.update(x[c])
        orcs.append(o)
    for bw in bws:
        for fl in FLAGS:
            encs, valid = q.getEncoding(bw, *fl)
            assert valid
            for c in range(C):
                assert encs[c].to_tuple() == orcs[c].compute(bw, *fl).as_tuple(), (c, bw, fl)


def test_tfe_split_search_equals_one_workgroup_per_channel():
    """The split TF-E search (fewer than 512 channels in the batch: candidates over one-wave
    workgroups, first minimum by (cost, index) across them) == one workgroup per channel (the same
    quantizers searched in a batch with a 512-channel quantizer beside them), for a batch of
    per-tensor quantizers (the activations' getEncodings) and every flag set."""
    rng = np.random.default_rng(33)
    qs = []
    for i in range(40):
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
        x = rng.standard_t(2 + i % 5, 4096 + 97 * i) * rng.uniform(1e-3, 10) + rng.uniform(-2, 2)
        if i % 7 == 3:
            x = np.abs(x)
        q.updateStats(gpu(x.astype(np.float32)), True)
        qs.append(q)
    big = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED, num_channels=512)
    big.updateStatsPerChannel(gpu(rng.standard_normal((512, 64)).astype(np.float32)), 0, True)
    for bw in (8, 16):
        for fl in FLAGS:
            split = AimetTensorQuantizer.getEncodings(qs, bw, *fl)
            whole = AimetTensorQuantizer.getEncodings(qs + [big], bw, *fl)[:len(qs)]
            assert [(e.to_tuple(), v) for e, v in split] == [(e.to_tuple(), v) for e, v in whole], (bw, fl)


def test_mse_device_search_per_tensor_large():
    """Per-tensor MSE (all 128 candidate slices of one channel) on a dense 16M-element histogram
    == the oracle."""
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(1 << 24, device=DEV, generator=g) * 2 + 0.5
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_MSE)
    q.updateStats(x, True)
    o = O.Analyzer(O.QUANTIZATION_MSE)
    o.update(host(x))
    for fl in FLAGS:
        assert q.getEncoding(8, *fl)[0].to_tuple() == o.compute(8, *fl).as_tuple(), fl


def test_get_encodings_batched_equals_individual():
    """AimetTensorQuantizer.getEncodings (one device search launch + one sync for all quantizers)
    == getEncoding of each, for every scheme, per-tensor and per-channel, with and without stats."""
    rng = np.random.default_rng(3)
    qs = []
    for scheme in (QuantizationMode.QUANTIZATION_TF, QuantizationMode.QUANTIZATION_TF_ENHANCED,
                   QuantizationMode.QUANTIZATION_PERCENTILE, QuantizationMode.QUANTIZATION_MSE,
                   QuantizationMode.QUANTIZATION_ENTROPY):
        for C in (1, 7, 1, 1):   # several per-tensor entropy quantizers: the host pool spans quantizers
            q = AimetTensorQuantizer(scheme, num_channels=C)
            if scheme == QuantizationMode.QUANTIZATION_PERCENTILE:
                q.setPercentileValue(99.0)
            x = (rng.standard_normal((C, 300)) * rng.uniform(0.1, 4)).astype(np.float32)
            if C == 1:
                q.updateStats(gpu(x), True)
            else:
                q.updateStatsPerChannel(gpu(x), 0, True)
            qs.append(q)
    qs.append(AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED))      # no stats
    qs.append(AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED, num_channels=3))
    z = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED, num_channels=4)
    z.updateStatsPerChannel(torch.zeros(4, 50, device=DEV), 0, True)                 # all-zero data
    qs.append(z)
    for fl in FLAGS:
        batched = AimetTensorQuantizer.getEncodings(qs, 8, *fl)
        for q, (e, v) in zip(qs, batched):
            e1, v1 = q.getEncoding(8, *fl)
            assert v == v1
            if isinstance(e1, list):
                assert [a.to_tuple() for a in e] == [a.to_tuple() for a in e1]
            else:
                assert e.to_tuple() == e1.to_tuple()


def test_minmax_and_histogram_full_size():
    """Stats of a 205M-element activation: TF encoding == oracle over the whole tensor, TF-E PDF
    == oracle PDF (bit-exact) and sums to the in-range fraction."""
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.relu(torch.randn(256, 64, 112, 112, device=DEV, generator=g) * 1.5 + 0.2)
    xh = host(x).ravel()
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
    q.updateStats(x, True)
    o = O.Analyzer(O.QUANTIZATION_TF)
    o.update(xh)
    assert q.getEncoding(8, False, False, False)[0].to_tuple() == o.compute(8).as_tuple()
    qe = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
    qe.updateStats(x, True)
    oe = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
    oe.update(xh)
    h = qe.getStatsHistogram()
    xl, pdf = oe.histogram()
    np.testing.assert_array_equal(np.array([t[1] for t in h]), pdf)
    np.testing.assert_array_equal(np.array([t[0] for t in h]), xl)
    assert qe.getEncoding(8, False, False, False)[0].to_tuple() == oe.compute(8).as_tuple()


# ------------------------------------------------------------------------------------------
# STE / autograd
# ------------------------------------------------------------------------------------------
def test_ste_golden(golden_torch):
    from aimet_amd.quantizers import compute_dloss_by_dx
    x, g = gpu(golden_torch["ste_x"]), gpu(golden_torch["ste_g"])
    got = compute_dloss_by_dx(x, g, golden_torch["ste_mins"].tolist(), golden_torch["ste_maxs"].tolist(), 0)
    np.testing.assert_array_equal(bits(host(got)), bits(golden_torch["ste_pc"]))
    got = compute_dloss_by_dx(x, g, -1.25, 0.8)
    np.testing.assert_array_equal(bits(host(got)), bits(golden_torch["ste_pt"]))


def test_quantize_dequantize_autograd_per_tensor_and_channel():
    from aimet_amd.quantizers import QuantScheme, StaticGridPerChannelQuantizer, StaticGridPerTensorQuantizer
    torch.manual_seed(0)
    x = torch.randn(8, 16, 5, 5, device=DEV, requires_grad=True)
    tq = StaticGridPerTensorQuantizer(8, "nearest", QuantScheme.post_training_tf, False, True)
    tq.update_encoding_stats(x.detach() * 0.5)
    tq.compute_encoding()
    y = tq.quantize_dequantize(x, NEAREST)
    y.backward(torch.ones_like(y))
    mn, mx = np.float32(tq.encoding.min), np.float32(tq.encoding.max)
    xh = host(x)
    np.testing.assert_array_equal(host(x.grad), ((xh >= mn) & (xh <= mx)).astype(np.float32))
    np.testing.assert_array_equal(bits(host(y)), bits(O.qdq_per_tensor(xh, tq.encoding.min, tq.encoding.max, 8)))

    w = torch.randn(16, 8, 3, 3, device=DEV, requires_grad=True)
    pq = StaticGridPerChannelQuantizer(8, "nearest", QuantScheme.post_training_tf_enhanced, True, 16, True)
    pq.update_encoding_stats(w.detach())
    pq.compute_encoding()
    assert len(pq.encoding) == 16
    yw = pq.quantize_dequantize(w, NEAREST)
    yw.sum().backward()
    wh = host(w)
    for c in range(16):
        o = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
        o.update(wh[c].ravel())
        assert pq.encoding[c].to_tuple() == o.compute(8, True, False, False).as_tuple()
        lo, hi = np.float32(pq.encoding[c].min), np.float32(pq.encoding[c].max)
        np.testing.assert_array_equal(host(w.grad)[c], ((wh[c] >= lo) & (wh[c] <= hi)).astype(np.float32))


# ------------------------------------------------------------------------------------------
# AdaRound
# ------------------------------------------------------------------------------------------
def _cpu_one_thread(fn):
    """Run the reference's torch-op arithmetic on the CPU with one thread (the reference's own
    platform; one thread so only each tensor's last numel % 32 elements take torch's scalar path)."""
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        return fn()
    finally:
        torch.set_num_threads(nt)


def test_adaround_forward_backward_vs_torch(kat):
    """Fused soft-quant forward / backward vs torch autograd of the reference formula on the CPU:
    bit-exact (numel is a multiple of 32, so every element takes torch's vectorized sigmoid)."""
    from aimet_amd.adaround import AdaroundFunction, round_loss_and_grad
    from oracle import torch_ref as T
    torch.manual_seed(0)
    w = torch.randn(32, 16, 3, 3, device=DEV) * 0.1
    delta = (torch.rand(32, device=DEV) * 0.01 + 0.001).view(32, 1, 1, 1)
    offset = torch.full((32, 1, 1, 1), -128.0, device=DEV)
    alpha = torch.randn_like(w)
    g = torch.randn_like(w)

    def ref():
        a = alpha.cpu().requires_grad_(True)
        wq = T.adaround_forward(w.cpu(), a, delta.cpu(), offset.cpu(), 8)
        (wq * g.cpu()).sum().backward()
        return wq.detach(), a.grad
    wq_ref, ga_ref = _cpu_one_thread(ref)
    a = alpha.clone().requires_grad_(True)
    wq = AdaroundFunction.apply(w, a, delta.view(-1), offset.view(-1), 8, 0)
    assert torch.equal(wq.cpu(), wq_ref)
    (wq * g).sum().backward()
    assert torch.equal(a.grad.cpu(), ga_ref)
    # round loss KAT (test_adaround_loss.py:83-100): float32 alpha, tolerance 1e-5 (places=5)
    k = kat["adaround_round_loss"]
    np.random.seed(k["seed"])
    al = torch.from_numpy(np.random.rand(*k["shape"]).astype(np.float32)).to(DEV)
    loss, _ = round_loss_and_grad(al, k["reg_param"], kat["adaround_beta"]["expected"])
    assert abs(float(loss) - k["expected"]) < 1e-5


@pytest.mark.parametrize("beta", [2.0, 7.5, 20.0])
@pytest.mark.parametrize("shape", [(64, 32, 3, 3), (32, 3, 3, 3)])   # 16-B path / scalar path
def test_adaround_backward_with_round_loss_vs_torch(beta, shape):
    """Fused backward with the rounding loss (reg != 0): dL/dalpha and the loss itself vs torch
    autograd of the reference formulas (adaround_wrapper.py:124-149 + adaround_loss.py:97-110).
    Wq bit-exact; loss rtol 1e-5 (fp32 sum order); gradient rtol 1e-5: the kernel restates the
    AVX512F build of Sleef's powf_u10 that produced the reference's golden vectors (bit-equal there,
    test_adaround_golden.py), while torch on this host may dispatch another Sleef build."""
    from aimet_amd.adaround import AdaroundFunction
    from oracle import torch_ref as T
    torch.manual_seed(1)
    C = shape[0]
    w = torch.randn(*shape, device=DEV) * 0.1
    delta = (torch.rand(C, device=DEV) * 0.01 + 0.001).view(C, 1, 1, 1)
    offset = torch.full((C, 1, 1, 1), -128.0, device=DEV)
    alpha = torch.randn_like(w) * 2
    g = torch.randn_like(w)
    reg = 0.01

    def ref():
        a_ref = alpha.cpu().requires_grad_(True)
        wq_ref = T.adaround_forward(w.cpu(), a_ref, delta.cpu(), offset.cpu(), 8)
        loss_ref = T.adaround_round_loss(a_ref, reg, beta)
        ((wq_ref * g.cpu()).sum() + loss_ref).backward()
        return wq_ref.detach(), a_ref.grad, loss_ref.item()
    wq_ref, ga_ref, loss_ref = _cpu_one_thread(ref)
    a = alpha.clone().requires_grad_(True)
    loss = torch.zeros(1, device=DEV)
    wq = AdaroundFunction.apply(w, a, delta.view(-1), offset.view(-1), 8, 0, True, reg, beta, loss)
    (wq * g).sum().backward()
    assert torch.equal(wq.cpu(), wq_ref)
    # only the rounding-loss branch's pow may differ (the host's Sleef build)
    torch.testing.assert_close(a.grad.cpu(), ga_ref, rtol=1e-5, atol=1e-9)
    assert abs(loss.item() - loss_ref) <= 1e-5 * abs(loss_ref)


@pytest.mark.parametrize("beta", [3.0, 4.0, 7.25, 20.0])   # beta - 1 = 2 / 3: x*x / x*x*x (no logarithm)
@pytest.mark.parametrize("want_loss", [False, True])
@pytest.mark.parametrize("n, C", [(1 << 19, 64), ((1 << 19) + 16, 1)])   # n % 32 == 16: the scalar pow tail
def test_adaround_backward_dense_waves_equal_compacted(beta, want_loss, n, C, exact_pow):
    """The fused backward evaluates the rounding-loss pows of a dense wave (>= 3/4 of its elements
    need the logarithm) in place (the exact pow two at a time in packed f32) and those of a sparse
    wave compacted through LDS (adaround.hip: ada_round_pows), in either pow form. The same
    element must give the same bits either way: run A has every alpha unsaturated (dense waves),
    run B saturates 3 of every 4 quads (sparse waves), and the unsaturated quads' gradients of the
    two runs are compared bit for bit."""
    from aimet_amd import _native
    g = torch.Generator(device=DEV).manual_seed(5)
    K = n // C
    w = torch.randn(n, device=DEV, generator=g) * 0.05
    grad = torch.randn(n, device=DEV, generator=g)
    delta = (w.view(C, K).abs().amax(1) / 127).contiguous()
    offset = torch.full((C,), -128.0, device=DEV)
    alpha_a = torch.randn(n, device=DEV, generator=g) * 0.7
    quad = torch.arange(n, device=DEV) // 4
    keep = quad % 4 == 0
    alpha_b = torch.where(keep, alpha_a, torch.full_like(alpha_a, 60.0))
    stream = torch.cuda.current_stream().cuda_stream
    outs = []
    for alpha in (alpha_a, alpha_b):
        out = torch.empty_like(w)
        loss = torch.zeros(1, device=DEV)
        _native.call("aimet_adaround_backward", w.data_ptr(), alpha.data_ptr(), grad.data_ptr(), out.data_ptr(), 1,
                     C, K, delta.data_ptr(), offset.data_ptr(), 8, ctypes.c_double(0.01), ctypes.c_double(beta),
                     loss.data_ptr() if want_loss else None, stream)
        outs.append(out)
    torch.cuda.synchronize()
    a, b = outs[0][keep].view(torch.int32), outs[1][keep].view(torch.int32)
    assert torch.equal(a, b), int((a != b).sum())
    # and the saturated quads took the exact |x| == 1 value: the Wq gradient alone (h's clamp passes none)
    assert torch.isfinite(outs[1]).all()


@pytest.mark.parametrize("reg", [0.0, 0.01])
@pytest.mark.parametrize("n, C", [(3 << 22, 96), ((3 << 22) + 16, 1)])   # n % 32 == 16: the scalar pow tail
def test_adaround_backward_grid_forms_equal(reg, n, C, exact_pow):
    """Above 8192 workgroups' worth of quads the backward without the loss value runs one tile per
    workgroup, with it a grid-stride loop over 8192 workgroups (adaround.hip: adaround_backward).
    Both forms must give the same gradient bits; 12.6 M elements (1.5 x the bounded grid's tile)."""
    from aimet_amd import _native
    g = torch.Generator(device=DEV).manual_seed(9)
    K = n // C
    w = torch.randn(n, device=DEV, generator=g) * 0.05
    grad = torch.randn(n, device=DEV, generator=g)
    alpha = torch.randn(n, device=DEV, generator=g) * 2
    delta = (w.view(C, K).abs().amax(1) / 127).contiguous()
    offset = torch.full((C,), -128.0, device=DEV)
    stream = torch.cuda.current_stream().cuda_stream
    outs = []
    for want_loss in (False, True):
        out = torch.full_like(w, float("nan"))
        loss = torch.zeros(1, device=DEV)
        _native.call("aimet_adaround_backward", w.data_ptr(), alpha.data_ptr(), grad.data_ptr(), out.data_ptr(), 1,
                     C, K, delta.data_ptr(), offset.data_ptr(), 8, ctypes.c_double(reg), ctypes.c_double(8.0),
                     loss.data_ptr() if want_loss else None, stream)
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    assert torch.isfinite(outs[0]).all()
    if reg == 0.0:   # no loss term at reg 0 (the launch takes the no-loss form): the value is untouched
        assert loss.item() == 0.0
    else:
        assert loss.item() > 0.0


def test_adaround_hard_rounding_floor_exact_at_multiples():
    """floor(W / delta) in the AdaRound kernels (reciprocal fast path, adaround.hip: floor_div) equals
    torch's IEEE floor(W / delta) bit for bit, on weights at exact multiples of delta and 1-2 ulp
    beside them; hard rounding makes Wq exact, so the comparison is equality."""
    from aimet_amd.adaround import AdaroundFunction
    torch.manual_seed(3)
    C, K = 64, 1024
    delta = (torch.rand(C, device=DEV) * 0.01 + 0.0005)
    k = torch.randint(-140, 140, (C, K), device=DEV).float()
    w = k * delta.view(C, 1)
    for step in (0, 1, -1, 2, -2):
        ws = w if step == 0 else torch.nextafter(w, w + step * float("inf"))
        if abs(step) == 2:
            ws = torch.nextafter(ws, ws + step * float("inf"))
        offset = torch.full((C,), -128.0, device=DEV)
        alpha = torch.randn(C, K, device=DEV)
        with torch.no_grad():
            wq = AdaroundFunction.apply(ws, alpha, delta, offset, 8, 0, False)
            ref = (torch.clamp(torch.floor(ws / delta.view(C, 1)) + (alpha >= 0).float() - offset.view(C, 1), 0, 255)
                   + offset.view(C, 1)) * delta.view(C, 1)
        assert torch.equal(wq, ref), step


def test_channel_plan_equals_individual_launches():
    """All parameter QDQs in one launch == one launch per tensor (incl. K % 4 != 0, axis 1)."""
    from aimet_amd.tensor_quantizer import ChannelQdqPlan, per_channel_view, qdq_per_channel_table
    torch.manual_seed(5)
    shapes = [((64, 3, 7, 7), 0), ((256, 64, 1, 1), 0), ((128, 128, 3, 3), 0), ((1000, 2048), 0),
              ((32, 16, 3, 3), 1), ((5,), 0)]
    entries, wants = [], []
    for shape, ax in shapes:
        w = torch.randn(shape, device=DEV) * 0.05
        C = shape[ax]
        encs = [enc_of(-0.1 - 0.001 * c, 0.12 + 0.001 * c, 8) for c in range(C)]
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
        table = q.channelTable(encs, torch.device(DEV)).clone()
        outer, C_, K = per_channel_view(shape, ax)
        wants.append(qdq_per_channel_table(w, table, outer, C_, K))
        entries.append((w, torch.empty_like(w), ax, table))
    plan = ChannelQdqPlan(entries)
    plan.run()
    for (w, y, ax, t), want in zip(entries, wants):
        assert torch.equal(y, want)


@pytest.mark.parametrize("case", range(5))
def test_learned_grid_vs_reference_golden(golden_dir, case):
    """Fused learned-grid fwd/bwd vs the reference module's outputs (golden_lg.npz): y and grad_x
    bit-exact; the encoding gradients are sums, so they are held to a stated bound instead: ours and
    the reference's both within LG_BOUND_C = 2 eps x (the sum of |terms|) of the float64 value of
    the same sum (the reference's own error is <= 1.3 of that unit on these cases)."""
    import os
    from aimet_amd.learned_grid import LearnedGridQuantizeDequantize
    from oracle import torch_ref as T
    g = dict(np.load(os.path.join(golden_dir, "golden_lg.npz")))
    i = case
    x = gpu(g["c%d_x" % i]).requires_grad_(True)
    grad = gpu(g["c%d_grad" % i])
    emin = gpu(g["c%d_emin" % i]).requires_grad_(True)
    emax = gpu(g["c%d_emax" % i]).requires_grad_(True)
    bw, sym = (int(v) for v in g["c%d_cfg" % i])
    y = LearnedGridQuantizeDequantize.apply(x, emin, emax, bw, bool(sym), False, False, 0)
    np.testing.assert_array_equal(bits(host(y)), bits(g["c%d_y" % i]))
    y.backward(grad)
    np.testing.assert_array_equal(bits(host(x.grad)), bits(g["c%d_gx" % i]))
    ex_min, ex_max, b_min, b_max = T.lg_encoding_grads_bound(x.detach().cpu(), grad.cpu(), emin.detach().cpu(),
                                                             emax.detach().cpu(), bw, bool(sym))
    for got, ex, b, what in ((emin.grad, ex_min, b_min, "grad_min"), (emax.grad, ex_max, b_max, "grad_max"),
                             (torch.from_numpy(g["c%d_gmin" % i]), ex_min, b_min, "reference grad_min"),
                             (torch.from_numpy(g["c%d_gmax" % i]), ex_max, b_max, "reference grad_max")):
        T.assert_within_sum_bound(got, ex, b, LG_BOUND_C, "golden c%d %s" % (i, what))


@pytest.mark.parametrize("shape,sym", [((4096, 4096), True), ((8, 1 << 20), False), ((96, 3, 7), True),
                                       ((1024, 14336), False)])
def test_learned_grid_large_vs_torch_ref(shape, sym):
    """Llama-like weight (4096 x 4096, per-channel 4-bit symmetric; one workgroup per channel),
    few long channels (channel x slice grid, atomic sums) and K % 4 != 0 (scalar path): kernel vs
    the torch restatement. grad_x bit-exact; encoding gradients within LG_BOUND_C = 2 eps x (sum of
    |terms|) of the float64 sum; torch's own fp32 sums of the restatement are reported beside them
    and held to 64 (they are the torch-op path's, not ours)."""
    from aimet_amd.learned_grid import LearnedGridQuantizeDequantize
    from oracle import torch_ref as T
    torch.manual_seed(2)
    w = (torch.randn(*shape, device=DEV) * 0.02).requires_grad_(True)
    red = tuple(range(1, w.dim()))
    emax = (w.detach().abs().amax(dim=red) * 0.9).requires_grad_(True)
    emin = (-emax.detach() * (1.0 if sym else 0.7)).clone().requires_grad_(True)
    grad = torch.randn_like(w)
    y = LearnedGridQuantizeDequantize.apply(w, emin, emax, 4, sym, False, False, 0)
    yr = T.lg_forward(w.detach(), emin.detach(), emax.detach(), 4, sym)[0]
    assert torch.equal(y, yr)
    y.backward(grad)
    gx, gmin, gmax = T.lg_gradients(w.detach(), grad, emin.detach(), emax.detach(), 4, sym)
    assert torch.equal(w.grad, gx)
    ex_min, ex_max, b_min, b_max = T.lg_encoding_grads_bound(w.detach(), grad, emin.detach(), emax.detach(), 4, sym)
    tag = "large %s sym=%d " % ("x".join(map(str, shape)), sym)
    for got, ex, b, what, c in ((emin.grad, ex_min, b_min, "grad_min", LG_BOUND_C),
                                (emax.grad, ex_max, b_max, "grad_max", LG_BOUND_C),
                                (gmin, ex_min, b_min, "torch restatement grad_min", 64),
                                (gmax, ex_max, b_max, "torch restatement grad_max", 64)):
        T.assert_within_sum_bound(got, ex, b, c, tag + what)


@pytest.mark.parametrize("bw,sym", [(16, False), (16, True), (8, False), (4, True)])
def test_learned_grid_quotients_at_half_integers(bw, sym):
    """The learned-grid kernels form x / delta from a per-encoding reciprocal with one Markstein
    correction (learned_grid.hip: div_rn). Inputs built to land on and +-1..3 ulp around every
    kind of rounding boundary of x / delta (half-integers, the clamp edges), zeros of both signs,
    tiny / huge / non-finite values: y and grad_x == the reference's torch ops bit for bit, on the
    float32 path, per tensor and per channel, and on the bf16 / fp16 per-tensor path (== the
    upcast chain)."""
    from aimet_amd.learned_grid import LearnedGridQuantizeDequantize
    from oracle import torch_ref as T
    g = torch.Generator(device=DEV).manual_seed(bw * 10 + sym)
    C = 4
    emax = torch.tensor([3.1, 0.37, 1e-3, 5e4], device=DEV)
    emin = -emax if sym else -emax * torch.tensor([0.3, 1.0, 0.01, 2.0], device=DEV)
    delta, offset, steps = T.lg_encodings(bw, emin, emax, sym, False, False)
    K = 1 << 14
    n = torch.randint(-(1 << (bw - 1)) - 4, (1 << (bw - 1)) + 4, (C, K), device=DEV, generator=g).float()
    x = ((n + 0.5) * delta.view(C, 1))
    ulps = torch.randint(-3, 4, (C, K), device=DEV, generator=g, dtype=torch.int32)
    x = (x.view(torch.int32) + ulps).view(torch.float32)
    x[:, :64] = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 3e38, -3e38, float("inf"), float("-inf")] * 8, device=DEV)
    x[:, 64:128] = n[:, 64:128] * delta.view(C, 1)            # exact integers
    grad = torch.randn(C, K, device=DEV, generator=g)
    for per_channel in (True, False):
        mn, mx = (emin, emax) if per_channel else (emin[:1], emax[:1])
        xt = x.clone().requires_grad_(True)
        y = LearnedGridQuantizeDequantize.apply(xt, mn, mx, bw, sym, False, False, 0)
        yr = T.lg_forward(x, mn, mx, bw, sym)[0]
        assert torch.equal(y.view(torch.int32), yr.view(torch.int32)), per_channel
        y.backward(grad)
        gx = T.lg_gradients(x, grad, mn, mx, bw, sym)[0]
        assert torch.equal(xt.grad.view(torch.int32), gx.view(torch.int32)), per_channel
    for dt in (torch.bfloat16, torch.float16):
        xh = x[:1].reshape(-1).to(dt)
        yh = LearnedGridQuantizeDequantize.apply(xh, emin[:1], emax[:1], bw, sym, False, False, 0)
        want = T.lg_forward(xh.float(), emin[:1], emax[:1], bw, sym)[0].to(dt)
        assert torch.equal(yh.view(torch.int16), want.view(torch.int16)), dt


@pytest.mark.parametrize("sym", [False, True])
def test_learned_grid_non_finite_inputs_follow_torch(sym):
    """NaN / inf / overflowing inputs: the reference's torch ops pass a NaN through torch.clamp
    (y = NaN), its mask * grad zeroes them, and its encoding-gradient sums turn NaN on a channel
    holding a non-finite x (sym: mask * (x / delta) -- also where x / delta overflows; asym:
    x * mask / delta -- only a non-finite x). y and grad_x bit for bit (NaN positions: the quieted
    input), the encoding gradients NaN on exactly the reference's channels and close elsewhere;
    per channel, per tensor, and the bf16 / fp16 per-tensor path (== the upcast chain)."""
    from aimet_amd.learned_grid import LearnedGridQuantizeDequantize
    from oracle import torch_ref as T
    g = torch.Generator(device=DEV).manual_seed(11 + sym)
    C, K = 5, 4096
    emax = torch.tensor([3.1, 0.37, 1e-3, 5e4, 2.0], device=DEV)
    emin = -emax if sym else -emax * torch.tensor([0.3, 1.0, 0.01, 2.0, 0.5], device=DEV)
    x = torch.randn(C, K, device=DEV, generator=g) * emax.view(C, 1)
    x[0, 7] = float("nan")
    x[0, 4000] = -float("nan")
    x[1, 100] = float("inf")
    x[2, 9] = 3e38                      # x / delta overflows on this channel (delta ~ 1e-5)
    x[3, 17] = torch.tensor(0x7FC00123, dtype=torch.int32).view(torch.float32)   # a NaN payload
    grad = torch.randn(C, K, device=DEV, generator=g)
    for per_channel in (True, False):
        mn, mx = (emin, emax) if per_channel else (emin[2:3], emax[2:3])
        xt = x.clone().requires_grad_(True)
        emn, emx = mn.clone().requires_grad_(True), mx.clone().requires_grad_(True)
        y = LearnedGridQuantizeDequantize.apply(xt, emn, emx, 8, sym, False, False, 0)
        # the reference on the host: x86 passes a NaN's payload through, as the kernels do
        yr = T.lg_forward(x.cpu(), mn.cpu(), mx.cpu(), 8, sym)[0]
        assert torch.equal(y.cpu().view(torch.int32), yr.view(torch.int32)), per_channel
        y.backward(grad)
        gx, gmin, gmax = T.lg_gradients(x.cpu(), grad.cpu(), mn.cpu(), mx.cpu(), 8, sym)
        assert torch.equal(xt.grad.cpu().view(torch.int32), gx.view(torch.int32)), per_channel
        for got, want in ((emn.grad.cpu(), gmin), (emx.grad.cpu(), gmax)):
            assert torch.equal(torch.isnan(got), torch.isnan(want)), (per_channel, got, want)
            fin = ~torch.isnan(want)
            torch.testing.assert_close(got[fin], want[fin], rtol=2e-4, atol=1e-4)
    for dt in (torch.bfloat16, torch.float16):
        xh = x[:2].reshape(-1).to(dt)
        yh = LearnedGridQuantizeDequantize.apply(xh, emin[:1], emax[:1], 8, sym, False, False, 0)
        # the float result from the host reference, cast on the device as the reference's device
        # tensors are (torch's CPU bf16 cast maps NaN to 0xFFFF in its vector part, 0x7FC0 else)
        want = T.lg_forward(xh.float().cpu(), emin[:1].cpu(), emax[:1].cpu(), 8, sym)[0].to(DEV).to(dt)
        assert torch.equal(yh.view(torch.int16), want.view(torch.int16)), dt


@pytest.mark.parametrize("outer,C,K", [(3, 5, 2048), (2, 7, 3072), (4, 3, 100)])
def test_learned_grid_backward_sums_channel_axis_inner(outer, C, K):
    """aimet_lg_backward on [outer][C][K] with outer > 1 (channel axis not first): grad_x exact and
    the per-channel sums A = sum((x_q + o) g), B = sum(mask x/delta g), D = sum(!mask g) against
    float64 numpy (rtol 1e-4: fp32 accumulation order). Covers the tile form (K % 1024 == 0, 4 and 2
    quads per lane) and the channel form."""
    from aimet_amd import _native
    g0 = torch.Generator(device=DEV).manual_seed(outer * 100 + C)
    x = torch.randn(outer, C, K, device=DEV, generator=g0) * 0.3
    g = torch.randn(outer, C, K, device=DEV, generator=g0)
    delta = torch.rand(C, device=DEV, generator=g0) * 0.01 + 0.002
    offset = torch.full((C,), -8.0, device=DEV)
    steps = 15.0
    gx = torch.empty_like(x)
    sums = torch.empty(3 * C, device=DEV)
    _native.call("aimet_lg_backward", x.data_ptr(), g.data_ptr(), gx.data_ptr(), sums.data_ptr(), outer, C, K,
                 delta.data_ptr(), offset.data_ptr(), ctypes.c_float(steps), None,
                 torch.cuda.current_stream().cuda_stream)
    d3, o3 = delta.view(1, C, 1), offset.view(1, C, 1)
    xr = torch.round(x / d3) - o3
    mask = (xr >= 0) & (xr <= steps)
    assert torch.equal(gx, mask.float() * g)
    xq = torch.clamp(xr, 0, steps)
    xd, gd, md = x.double(), g.double(), mask.double()
    A = ((xq.double() + o3.double()) * gd).sum(dim=(0, 2))
    B = (md * (xd / d3.double()) * gd).sum(dim=(0, 2))
    D = ((1 - md) * gd).sum(dim=(0, 2))
    want = torch.stack([A, B, D], 1).reshape(-1).float()
    torch.testing.assert_close(sums, want, rtol=1e-4, atol=1e-3)


# ------------------------------------------------------------------------------------------
# fp16 / bf16 I/O (fused casts) == the reference's upcast -> fp32 kernel -> downcast
# ------------------------------------------------------------------------------------------
def _bits16(t):
    return t.view(torch.int16).cpu().numpy()


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("rm", [0, 1])
def test_16bit_io_qdq_equals_upcast_path(dtype, rm):
    from aimet_amd import _native
    from aimet_amd.tensor_quantizer import IO_DTYPES
    g = torch.Generator(device=DEV).manual_seed(4)
    code = IO_DTYPES[dtype]
    stream = torch.cuda.current_stream().cuda_stream
    for n, off in ((1 << 20, 0), (100003, 1), (7, 0)):
        x = (torch.randn(n + off, device=DEV, generator=g) * 3).to(dtype)[off:]
        if n > 16:
            x[:6] = torch.tensor([float("nan"), float("inf"), -float("inf"), 0.0, -0.0, 1e-7], dtype=dtype)
        enc = enc_of(-2.5, 4.0, 8)
        out16 = torch.empty_like(x)
        _native.call("aimet_qdq_per_tensor_16", x.data_ptr(), out16.data_ptr(), n, code, enc.to_c(), rm, 77, stream)
        xf = x.float()
        out32 = torch.empty_like(xf)
        _native.call("aimet_qdq_per_tensor", xf.data_ptr(), out32.data_ptr(), n, enc.to_c(), rm, 77, stream)
        np.testing.assert_array_equal(_bits16(out16), _bits16(out32.to(dtype)))
    # per-channel: K % 8 == 0 (16-B path) and K % 8 != 0 (scalar path), axis 0 and 1
    for shape, axis in (((64, 16, 3, 3), 0), ((40, 24), 0), ((6, 10, 5), 1)):
        x = (torch.randn(*shape, device=DEV, generator=g) * 0.5).to(dtype)
        C = shape[axis]
        encs = [enc_of(-1.0 - 0.1 * c, 0.8 + 0.05 * c, 8) for c in range(C)]
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF, num_channels=C)
        table = q.channelTable(encs, torch.device(DEV))
        from aimet_amd.tensor_quantizer import per_channel_view
        outer, C, K = per_channel_view(x.shape, axis)
        out16 = torch.empty_like(x)
        _native.call("aimet_qdq_per_channel_16", x.data_ptr(), out16.data_ptr(), outer, C, K, code, table.data_ptr(),
                     rm, 5, stream)
        xf = x.float()
        out32 = torch.empty_like(xf)
        _native.call("aimet_qdq_per_channel", xf.data_ptr(), out32.data_ptr(), outer, C, K, table.data_ptr(), rm, 5,
                     stream)
        np.testing.assert_array_equal(_bits16(out16), _bits16(out32.to(dtype)), err_msg=str(shape))


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_16bit_io_qdq_per_tensor_all_bit_patterns(dtype):
    """Per-tensor nearest QDQ with 16-bit I/O (qdq16_vec_kernel, hoisted rounding threshold): every
    16-bit input pattern, tiled to a large tensor, equals upcast -> fp32 QDQ -> downcast."""
    from aimet_amd import _native
    from aimet_amd.tensor_quantizer import IO_DTYPES
    code = IO_DTYPES[dtype]
    stream = torch.cuda.current_stream().cuda_stream
    n = (1 << 23) + 13
    pat = torch.arange(65536, dtype=torch.int32, device=DEV).to(torch.int16).view(dtype)
    x = pat.repeat(n // 65536 + 1)[:n].contiguous()
    for lo, hi, bw in ((-2.5, 4.0, 8), (-1e-3, 7e4, 16), (0.0, 1.0, 4), (-6e4, 6e4, 8)):
        enc = enc_of(lo, hi, bw)
        out16 = torch.empty_like(x)
        _native.call("aimet_qdq_per_tensor_16", x.data_ptr(), out16.data_ptr(), n, code, enc.to_c(), 0, 0, stream)
        xf = x.float()
        out32 = torch.empty_like(xf)
        _native.call("aimet_qdq_per_tensor", xf.data_ptr(), out32.data_ptr(), n, enc.to_c(), 0, 0, stream)
        np.testing.assert_array_equal(_bits16(out16), _bits16(out32.to(dtype)), err_msg=str((lo, hi, bw)))


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_16bit_io_qdq_per_channel_all_bit_patterns(dtype):
    """Per-channel 16-bit QDQ (qdq16_vec_kernel, hoisted rounding threshold): every 16-bit input
    pattern in every channel, channels with dyadic deltas (exact half-integer quotients: the exact
    division path), zero / non-zero offsets, tiny and huge ranges, non-finite encodings; equals
    upcast -> fp32 per-channel QDQ (IEEE division) -> downcast bit for bit."""
    from aimet_amd import _native
    from aimet_amd.tensor_quantizer import IO_DTYPES
    code = IO_DTYPES[dtype]
    stream = torch.cuda.current_stream().cuda_stream
    ranges = [(-1.0, 1.0, 8), (-0.5, 0.5, 4), (0.0, 1.0, 8), (-1e-3, 7e4, 16), (-6e4, 6e4, 8), (-3e-5, 3e-5, 8),
              (-2.0, 2.0 * 127 / 128, 8), (-2.5, 4.0, 8), (-1e-30, 1e-30, 8), (0.0, 255.0, 8), (-8.0, 7.0, 4),
              (float("-inf"), 1.0, 8), (-1.0, float("nan"), 8),
              # 16-bit grids: products delta * (q + off) on fine grids, where rounding the fp32
              # product to fp16 (torch's two-step cast) and rounding the exact product differ
              (-0.37, 11.3, 16), (-123.4, 77.7, 16), (-3.3e4, 6.1e4, 16), (-0.0123, 0.0456, 16)]
    encs = [enc_of(lo, hi, bw) for lo, hi, bw in ranges]
    C = len(encs)
    pat = torch.arange(65536, dtype=torch.int32, device=DEV).to(torch.int16).view(dtype)
    x = pat.repeat(C).view(C, 65536).contiguous()
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF, num_channels=C)
    table = q.channelTable(encs, torch.device(DEV))
    out16 = torch.empty_like(x)
    _native.call("aimet_qdq_per_channel_16", x.data_ptr(), out16.data_ptr(), 1, C, 65536, code, table.data_ptr(),
                 0, 0, stream)
    xf = x.float()
    out32 = torch.empty_like(xf)
    _native.call("aimet_qdq_per_channel", xf.data_ptr(), out32.data_ptr(), 1, C, 65536, table.data_ptr(), 0, 0,
                 stream)
    got, want = _bits16(out16).reshape(C, -1), _bits16(out32.to(dtype)).reshape(C, -1)
    for c in range(C):
        np.testing.assert_array_equal(got[c], want[c], err_msg=str(ranges[c]))


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_16bit_io_ste_and_autograd(dtype):
    from aimet_amd.quantizers import (QuantScheme, StaticGridPerChannelQuantizer, StaticGridPerTensorQuantizer,
                                      compute_dloss_by_dx)
    g = torch.Generator(device=DEV).manual_seed(6)
    x = (torch.randn(1 << 16, device=DEV, generator=g) * 3).to(dtype)
    gr = torch.randn(1 << 16, device=DEV, generator=g).to(dtype)
    got = compute_dloss_by_dx(x, gr, -2.0, 2.5)
    want = compute_dloss_by_dx(x.float(), gr.float(), -2.0, 2.5).to(dtype)
    np.testing.assert_array_equal(_bits16(got), _bits16(want))
    w = (torch.randn(32, 16, 3, 3, device=DEV, generator=g) * 0.1).to(dtype)
    gw = torch.randn_like(w)
    mins = [-0.1 - 0.01 * c for c in range(32)]
    maxs = [0.12 + 0.01 * c for c in range(32)]
    got = compute_dloss_by_dx(w, gw, mins, maxs, 0)
    want = compute_dloss_by_dx(w.float(), gw.float(), mins, maxs, 0).to(dtype)
    np.testing.assert_array_equal(_bits16(got), _bits16(want))
    # through the quantizer's autograd function: forward / backward == the upcast path
    for tq in (StaticGridPerTensorQuantizer(8, "nearest", QuantScheme.post_training_tf, False, True),
               StaticGridPerChannelQuantizer(8, "nearest", QuantScheme.post_training_tf, True, 32, True)):
        src = w if isinstance(tq, StaticGridPerChannelQuantizer) else w.flatten()
        tq.update_encoding_stats(src.float())
        tq.compute_encoding()
        a = src.clone().requires_grad_(True)
        y = tq.quantize_dequantize(a, "nearest")
        assert y.dtype == dtype
        y.backward(torch.ones_like(y))
        b = src.float().clone().requires_grad_(True)
        y32 = tq.quantize_dequantize(b, "nearest")
        y32.backward(torch.ones_like(y32))
        np.testing.assert_array_equal(_bits16(y.detach()), _bits16(y32.detach().to(dtype)))
        if isinstance(tq, StaticGridPerChannelQuantizer):
            # 1-D float32 bounds: the 16-bit mask equals the fp32 one
            np.testing.assert_array_equal(_bits16(a.grad), _bits16(b.grad.to(dtype)))
        else:
            # scalar bounds are compared in x's dtype (the reference's 0-dim bound tensor)
            emn, emx = torch.tensor(tq.encoding.min), torch.tensor(tq.encoding.max)
            xc = src.cpu()
            want = torch.ones_like(xc) * (emn <= xc).logical_and(xc <= emx)
            np.testing.assert_array_equal(_bits16(a.grad), _bits16(want))


def test_qdq_and_histogram_near_rounding_boundaries():
    """Inputs within a few ulp of every rounding boundary (x / delta - offset = k + 1/2): the
    reciprocal fast path must defer to the IEEE division exactly there (bit-exact vs the oracle),
    for QDQ (fp32 and bf16 I/O) and the histogram binning."""
    rng = np.random.default_rng(31)
    for bw, mn, mx in ((8, -3.1, 5.7), (4, -0.37, 0.9), (16, -1e-3, 2e-3), (8, 0.0, 6.0), (8, -1e4, 3e4)):
        e = O.fill_encoding_info(bw, mn, mx)
        d, o = np.float32(e.delta), np.float32(e.offset)
        k = np.arange(0, 2 ** bw, max(1, 2 ** bw // 4096), dtype=np.float32)
        base = ((k + np.float32(0.5) + o) * d).astype(np.float32)
        xs = [base]
        for s in (1, 2, 3):
            xs.append(np.nextafter(base, np.float32(np.inf)))
            xs.append(np.nextafter(base, np.float32(-np.inf)))
            base = xs[-2]
        x = np.concatenate(xs + [rng.uniform(mn, mx, 100000).astype(np.float32)]).astype(np.float32)
        y = host(AimetTensorQuantizer.quantize_dequantize_tensor(gpu(x), enc_of(mn, mx, bw)))
        np.testing.assert_array_equal(bits(y), bits(O.qdq_per_tensor(x, mn, mx, bw)), err_msg=str((bw, mn, mx)))
        # quantize-only exposes the sign of a zero code (x / delta ~ offset): code-0 neighbourhood
        z = ((o + np.float32(0.0)) * d).astype(np.float32)
        zs = [np.nextafter(z, np.float32(np.inf) if s > 0 else np.float32(-np.inf)) for s in (1, -1)]
        xz = np.concatenate([x, np.array([z] + zs, np.float32).ravel(),
                             (z + rng.uniform(-1, 1, 1000).astype(np.float32) * d * np.float32(0.6))
                             .astype(np.float32)])
        qz = host(AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF).quantize(gpu(xz), enc_of(mn, mx, bw),
                                                                                  NEAREST, True, False))
        np.testing.assert_array_equal(bits(qz), bits(O.quantize_per_tensor(xz, mn, mx, bw, False)))
        # histogram over the same values (bins = round(x / bucket - offset))
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
        a = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
        q.updateStats(gpu(x), True)
        a.update(x)
        xl, _ = a.histogram()
        bucket = np.float32(xl[1] - xl[0])
        off = np.float32(np.float32(xl[0]) / bucket)
        edges = ((np.arange(512, dtype=np.float32) + np.float32(0.5) + off) * bucket).astype(np.float32)
        x2 = np.concatenate([edges, np.nextafter(edges, np.float32(np.inf)), np.nextafter(edges, np.float32(-np.inf))])
        q.updateStats(gpu(x2), True)
        a.update(x2)
        np.testing.assert_array_equal(np.array([t[1] for t in q.getStatsHistogram()]), a.histogram()[1])


def test_update_stats_many_equals_individual():
    """aimet_tq_update_stats_many (one launch per phase for all quantizers) == updateStats per
    quantizer: every scheme, sizes from 1 element to 2^22 (unaligned views, an all-zero first
    batch, NaN / inf), three batches, then encodings and histograms bit-identical."""
    rng = np.random.default_rng(12)
    schemes = [QuantizationMode.QUANTIZATION_TF, QuantizationMode.QUANTIZATION_TF_ENHANCED,
               QuantizationMode.QUANTIZATION_PERCENTILE, QuantizationMode.QUANTIZATION_MSE]
    sizes = [1, 3, 1000, 4097, 65536, 1 << 22]
    specs = [(s, n) for s in schemes for n in sizes]
    a = [AimetTensorQuantizer(s) for s, _ in specs]
    b = [AimetTensorQuantizer(s) for s, _ in specs]
    for q in a + b:
        if q.quant_scheme == QuantizationMode.QUANTIZATION_PERCENTILE:
            q.setPercentileValue(99.5)
    for batch in range(3):
        ts = []
        for i, (s, n) in enumerate(specs):
            x = (rng.standard_normal(n + 1) * (1 + batch + i % 3)).astype(np.float32)
            if batch == 0 and i % 5 == 0:
                x[:] = 0.0
            if n > 100 and batch == 1:
                x[7], x[8] = np.nan, np.inf
            ts.append(gpu(x)[1:])          # 4-byte offset: exercises the scalar path
        AimetTensorQuantizer.updateStatsMany(a, ts)
        for q, t in zip(b, ts):
            q.updateStats(t, True)
    for fl in FLAGS:
        for qa, qb in zip(a, b):
            assert qa.getEncoding(8, *fl)[0].to_tuple() == qb.getEncoding(8, *fl)[0].to_tuple()
    for qa, qb in zip(a, b):
        if qa.quant_scheme != QuantizationMode.QUANTIZATION_TF:
            assert qa.getStatsHistogram() == qb.getStatsHistogram()


def test_update_stats_channels_many_equals_individual():
    """aimet_tq_update_stats_channels_many (min/max + fold, histogram + fold: two launches for
    every channel of every quantizer) == updateStatsPerChannel per quantizer, for every scheme
    incl. entropy, channel axes 0 and 1, ragged K, unaligned views, all-zero channels and first
    batches, NaN / inf, three batches; then encodings, histograms and entropy state bit-identical,
    and a few channels against the CPU oracle."""
    rng = np.random.default_rng(31)
    schemes = [QuantizationMode.QUANTIZATION_TF, QuantizationMode.QUANTIZATION_TF_ENHANCED,
               QuantizationMode.QUANTIZATION_PERCENTILE, QuantizationMode.QUANTIZATION_MSE,
               QuantizationMode.QUANTIZATION_ENTROPY]
    shapes = [((64, 3, 7, 7), 0), ((96, 32, 3, 3), 0), ((16, 24, 3, 3), 1), ((40, 130), 0), ((7, 1), 0),
              ((3, 1000), 0)]
    specs = [(s, sh, ax) for s in schemes for sh, ax in shapes]
    a = [AimetTensorQuantizer(s, num_channels=sh[ax]) for s, sh, ax in specs]
    b = [AimetTensorQuantizer(s, num_channels=sh[ax]) for s, sh, ax in specs]
    for q in a + b:
        if q.quant_scheme == QuantizationMode.QUANTIZATION_PERCENTILE:
            q.setPercentileValue(99.5)
    orc = {}
    for batch in range(3):
        ts = []
        for i, (s, sh, ax) in enumerate(specs):
            n = int(np.prod(sh))
            xt = (rng.standard_normal(n) * (1 + batch + i % 3)).astype(np.float32)
            if batch == 0 and i % 4 == 0:
                xt[:] = 0.0
            if n > 100 and batch == 1:
                xt[7], xt[8] = np.nan, np.inf
            xt = xt.reshape(sh)
            xt[(slice(None),) * ax + (min(1, sh[ax] - 1),)] = 0.0   # an all-zero channel
            if i % 2:   # odd specs: a 4-byte offset view (scalar path)
                ts.append(gpu(np.concatenate([[0], xt.ravel()]))[1:].view(sh))
            else:
                ts.append(gpu(xt))
            if s in (QuantizationMode.QUANTIZATION_TF_ENHANCED, QuantizationMode.QUANTIZATION_TF) and i % 3 == 0:
                C = sh[ax]
                oc = orc.setdefault(i, [O.Analyzer(int(s)) for _ in range(C)])
                for c in range(C):
                    oc[c].update(np.ascontiguousarray(np.take(xt, c, axis=ax)))
        keep = AimetTensorQuantizer.updateStatsPerChannelMany(a, ts, [ax for _, _, ax in specs])
        for q, t, (_, _, ax) in zip(b, ts, specs):
            q.updateStatsPerChannel(t, ax, True)
        torch.cuda.synchronize()
        del keep
    for fl in FLAGS:
        for i, (qa, qb) in enumerate(zip(a, b)):
            if qa.quant_scheme == QuantizationMode.QUANTIZATION_MSE and fl[1]:
                continue
            ea, va = qa.getEncoding(8, *fl)
            eb, vb = qb.getEncoding(8, *fl)
            assert va == vb
            ta = np.array([e.to_tuple() for e in ea], np.float64)
            tb = np.array([e.to_tuple() for e in eb], np.float64)
            assert np.array_equal(ta.view(np.uint64), tb.view(np.uint64)), (i, fl)   # NaN-safe
            if i in orc:
                for c, o in enumerate(orc[i]):
                    assert ea[c].to_tuple() == o.compute(8, *fl).as_tuple(), (i, c, fl)
    for qa, qb in zip(a, b):
        for c in range(qa.num_channels):
            if qa.quant_scheme == QuantizationMode.QUANTIZATION_ENTROPY:
                sa, sb = qa.entropy_state(c), qb.entropy_state(c)
                assert sa.keys() == sb.keys()
                assert all(np.array_equal(np.asarray(sa[k]), np.asarray(sb[k])) for k in sa), c
            elif qa.quant_scheme != QuantizationMode.QUANTIZATION_TF:
                assert qa.getStatsHistogram(c) == qb.getStatsHistogram(c)


def test_reset_many_then_recompute_equals_fresh_quantizers():
    """aimet_tq_reset_encoding_stats_many (one zeroing launch + one re-initialisation, no sync)
    leaves quantizers that calibrate exactly like new ones (TF, TF-E, percentile, MSE, entropy;
    per-tensor and per-channel)."""
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    g = torch.Generator(device=DEV).manual_seed(21)
    modes = [QuantizationMode.QUANTIZATION_TF, QuantizationMode.QUANTIZATION_TF_ENHANCED,
             QuantizationMode.QUANTIZATION_PERCENTILE, QuantizationMode.QUANTIZATION_MSE,
             QuantizationMode.QUANTIZATION_ENTROPY]

    def make():
        return [AimetTensorQuantizer(m) for m in modes] + [AimetTensorQuantizer(m, num_channels=6) for m in modes]

    def feed(qs, seed):
        gg = torch.Generator(device=DEV).manual_seed(seed)
        x = torch.randn(4, 6, 9, 9, device=DEV, generator=gg) * 3 + 1
        for q in qs:
            if q.num_channels == 1:
                q.updateStats(x, True)
            else:
                q.updateStatsPerChannel(x, 1, True)

    def encs(qs):
        out = []
        for q in qs:
            e, v = q.getEncoding(8, False, False, False)
            out.append(([t.to_tuple() for t in e] if isinstance(e, list) else e.to_tuple(), v))
        return out

    used = make()
    feed(used, 1)
    feed(used, 2)
    AimetTensorQuantizer.resetEncodingStatsMany(used)
    assert all(not v for _, v in encs(used))
    feed(used, 3)
    fresh = make()
    feed(fresh, 3)
    assert encs(used) == encs(fresh)


@pytest.mark.parametrize("act", [None, torch.nn.ReLU(), torch.nn.ReLU6()])
@pytest.mark.parametrize("shape", [(32, 24, 12, 12), (32, 1000), (3, 5, 7)])
def test_recon_loss_backward_fused_vs_torch(act, shape):
    """aimet_adaround_recon_grad (one pass) == the gradient of adaround_loss.py:70-80's
    recon_loss(act(q), act(t)) through torch autograd, to fp32 rounding."""
    from aimet_amd.adaround_optimizer import recon_loss, recon_loss_backward
    g = torch.Generator(device=DEV).manual_seed(8)
    q0 = torch.randn(*shape, device=DEV, generator=g) * 4
    t = q0 + torch.randn(*shape, device=DEV, generator=g)
    q0[0].view(-1)[:3] = torch.tensor([0.0, 6.0, -0.0], device=DEV)   # activation edges
    qa = q0.clone().requires_grad_(True)
    recon_loss_backward(qa, t, act)
    qb = q0.clone().requires_grad_(True)
    a, b = (act(qb), act(t)) if act is not None else (qb, t)
    recon_loss(a, b).backward()
    torch.testing.assert_close(qa.grad, qb.grad, rtol=2e-6, atol=1e-12)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("K", [4096, 1000])
def test_learned_grid_cast_fused_weight_equals_cast_after(dtype, sym, K):
    """out_dtype: aimet_lg_forward_cast == the float32 op then .to(dtype); aimet_lg_backward_grad16
    on the 16-bit gradient == the float32 backward on grad.to(float32) -- y, grad_x and both range
    gradients bit for bit (per-channel [C, K] weights with K a multiple of 1024)."""
    from aimet_amd.learned_grid import LearnedGridQuantizeDequantize as LG
    g = torch.Generator(device=DEV).manual_seed(41 + int(sym))
    C = 96   # K = 1000: rows not a multiple of 1024 -> the backward upcasts the gradient first
    w = torch.randn(C, K, device=DEV, generator=g) * 0.02
    amax = w.abs().amax(dim=1) * 0.8
    gy = torch.randn(C, K, device=DEV, generator=g).to(dtype)
    outs = []
    for fused in (True, False):
        x = w.clone().requires_grad_(True)
        emin = (-amax if sym else w.amin(dim=1) * 0.9).clone().requires_grad_(True)
        emax = amax.clone().requires_grad_(True)
        if fused:
            y = LG.apply(x, emin, emax, 4, sym, False, False, 0, dtype)
            assert y.dtype == dtype
            y.backward(gy)
        else:
            y = LG.apply(x, emin, emax, 4, sym, False, False, 0).to(dtype)
            y.backward(gy)
        outs.append((y.detach(), x.grad, emin.grad, emax.grad))
    (y_a, gx_a, gn_a, gm_a), (y_b, gx_b, gn_b, gm_b) = outs
    assert torch.equal(y_a.view(torch.int16), y_b.view(torch.int16))
    assert torch.equal(gx_a.view(torch.int32), gx_b.view(torch.int32))
    assert torch.equal(gn_a.view(torch.int32), gn_b.view(torch.int32))
    assert torch.equal(gm_a.view(torch.int32), gm_b.view(torch.int32))


def test_learned_grid_wrapper_autocast_cast_fusion_is_exact(monkeypatch):
    """LearnedGridQuantWrapper around a Linear under bf16 autocast: with the weight's cast fused
    into the quantizer kernels and without it, the forward output and every gradient (input,
    weight, both ranges of the weight and output quantizers) are bit-identical."""
    from aimet_amd import qc_quantize_op as Q
    from aimet_amd.quantizers import QuantScheme
    from aimet_amd.quantsim import QuantizationSimModel
    torch.manual_seed(5)
    cfg = {"defaults": {"ops": {"is_output_quantized": "True"},
                        "params": {"is_quantized": "True", "is_symmetric": "True"},
                        "strict_symmetric": "False", "per_channel_quantization": "True"}}
    x = torch.randn(8, 64, 2048, device=DEV)
    results = []
    for fuse in (True, False):
        monkeypatch.setattr(Q, "_FUSE_AUTOCAST_CAST", fuse)
        torch.manual_seed(5)
        model = torch.nn.Sequential(torch.nn.Linear(2048, 512, bias=False)).to(DEV)
        sim = QuantizationSimModel(model, quant_scheme=QuantScheme.training_range_learning_with_tf_init,
                                   default_param_bw=4, default_output_bw=16, config_file=cfg,
                                   dummy_input=x[:1])

        def cal(m, _):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                m(x)
        sim.compute_encodings(cal, None)
        xin = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = sim.model(xin)
        out.float().square().mean().backward()
        grads = {n: p.grad.clone() for n, p in sim.model.named_parameters() if p.grad is not None}
        results.append((out.detach(), xin.grad.clone(), grads))
    (o_a, gx_a, g_a), (o_b, gx_b, g_b) = results
    assert o_a.dtype == o_b.dtype and torch.equal(o_a, o_b)
    assert torch.equal(gx_a, gx_b)
    assert g_a.keys() == g_b.keys() and len(g_a) >= 3
    for k in g_a:
        assert torch.equal(g_a[k], g_b[k]), k


def _same_bits_or_nan(a, b):
    """Bit-equal float32 tensors, except that a NaN only has to be a NaN (its sign and payload
    follow the instruction sequence that produced it, not the arithmetic)."""
    na, nb = torch.isnan(a), torch.isnan(b)
    return torch.equal(na, nb) and torch.equal(a.view(torch.int32)[~na], b.view(torch.int32)[~nb])


def test_learned_grid_gate_and_range_grads_equal_torch_ops_on_device():
    """aimet_lg_gate_range == the reference's clamp_ / clamp_ / maximum(max, min + 1e-5) and
    aimet_lg_range_grads == asymmetric_gradients / symmetric_gradients' torch expressions on the
    sums, on the device, bit for bit (NaN and signed-zero ranges included)."""
    from aimet_amd import _native
    from aimet_amd.learned_grid import set_encoding_min_max_gating_threshold
    g = torch.Generator(device=DEV).manual_seed(43)
    n = 5000
    mn = torch.randn(n, device=DEV, generator=g)
    mx = torch.randn(n, device=DEV, generator=g)
    mn[:6] = torch.tensor([float("nan"), 0.0, -0.0, 1e-30, -1e-6, 3.0], device=DEV)
    mx[6:12] = torch.tensor([float("nan"), 0.0, -0.0, -1e-30, 2e-6, -3.0], device=DEV)
    a, b = mn.clone(), mx.clone()
    with torch.no_grad():
        a.clamp_(max=0.0)
        b.clamp_(min=0.0)
        b.copy_(torch.maximum(b, a + torch.full_like(a, 1e-5)))
    c, d = mn.clone(), mx.clone()
    set_encoding_min_max_gating_threshold(c, d)
    assert _same_bits_or_nan(c, a)
    assert _same_bits_or_nan(d, b)
    # range gradients from random sums, both flavours
    from aimet_amd.learned_grid import _delta_offset
    emin, emax = -(torch.rand(n, device=DEV, generator=g) + 0.1), torch.rand(n, device=DEV, generator=g) + 0.1
    sums = torch.randn(n, 3, device=DEV, generator=g) * 100
    for bw, sym in ((4, True), (8, False), (16, False), (8, True)):
        delta, _, steps = _delta_offset(bw, emin, emax, sym, False, False)
        st = torch.full_like(emin, steps)
        A, B, D = sums[:, 0], sums[:, 1], sums[:, 2]
        gss = A - B
        if sym:
            want_max = gss / torch.div(st, 2, rounding_mode="floor")
            want_min = -want_max
        else:
            term1 = gss / st
            term2 = st / (emax - emin) ** 2 * (delta * D)
            want_min, want_max = -term1 + emax * term2, term1 - emin * term2
        gmin, gmax = torch.empty_like(emin), torch.empty_like(emax)
        _native.call("aimet_lg_range_grads", sums.data_ptr(), emin.data_ptr(), emax.data_ptr(), delta.data_ptr(), n,
                     steps, int(sym), gmin.data_ptr(), gmax.data_ptr(), torch.cuda.current_stream().cuda_stream)
        assert torch.equal(gmin.view(torch.int32), want_min.view(torch.int32)), (bw, sym)
        assert torch.equal(gmax.view(torch.int32), want_max.view(torch.int32)), (bw, sym)


@pytest.mark.parametrize("shape", [(1, 1, 300001), (1, 64, 4096), (3, 16, 1000), (1, 8, 77)])
@pytest.mark.parametrize("sym", [False, True])
def test_learned_grid_range_epilogue_equals_separate_launch(shape, sym):
    """The encoding gradients written by the backward's fold (aimet_lg_range_spec) == aimet_lg_range_grads
    on the sums the same call returns, bit for bit, on every backward path (per tensor, tile,
    channel x slice, channel)."""
    from aimet_amd import _native
    from aimet_amd.learned_grid import _RangeSpec, _device_delta_offset
    outer, C, K = shape
    g = torch.Generator(device=DEV).manual_seed(C * 7 + int(sym))
    x = torch.randn(outer, C, K, device=DEV, generator=g)
    gr = torch.randn(outer, C, K, device=DEV, generator=g)
    emin = -(torch.rand(C, device=DEV, generator=g) + 0.5)
    emax = torch.rand(C, device=DEV, generator=g) + 0.5
    delta, offset, steps = _device_delta_offset(8, emin, emax, sym, False, False)
    sums = torch.empty(C, 3, device=DEV)
    gmin, gmax = torch.empty_like(emin), torch.empty_like(emax)
    spec = ctypes.byref(_RangeSpec(emin.data_ptr(), emax.data_ptr(), delta.data_ptr(), gmin.data_ptr(),
                                   gmax.data_ptr(), int(sym)))
    s = torch.cuda.current_stream().cuda_stream
    _native.call("aimet_lg_backward", x.data_ptr(), gr.data_ptr(), None, sums.data_ptr(), outer, C, K,
                 delta.data_ptr(), offset.data_ptr(), ctypes.c_float(steps), spec, s)
    want_min, want_max = torch.empty_like(emin), torch.empty_like(emax)
    _native.call("aimet_lg_range_grads", sums.data_ptr(), emin.data_ptr(), emax.data_ptr(), delta.data_ptr(), C,
                 ctypes.c_float(steps), int(sym), want_min.data_ptr(), want_max.data_ptr(), s)
    assert torch.equal(gmin, want_min) and torch.equal(gmax, want_max)


@pytest.mark.parametrize("shape", [(1, 1, 100003), (1, 48, 1024), (2, 16, 777), (1, 5, 3)])
@pytest.mark.parametrize("flags", [(True, False, False), (False, False, False), (True, True, False), (True, False, True)])
def test_learned_grid_forward_range_equals_tables(shape, flags):
    """aimet_lg_forward_range (encodings computed in the forward kernel) == aimet_lg_encodings +
    aimet_lg_forward: delta, offset and y bit for bit; the 16-bit per-tensor form likewise."""
    from aimet_amd import _native
    from aimet_amd.learned_grid import _device_delta_offset
    outer, C, K = shape
    sym, strict, uns = flags
    g = torch.Generator(device=DEV).manual_seed(C + K)
    x = torch.randn(outer, C, K, device=DEV, generator=g) * 2
    emin = -(torch.rand(C, device=DEV, generator=g) + 0.3) if not uns else torch.zeros(C, device=DEV)
    emax = torch.rand(C, device=DEV, generator=g) + 0.3
    s = torch.cuda.current_stream().cuda_stream
    d_ref, o_ref, steps = _device_delta_offset(8, emin, emax, sym, strict, uns)
    y_ref = torch.empty_like(x)
    _native.call("aimet_lg_forward", x.data_ptr(), y_ref.data_ptr(), outer, C, K, d_ref.data_ptr(), o_ref.data_ptr(),
                 ctypes.c_float(steps), s)
    y, d, o = torch.empty_like(x), torch.empty_like(emin), torch.empty_like(emin)
    rng = torch.full((2, C), float("nan"), device=DEV)
    _native.call("aimet_lg_forward_range", x.data_ptr(), y.data_ptr(), outer, C, K, 0, emin.data_ptr(),
                 emax.data_ptr(), 8, int(sym), int(strict), int(uns), d.data_ptr(), o.data_ptr(), rng.data_ptr(), s)
    assert torch.equal(d, d_ref) and torch.equal(o, o_ref) and torch.equal(y, y_ref)
    assert torch.equal(rng[0], emin) and torch.equal(rng[1], emax)   # the saved copy of the range
    if C == 1:
        xb = x.reshape(-1).to(torch.bfloat16)
        yb_ref, yb = torch.empty_like(xb), torch.empty_like(xb)
        _native.call("aimet_lg_forward_16", xb.data_ptr(), yb_ref.data_ptr(), xb.numel(), 2, d_ref.data_ptr(),
                     o_ref.data_ptr(), ctypes.c_float(steps), s)
        d2, o2 = torch.empty_like(emin), torch.empty_like(emin)
        _native.call("aimet_lg_forward_16_range", xb.data_ptr(), yb.data_ptr(), xb.numel(), 2, emin.data_ptr(),
                     emax.data_ptr(), 8, int(sym), int(strict), int(uns), d2.data_ptr(), o2.data_ptr(), None, s)
        assert torch.equal(yb.view(torch.int16), yb_ref.view(torch.int16))
        assert torch.equal(d2, d_ref) and torch.equal(o2, o_ref)


def test_learned_grid_encodings_equal_reference_torch_ops_on_device():
    """learned_grid._delta_offset (cached 0-dim device constants, fewer launches) == the reference's
    get_computed_encodings with its full_like tensors (oracle/torch_ref.lg_encodings), on the
    device, bit for bit -- including the sign of a zero offset; a NaN range gives NaN."""
    from aimet_amd.learned_grid import _delta_offset, _device_delta_offset
    from oracle import torch_ref as T
    g = torch.Generator(device=DEV).manual_seed(31)
    for bw in (2, 4, 8, 16):
        for sym in (False, True):
            for strict in (False, True):
                for uns in (False, True):
                    emin = torch.randn(4099, device=DEV, generator=g) * 3 - 1
                    emax = emin.abs() + torch.rand(4099, device=DEV, generator=g) * 5
                    emin[:4] = torch.tensor([float("nan"), 0.0, -0.0, float("inf")], device=DEV)
                    emax[4:8] = torch.tensor([float("nan"), 0.0, 1e-30, -1.0], device=DEV)
                    d_ref, o_ref, _ = T.lg_encodings(bw, emin, emax, sym, strict, uns)
                    for fn in (_delta_offset, _device_delta_offset):
                        d, o, steps = fn(bw, emin, emax, sym, strict, uns)
                        assert _same_bits_or_nan(d, d_ref), (fn, bw, sym, strict, uns)
                        assert _same_bits_or_nan(o, o_ref), (fn, bw, sym, strict, uns)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [4096 * 33 + 3, 1 << 22])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("specials", [(0.0, -0.0, 6e4, -6e4), (0.0, -0.0, float("inf"), float("nan"))])
def test_learned_grid_16bit_io_equals_upcast_chain(dtype, n, sym, specials):
    """aimet_lg_forward_16 / aimet_lg_backward_16 == x.to(float32) -> the fp32 kernels -> .to(dtype),
    bit for bit: y, grad_x and both encoding gradients (the sums run in the same order; with a
    non-finite input both are NaN, as the reference's)."""
    from aimet_amd.learned_grid import LearnedGridQuantizeDequantize as LG
    g = torch.Generator(device=DEV).manual_seed(n % 1000 + int(sym))
    x16 = (torch.randn(n, device=DEV, generator=g) * 3).to(dtype)
    x16[:4] = torch.tensor(specials, device=DEV).to(dtype)
    g16 = torch.randn(n, device=DEV, generator=g).to(dtype)
    outs = []
    for x_in, g_in in ((x16.clone(), g16), (x16.float(), g16.float())):
        x_in.requires_grad_(True)
        emin = torch.tensor([-2.5], device=DEV, requires_grad=True)
        emax = torch.tensor([3.25], device=DEV, requires_grad=True)
        y = LG.apply(x_in, emin, emax, 16 if dtype == torch.bfloat16 else 8, sym, False, False, 0)
        y.backward(g_in)
        outs.append((y.detach().to(dtype), x_in.grad.to(dtype), emin.grad, emax.grad))
    (y_a, gx_a, gmin_a, gmax_a), (y_b, gx_b, gmin_b, gmax_b) = outs
    assert torch.equal(y_a.view(torch.int16), y_b.view(torch.int16))
    assert torch.equal(gx_a.view(torch.int16), gx_b.view(torch.int16))
    assert torch.equal(gmin_a.view(torch.int32), gmin_b.view(torch.int32))
    assert torch.equal(gmax_a.view(torch.int32), gmax_b.view(torch.int32))
    assert bool(torch.isfinite(gmin_a).all()) == all(abs(v) < float("inf") for v in specials)


_LG_FOLD_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from aimet_amd.learned_grid import LearnedGridQuantizeDequantize as LG
dev = torch.device("cuda", 0)
out = []
for n, dtype in ((13_690_000, torch.bfloat16), (2_100_000, torch.float16), (1_000_003, torch.float32)):
    g = torch.Generator(device=dev).manual_seed(n)
    x = (torch.randn(n, device=dev, generator=g) * 3).to(dtype).requires_grad_(True)
    gy = torch.randn(n, device=dev, generator=g).to(dtype)
    emin = torch.tensor([-2.5], device=dev, requires_grad=True)
    emax = torch.tensor([3.25], device=dev, requires_grad=True)
    LG.apply(x, emin, emax, 16 if dtype != torch.float32 else 8, False, False, False, 0).backward(gy)
    out += [emin.grad.view(torch.int32).item(), emax.grad.view(torch.int32).item()]
print(" ".join(str(v) for v in out))
"""


def test_learned_grid_fold_is_reproducible_across_processes():
    """The per-tensor backward's encoding gradients (per-tile partials folded in one fixed order,
    fold_partials) are the same bits in two processes, fp32 and 16-bit, on Llama-3-8B call sizes:
    nothing in them depends on scheduling."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for _ in range(2):
        r = subprocess.run([sys.executable, "-c", _LG_FOLD_CHILD, repo], capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        res.append(r.stdout.strip().splitlines()[-1])
    assert res[0] == res[1], res


@pytest.mark.parametrize("N,C,H,K,stride,pad,dil", [(32, 32, 112, 3, 1, 1, 1), (32, 96, 112, 3, 2, 1, 1),
                                                    (5, 7, 13, 3, 2, 0, 1), (4, 16, 19, 5, 1, 2, 1),
                                                    (3, 12, 17, 3, 1, 2, 2), (32, 960, 7, 3, 1, 1, 1)])
def test_depthwise_conv_kernels_vs_torch(N, C, H, K, stride, pad, dil):
    """aimet_dwconv2d_forward == torch's depthwise conv2d (native kernel, bias included) and
    aimet_dwconv2d_grad_weight == autograd's weight gradient, to fp32 summation-order tolerance."""
    import ctypes
    from aimet_amd import _native
    g = torch.Generator(device=DEV).manual_seed(N * C + K)
    x = torch.randn(N, C, H, H, device=DEV, generator=g)
    w = torch.randn(C, 1, K, K, device=DEV, generator=g) * 0.3
    b = torch.randn(C, device=DEV, generator=g)
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    try:
        wr = w.clone().requires_grad_(True)
        ref = torch.nn.functional.conv2d(x, wr, b, stride, pad, dil, C)
        gy = torch.randn(ref.shape, device=DEV, generator=g)
        ref.backward(gy)
    finally:
        torch.backends.cudnn.enabled = prev
    OH, OW = ref.shape[2], ref.shape[3]
    y = torch.empty_like(ref)
    s = torch.cuda.current_stream().cuda_stream
    _native.call("aimet_dwconv2d_forward", x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), N, C, H, H, OH, OW,
                 K, stride, pad, dil, s)
    torch.testing.assert_close(y, ref.detach(), rtol=1e-6, atol=1e-5)
    gw = torch.empty_like(w)
    _native.call("aimet_dwconv2d_grad_weight", x.data_ptr(), gy.data_ptr(), gw.data_ptr(), None, N, C, H, H, OH, OW,
                 K, stride, pad, dil, s)
    n_ws = ctypes.c_int64()
    _native.call("aimet_dwconv2d_grad_weight_workspace", N, C, OH, OW, K, ctypes.byref(n_ws))
    ws = torch.empty(n_ws.value, device=DEV)
    gw2 = torch.empty_like(w)
    _native.call("aimet_dwconv2d_grad_weight", x.data_ptr(), gy.data_ptr(), gw2.data_ptr(), ws.data_ptr(), N, C, H, H,
                 OH, OW, K, stride, pad, dil, s)
    torch.testing.assert_close(gw2, gw, rtol=0, atol=0)          # deterministic
    scale = float((gy.abs().sum() * x.abs().max()) / (N * OH * OW) ** 0.5)
    torch.testing.assert_close(gw, wr.grad, rtol=2e-5, atol=1e-6 * scale)


@pytest.mark.parametrize("N,C,H,K,stride,pad,dil,act,with_bias", [(32, 32, 112, 3, 1, 1, 1, 2, False),
                                                                   (8, 96, 56, 3, 2, 1, 1, 2, True),
                                                                   (5, 7, 13, 3, 2, 0, 1, 0, True),
                                                                   (4, 16, 19, 5, 1, 2, 1, 1, False),
                                                                   (3, 12, 17, 3, 1, 2, 2, 1, True),
                                                                   (32, 960, 7, 3, 1, 1, 1, 2, False)])
def test_adaround_dw_step_equals_unfused_chain(N, C, H, K, stride, pad, dil, act, with_bias):
    """aimet_adaround_dw_step (the depthwise AdaRound iteration in one pass over the cached rows)
    == aimet_adaround_gather -> aimet_dwconv2d_forward -> aimet_adaround_recon_grad_indexed ->
    aimet_dwconv2d_grad_weight, bit for bit, and moves the iteration counter the same way."""
    import ctypes
    from aimet_amd import _native
    g = torch.Generator(device=DEV).manual_seed(N * C + K + act)
    rows = N + 5
    OH = (H + 2 * pad - dil * (K - 1) - 1) // stride + 1
    x_cache = torch.randn(rows, C, H, H, device=DEV, generator=g)
    t_cache = torch.randn(rows, C, OH, OH, device=DEV, generator=g) * 2 + 1
    w = torch.randn(C, 1, K, K, device=DEV, generator=g) * 0.3
    b = torch.randn(C, device=DEV, generator=g) if with_bias else None
    iters = 3
    idx = torch.stack([torch.randperm(rows, device=DEV, generator=g)[:N] for _ in range(iters)]).contiguous()
    s = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr() if t is not None else None   # noqa: E731
    n_ws = ctypes.c_int64()
    _native.call("aimet_dwconv2d_grad_weight_workspace", N, C, OH, OH, K, ctypes.byref(n_ws))
    ws = torch.empty(n_ws.value, device=DEV)
    for it in (0, 2):
        # unfused chain
        ctr = torch.tensor([it, -1], dtype=torch.long, device=DEV)
        inp = torch.empty(N, C, H, H, device=DEV)
        _native.call("aimet_adaround_gather", P(x_cache), P(t_cache), P(inp), None, P(idx), ctr.data_ptr(),
                     ctr.data_ptr() + 8, N, C * H * H, C * OH * OH, s)
        q = torch.empty(N, C, OH, OH, device=DEV)
        _native.call("aimet_dwconv2d_forward", P(inp), P(w), P(b), P(q), N, C, H, H, OH, OH, K, stride, pad, dil, s)
        gq = torch.empty_like(q)
        _native.call("aimet_adaround_recon_grad_indexed", P(q), P(t_cache), P(idx), ctr.data_ptr(), P(gq), N, C,
                     OH * OH, None, act, s)
        gw_ref = torch.empty_like(w)
        _native.call("aimet_dwconv2d_grad_weight", P(inp), P(gq), P(gw_ref), P(ws), N, C, H, H, OH, OH, K, stride,
                     pad, dil, s)
        # fused
        ctr2 = torch.tensor([it, -1], dtype=torch.long, device=DEV)
        gw = torch.empty_like(w)
        _native.call("aimet_adaround_dw_step", P(x_cache), P(t_cache), P(idx), ctr2.data_ptr(), ctr2.data_ptr() + 8,
                     P(w), P(b), P(gw), P(ws), N, C, H, H, OH, OH, K, stride, pad, dil, act, s)
        assert torch.equal(gw.view(torch.int32), gw_ref.view(torch.int32)), it
        assert ctr2.tolist() == ctr.tolist() == [it, it + 1]
        assert bool(gw.abs().sum() > 0)


@pytest.mark.parametrize("N,Cin,Cout,HW,act,with_bias", [(32, 16, 96, 112 * 112, 2, False),
                                                          (32, 144, 24, 56 * 56, 0, True),
                                                          (32, 32, 192, 28 * 28, 2, True),
                                                          (7, 27, 32, 100, 1, False),
                                                          (5, 3, 5, 12, 2, True),
                                                          (4, 192, 32, 196, 0, False),
                                                          (32, 64, 384, 196, 2, True),
                                                          (6, 96, 576, 196, 1, False),
                                                          (3, 160, 200, 100, 0, True),
                                                          (4, 32, 2, 64 * 64, 0, True),
                                                          (4, 24, 1, 32 * 32, 1, False),
                                                          (4, 192, 3, 64, 0, False)])
def test_adaround_pw_step_vs_torch(N, Cin, Cout, HW, act, with_bias):
    """aimet_adaround_pw_step (a 1x1 layer's AdaRound iteration in one pass over the cached rows)
    == the fp32 torch ops it replaces (index_select, W @ x, the reconstruction-loss gradient, the
    weight gradient) to summation-order tolerance; deterministic; moves the iteration counter."""
    import ctypes
    from aimet_amd import _native
    g = torch.Generator(device=DEV).manual_seed(Cin * Cout + HW)
    rows = N + 3
    x_cache = torch.rand(rows, Cin, HW, device=DEV, generator=g)
    w = torch.randn(Cout, Cin, device=DEV, generator=g) / Cin ** 0.5
    b = torch.randn(Cout, device=DEV, generator=g) * 0.1 if with_bias else None
    t_cache = torch.randn(rows, Cout, HW, device=DEV, generator=g) * 0.5
    idx = torch.stack([torch.randperm(rows, device=DEV, generator=g)[:N] for _ in range(2)]).contiguous()
    it = 1
    xb, tb = x_cache[idx[it]].double(), t_cache[idx[it]].double()
    q = torch.einsum("oc,nch->noh", w.double(), xb) + (b.double()[None, :, None] if with_bias else 0)
    actf = {0: lambda v: v, 1: torch.relu, 2: lambda v: v.clamp(0, 6)}[act]
    mask = {0: lambda v: torch.ones_like(v), 1: lambda v: (v > 0).double(),
            2: lambda v: ((v > 0) & (v < 6)).double()}[act]
    gq = 2.0 / (N * HW) * (actf(q) - actf(tb)) * mask(q)
    gw_ref = torch.einsum("noh,nch->oc", gq, xb)
    n_ws = ctypes.c_int64()
    _native.call("aimet_adaround_pw_step_workspace", N, Cin, Cout, HW, ctypes.byref(n_ws))
    ws = torch.empty(n_ws.value, device=DEV)
    s = torch.cuda.current_stream().cuda_stream
    outs = []
    for use_ws in (True, False):
        ctr = torch.tensor([it, -1], dtype=torch.long, device=DEV)
        gw = torch.empty(Cout, Cin, device=DEV)
        _native.call("aimet_adaround_pw_step", x_cache.data_ptr(), t_cache.data_ptr(), idx.data_ptr(),
                     ctr.data_ptr(), ctr.data_ptr() + 8, w.data_ptr(), b.data_ptr() if with_bias else None,
                     gw.data_ptr(), ws.data_ptr() if use_ws else None, N, Cin, Cout, HW, act, s)
        assert ctr.tolist() == [it, it + 1]
        outs.append(gw)
    assert torch.equal(outs[0], outs[1])   # deterministic
    # fp32 sums over N * HW positions: the error is bounded by a small multiple of eps * sum |g x|
    bound = torch.einsum("noh,nch->oc", gq.abs(), xb.abs())
    err = (outs[0].double() - gw_ref).abs()
    assert bool((err <= 2e-5 * bound + 1e-12).all()), float((err / (bound + 1e-30)).max())


def test_adam_bias_correction_table_equals_in_kernel():
    """aimet_adaround_adam_bias_corrections' per-step table read by the Adam step gives the same
    alpha / moments / soft weight bit for bit as the bias corrections computed in the kernel, at
    steps across a 10k-iteration loop; the table equals ATen's 1 - beta^step (double, rounded to
    float; the second as its square root) to one float ulp."""
    import ctypes
    from aimet_amd import _native
    s = torch.cuda.current_stream().cuda_stream
    steps = 10000
    b1, b2 = 0.9, 0.999
    bc = torch.empty(steps, 2, device=DEV)
    _native.call("aimet_adaround_adam_bias_corrections", ctypes.c_double(b1), ctypes.c_double(b2), steps,
                 bc.data_ptr(), s)
    st = torch.arange(1, steps + 1, dtype=torch.float64)
    ref = torch.stack([(1 - b1 ** st).float(), (1 - b2 ** st).sqrt().float()], 1)
    ulp = torch.finfo(torch.float32).eps * ref.abs()
    assert bool(((bc.cpu() - ref).abs() <= ulp).all())
    g = torch.Generator(device=DEV).manual_seed(11)
    C, K = 24, 40
    w = torch.randn(C, K, device=DEV, generator=g) * 0.05
    d = (w.abs().amax(1) / 7).contiguous()
    o = torch.full((C,), -8.0, device=DEV)
    grad = torch.randn(C, K, device=DEV, generator=g) * 1e-3
    rb = torch.tensor([[0.01, 10.0, 9.0]] * steps, device=DEV)
    for step in (1, 2, 7, 100, 999, 5000, 10000):
        res = []
        for tab in (None, bc.data_ptr()):
            alpha = torch.randn(C, K, device=DEV, generator=torch.Generator(device=DEV).manual_seed(step))
            m = torch.full_like(alpha, 1e-4)
            v = torch.full_like(alpha, 1e-7)
            wq = torch.empty_like(alpha)
            ctr = torch.tensor([step - 1, step], dtype=torch.long, device=DEV)
            _native.call("aimet_adaround_backward_adam_parts", w.data_ptr(), alpha.data_ptr(), grad.data_ptr(), 1, 0,
                         m.data_ptr(), v.data_ptr(), 1, C, K, d.data_ptr(), o.data_ptr(), 4, rb.data_ptr(),
                         ctr.data_ptr() + 8, ctr.data_ptr(), ctypes.c_double(1e-3), ctypes.c_double(b1),
                         ctypes.c_double(b2), ctypes.c_double(1e-8), None, wq.data_ptr(), tab, s)
            res.append((alpha, m, v, wq))
        for a_, b_ in zip(*res):
            assert torch.equal(a_, b_), step


@pytest.mark.parametrize("layer", ["conv", "depthwise", "pointwise", "linear", "linear_noact", "conv_gelu"])
def test_adaround_fused_step_graph_equals_torch_adam_graph(layer):
    """The single-process loop with the batch draw and backward + Adam fused into two kernels
    (aimet_adaround_gather, aimet_adaround_backward_adam) follows the graph of torch ops (index_select
    x4, backward, grad accumulate, torch.optim.Adam(fused, capturable)): same batches, same
    gradients; the Adam first moment can differ from torch's fused kernel by 1 ulp in ~0.1 % of
    elements (profiles/r02/adam_probe.txt), so alpha agrees to fp32 tolerance after 80 steps."""
    from aimet_amd.adaround_optimizer import AdaroundHyperParameters, AdaroundOptimizer, conv_backend
    torch.manual_seed(4)
    if layer in ("conv", "conv_gelu"):
        mod, x = torch.nn.Conv2d(16, 24, 3, padding=1), torch.randn(96, 16, 10, 10)
    elif layer == "depthwise":
        mod, x = torch.nn.Conv2d(24, 24, 3, padding=1, groups=24), torch.randn(96, 24, 10, 10)
    elif layer == "pointwise":
        mod, x = torch.nn.Conv2d(24, 40, 1), torch.randn(96, 24, 10, 10)
    else:
        mod, x = torch.nn.Linear(40, 30), torch.randn(96, 40)
    # GELU has no fused reconstruction-gradient form: the target is gathered and autograd runs it
    act = None if layer == "linear_noact" else torch.nn.GELU() if layer == "conv_gelu" else torch.nn.ReLU()
    mod, x = mod.to(DEV), x.to(DEV)
    with torch.no_grad():
        out = mod(x) + 0.01 * torch.randn_like(mod(x))
    w = mod.weight.detach()
    d = (w.abs().flatten(1).amax(dim=1) / 7).contiguous()
    o = torch.full((w.shape[0],), -8.0, device=DEV)
    params = AdaroundHyperParameters(num_iterations=80, warm_start=0.25)
    res = {}
    for fused in (True, False):
        loss = torch.zeros(1, device=DEV)
        with conv_backend(mod):
            a = AdaroundOptimizer._optimize_graphed(mod, x, out, d, o, 4, 0, params, act,
                                                    torch.Generator().manual_seed(9), loss, fused_step=fused)
        res[fused] = (a.detach().clone(), loss.clone())
    torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(res[True][1], res[False][1], rtol=1e-4, atol=1e-7)
    assert float(res[True][1]) > 0


def test_adaround_optimizer_matches_reference_loop():
    """AdaroundOptimizer (fused soft-quant + rounding-loss kernels) follows the reference's loop
    (torch-op soft quantization + AdaroundLoss, adaround_optimizer.py:181-218) iteration for
    iteration: same Adam trajectory of alpha within fp32 tolerance, same hard rounding."""
    from aimet_amd.adaround import compute_beta, init_alpha
    from aimet_amd.adaround_optimizer import (AdaroundHyperParameters, AdaroundOptimizer, layer_forward,
                                              recon_loss)
    from oracle import torch_ref as T
    torch.manual_seed(3)
    conv = torch.nn.Conv2d(16, 24, 3, padding=1).to(DEV)
    inp = torch.randn(256, 16, 12, 12, device=DEV)
    with torch.no_grad():
        out = conv(inp) + 0.01 * torch.randn(256, 24, 12, 12, device=DEV)
    w = conv.weight.detach()
    d = (w.abs().amax(dim=(1, 2, 3)) / 127).contiguous()
    o = torch.full((24,), -128.0, device=DEV)
    params = AdaroundHyperParameters(num_iterations=120, warm_start=0.25)
    act = torch.nn.ReLU6()
    loss_eager = torch.zeros(1, device=DEV)
    a_ours = AdaroundOptimizer.optimize_rounding(conv, inp, out, d, o, 8, 0, params, act,
                                                 torch.Generator().manual_seed(5), loss_eager, use_graph=False)
    # the HIP-graph form (one captured iteration replayed): the same trajectory
    loss_graph = torch.zeros(1, device=DEV)
    a_graph = AdaroundOptimizer.optimize_rounding(conv, inp, out, d, o, 8, 0, params, act,
                                                  torch.Generator().manual_seed(5), loss_graph, use_graph=True)
    torch.testing.assert_close(a_graph.detach(), a_ours.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(loss_graph, loss_eager, rtol=1e-4, atol=1e-6)
    assert float(loss_graph) > 0
    # the reference loop
    a_ref = init_alpha(w, d.view(-1, 1, 1, 1))
    opt = torch.optim.Adam([a_ref])
    g = torch.Generator().manual_seed(5)
    for it in range(params.num_iterations):
        idx = torch.randperm(256, generator=g)[:32].to(DEV)
        x, target = inp.index_select(0, idx), out.index_select(0, idx)
        opt.zero_grad()
        qo = layer_forward(conv, x, T.adaround_forward(w, a_ref, d.view(-1, 1, 1, 1), o.view(-1, 1, 1, 1), 8))
        loss = recon_loss(act(qo), act(target))
        if it >= params.num_iterations * params.warm_start:
            beta = compute_beta(params.num_iterations, it, params.beta_range, params.warm_start)
            loss = loss + T.adaround_round_loss(a_ref, params.reg_param, beta)
        loss.backward()
        opt.step()
    torch.testing.assert_close(a_ours.detach(), a_ref.detach(), rtol=1e-3, atol=2e-4)
    hard_ours = AdaroundOptimizer.hard_rounded_weight(conv, a_ours, d, o, 8)
    hard_ref = T.adaround_forward(w, torch.where(a_ref.detach() >= 0, 100.0, -100.0), d.view(-1, 1, 1, 1),
                                  o.view(-1, 1, 1, 1), 8)
    # the hard rounding (AdaRound's integer output) is identical wherever alpha is farther from 0
    # than the alpha tolerance above: a flip is possible only for an alpha within it of 0
    decisive = a_ref.detach().abs() > 2e-4 + 1e-3 * a_ref.detach().abs()
    assert torch.equal(hard_ours[decisive], hard_ref[decisive])
    assert (hard_ours != hard_ref).float().mean() < 1e-3


def test_create_many_shared_state_lifetime():
    """aimet_tq_create_many: quantizers sharing one allocation behave like individually created
    ones, and destroying some of them (the slab is freed with the last) leaves the others intact."""
    import gc
    rng = np.random.default_rng(5)
    schemes = [QuantizationMode.QUANTIZATION_TF, QuantizationMode.QUANTIZATION_TF_ENHANCED,
               QuantizationMode.QUANTIZATION_PERCENTILE, QuantizationMode.QUANTIZATION_MSE,
               QuantizationMode.QUANTIZATION_ENTROPY] * 2
    xs = [gpu(rng.standard_normal(5000 + 17 * i).astype(np.float32) * (i + 1)) for i in range(len(schemes))]
    shared = [AimetTensorQuantizer(s) for s in schemes]
    shared[2].setPercentileValue(99.0)
    AimetTensorQuantizer.updateStatsMany(shared, xs)
    for i in (0, 3, 4, 8):
        shared[i] = None
    gc.collect()
    for i, (s, x) in enumerate(zip(schemes, xs)):
        if shared[i] is None:
            continue
        single = AimetTensorQuantizer(s)
        if i == 2:
            single.setPercentileValue(99.0)
        single.updateStats(x, True)
        shared[i].updateStats(x * 1.5, True)
        single.updateStats(x * 1.5, True)
        assert shared[i].getEncoding(8, False, False, False)[0] == single.getEncoding(8, False, False, False)[0], i
    shared = None
    gc.collect()
    torch.cuda.synchronize()


def test_reset_of_quantizers_bound_to_exchange_buffers():
    """Quantizers whose {-min, max} and counts live in the packed exchange buffers of the sharded
    path (aimet_amd.distributed, 8-B slots at any offset) reset in the batched reset and then
    recompute exactly what fresh quantizers compute."""
    from aimet_amd import distributed as D
    g = torch.Generator(device=DEV).manual_seed(23)
    TFE = QuantizationMode.QUANTIZATION_TF_ENHANCED
    tensors = [torch.relu(torch.randn(n, device=DEV, generator=g) * (i + 1)) for i, n in
               enumerate((1 << 16, 1001, 3 << 14, 77))]
    qs = [AimetTensorQuantizer(TFE) for _ in tensors]
    D.sharded_update_stats(qs, [t * 3 for t in tensors], fused=False)       # bound to packed buffers
    AimetTensorQuantizer.resetEncodingStatsMany(qs)
    D.sharded_update_stats(qs, tensors, fused=False)
    got = [e.to_tuple() for e, _ in AimetTensorQuantizer.getEncodings(qs, 8, False, False, False)]
    fresh = [AimetTensorQuantizer(TFE) for _ in tensors]
    for q, t in zip(fresh, tensors):
        q.updateStats(t, True)
    want = [e.to_tuple() for e, _ in AimetTensorQuantizer.getEncodings(fresh, 8, False, False, False)]
    assert got == want


@pytest.mark.parametrize("schemes", ["tfe", "mixed"])
def test_calibrate_native_call_equals_phased_path_with_reset(schemes, monkeypatch):
    """compute_encodings_resident's calibration plan and native calls (aimet_calibrate_launch, reset
    folded in; the activations' and the parameters' calls apart, and both in one call) ==
    the phase-by-phase path from Python (resetEncodingStatsMany + per-phase *_many launches + the
    two requests), on quantizers that already hold the previous batch's statistics; and a second
    reset + recompute of the same data == the first (nothing of the earlier batch survives)."""
    from aimet_amd import calibration
    from aimet_amd.calibration import compute_encodings_resident
    g = torch.Generator(device=DEV).manual_seed(21)
    M = QuantizationMode
    a_modes = [M.QUANTIZATION_TF_ENHANCED] * 4 if schemes == "tfe" else \
        [M.QUANTIZATION_TF, M.QUANTIZATION_TF_ENHANCED, M.QUANTIZATION_PERCENTILE, M.QUANTIZATION_MSE]
    p_modes = [M.QUANTIZATION_TF_ENHANCED] * 3 if schemes == "tfe" else \
        [M.QUANTIZATION_TF, M.QUANTIZATION_TF_ENHANCED, M.QUANTIZATION_MSE]

    def batch(scale):
        acts = [torch.relu(torch.randn(n, device=DEV, generator=g) * scale * (1 + i)) for i, n in
                enumerate((1 << 20, 3001, 77777, 1 << 18))]
        params = [torch.randn(c, k, device=DEV, generator=g) * 0.05 * scale
                  for c, k in ((64, 27), (128, 576), (10, 2048))]
        return acts, params

    from aimet_amd import tensor_quantizer
    old, new_ = batch(3.0), batch(1.0)
    results = []
    # the calibration plan, two native calls (activations, then parameters), one native call, the
    # phased path
    for sched, split in (("plan", True), ("native", True), ("native", False), ("phased", False)):
        monkeypatch.setattr(calibration, "_SCHEDULE", sched)
        monkeypatch.setattr(tensor_quantizer, "_CAL_SPLIT", split)
        aq = [AimetTensorQuantizer(m) for m in a_modes]
        pq = [AimetTensorQuantizer(m, num_channels=p.shape[0]) for m, p in zip(p_modes, new_[1])]
        compute_encodings_resident(aq, old[0], pq, old[1])                 # earlier statistics
        r1 = compute_encodings_resident(aq, new_[0], pq, new_[1], reset=True)
        r2 = compute_encodings_resident(aq, new_[0], pq, new_[1], reset=True)
        flat = lambda r: ([e.to_tuple() for e, _ in r[0]],
                          [[x.to_tuple() for x in (es if isinstance(es, list) else [es])] for es, _ in r[1]])
        assert flat(r1) == flat(r2)
        results.append(flat(r1))
    assert results[0] == results[1] == results[2] == results[3]
    # and == fresh quantizers fed only the new batch
    fa = [AimetTensorQuantizer(m) for m in a_modes]
    fp = [AimetTensorQuantizer(m, num_channels=p.shape[0]) for m, p in zip(p_modes, new_[1])]
    monkeypatch.setattr(calibration, "_SCHEDULE", "plan")
    fresh = compute_encodings_resident(fa, new_[0], fp, new_[1])
    assert ([e.to_tuple() for e, _ in fresh[0]]) == results[0][0]


def test_calibrate_two_calls_bad_parameter_is_refused_before_any_launch():
    """A parameter the two-call form refuses (float16) raises TypeError before anything is
    launched: the activation quantizers keep the statistics of their earlier batch (their encodings
    equal those of quantizers that never saw the refused call), and the same quantizers then
    calibrate normally, equal to fresh ones."""
    from aimet_amd import calibration
    from aimet_amd.calibration import compute_encodings_resident
    g = torch.Generator(device=DEV).manual_seed(4)
    TFE = QuantizationMode.QUANTIZATION_TF_ENHANCED
    acts = [torch.randn(n, device=DEV, generator=g) for n in (1 << 20, 4099)]
    acts2 = [a * 3 + 1 for a in acts]
    params = [torch.randn(16, 75, device=DEV, generator=g) * 0.1]
    aq = [AimetTensorQuantizer(TFE) for _ in acts]
    pq = [AimetTensorQuantizer(TFE, num_channels=16)]
    before = compute_encodings_resident(aq, acts, pq, params, reset=True)
    dev = torch.device(DEV, torch.cuda.current_device())
    side = calibration._side_stream(dev)
    with pytest.raises(TypeError):
        AimetTensorQuantizer.calibrateResidentAsync(aq, acts2, pq, [params[0].half()], reset=True,
                                                    main_stream=torch.cuda.current_stream(dev), side_stream=side)
    untouched = AimetTensorQuantizer.getEncodings(aq, 8, False, False, False)
    assert [e.to_tuple() for e, _ in untouched] == [e.to_tuple() for e, _ in before[0]]
    got = compute_encodings_resident(aq, acts2, pq, params, reset=True)
    fa, fp = [AimetTensorQuantizer(TFE) for _ in acts], [AimetTensorQuantizer(TFE, num_channels=16)]
    want = compute_encodings_resident(fa, acts2, fp, params)
    assert [e.to_tuple() for e, _ in got[0]] == [e.to_tuple() for e, _ in want[0]]
    assert [x.to_tuple() for x in got[1][0][0]] == [x.to_tuple() for x in want[1][0][0]]


@pytest.mark.parametrize("split", [True, False])
def test_calibrate_non_contiguous_parameters_and_activations(monkeypatch, split):
    """Non-contiguous inputs (a transposed weight, a channels_last conv weight, a strided
    activation) are copied on the stream that consumes them: the encodings equal those of the
    contiguous tensors, in the two-call and the one-call form, with torch's current stream a
    different one from the call's main stream."""
    from aimet_amd import calibration, tensor_quantizer
    monkeypatch.setattr(tensor_quantizer, "_CAL_SPLIT", split)
    g = torch.Generator(device=DEV).manual_seed(9)
    TFE = QuantizationMode.QUANTIZATION_TF_ENHANCED
    w_t = (torch.randn(300, 64, device=DEV, generator=g) * 0.1).t()          # [64, 300], not contiguous
    w_cl = (torch.randn(96, 48, 3, 3, device=DEV, generator=g) * 0.05).to(memory_format=torch.channels_last)
    act = torch.randn(4096, 513, device=DEV, generator=g)[:, :512]           # strided rows
    assert not (w_t.is_contiguous() or w_cl.is_contiguous() or act.is_contiguous())
    dev = torch.device(DEV, torch.cuda.current_device())
    main = torch.cuda.Stream(dev)
    side = calibration._side_stream(dev)

    def run(acts, params):
        aq = [AimetTensorQuantizer(TFE) for _ in acts]
        pq = [AimetTensorQuantizer(TFE, num_channels=p.shape[0]) for p in params]
        main.wait_stream(torch.cuda.current_stream(dev))
        a_p, p_p, keep = AimetTensorQuantizer.calibrateResidentAsync(aq, acts, pq, params, reset=True,
                                                                      main_stream=main, side_stream=side)
        res = a_p.result(), p_p.result()
        torch.cuda.current_stream(dev).wait_stream(main)
        return [e.to_tuple() for e, _ in res[0]], [[x.to_tuple() for x in es] for es, _ in res[1]]

    # the tensors' values are written on the current stream right before the call
    got = run([act], [w_t, w_cl])
    want = run([act.contiguous()], [w_t.contiguous(), w_cl.contiguous()])
    assert got == want


@pytest.mark.parametrize("schemes", ["tfe", "mixed"])
def test_calibration_plan_equals_per_quantizer_updates(schemes):
    """aimet_amd.calibration.CalibrationPlan (every job table prepared once; the TF-E searches write
    straight into the plan's pinned blocks; the parameters' light reset): two batches without a
    reset == each quantizer's own updateStats over both batches; then run(reset=True) on a third
    batch, twice, == fresh quantizers fed only that batch (nothing of the earlier batches survives,
    the PDFs the light reset left in place included); a second launch before the first request is
    finished is refused."""
    from aimet_amd.calibration import CalibrationPlan
    g = torch.Generator(device=DEV).manual_seed(31)
    M = QuantizationMode
    a_modes = [M.QUANTIZATION_TF_ENHANCED] * 3 if schemes == "tfe" else \
        [M.QUANTIZATION_TF, M.QUANTIZATION_TF_ENHANCED, M.QUANTIZATION_PERCENTILE, M.QUANTIZATION_MSE,
         M.QUANTIZATION_ENTROPY]
    p_modes = [M.QUANTIZATION_TF_ENHANCED] * 2 if schemes == "tfe" else \
        [M.QUANTIZATION_TF, M.QUANTIZATION_TF_ENHANCED, M.QUANTIZATION_MSE, M.QUANTIZATION_PERCENTILE,
         M.QUANTIZATION_ENTROPY]
    sizes = [1 << 20, 3001, 77777, 1 << 18, 4099][:len(a_modes)]
    shapes = [(64, 27), (128, 576), (10, 2048), (33, 5), (17, 300)][:len(p_modes)]

    def batch(scale):
        acts = [torch.relu(torch.randn(n, device=DEV, generator=g) * scale * (1 + i)) - 0.1 * i
                for i, n in enumerate(sizes)]
        params = [torch.randn(c, k, device=DEV, generator=g) * 0.05 * scale for c, k in shapes]
        return acts, params

    def flat(a_res, p_res):
        return ([e.to_tuple() for e, _ in a_res],
                [[x.to_tuple() for x in (es if isinstance(es, list) else [es])] for es, _ in p_res])

    def individual(batches):
        aq = [AimetTensorQuantizer(m) for m in a_modes]
        pq = [AimetTensorQuantizer(m, num_channels=c) for m, (c, _) in zip(p_modes, shapes)]
        for acts, params in batches:
            for q, t in zip(aq, acts):
                q.updateStats(t, True)
            for q, t in zip(pq, params):
                q.updateStatsPerChannel(t, 0, True)
        return (flat([q.getEncoding(8, False, False, False) for q in aq],
                     [q.getEncoding(8, True, False, False) for q in pq]))

    b1, b2, b3 = batch(2.0), batch(1.0), batch(0.5)
    aq = [AimetTensorQuantizer(m) for m in a_modes]
    pq = [AimetTensorQuantizer(m, num_channels=c) for m, (c, _) in zip(p_modes, shapes)]
    bufs = [t.clone() for t in b1[0]], [t.clone() for t in b1[1]]
    plan = CalibrationPlan(aq, bufs[0], pq, bufs[1])
    plan.run()
    for t, s in zip(bufs[0] + bufs[1], b2[0] + b2[1]):
        t.copy_(s)
    assert flat(*plan.run()) == individual([b1, b2])
    for t, s in zip(bufs[0] + bufs[1], b3[0] + b3[1]):
        t.copy_(s)
    want = individual([b3])
    assert flat(*plan.run(reset=True)) == want
    assert flat(*plan.run(reset=True)) == want
    a_p, p_p = plan.launch(reset=True)
    with pytest.raises(ValueError):
        plan.launch(reset=True)
    assert flat(a_p.result(), p_p.result()) == want
    plan.close()


def test_compute_encodings_resident_equals_individual():
    """aimet_amd.calibration.compute_encodings_resident (batched activation statistics, parameter
    statistics + searches on a second stream) == updateStats / getEncoding quantizer by quantizer."""
    from aimet_amd.calibration import compute_encodings_resident
    g = torch.Generator(device=DEV).manual_seed(14)
    acts = [torch.relu(torch.randn(n, device=DEV, generator=g) * (1 + i)) for i, n in
            enumerate((1 << 20, 3000, 77777, 1 << 18))]
    params = [torch.randn(c, k, device=DEV, generator=g) * 0.05 for c, k in ((64, 27), (128, 576), (10, 2048))]
    TFE = QuantizationMode.QUANTIZATION_TF_ENHANCED
    aq = [AimetTensorQuantizer(TFE) for _ in acts]
    pq = [AimetTensorQuantizer(TFE, num_channels=p.shape[0]) for p in params]
    a_res, p_res = compute_encodings_resident(aq, acts, pq, params)
    for t, (e, v) in zip(acts, a_res):
        q = AimetTensorQuantizer(TFE)
        q.updateStats(t, True)
        e1, v1 = q.getEncoding(8, False, False, False)
        assert v and v1 and e.to_tuple() == e1.to_tuple()
    for p, (es, v) in zip(params, p_res):
        q = AimetTensorQuantizer(TFE, num_channels=p.shape[0])
        q.updateStatsPerChannel(p, 0, True)
        e1, v1 = q.getEncoding(8, True, False, False)
        assert v and v1 and [e.to_tuple() for e in es] == [e.to_tuple() for e in e1]


def test_learned_grid_gate_ranges_equals_single_range_gate():
    """aimet_lg_gate_ranges (a wrapper's ranges in one launch) == aimet_lg_gate_range per range,
    bit for bit (NaN and signed-zero ranges, ragged channel counts, more than 8 ranges)."""
    from aimet_amd.learned_grid import (set_encoding_min_max_gating_threshold,
                                        set_encoding_min_max_gating_threshold_many)
    g = torch.Generator(device=DEV).manual_seed(47)
    sizes = [1, 5000, 3, 4096, 257, 1, 64, 9, 1000, 2]
    ranges = []
    for k in sizes:
        mn, mx = torch.randn(k, device=DEV, generator=g), torch.randn(k, device=DEV, generator=g)
        if k >= 6:
            mn[:6] = torch.tensor([float("nan"), 0.0, -0.0, 1e-30, -1e-6, 3.0], device=DEV)
            mx[:6] = torch.tensor([-0.0, float("nan"), 0.0, -1e-30, 2e-6, -3.0], device=DEV)
        ranges.append((mn, mx))
    expect = [(a.clone(), b.clone()) for a, b in ranges]
    for a, b in expect:
        set_encoding_min_max_gating_threshold(a, b)
    v0 = [a._version for a, _ in ranges]
    set_encoding_min_max_gating_threshold_many(ranges)
    for (a, b), (ea, eb), v in zip(ranges, expect, v0):
        assert _same_bits_or_nan(a, ea) and _same_bits_or_nan(b, eb)
        assert a._version > v


@pytest.mark.parametrize("outer,C,K", [(5, 3, 300), (2, 9, 1024), (3, 2, 5000), (1, 1, 20000)])
@pytest.mark.parametrize("out_dtype", [0, 2])
def test_learned_grid_forward_chunking_is_exact(outer, C, K, out_dtype):
    """The fp32-input forward splits passes of more than 2^30 elements into sub-problems (whole
    rows, channel ranges of a row, pieces of a channel). With the bound lowered to 4096 elements
    (aimet_lg_set_chunk_limit) each split mode runs on a small tensor: y, delta, offset and the
    saved range == the unsplit pass, bit for bit (float32 and the bf16-cast output)."""
    from aimet_amd import _native
    g = torch.Generator(device=DEV).manual_seed(outer * 7 + C)
    x = torch.randn(outer, C, K, device=DEV, generator=g) * 0.7
    emax = torch.rand(C, device=DEV, generator=g) + 0.5
    emin = -emax * 0.6
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.float32 if out_dtype == 0 else torch.bfloat16

    def run():
        y = torch.empty(x.shape, dtype=dt, device=DEV)
        enc = torch.full((4, C), float("nan"), device=DEV)
        _native.call("aimet_lg_forward_range", x.data_ptr(), y.data_ptr(), outer, C, K, out_dtype, emin.data_ptr(),
                     emax.data_ptr(), 4, 0, 0, 0, enc[0].data_ptr(), enc[1].data_ptr(), enc[2].data_ptr(), s)
        return y, enc
    y_ref, enc_ref = run()
    try:
        _native.call("aimet_lg_set_chunk_limit", 4096)
        y, enc = run()
    finally:
        _native.call("aimet_lg_set_chunk_limit", 0)
    assert torch.equal(y.view(torch.int16 if out_dtype else torch.int32),
                       y_ref.view(torch.int16 if out_dtype else torch.int32))
    assert torch.equal(enc, enc_ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_learned_grid_past_2_31_elements(dtype):
    """A per-tensor learned-grid forward + backward over 2^31 + 4100 elements (an activation the
    size of Llama-3-8B's logits at micro-batch 2 x seq 8192; the reference's torch ops have no
    element limit): y and grad_x bit-exact vs the reference's torch ops (oracle/torch_ref.py) on
    slices at the start, across 2^31 and at the ragged end; the encoding gradients vs the torch
    ops over the whole tensor (rtol 1e-4: fp32 summation order)."""
    from aimet_amd.learned_grid import LearnedGridQuantizeDequantize
    from oracle import torch_ref as T
    n = (1 << 31) + 4100
    g = torch.Generator(device=DEV).manual_seed(31)
    x = torch.randn(n, device=DEV, generator=g, dtype=torch.float32).to(dtype)
    grad = torch.randn(n, device=DEV, generator=g, dtype=torch.float32).to(dtype)
    emin = torch.tensor([-2.9], device=DEV, requires_grad=True)
    emax = torch.tensor([3.3], device=DEV, requires_grad=True)
    xt = x.requires_grad_(True)
    y = LearnedGridQuantizeDequantize.apply(xt, emin, emax, 8)
    y.backward(grad)
    gx = xt.grad
    for a, b in ((0, 1 << 20), ((1 << 31) - (1 << 20), (1 << 31) + (1 << 20)), (n - (1 << 20), n)):
        xs = x[a:b].detach().float()
        want = T.lg_forward(xs, emin.detach(), emax.detach(), 8)[0].to(dtype)
        got = LearnedGridQuantizeDequantize.apply(x[a:b].detach(), emin.detach(), emax.detach(), 8)
        assert torch.equal(got.view(torch.int16 if dtype != torch.float32 else torch.int32),
                           want.view(torch.int16 if dtype != torch.float32 else torch.int32)), (a, b)
        wgx = T.lg_gradients(xs, grad[a:b].float(), emin.detach(), emax.detach(), 8)[0].to(dtype)
        assert torch.equal(gx[a:b], wgx), (a, b)
    del gx
    _, gmin, gmax = T.lg_gradients(x.detach().float(), grad.float(), emin.detach(), emax.detach(), 8)
    torch.testing.assert_close(emin.grad, gmin, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(emax.grad, gmax, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("scheme", ["TF_ENHANCED", "MSE", "ENTROPY", "TF"])
def test_get_encodings_results_independent_across_calls(scheme):
    """getEncodings' per-channel TfEncoding objects are views into the call's own result block,
    built while the searches run (tensor_quantizer.PendingEncodings): a later call, on other
    statistics, leaves an earlier call's objects as they were; every channel equals its own
    getEncoding."""
    mode = getattr(QuantizationMode, "QUANTIZATION_" + scheme)
    g = torch.Generator(device=DEV).manual_seed(31)
    shapes = [(16, 40), (1, 300), (7, 9)]
    qs = [AimetTensorQuantizer(mode, num_channels=s[0]) for s in shapes]
    ws = [torch.randn(s, device=DEV, generator=g) * 0.1 for s in shapes]
    AimetTensorQuantizer.updateStatsPerChannelMany(qs, ws)
    first = AimetTensorQuantizer.getEncodings(qs, 8, True, False, False)
    snap = [[(e.min, e.max, e.delta, e.offset, e.bw) for e in (encs if isinstance(encs, list) else [encs])]
            for encs, _ in first]
    # other statistics, a second batched call
    qs2 = [AimetTensorQuantizer(mode, num_channels=s[0]) for s in shapes]
    AimetTensorQuantizer.updateStatsPerChannelMany(qs2, [w * 3 + 0.05 for w in ws])
    second = AimetTensorQuantizer.getEncodings(qs2, 8, False, False, False)
    again = [[(e.min, e.max, e.delta, e.offset, e.bw) for e in (encs if isinstance(encs, list) else [encs])]
             for encs, _ in first]
    assert again == snap
    for q, (encs, valid) in zip(qs2, second):
        assert valid
        one, _ = q.getEncoding(8, False, False, False)
        encs = encs if isinstance(encs, list) else [encs]
        one = one if isinstance(one, list) else [one]
        assert [(e.min, e.max, e.delta, e.offset, e.bw) for e in encs] == \
            [(e.min, e.max, e.delta, e.offset, e.bw) for e in one]
