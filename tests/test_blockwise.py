"""Blockwise (broadcast) QDQ, LPBQ encodings and the ONNX QcQuantizeOp.

Reference: quantizeDequantizeBroadcast (trim_functions.cpp:633-687, trim_functions.cu:96-122),
BroadcastShapeInfo / copyToContiguousBlockLayout (onnx/src/QuantizeDequantizeUtils.cpp:64-213),
QcQuantizeOp::computeImpl + AimetOpUtils.h:101-330, lpbq_utils.py.

Pinning: golden_broadcast.npz holds the reference C++ quantizeDequantizeBroadcastCpu outputs
(make_golden.py); BroadcastShapeInfo and the block permutation (onnx sources, which need
onnxruntime headers and so are not compiled here) are pinned by the KATs of
onnx/test/TestOnnxTensorOps.cpp; the op and LPBQ by the KATs of onnx/test/python/test_qc_quantize_op.py.
"""
import ctypes

import numpy as np
import pytest

from conftest import bits, gpu_available
from oracle import oracle as O

gpu = pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")


@pytest.fixture(scope="module")
def golden_broadcast(golden_dir):
    import os
    return dict(np.load(os.path.join(golden_dir, "golden_broadcast.npz")))


def _cases(g):
    for i in range(int(g["count"])):
        ch, ba, bs = (int(v) for v in g["b%d_cfg" % i])
        yield dict(shape=tuple(int(v) for v in g["b%d_shape" % i]), ch=ch, ba=ba, bs=bs, x=g["b%d_x" % i],
                   encs=g["b%d_encs" % i], y=g["b%d_y" % i])


# TestOnnxTensorOps.cpp:298-415: (shape, channel axis, block axis, block size) ->
# (numEncodings, tensor strides, encoding strides, hasContiguousBlocks)
SHAPE_KATS = [
    (((8, 12, 5, 2), 0, 1, 3), (32, [120, 30, 10, 2, 1], [4, 1, 0, 0, 0], True)),
    (((10, 4, 10), 1, 0, 2), (20, [80, 40, 10, 1], [4, 0, 1, 0], False)),
    (((4, 2, 2), 2, 0, 2), (4, [8, 4, 2, 1], [2, 0, 0, 1], False)),
]

# TestOnnxTensorOps.cpp:167-296 TensorBlockPermute{,2,3}
_IN16 = np.arange(1, 17, dtype=np.float32)
_P2 = np.array([[[[k + 2.0 * i for _m in range(4)] for k in range(2)] for _j in range(2)] for i in range(4)],
               np.float32).ravel()
PERMUTE_KATS = [
    (_IN16, ((4, 2, 2), 2, 0, 2), [1, 3, 5, 7, 2, 4, 6, 8, 9, 11, 13, 15, 10, 12, 14, 16]),
    (_P2, ((4, 2, 8), 0, 2, 4), [i // 8 for i in range(64)]),
    (_IN16, ((4, 2, 2), 1, -1, 0), [1, 2, 5, 6, 9, 10, 13, 14, 3, 4, 7, 8, 11, 12, 15, 16]),
]


def _delta_offset(mn, mx, bw, sym=False, strict=False):
    """aimet_common/quantsim.py:123-152 calculate_delta_offset (the KATs' create_encoding)."""
    steps = 2 ** bw - 1
    if sym and strict:
        steps -= 1
    mn, mx = min(mn, 0.0), max(mx, 0.0)
    mx = max(mx, mn + 1e-5)
    if sym and mn < 0:
        pos = np.floor(steps / 2)
        return mx / pos, -pos - (0 if strict else 1)
    d = (mx - mn) / steps
    return d, round(mn / d)


# test_qc_quantize_op.py:536-641 blockwise_qdq_test_{1,2,3}
BLOCKWISE_KATS = [
    dict(shape=(2, 3, 4), block_axis=0, block_size=1, channel_axis=1,
         min=[0, 0, 0, -2, -2.5, 0], max=[255. * 0.25, 255.0, 127.5, 508., 245. * 0.25, 2550.],
         x=[0.126, 10.4, -12.3, 10000] * 6,
         y=[0.25, 10.5, 0, 63.75, 0., 10., 0., 255., 0., 10.5, 0., 127.5, 0., 10., -2., 508.,
            0.25, 10.5, -2.5, 61.25, 0., 10., 0, 2550.]),
    dict(shape=(4, 2, 2), block_axis=0, block_size=2, channel_axis=2,
         min=[-64.0, -128.0, -256.0, -512.0], max=[63.5, 127.0, 254.0, 508.0],
         x=[-125.1, -125.1, 48.3, 48.3, 68.3, 68.3, -3.1, -3.1] * 2,
         y=[-64.0, -125.0, 48.5, 48.0, 63.5, 68.0, -3.0, -3.0, -126.0, -124.0, 48.0, 48.0, 68.0, 68.0, -4.0, -4.0]),
    dict(shape=(4, 4), block_axis=1, block_size=2, channel_axis=0,
         min=[-1.28, -12.8, -128, -1280, 0, 0, 0, 0], max=[1.27, 12.7, 127, 1270, 2.55, 25.5, 255, 2550],
         x=[40.23, .0321, -40.23, -.0321, 23.44, -2.3111, 23.44, -2.3111,
            -1000.1, 334, 23.1111, -23.1111, 23.1111, -23.1111, -1, 100000],
         y=[1.27, .03, -12.8, 0.0, 23, -2, 20., 0, 0, 2.55, 23.1, 0., 23, 0., 0, 2550]),
]


def _kat_encodings(k):
    out = []
    for mn, mx in zip(k["min"], k["max"]):
        d, o = _delta_offset(mn, mx, 8)
        out.append((mn, mx, d, o))
    return np.array(out, dtype=np.float32)


# ---- CPU ------------------------------------------------------------------------------------------
def test_broadcast_shape_info_kats():
    """Oracle restatement and the product's host BroadcastShapeInfo vs TestOnnxTensorOps.cpp."""
    from aimet_amd.onnx_op import BroadcastShapeInfo
    for (shape, ch, ba, bs), (nenc, tstr, estr, contig) in SHAPE_KATS:
        o = O.broadcast_shape_info(shape, ch, ba, bs)
        assert (o["num_encodings"], o["tensor_strides"], o["encoding_strides"], o["contiguous_blocks"]) == \
            (nenc, tstr, estr, contig)
        p = BroadcastShapeInfo(shape, ch, ba, bs)
        assert (p.numEncodings, p.tensorStrides, p.encodingStrides, p.hasContiguousBlocks()) == \
            (nenc, tstr, estr, contig)
        assert p.tensorShape == o["tensor_shape"] and p.encodingShape == o["encoding_shape"]
    for shape, ch, ba, bs in [((3, 5, 7), -1, 2, 7), ((6, 2), 1, 0, 2), ((5, 12, 4), 2, 1, 4), ((7,), 0, -1, 0)]:
        o = O.broadcast_shape_info(shape, ch, ba, bs)
        p = BroadcastShapeInfo(shape, ch, ba, bs)
        assert (p.tensorShape, p.encodingShape, p.encodingStrides, p.numEncodings, p.hasContiguousBlocks()) == \
            (o["tensor_shape"], o["encoding_shape"], o["encoding_strides"], o["num_encodings"],
             o["contiguous_blocks"])
    with pytest.raises(RuntimeError, match="evenly divisible"):
        BroadcastShapeInfo((4, 6), 0, 1, 4)


def test_oracle_block_permute_kats():
    for x, (shape, ch, ba, bs), want in PERMUTE_KATS:
        info = O.broadcast_shape_info(shape, ch, ba, bs)
        np.testing.assert_array_equal(O.copy_to_contiguous_block_layout(x, info), np.array(want, np.float32))


def test_oracle_broadcast_golden(golden_broadcast):
    for c in _cases(golden_broadcast):
        info = O.broadcast_shape_info(c["shape"], c["ch"], c["ba"], c["bs"])
        f = c["encs"][:, :4].astype(np.float32)
        y = O.qdq_broadcast(c["x"], info["tensor_strides"], info["encoding_strides"], f[:, 0], f[:, 1], f[:, 2],
                            f[:, 3])
        np.testing.assert_array_equal(bits(y), bits(c["y"]), err_msg=str(c["shape"]))


def test_oracle_blockwise_qdq_kats():
    for k in BLOCKWISE_KATS:
        info = O.broadcast_shape_info(k["shape"], k["channel_axis"], k["block_axis"], k["block_size"])
        e = _kat_encodings(k)
        y = O.qdq_broadcast(np.array(k["x"], np.float32), info["tensor_strides"], info["encoding_strides"],
                            e[:, 0], e[:, 1], e[:, 2], e[:, 3])
        np.testing.assert_allclose(y, np.array(k["y"], np.float32), rtol=1e-5, atol=1e-8)


@pytest.mark.ref
def test_oracle_broadcast_vs_compiled_reference_random():
    from oracle import ref as R
    if not R.available():
        pytest.skip("reference not present")
    rng = np.random.default_rng(31)
    for shape, ch, ba, bs in [((6, 8, 5), 1, 0, 3), ((9, 16), 0, 1, 4), ((4, 3, 10), 2, 0, 2), ((12, 12), 1, 0, 6)]:
        info = O.broadcast_shape_info(shape, ch, ba, bs)
        E = info["num_encodings"]
        x = (rng.standard_normal(int(np.prod(shape))) * 3).astype(np.float32)
        mn = -rng.uniform(0.5, 2, E).astype(np.float32)
        mx = rng.uniform(0.5, 2, E).astype(np.float32)
        d = ((mx - mn) / 255).astype(np.float32)
        o = np.round(mn / d).astype(np.float32)
        args = (info["tensor_strides"], info["encoding_strides"], mn, mx, d, o)
        np.testing.assert_array_equal(bits(O.qdq_broadcast(x, *args)), bits(R.qdq_broadcast(x, *args)))


def test_lpbq_kats():
    """test_qc_quantize_op.py:902-1000 TestLPBQOp (encoding side)."""
    from aimet_amd import lpbq
    scale = np.asarray([[1.6, 1.1222, .00001], [16, 2.56, 4.9]], np.float32)
    offset = np.ones_like(scale) * -8
    encs = lpbq.scale_offset_arrays_to_encodings(scale, offset, 4)
    shape, grouping = lpbq.lpbq_encoding_shape((2, 9), 0, 1, 3)
    assert shape == [2, 3] and grouping == [1, -1]
    out = lpbq.compress_encoding_scales(encs, shape, grouping, scale_bitwidth=8 - 4)
    s, o = lpbq.encodings_to_scale_offset_arrays(out, (2, 3))
    np.testing.assert_allclose(s, [[1.6, 1.1, .1], [16, 3, 5]], rtol=1e-5)
    np.testing.assert_allclose(o, offset)
    q, per_block = lpbq.grouped_dynamic_quantize(s, grouping, 4)
    assert q.flatten().tolist() == [16, 11, 1, 16, 3, 5]
    np.testing.assert_allclose(per_block.flatten(), [1.6 / 16, 16 / 16], rtol=1e-6)


# ---- GPU ------------------------------------------------------------------------------------------
def _encs_from(arr):
    from aimet_amd.libpymo import TfEncoding
    out = []
    for r in arr:
        e = TfEncoding()
        e.min, e.max, e.delta, e.offset = (float(v) for v in r[:4])
        e.bw = int(r[4]) if len(r) > 4 else 8
        out.append(e)
    return out


@pytest.mark.gpu
@gpu
def test_broadcast_qdq_golden(golden_broadcast):
    import torch
    from aimet_amd.onnx_op import BroadcastShapeInfo, quantize_dequantize_broadcast
    for c in _cases(golden_broadcast):
        info = BroadcastShapeInfo(c["shape"], c["ch"], c["ba"], c["bs"])
        x = torch.from_numpy(c["x"]).cuda()
        y = quantize_dequantize_broadcast(x, info, _encs_from(c["encs"])).cpu().numpy()
        np.testing.assert_array_equal(bits(y), bits(c["y"]), err_msg=str(c["shape"]))
    for k in BLOCKWISE_KATS:
        info = BroadcastShapeInfo(k["shape"], k["channel_axis"], k["block_axis"], k["block_size"])
        y = quantize_dequantize_broadcast(torch.tensor(k["x"], dtype=torch.float32).cuda(), info,
                                          _encs_from(_kat_encodings(k)))
        np.testing.assert_allclose(y.cpu().numpy(), np.array(k["y"], np.float32), rtol=1e-5, atol=1e-8)


@pytest.mark.gpu
@gpu
def test_broadcast_qdq_large_vs_oracle():
    """The vectorised path (innermost run % 4 == 0) and the scalar path on LPBQ-sized weights."""
    import torch
    from aimet_amd.onnx_op import BroadcastShapeInfo, quantize_dequantize_broadcast
    rng = np.random.default_rng(4)
    for shape, ch, ba, bs in [((1024, 2048), 0, 1, 64), ((2048, 768), 1, 0, 32), ((96, 130, 3, 3), 0, 1, 10),
                              ((333, 1001), 0, 1, 7)]:
        info = BroadcastShapeInfo(shape, ch, ba, bs)
        E = info.numEncodings
        x = (rng.standard_normal(int(np.prod(shape))) * 0.05).astype(np.float32)
        mx = rng.uniform(0.01, 0.2, E).astype(np.float32)
        d = (mx / 7).astype(np.float32)
        tab = np.stack([-8 * d, mx, d, np.full(E, -8, np.float32)], 1)
        y = quantize_dequantize_broadcast(torch.from_numpy(x).cuda(), info, _encs_from(tab)).cpu().numpy()
        want = O.qdq_broadcast(x, info.tensorStrides, info.encodingStrides, tab[:, 0], tab[:, 1], tab[:, 2], tab[:, 3])
        np.testing.assert_array_equal(bits(y), bits(want), err_msg=str(shape))
        # the same through the C-ABI with encoding arrays that are not 16-B aligned (gather path)
        from aimet_amd import _native
        buf = torch.zeros(4 * E + 1, device="cuda")
        arrs = [buf[1 + k * E: 1 + (k + 1) * E] for k in range(4)]
        for k in range(4):
            arrs[k].copy_(torch.from_numpy(np.ascontiguousarray(tab[:, k])))
        xt, yt = torch.from_numpy(x).cuda(), torch.empty(x.size, device="cuda")
        nd = info.numDims
        _native.call("aimet_qdq_broadcast", xt.data_ptr(), yt.data_ptr(), x.size, nd,
                     (ctypes.c_int64 * nd)(*info.tensorStrides), (ctypes.c_int64 * nd)(*info.encodingStrides),
                     *[a.data_ptr() for a in arrs], torch.cuda.current_stream().cuda_stream)
        np.testing.assert_array_equal(bits(yt.cpu().numpy()), bits(want), err_msg=str(shape))


@pytest.mark.gpu
@gpu
def test_broadcast_qdq_rounding_ties_vs_oracle():
    """Blockwise QDQ with a per-vector reciprocal (contiguous blocks) and per-column reciprocals
    (strided blocks): dyadic deltas and inputs on exact half-integer quotients (the exact-division
    fallback), zero and non-zero offsets, signed zeros, NaN / inf inputs; bit-exact vs the oracle."""
    import torch
    from aimet_amd.onnx_op import BroadcastShapeInfo, quantize_dequantize_broadcast
    rng = np.random.default_rng(9)
    for shape, ch, ba, bs in [((256, 512), 0, 1, 64), ((512, 256), 1, 0, 32)]:
        info = BroadcastShapeInfo(shape, ch, ba, bs)
        E = info.numEncodings
        d = (2.0 ** rng.integers(-12, 2, E)).astype(np.float32)
        off = rng.choice(np.array([-8, 0, -0.0, -3, -128], np.float32), E)
        steps = rng.choice(np.array([15, 255], np.float32), E)
        tab = np.stack([off * d, (off + steps) * d, d, off], 1).astype(np.float32)
        n = int(np.prod(shape))
        # each element's encoding index: a QDQ with min = max = index, delta 1, offset 0
        ar = np.arange(E, dtype=np.float32)
        eidx = O.qdq_broadcast(np.zeros(n, np.float32), info.tensorStrides, info.encodingStrides, ar, ar,
                               np.ones(E, np.float32), np.zeros(E, np.float32)).astype(np.int64)
        # multiples of delta/2 of every element's own encoding: exact half-integer quotients
        x = (rng.integers(-600, 600, n) * 0.5 * d[eidx]).astype(np.float32)
        x[:8] = [0.0, -0.0, np.nan, np.inf, -np.inf, 1e-30, -1e-30, 3.0]
        y = quantize_dequantize_broadcast(torch.from_numpy(x).cuda(), info, _encs_from(tab)).cpu().numpy()
        want = O.qdq_broadcast(x, info.tensorStrides, info.encodingStrides, tab[:, 0], tab[:, 1], tab[:, 2], tab[:, 3])
        np.testing.assert_array_equal(bits(y), bits(want), err_msg=str(shape))


@pytest.mark.gpu
@gpu
def test_block_permute_and_fp16_on_device():
    import torch
    from aimet_amd.onnx_op import BroadcastShapeInfo, copy_to_contiguous_block_layout, quantize_dequantize_fp16
    for x, (shape, ch, ba, bs), want in PERMUTE_KATS:
        y = copy_to_contiguous_block_layout(torch.from_numpy(x).cuda(), BroadcastShapeInfo(shape, ch, ba, bs))
        np.testing.assert_array_equal(y.cpu().numpy(), np.array(want, np.float32))
    rng = np.random.default_rng(2)
    info = BroadcastShapeInfo((64, 48, 20), 2, 0, 8)
    x = rng.standard_normal(64 * 48 * 20).astype(np.float32)
    y = copy_to_contiguous_block_layout(torch.from_numpy(x).cuda(), info).cpu().numpy()
    np.testing.assert_array_equal(y, O.copy_to_contiguous_block_layout(x, O.broadcast_shape_info((64, 48, 20), 2, 0, 8)))
    x = np.concatenate([rng.standard_normal(100003).astype(np.float32) * 1000,
                        np.array([6e-8, 3e-8, 65519.99, 65520, 1e6, -1e-10, np.nan, np.inf, -np.inf, -0.0],
                                 np.float32)])
    for off in (0, 1):   # aligned (vector) and misaligned (scalar) paths
        xt = torch.from_numpy(x).cuda()[off:]
        y = quantize_dequantize_fp16(xt).cpu().numpy()
        np.testing.assert_array_equal(bits(y), bits(O.qdq_fp16(x[off:])))


def _info(encs, quantizers, mode, sym=False, per_channel=False, ch=0, ba=0, bs=0, enabled=True, is_int=True):
    from aimet_amd.onnx_op import QcQuantizeInfo
    q = QcQuantizeInfo()
    q.encoding, q.tensorQuantizerRef = encs, quantizers
    q.opMode, q.useSymmetricEncoding, q.enabled = mode, sym, enabled
    q.isIntDataType, q.usePerChannelMode, q.channelAxis = is_int, per_channel, ch
    q.blockAxis, q.blockSize = ba, bs
    return q


def _tq(n, scheme=0):
    from aimet_amd import libpymo
    return [libpymo.TensorQuantizer(scheme, libpymo.RoundingMode.ROUND_NEAREST) for _ in range(n)]


def _fresh(n, bw=8):
    from aimet_amd.libpymo import TfEncoding
    out = []
    for _ in range(n):
        e = TfEncoding()
        e.bw = bw
        out.append(e)
    return out


@pytest.mark.gpu
@gpu
def test_qc_op_blockwise_kats():
    """test_qc_quantize_op.py:645-803: blockwise QDQ, updateStats (+ computeEncoding on every
    tensorQuantizerRef) and oneShot, symmetric and asymmetric, contiguous and permuted blocks."""
    import torch
    from aimet_amd.libpymo import TensorQuantizerOpMode as M
    from aimet_amd.onnx_op import qc_quantize_op
    for k in BLOCKWISE_KATS:
        encs = _encs_from(_kat_encodings(k))
        info = _info(encs, _tq(len(encs)), M.quantizeDequantize, True, True, k["channel_axis"], k["block_axis"],
                     k["block_size"])
        y = qc_quantize_op(info, torch.tensor(k["x"], dtype=torch.float32).reshape(k["shape"]).cuda())
        np.testing.assert_allclose(y.cpu().numpy().ravel(), np.array(k["y"], np.float32), rtol=1e-5, atol=1e-8)
    data = np.asarray([-5.4, 10, -2, 3.5, 23.1, 2., -10, -2, -1, -.1, 0.3, 0.1], np.float32)
    # symmetric, blocks contiguous: (2, 6), block axis 1, size 3
    tq = _tq(4)
    info = _info(_fresh(4), tq, M.updateStats, True, True, 0, 1, 3)
    x = torch.from_numpy(data.reshape(2, 6)).cuda()
    assert torch.equal(qc_quantize_op(info, x), x)
    expected_max = np.max(np.abs(data.reshape(4, 3)), axis=1)
    for i, q in enumerate(tq):
        e = q.computeEncoding(8, True)
        assert abs(e.max - expected_max[i]) <= 1e-4 and abs(e.max + e.min + e.delta) <= 1e-4
        assert e.offset == -128 and abs(e.delta - e.max / 127) <= 1e-4
        want = O.Analyzer(O.QUANTIZATION_TF)
        want.update(data.reshape(4, 3)[i])
        assert e.to_tuple() == want.compute(8, True).as_tuple()
    # asymmetric, blocks NOT contiguous: (6, 2), block axis 0 size 2, channel axis 1 -> permuted
    tq = _tq(6)
    info = _info(_fresh(6), tq, M.updateStats, False, True, 1, 0, 2)
    qc_quantize_op(info, torch.from_numpy(data.reshape(6, 2)).cuda())
    blocks = data.reshape(3, 2, 2).transpose(0, 2, 1).reshape(6, 2)     # block (b, c) = x[2b:2b+2, c]
    for i, q in enumerate(tq):
        want = O.Analyzer(O.QUANTIZATION_TF)
        want.update(blocks[i])
        assert q.computeEncoding(8, False).to_tuple() == want.compute(8, False).as_tuple()
    # oneShot: encodings written into the info, output = blockwise QDQ with them, mode -> QDQ
    encs = _fresh(4)
    info = _info(encs, _tq(4), M.oneShotQuantizeDequantize, True, True, 0, 1, 3)
    y = qc_quantize_op(info, torch.from_numpy(data.reshape(2, 6)).cuda()).cpu().numpy()
    assert info.opMode == M.quantizeDequantize
    for i, e in enumerate(encs):
        a = O.Analyzer(O.QUANTIZATION_TF)
        a.update(data.reshape(4, 3)[i])
        w = a.compute(8, True)
        assert (e.min, e.max, e.delta, e.offset, e.bw) == (w.min, w.max, w.delta, w.offset, 8)
    oi = O.broadcast_shape_info((2, 6), 0, 1, 3)
    t = np.array([[e.min, e.max, e.delta, e.offset] for e in encs], np.float32)
    np.testing.assert_array_equal(bits(y.ravel()), bits(O.qdq_broadcast(data, oi["tensor_strides"],
                                                                         oi["encoding_strides"], *t.T)))


@pytest.mark.gpu
@gpu
def test_qc_op_per_tensor_per_channel_and_float_modes():
    """modeSpecificAction{Int,PerChannelInt,Float} (AimetOpUtils.h:101-330) against the oracle."""
    import torch
    from aimet_amd.libpymo import TensorQuantizerOpMode as M
    from aimet_amd.onnx_op import qc_quantize_op
    rng = np.random.default_rng(12)
    x = (rng.standard_normal((4, 6, 25)) * 2 + 0.5).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    # per-tensor: updateStats (pass-through) -> computeEncoding -> quantizeDequantize
    tq = _tq(1, scheme=1)    # TF-Enhanced
    enc = _fresh(1)
    info = _info(enc, tq, M.updateStats, sym=False)
    assert torch.equal(qc_quantize_op(info, xt), xt)
    a = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
    a.update(x.ravel())
    e = tq[0].computeEncoding(8, False)
    assert e.to_tuple() == a.compute(8).as_tuple()
    enc[0].min, enc[0].max = e.min, e.max
    info.opMode = M.quantizeDequantize
    y = qc_quantize_op(info, xt).cpu().numpy()
    np.testing.assert_array_equal(bits(y.ravel()), bits(O.qdq_per_tensor(x.ravel(), e.min, e.max, 8)))
    # per-tensor oneShot on a fresh TF quantizer
    enc = _fresh(1)
    info = _info(enc, _tq(1), M.oneShotQuantizeDequantize, sym=True)
    y = qc_quantize_op(info, xt).cpu().numpy()
    a = O.Analyzer(O.QUANTIZATION_TF)
    a.update(x.ravel())
    w = a.compute(8, True)
    assert (enc[0].min, enc[0].max, enc[0].delta, enc[0].offset) == (w.min, w.max, w.delta, w.offset)
    np.testing.assert_array_equal(bits(y.ravel()), bits(O.qdq_per_tensor(x.ravel(), w.min, w.max, 8)))
    assert info.opMode == M.quantizeDequantize
    # per-channel (axis 1) oneShot: per-channel analyzers, QDQ with the raw encodings
    encs = _fresh(6)
    info = _info(encs, _tq(6), M.oneShotQuantizeDequantize, sym=False, per_channel=True, ch=1)
    y = qc_quantize_op(info, xt).cpu().numpy()
    tab = []
    for c in range(6):
        a = O.Analyzer(O.QUANTIZATION_TF)
        a.update(np.ascontiguousarray(x[:, c, :]).ravel())
        w = a.compute(8, False)
        assert (encs[c].min, encs[c].max, encs[c].delta, encs[c].offset) == (w.min, w.max, w.delta, w.offset)
        tab.append([w.min, w.max, w.delta, w.offset])
    tab = np.array(tab, np.float32).T.ravel()
    np.testing.assert_array_equal(bits(y.ravel()), bits(O.qdq_per_channel(x.ravel(), 6, 25, tab)))
    with pytest.raises(RuntimeError, match="Channel dimensions"):
        qc_quantize_op(_info(_fresh(5), _tq(5), M.quantizeDequantize, per_channel=True, ch=1), xt)
    # disabled -> pass-through; float quantizer -> fp16 round trip
    info = _info(_fresh(1), _tq(1), M.quantizeDequantize, enabled=False)
    assert torch.equal(qc_quantize_op(info, xt), xt)
    info = _info([], [], M.quantizeDequantize, is_int=False)
    y = qc_quantize_op(info, xt).cpu().numpy()
    np.testing.assert_array_equal(bits(y.ravel()), bits(O.qdq_fp16(x.ravel())))
    info.opMode = M.updateStats
    assert torch.equal(qc_quantize_op(info, xt), xt)
