"""The ONNX QcQuantizeOp on MI355X: ``libquant_info.QcQuantizeInfo`` and the op's Compute.

Reference: TrainingExtensions/onnx/src/QcQuantizeInfo.{h,cpp} (the pybind ``libquant_info``
module), QcQuantizeOp.cpp:62-113 (computeImpl) and AimetOpUtils.h:101-330 (the op-mode state
machine: oneShotQuantizeDequantize / updateStats / quantizeDequantize / passThrough, for int
per-tensor, per-channel and blockwise (broadcast) quantizers and fp16 float quantizers).

The reference op is an onnxruntime custom op; onnxruntime is not part of this stack, so the op is
exposed as ``aimet_qc_quantize_op_compute`` in libaimet_amd (what an ORT-ROCm custom op's Compute
calls with its stream) and, here, as :func:`qc_quantize_op` on torch device
tensors. The reference keeps one ``libpymo.TensorQuantizer`` per encoding in
``tensorQuantizerRef``; here their analyzers are the channels of ONE device quantizer, and each
``TensorQuantizer`` of ``tensorQuantizerRef`` is bound to its channel so that
``computeEncoding`` on it returns that channel's (block's) encoding, as in the reference tests.
"""
import ctypes
from typing import List

import torch

from aimet_amd import _native
from aimet_amd._native import QcQuantizeInfoC, TfEncodingC
from aimet_amd.libpymo import (QuantizationMode, RoundingMode, TensorQuantizer, TensorQuantizerOpMode, TfEncoding)
from aimet_amd.tensor_quantizer import AimetTensorQuantizer, _require_gpu


class BroadcastShapeInfo:
    """onnx/src/QuantizeDequantizeUtils.hpp:166-178 (computed by the library, host side)."""

    def __init__(self, input_shape, channel_axis: int, block_axis: int, block_size: int):
        shape = (ctypes.c_int64 * max(1, len(input_shape)))(*[int(d) for d in input_shape])
        c = _native.BroadcastShapeInfoC()
        _native.call("aimet_broadcast_shape_info_init", shape, len(input_shape), int(channel_axis), int(block_axis),
                     int(block_size), ctypes.byref(c))
        nd = c.num_dims
        self._c = c
        self.numDims = nd
        self.tensorShape = list(c.tensor_shape[:nd])
        self.encodingShape = list(c.encoding_shape[:nd])
        self.tensorStrides = list(c.tensor_strides[:nd])
        self.encodingStrides = list(c.encoding_strides[:nd])
        self.numElements = c.num_elements
        self.numEncodings = c.num_encodings

    def hasContiguousBlocks(self) -> bool:
        return bool(self._c.contiguous_blocks)


def copy_to_contiguous_block_layout(x: torch.Tensor, shape_info: BroadcastShapeInfo) -> torch.Tensor:
    """QuantizeDequantizeUtils.cpp:173-213: x with every quantization block contiguous."""
    _require_gpu(x)
    x = x.contiguous()
    out = torch.empty_like(x)
    _native.call("aimet_copy_to_contiguous_block_layout", x.data_ptr(), out.data_ptr(), ctypes.byref(shape_info._c),
                 torch.cuda.current_stream(x.device).cuda_stream)
    return out


class QcQuantizeInfo:
    """libquant_info.QcQuantizeInfo: value-initialised like ``py::init<>()`` (all zero / False)."""

    def __init__(self):
        self.encoding: List[TfEncoding] = []
        self.opMode = TensorQuantizerOpMode.updateStats
        self.name = ""
        self.enabled = False
        self.useSymmetricEncoding = False
        self.usePerChannelMode = False
        self.isIntDataType = False
        self.channelAxis = 0
        self.blockSize = 0
        self.blockAxis = 0
        self._refs: List[TensorQuantizer] = []
        self._shared = None

    @property
    def tensorQuantizerRef(self):
        return list(self._refs)

    @tensorQuantizerRef.setter
    def tensorQuantizerRef(self, quantizers):
        # the reference stores raw TensorQuantizer pointers (libpymo.PtrToInt64); the mirror keeps
        # the objects themselves
        self._refs = [q for q in quantizers]
        self._shared = None

    def _device_quantizer(self, n_enc: int, device) -> AimetTensorQuantizer:
        """ONE device quantizer whose channels are the analyzers of tensorQuantizerRef."""
        if not self._refs:
            raise RuntimeError("QcQuantizeInfo.tensorQuantizerRef is empty")
        ref0 = self._refs[0]
        if n_enc == 1 and len(self._refs) == 1:
            return ref0._op                    # the TensorQuantizer's own analyzer
        if len(self._refs) != n_enc:
            raise RuntimeError("tensorQuantizerRef holds %d quantizers, the op needs %d" % (len(self._refs), n_enc))
        if self._shared is None or self._shared.num_channels != n_enc:
            self._shared = AimetTensorQuantizer(ref0.getQuantScheme(), num_channels=n_enc)
            for i, q in enumerate(self._refs):
                q._bind(self._shared, i)
        return self._shared


def qc_quantize_op(info: QcQuantizeInfo, x: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """QcQuantizeOp::Compute on a fp32 device tensor (QcQuantizeOp.cpp:62-113); returns the output."""
    _require_gpu(x)
    x = x.contiguous()
    y = torch.empty_like(x) if out is None else out
    encs = info.encoding
    n_enc = len(encs)
    arr = (TfEncodingC * max(1, n_enc))()
    for i, e in enumerate(encs):
        arr[i] = TfEncodingC(e.min, e.max, e.delta, e.offset, e.bw)
    c = QcQuantizeInfoC()
    c.op_mode = int(info.opMode)
    c.enabled = int(bool(info.enabled))
    c.is_int_data_type = int(bool(info.isIntDataType))
    c.use_per_channel_mode = int(bool(info.usePerChannelMode))
    c.channel_axis, c.block_axis, c.block_size = int(info.channelAxis), int(info.blockAxis), int(info.blockSize)
    c.use_symmetric_encoding = int(bool(info.useSymmetricEncoding))
    c.num_encodings = n_enc
    c.encodings = ctypes.cast(arr, ctypes.POINTER(TfEncodingC))
    mode = int(info.opMode) if info.enabled else int(TensorQuantizerOpMode.passThrough)
    needs_stats = info.isIntDataType and mode in (int(TensorQuantizerOpMode.updateStats),
                                                  int(TensorQuantizerOpMode.oneShotQuantizeDequantize))
    ref0 = info._refs[0] if info._refs else None
    c.rounding_mode = int(ref0.roundingMode) if ref0 is not None else int(RoundingMode.ROUND_NEAREST)
    if ref0 is not None:
        c.use_strict_symmetric = int(ref0.getStrictSymmetric())
        c.use_unsigned_symmetric = int(ref0.getUnsignedSymmetric())
    if needs_stats:
        q = info._device_quantizer(n_enc if info.usePerChannelMode else 1, x.device)
        c.quantizer = q._ensure(x.device).value
    shape = (ctypes.c_int64 * max(1, x.dim()))(*x.shape)
    with torch.cuda.device(x.device):
        _native.call("aimet_qc_quantize_op_compute", ctypes.byref(c), x.data_ptr(), y.data_ptr(), shape, x.dim(),
                     torch.cuda.current_stream(x.device).cuda_stream)
    if needs_stats:
        q._is_encoding_valid = True
        for r in info._refs:
            r._valid_stats = True
    if mode == int(TensorQuantizerOpMode.oneShotQuantizeDequantize):
        for e, ce in zip(encs, arr):
            e.min, e.max, e.offset, e.delta = ce.min, ce.max, ce.offset, ce.delta
    info.opMode = TensorQuantizerOpMode(c.op_mode)
    return y


def quantize_dequantize_broadcast(x: torch.Tensor, shape_info: BroadcastShapeInfo, encodings) -> torch.Tensor:
    """quantizeDequantizeBroadcast (QuantizeDequantizeUtils.hpp:186-245 -> trim_functions.cpp:633-687)
    with a list of TfEncoding (used as given)."""
    _require_gpu(x)
    x = x.contiguous()
    E = shape_info.numEncodings
    if len(encodings) != E:
        raise RuntimeError("encodings.size() does not match shapeInfo.numEncodings")
    t = torch.tensor([[e.min for e in encodings], [e.max for e in encodings], [e.delta for e in encodings],
                      [e.offset for e in encodings]], dtype=torch.float32).to(x.device)
    y = torch.empty_like(x)
    nd = shape_info.numDims
    ts = (ctypes.c_int64 * nd)(*shape_info.tensorStrides)
    es = (ctypes.c_int64 * nd)(*shape_info.encodingStrides)
    _native.call("aimet_qdq_broadcast", x.data_ptr(), y.data_ptr(), x.numel(), nd, ts, es, t[0].data_ptr(),
                 t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), torch.cuda.current_stream(x.device).cuda_stream)
    return y


def quantize_dequantize_fp16(x: torch.Tensor) -> torch.Tensor:
    """quantizeDequantizeFp16Gpu: float -> half (RNE) -> float, one fused pass."""
    _require_gpu(x)
    x = x.contiguous()
    y = torch.empty_like(x)
    _native.call("aimet_qdq_fp16", x.data_ptr(), y.data_ptr(), x.numel(), torch.cuda.current_stream(x.device).cuda_stream)
    return y


__all__ = ["BroadcastShapeInfo", "QcQuantizeInfo", "QuantizationMode", "TensorQuantizerOpMode",
           "copy_to_contiguous_block_layout", "qc_quantize_op", "quantize_dequantize_broadcast",
           "quantize_dequantize_fp16"]
