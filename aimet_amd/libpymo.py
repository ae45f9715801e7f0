"""Drop-in for the quantization subset of ``aimet_common._libpymo``
(ModelOptimizations/PyModelOptimizations/PyModelOptimizations.cpp:147-261).

Same names, same argument meaning. The numpy entry points (`EncodingAnalyzerForPython`,
`TensorQuantizationSimForPython`, `TensorQuantizer`) run on the MI355X: arrays are copied to
HBM, processed by the gfx950 kernels and copied back (the reference ran them on the CPU unless
``use_cuda``). Names of the reference module that belong to other subsystems (SVD, CLE, BN fold,
bias correction, op-def parser, encoding rescaling) exist as stubs that raise on use, like
``aimet_common/py_libpymo.py:50-127``.
"""
import enum

import numpy as np
import torch

from aimet_amd import _native
from aimet_amd._native import TfEncodingC


class ComputationMode(enum.IntEnum):       # Quantization.hpp:52-56
    COMP_MODE_CPU = 0
    COMP_MODE_GPU = 1


class QuantizationMode(enum.IntEnum):      # Quantization.hpp:84-106
    QUANTIZATION_TF = 0
    QUANTIZATION_TF_ENHANCED = 1
    QUANTIZATION_RANGE_LEARNING = 2
    QUANTIZATION_PERCENTILE = 3
    QUANTIZATION_MSE = 4
    QUANTIZATION_ENTROPY = 5


class LayerInOut(enum.IntEnum):            # Quantization.hpp:131-135
    LAYER_INPUT = 0
    LAYER_OUTPUT = 1


class RoundingMode(enum.IntEnum):          # Quantization.hpp:140-144
    ROUND_NEAREST = 0
    ROUND_STOCHASTIC = 1


class TensorQuantizerOpMode(enum.IntEnum):  # TensorQuantizerOpFacade.h:48-54
    updateStats = 0
    oneShotQuantizeDequantize = 1
    quantizeDequantize = 2
    passThrough = 3


# pybind11 enums export their values into the module namespace (export_values())
for _e in (ComputationMode, QuantizationMode, LayerInOut, RoundingMode):
    globals().update(_e.__members__)


class TfEncoding(TfEncodingC):
    """``DlQuantization::TfEncoding`` (Quantization.hpp:113-120); default-constructed to zeros.

    The object IS the C struct the library reads and writes (no conversion at the boundary), so
    a per-channel getEncoding of 27,560 channels materialises its list in one C-level pass.
    Every field assignment bumps a process-wide version number, so device-side caches built from
    encodings (per-channel QDQ tables) can tell in O(1) that any encoding changed.
    """
    _version = 0

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        TfEncoding._version += 1

    def __setattr__(self, name, value):
        if name == "bw":
            value = int(value)
        super().__setattr__(name, value)
        TfEncoding._version += 1

    def __repr__(self):
        return "TfEncoding(min=%r, max=%r, delta=%r, offset=%r, bw=%d)" % (
            self.min, self.max, self.delta, self.offset, self.bw)

    def __eq__(self, other):
        return isinstance(other, TfEncodingC) and self.to_tuple() == TfEncoding.to_tuple(other)

    __hash__ = None

    def to_tuple(self):
        return (self.min, self.max, self.delta, self.offset, self.bw)

    def to_c(self) -> TfEncodingC:
        return self

    @staticmethod
    def from_c(c: TfEncodingC) -> "TfEncoding":
        TfEncoding._version += 1
        return TfEncoding.from_buffer_copy(c)

    @staticmethod
    def array(n: int):
        """A C array of n zero encodings; ``list(arr)`` gives TfEncoding views into it."""
        TfEncoding._version += 1
        return (TfEncoding * n)()


def encodings_to_c(encodings):
    """Contiguous C copy of a sequence of TfEncoding (one C-level pass)."""
    n = len(encodings)
    return (TfEncodingC * n).from_buffer_copy(b"".join(map(bytes, encodings))) if n else (TfEncodingC * 0)()


def getComputedEncodings(bw, min_val, max_val, use_symmetric, use_strict_symmetric, use_unsigned_symmetric):
    """quantization_utils.cpp:58-143 (exposed for tests and encoding import/export)."""
    out = TfEncodingC()
    _native.call("aimet_get_computed_encodings", int(bw), float(min_val), float(max_val), int(use_symmetric),
                 int(use_strict_symmetric), int(use_unsigned_symmetric), out)
    return TfEncoding.from_c(out)


def fillEncodingInfo(bw, min_val, max_val):
    """TensorQuantizationSim.cpp:62-92."""
    out = TfEncodingC()
    _native.call("aimet_fill_encoding_info", int(bw), float(min_val), float(max_val), out)
    return TfEncoding.from_c(out)


def PtrToInt64(ptr):
    return int(ptr)


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("aimet_amd needs an MI355X (HIP device); there is no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


def _to_device(arr):
    a = np.ascontiguousarray(arr, dtype=np.float32)
    return torch.from_numpy(a).to(_device())


class EncodingAnalyzerForPython:
    """EncodingAnalyzerForPython.cpp: numpy updateStats / computeEncoding."""

    def __init__(self, quant_mode):
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        self._op = AimetTensorQuantizer(quant_mode)

    def updateStats(self, tensor, use_cuda=True):
        self._op.updateStats(_to_device(tensor), True)

    def computeEncoding(self, bw, use_symmetric_encodings, use_strict_symmetric, use_unsigned_symmetric):
        return self._op.getEncoding(bw, use_symmetric_encodings, use_strict_symmetric, use_unsigned_symmetric)


class TensorQuantizationSimForPython:
    """TensorQuantizationSimForPython.cpp: numpy QDQ, result written into the input array."""

    def quantizeDequantize(self, tensor, encoding, rounding_mode, *args):
        # overloads: (arr, enc, rm, use_cuda) and (arr, enc, rm, bitwidth, use_cuda)
        bw = int(args[0]) if len(args) == 2 else int(encoding.bw)
        enc = TfEncoding()
        enc.min, enc.max, enc.bw = encoding.min, encoding.max, bw
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        x = _to_device(tensor)
        y = AimetTensorQuantizer.quantize_dequantize_tensor(x, enc, rounding_mode)
        out = np.asarray(tensor)
        out[...] = y.cpu().numpy().reshape(out.shape)
        return out


class TensorQuantizer:
    """PyTensorQuantizer (PyModelOptimizations/PyTensorQuantizer.cpp): the libpymo TensorQuantizer."""

    def __init__(self, quant_scheme, rounding_mode):
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        self._scheme = QuantizationMode(quant_scheme)
        self.roundingMode = RoundingMode(rounding_mode)
        self.isEncodingValid = False
        self._strict = False
        self._unsigned = False
        self._valid_stats = False
        self._op = AimetTensorQuantizer(self._scheme)
        self._channel = None   # bound to channel c of a shared device quantizer (onnx_op.QcQuantizeInfo)

    def _bind(self, shared, channel):
        """Read statistics from channel `channel` of `shared` (the analyzers of a QcQuantizeOp)."""
        self._op, self._channel = shared, int(channel)

    def resetEncodingStats(self):
        self._valid_stats = False
        self.isEncodingValid = False
        if self._channel is None:   # a bound quantizer shares its statistics with its op
            self._op.resetEncodingStats()

    def updateStats(self, tensor, use_cuda=True):
        self._valid_stats = True
        self._op.updateStats(_to_device(tensor), True)

    def computeEncoding(self, bitwidth, use_symmetric_encoding):
        enc = TfEncoding()
        if self._valid_stats:
            enc, _ = self._op.getEncoding(bitwidth, use_symmetric_encoding, self._strict, self._unsigned)
            if self._channel is not None:
                enc = enc[self._channel] if isinstance(enc, list) else enc
            self.isEncodingValid = True
        return enc

    def quantizeDequantize(self, tensor, output, encoding_min, encoding_max, bitwidth, use_cuda=True):
        if not self.isEncodingValid:
            raise RuntimeError("quantizeDequantize called before computeEncoding (TensorQuantizer.cpp:177)")
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        enc = TfEncoding()
        enc.min, enc.max, enc.bw = encoding_min, encoding_max, bitwidth
        y = AimetTensorQuantizer.quantize_dequantize_tensor(_to_device(tensor), enc, self.roundingMode)
        out = np.asarray(output)
        out[...] = y.cpu().numpy().reshape(out.shape)

    def setQuantScheme(self, quant_scheme):
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        self._scheme = QuantizationMode(quant_scheme)
        self._op = AimetTensorQuantizer(self._scheme)
        self.resetEncodingStats()

    def getQuantScheme(self):
        return self._scheme

    def setStrictSymmetric(self, v):
        self._strict = bool(v)
        self.resetEncodingStats()

    def getStrictSymmetric(self):
        return self._strict

    def setUnsignedSymmetric(self, v):
        self._unsigned = bool(v)
        self.resetEncodingStats()

    def getUnsignedSymmetric(self):
        return self._unsigned

    def getStatsHistogram(self):
        return self._op.getStatsHistogram()

    def setPercentileValue(self, p):
        self._op.setPercentileValue(p)

    def getPercentileValue(self):
        return self._op.getPercentileValue()

    def computePartialEncoding(self, bw, encoding, use_symmetric, use_unsigned_symmetric, use_strict_symmetric):
        c = encoding.to_c()
        _native.call("aimet_compute_partial_encoding", int(bw), c, int(use_symmetric),
                     int(use_unsigned_symmetric), int(use_strict_symmetric))
        for f in ("min", "max", "delta", "offset", "bw"):
            setattr(encoding, f, getattr(c, f))


def GetQuantizationEncodingAnalyzerInstance(quant_mode):
    """QuantizerFactory.cpp:74-104 (bound at PyModelOptimizations.cpp:187)."""
    return EncodingAnalyzerForPython(quant_mode)


def _stub(name):
    def _raise(*_a, **_k):
        raise NotImplementedError("libpymo.%s belongs to a subsystem outside the MI355X quantization-simulation "
                                  "core (SURVEY §2: OUT OF SCOPE)" % name)
    _raise.__name__ = name
    return _raise


for _name in ("GetQuantizationInstance", "GetSVDInstance", "Svd", "LayerAttributes", "EqualizationParams",
              "scaleLayerParams", "scaleDepthWiseSeparableLayer", "BNParams", "BNParamsHighBiasFold",
              "updateBias", "BiasCorrection", "LayerParams", "ModelOpDefParser", "getRescaledOutputAndBias",
              "str_to_dtype", "str_to_rank"):
    globals()[_name] = _stub(_name)
