"""aimet_amd -- MI355X-native (gfx950) quantization-simulation core for AIMET.

The DlQuantization hot path (QcQuantize quantize-dequantize forward/backward, per-tensor and
per-channel; TF / TF-Enhanced / percentile / MSE encoding statistics; AdaRound soft rounding)
as hand-written HIP kernels behind a C-ABI (include/aimet_amd.h), with the reference's Python
operator surface on top:

* ``aimet_amd.libpymo``            -- the quantization subset of ``aimet_common._libpymo``
* ``aimet_amd.tensor_quantizer``   -- ``AimetTensorQuantizer`` (the torch extension)
* ``aimet_amd.quantizers``         -- v1 StaticGrid{PerTensor,PerChannel}Quantizer + STE autograd
* ``aimet_amd.quantsim``           -- QcQuantize wrapper / compute_encodings driver
* ``aimet_amd.adaround``           -- AdaRound soft-rounding autograd on the fused kernels
* ``aimet_amd.distributed``        -- calibration sharded over ranks (RCCL stats exchange)

There is no CPU fallback: without libaimet_amd.so or an MI355X every compute call raises.
"""
from aimet_amd import _native  # noqa: F401
from aimet_amd.libpymo import QuantizationMode, RoundingMode, TfEncoding  # noqa: F401
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: F401

__version__ = "0.1.0"


def native_library():
    """Load (and return) libaimet_amd.so; raises NativeLibraryError when it is unusable."""
    return _native.load()
