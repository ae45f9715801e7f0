"""Quantization wrappers around torch modules: the Python callers of the QDQ / statistics core.

Mirrors aimet_torch/v1/qc_quantize_op.py (QcQuantizeOpMode :63-70, tensor_quantizer_factory
:77-110, QcQuantizeWrapper :198-676, StaticGridQuantWrapper :679-938,
SteGatingFuncForParameters :1314-1366): same names, modes, quantizer layout
(input_quantizers / output_quantizers lists, param_quantizers dict), same ANALYSIS / ACTIVE
behaviour and encoding import/export format. Every statistic and every QDQ runs on the gfx950
kernels of aimet_amd (no CPU path; CPU tensors are refused by the core).
"""
import contextlib
import enum
import os
import threading
from typing import Dict, Mapping, Optional

import torch
from torch import nn

from aimet_amd.encodings_io import (compute_partial_encoding, create_encoding_from_dict, export_quantizer_encoding,
                                    validate_is_symmetric_flag)
from aimet_amd.learned_grid import (LearnedGridTensorQuantizer, initialize_learned_grid_quantizer_attributes,
                                    set_encoding_min_max_gating_threshold_many)
from aimet_amd.libpymo import RoundingMode
from aimet_amd.quantizers import (MAP_ROUND_MODE_TO_PYMO, QuantizationDataType, QuantScheme,
                                  StaticGridPerChannelQuantizer, StaticGridPerTensorQuantizer, compute_dloss_by_dx)


class QcQuantizeOpMode(enum.Enum):
    """v1/qc_quantize_op.py:63-70."""
    PASSTHROUGH = 1
    ANALYSIS = 2
    ACTIVE = 3
    LEARN_ENCODINGS = 4


QUANTIZER_TYPE_INPUT = "input"
QUANTIZER_TYPE_OUTPUT = "output"
# v1/qc_quantize_op.py:74-76: optional 2x downsampling of TF-Enhanced statistics
TF_ENHANCED_USE_DOWNSAMPLING = bool(int(os.environ.get("AIMET_TFE_USE_DOWNSAMPLING", "0")))
TF_ENHANCED_OFFSET_FACTOR = 0
TF_ENHANCED_STRIDE_FACTOR = 2

# DataParallel replicas share their quantizer objects (replicate() copies module __dict__s) and run
# in one thread per device; a parameter quantizer's reset -> statistics -> encoding -> QDQ sequence
# runs under this lock so the replicas never interleave on one quantizer's device state
_REPLICA_LOCK = threading.Lock()


class StatsBatch:
    """The activation statistics of QuantizationSimModel.compute_encodings' ANALYSIS forwards,
    batched: a wrapper hands (quantizer, a copy of the tensor) here instead of launching the
    quantizer's update (aimet_tq_update_stats: ~4 launches and ~25 us of host time each; the copy
    is one), and flush() updates every pending quantizer with one AimetTensorQuantizer.updateStatsMany
    call per device (one launch per phase). Each quantizer still sees its tensors in the order the forward produced them: a second
    tensor for a pending quantizer flushes first. The tensors stay alive until flushed, so at most
    `limit` elements are held (then flushed); compute_encodings flushes after every forward of the
    model and at the end. Shared by DataParallel replicas (their wrappers' __dict__ is a shallow copy)."""

    def __init__(self, limit: int = 1 << 30):
        self.limit = limit
        self.lock = threading.Lock()
        self.items = []
        self.pending = set()
        self.elems = 0

    @staticmethod
    def eligible(q, t) -> bool:
        from aimet_amd.quantizers import StaticGridPerTensorQuantizer
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        return (type(q) is StaticGridPerTensorQuantizer and q.enabled and not q._is_encoding_frozen and
                q.bitwidth != 32 and q.data_type == QuantizationDataType.int and
                q.encoding_min_max_fixed_vals is None and isinstance(t, torch.Tensor) and t.is_cuda and
                t.dtype == torch.float32 and type(q._op()) is AimetTensorQuantizer)

    def add(self, q, t, owned: bool = False):
        """Queue q's update with t. Unless the caller owns t (a copy nobody else sees), t is copied
        first: the network may overwrite it in place before the flush (nn.ReLU(inplace=True),
        `out += identity`), and the statistics must see the values the quantizer was given -- what
        the per-call update, launched at once on the stream, reads."""
        if not owned or not t.is_contiguous():
            t = t.clone(memory_format=torch.contiguous_format)
        with self.lock:
            if id(q) in self.pending or self.elems + t.numel() > self.limit:
                self._flush_locked()
            self.items.append((q, t))
            self.pending.add(id(q))
            self.elems += t.numel()

    def flush(self):
        with self.lock:
            self._flush_locked()

    def _flush_locked(self):
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        items, self.items, self.pending, self.elems = self.items, [], set(), 0
        by_dev = {}
        for q, t in items:
            by_dev.setdefault(t.device, []).append((q, t))
        for dev, group in by_dev.items():
            with torch.cuda.device(dev):
                AimetTensorQuantizer.updateStatsMany([q._op() for q, _ in group], [t for _, t in group])

_IGNORED_DTYPES = (torch.int8, torch.uint8, torch.int16, torch.int32, torch.int64, torch.bool)
# wrapped modules that never modify their inputs in place
_INPUT_PRESERVING_TYPES = (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.ConvTranspose1d, nn.ConvTranspose2d,
                           nn.ConvTranspose3d, nn.Linear)


def tensor_quantizer_factory(bitwidth, round_mode, quant_scheme, use_symmetric_encodings, enabled_by_default,
                             data_type=QuantizationDataType.int):
    """v1/qc_quantize_op.py:77-110."""
    if quant_scheme in (QuantScheme.post_training_tf_enhanced, QuantScheme.post_training_tf,
                        QuantScheme.post_training_percentile):
        return StaticGridPerTensorQuantizer(bitwidth, round_mode, quant_scheme, use_symmetric_encodings,
                                            enabled_by_default, data_type=data_type)
    if quant_scheme in (QuantScheme.training_range_learning_with_tf_init,
                        QuantScheme.training_range_learning_with_tf_enhanced_init):
        return LearnedGridTensorQuantizer(bitwidth, round_mode, quant_scheme, use_symmetric_encodings,
                                          enabled_by_default, data_type)
    raise AssertionError("Unsupported quant_scheme: " + str(quant_scheme))


class QcQuantizeWrapper(nn.Module):
    """v1/qc_quantize_op.py:198-676."""

    def __init__(self, module_to_wrap: nn.Module, weight_bw: int, activation_bw: int, round_mode,
                 quant_scheme: QuantScheme, is_output_quantized=True, is_symmetric=False, num_inputs=1,
                 num_outputs=1, data_type: QuantizationDataType = QuantizationDataType.int):
        super().__init__()
        if data_type == QuantizationDataType.float:
            raise NotImplementedError("float (fp8/fp16) quantization is outside the MI355X integer QDQ core")
        self.output_quantizers = [tensor_quantizer_factory(activation_bw, round_mode, quant_scheme, is_symmetric,
                                                           enabled_by_default=is_output_quantized,
                                                           data_type=data_type) for _ in range(num_outputs)]
        self._mode = QcQuantizeOpMode.ANALYSIS
        self._module_to_wrap = module_to_wrap
        self.param_quantizers = {}
        for name, _ in module_to_wrap.named_parameters():
            self.param_quantizers[name] = tensor_quantizer_factory(weight_bw, round_mode, quant_scheme, is_symmetric,
                                                                   enabled_by_default=True, data_type=data_type)
        self.input_quantizers = [tensor_quantizer_factory(activation_bw, round_mode, quant_scheme, is_symmetric,
                                                          enabled_by_default=False, data_type=data_type)
                                 for _ in range(num_inputs)]
        self.supported_kernels = {}

    def get_named_parameters(self):
        """v1/qc_quantize_op.py:257-269: a torch.nn.DataParallel replica holds its (broadcast)
        parameters outside ``_parameters``; they are listed in ``_former_parameters``."""
        if getattr(self, "_is_replica", False):
            yield from self._module_to_wrap._former_parameters.items()
        else:
            yield from self._module_to_wrap.named_parameters()

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self._module_to_wrap, name)

    def set_output_bw(self, output_bw: int):
        self.output_quantizers[0].bitwidth = output_bw

    def set_mode(self, mode):
        self._mode = mode

    def enable_param_quantizers(self, enabled: bool, param_name_to_exclude=("bias",)):
        for name, q in self.param_quantizers.items():
            if name not in (param_name_to_exclude or ()):
                q.enabled = enabled

    def enable_input_quantizers(self, enabled: bool):
        for q in self.input_quantizers:
            q.enabled = enabled

    def enable_output_quantizers(self, enabled: bool):
        for q in self.output_quantizers:
            q.enabled = enabled

    def enable_activation_quantizers(self, enabled: bool):
        self.enable_input_quantizers(enabled)
        self.enable_output_quantizers(enabled)

    def reset_encodings(self):
        for q in list(self.input_quantizers) + list(self.output_quantizers) + list(self.param_quantizers.values()):
            q.reset_encoding_stats()

    def get_original_module(self) -> nn.Module:
        return self._module_to_wrap

    @staticmethod
    def should_perform_quant_dequant(tensor, tensor_quantizer) -> bool:
        """v1/qc_quantize_op.py:451-473."""
        if not isinstance(tensor, torch.Tensor) or tensor.dtype in _IGNORED_DTYPES or \
                (tensor_quantizer.is_const and tensor.numel() == 1) or not tensor_quantizer.enabled:
            tensor_quantizer.enabled = False
            return False
        return True

    # -- encodings export / import (v1/qc_quantize_op.py:363-676) -------------------------------
    def export_param_encodings(self):
        return {name: export_quantizer_encoding(q) for name, q in self.param_quantizers.items()}

    def export_output_encodings(self):
        return [export_quantizer_encoding(q) for q in self.output_quantizers]

    def export_input_encodings(self):
        return [export_quantizer_encoding(q) for q in self.input_quantizers]

    def set_activation_encoding(self, module_name: str, activation_encodings: Dict,
                                ignore_when_quantizer_disabled: bool = False,
                                disable_quantizer_without_encoding: bool = True):
        entry = activation_encodings.get(module_name, {})
        self.import_input_encodings(entry.get(QUANTIZER_TYPE_INPUT, {}), strict=not ignore_when_quantizer_disabled,
                                    partial=not disable_quantizer_without_encoding, requires_grad=None,
                                    allow_overwrite=None)
        self.import_output_encodings(entry.get(QUANTIZER_TYPE_OUTPUT, {}),
                                     strict=not ignore_when_quantizer_disabled,
                                     partial=not disable_quantizer_without_encoding, requires_grad=None,
                                     allow_overwrite=None)

    def set_param_encoding(self, module_name: str, param_encodings: Dict, ignore_when_quantizer_disabled: bool = False,
                           disable_quantizer_without_encoding: bool = True):
        enc = {p: param_encodings["%s.%s" % (module_name, p)] for p in self.param_quantizers
               if "%s.%s" % (module_name, p) in param_encodings}
        self.import_param_encodings(enc, strict=not ignore_when_quantizer_disabled,
                                    partial=not disable_quantizer_without_encoding, requires_grad=None,
                                    allow_overwrite=None)

    def freeze_param_encoding(self, module_name: str, param_encodings: Dict):
        for p, q in self.param_quantizers.items():
            if "%s.%s" % (module_name, p) in param_encodings and q.enabled:
                q.freeze_encoding()

    def import_param_encodings(self, encodings: Mapping, strict: bool, partial: bool,
                               requires_grad: Optional[bool], allow_overwrite: bool):
        """v1/qc_quantize_op.py:499-584."""
        for name in list(self.param_quantizers):
            q = self.param_quantizers[name]
            if q._is_encoding_frozen:
                continue
            encoding = encodings.get(name, None)
            if not encoding:
                if not partial:
                    q.enabled = False
                continue
            if not q.enabled:
                if strict:
                    raise RuntimeError("The quantsim passed for loading encodings does not have the same "
                                       "configuration as the quantsim which was used to export the encodings")
                continue
            per_channel = isinstance(q, StaticGridPerChannelQuantizer)
            if isinstance(q, LearnedGridTensorQuantizer):
                pass   # the range parameters take the encoding's channel count
            elif per_channel and q._num_channels != len(encoding):
                if len(encoding) != 1:
                    raise AssertionError("Number of Per Channel encodings provided (%d) is not same as number of "
                                         "channels (%d)" % (len(encoding), q._num_channels))
                if strict:
                    raise ValueError("Invalid PerChannel encodings for %s, the quantizer is a PerChannelQuantizer. "
                                     "To avoid this, disable per_channel_quantization" % name)
                q = _per_tensor_from_per_channel(q)
                self.param_quantizers[name] = q
            elif not per_channel and len(encoding) != 1:
                if strict:
                    raise ValueError("Invalid PerTensor encodings for %s, the quantizer is a PerTensorQuantizer. "
                                     "To avoid this, enable per_channel_quantization" % name)
                q = _per_channel_from_per_tensor(q, self._module_to_wrap, name)
                if q._num_channels != len(encoding):
                    raise AssertionError("Number of per channel encodings (%d) should match the number of output "
                                         "channels (%d)" % (len(encoding), q._num_channels))
                self.param_quantizers[name] = q
            if encoding[0]["dtype"] == "int":
                validate_is_symmetric_flag(q, encoding[0], strict)
                sym = encoding[0]["is_symmetric"] == "True"
                q.use_symmetric_encodings = sym
                q.use_unsigned_symmetric = q.use_unsigned_symmetric if sym else False
                q.use_strict_symmetric = q.use_strict_symmetric if sym else False
                encoding = [compute_partial_encoding(q, dict(e)) for e in encoding]
                q.bitwidth = encoding[0]["bitwidth"]
                q.encoding = [create_encoding_from_dict(e) for e in encoding]
                q.data_type = QuantizationDataType.int
            elif encoding[0]["dtype"] == "float":
                q.bitwidth = encoding[0]["bitwidth"]
                q.data_type = QuantizationDataType.float
            else:
                raise RuntimeError("Data type does not match int or float in encodings file")
            if not allow_overwrite and q.encoding is not None:
                q.freeze_encoding()

    def import_output_encodings(self, encodings: Mapping, strict: bool, partial: bool,
                                requires_grad: Optional[bool], allow_overwrite: bool):
        self._import_encoding(encodings, self.output_quantizers, strict, partial, allow_overwrite)

    def import_input_encodings(self, encodings: Mapping, strict: bool, partial: bool,
                               requires_grad: Optional[bool], allow_overwrite: bool):
        self._import_encoding(encodings, self.input_quantizers, strict, partial, allow_overwrite)

    def _import_encoding(self, encodings, quantizers, strict, partial, allow_overwrite):
        """v1/qc_quantize_op.py:620-676."""
        for i, q in enumerate(quantizers):
            if q._is_encoding_frozen:
                continue
            encoding = encodings.get(str(i), encodings.get(i, None))
            if not encoding:
                if not partial:
                    q.enabled = False
                continue
            if not q.enabled:
                if not strict:
                    continue
                raise RuntimeError("The quantsim passed for loading encodings does not have the same "
                                   "configuration as the quantsim which was used to export the encodings")
            if encoding["dtype"] == "int":
                validate_is_symmetric_flag(q, encoding, strict)
                sym = encoding["is_symmetric"] == "True"
                q.use_symmetric_encodings = sym
                q.use_unsigned_symmetric = q.use_unsigned_symmetric if sym else False
                q.use_strict_symmetric = q.use_strict_symmetric if sym else False
                enc = create_encoding_from_dict(compute_partial_encoding(q, dict(encoding)))
                q.bitwidth = enc.bw
                q.encoding = enc
                q.data_type = QuantizationDataType.int
            elif encoding["dtype"] == "float":
                q.bitwidth = encoding["bitwidth"]
                q.data_type = QuantizationDataType.float
            else:
                raise RuntimeError("Unrecognized encodings datatype")
            if not allow_overwrite and q.encoding is not None:
                q.freeze_encoding()


def _param_channel_axis(module, param):
    """v1/qc_quantize_op.py:905-911: ConvTranspose weights are quantized along axis 1."""
    if isinstance(module, (nn.ConvTranspose1d, nn.ConvTranspose2d, nn.ConvTranspose3d)) and param.dim() > 1:
        return 1
    return 0


def _per_channel_from_per_tensor(q, module, name):
    param = dict(module.named_parameters())[name]
    ax = _param_channel_axis(module, param)
    pc = StaticGridPerChannelQuantizer(q.bitwidth, q.round_mode, q.quant_scheme, q.use_symmetric_encodings,
                                       num_channels=param.shape[ax], enabled_by_default=q.enabled, ch_axis=ax,
                                       data_type=q.data_type)
    pc.use_strict_symmetric = q.use_strict_symmetric
    pc.use_unsigned_symmetric = q.use_unsigned_symmetric
    return pc


def _per_tensor_from_per_channel(q):
    pt = StaticGridPerTensorQuantizer(q.bitwidth, q.round_mode, q.quant_scheme, q.use_symmetric_encodings,
                                      enabled_by_default=q.enabled, data_type=q.data_type)
    pt.use_strict_symmetric = q.use_strict_symmetric
    pt.use_unsigned_symmetric = q.use_unsigned_symmetric
    return pt


class StaticGridQuantWrapper(QcQuantizeWrapper):
    """v1/qc_quantize_op.py:679-938."""

    def __init__(self, module_to_wrap: nn.Module, weight_bw: int, activation_bw: int, round_mode, quant_scheme,
                 is_output_quantized=True, is_symmetric=False, num_inputs=1, num_outputs=1,
                 data_type: QuantizationDataType = QuantizationDataType.int):
        round_mode = MAP_ROUND_MODE_TO_PYMO[round_mode] if isinstance(round_mode, str) else round_mode
        super().__init__(module_to_wrap, weight_bw, activation_bw, round_mode, quant_scheme, is_output_quantized,
                         is_symmetric, num_inputs, num_outputs, data_type)

    def forward(self, *inputs, **kwargs):
        """v1/qc_quantize_op.py:705-745."""
        ran = self.__dict__.get("_analysis_ran")   # QuantizationSimModel.compute_encodings is watching
        if ran is not None:
            ran[0] = True
        quantized_inputs = self._quantize_activation(self.input_quantizers, list(inputs))
        shadow_params = self._quantize_dequantize_params()
        if torch.is_grad_enabled() or not isinstance(self._module_to_wrap, _INPUT_PRESERVING_TYPES):
            quantized_inputs = SteGatingFuncForParameters.apply(self, *quantized_inputs)
            # the reference clones the custom Function's outputs (in-place ops on a view of them
            # would corrupt the gradient)
            quantized_inputs = [t.clone() if isinstance(t, torch.Tensor) else t for t in quantized_inputs]
        # else: no autograd graph is recorded and conv / linear never write to their inputs, so the
        # gating node is an identity and the clone (a full copy of every input activation: 23 GB
        # per ResNet-50 bs256 forward) changes nothing
        wrapped_output = self._module_to_wrap(*quantized_inputs, **kwargs)
        self._restore_shadow_params(shadow_params)
        if not isinstance(wrapped_output, (list, tuple)):
            wrapped_output = [wrapped_output]
        output = self._quantize_activation(self.output_quantizers, list(wrapped_output))
        return output[0] if len(output) == 1 else output

    def _restore_shadow_params(self, shadow_params):
        for name, param in self.get_named_parameters():
            if name in shadow_params:
                param.data = shadow_params[name]

    def _quantize_dequantize_params(self):
        """v1/qc_quantize_op.py:753-798. The reference saves a clone of every parameter and copies it
        back after the forward; here the fp32 original is kept by reference and the QDQ result
        (a new tensor) is swapped in for the wrapped forward -- same values, no clone / copy. A
        DataParallel replica (``_is_replica``, v1/qc_quantize_op.py:785-796) quantizes its
        broadcast copy the same way, on its own device, under _REPLICA_LOCK."""
        shadow_params = {}
        replica = getattr(self, "_is_replica", False)
        for name, param in self.get_named_parameters():
            q = self.param_quantizers[name]
            if not (q.enabled and q.bitwidth != 32):
                continue
            with _REPLICA_LOCK if replica else contextlib.nullcontext():
                if self._module_to_wrap.training or q.encoding is None:
                    q.reset_encoding_stats()
                    q.update_encoding_stats(param.data)
                    if q.quant_scheme == QuantScheme.post_training_percentile:
                        q.set_percentile_value(100)
                    q.compute_encoding()
                    if not q.enabled:
                        continue
                round_mode = q.round_mode if self.training else RoundingMode.ROUND_NEAREST
                shadow_params[name] = param.data
                param.data = q.quantize_dequantize(param.data, round_mode)
        return shadow_params

    def compute_weight_encodings(self):
        if "weight" in self.param_quantizers:
            return self.param_quantizers["weight"].encoding
        return None

    def compute_encoding(self):
        """v1/qc_quantize_op.py:811-825."""
        for q in self.input_quantizers:
            q.compute_encoding()
        for q in self.param_quantizers.values():
            q.compute_encoding()
        for q in self.output_quantizers:
            q.compute_encoding()

    def set_percentile_value(self, percentile_value: float):
        for q in list(self.input_quantizers) + list(self.output_quantizers):
            q.set_percentile_value(percentile_value)

    def _quantize_activation(self, tensor_quantizers, tensors_to_quantize):
        """v1/qc_quantize_op.py:837-897."""

        def inner(t, index):
            if isinstance(t, (list, tuple)):
                return [inner(x, index) for x in t]
            q = tensor_quantizers[index]
            if not self.should_perform_quant_dequant(t, q):
                return t
            if self._mode is QcQuantizeOpMode.ANALYSIS and not q.is_encoding_frozen:
                if TF_ENHANCED_USE_DOWNSAMPLING and q.quant_scheme == QuantScheme.post_training_tf_enhanced:
                    x = t.reshape(-1)[TF_ENHANCED_OFFSET_FACTOR::TF_ENHANCED_STRIDE_FACTOR].contiguous()
                else:
                    x = t
                batch = self.__dict__.get("_stats_batch")   # QuantizationSimModel.compute_encodings
                if batch is not None and StatsBatch.eligible(q, x):
                    batch.add(q, x, owned=x is not t and x._base is None)
                else:
                    q.update_encoding_stats(x)
                return t
            if self._mode is QcQuantizeOpMode.ACTIVE or \
                    (self._mode is QcQuantizeOpMode.ANALYSIS and q.is_encoding_frozen):
                round_mode = q.round_mode if self.training else RoundingMode.ROUND_NEAREST
                return q.quantize_dequantize(t, round_mode)
            return t

        outputs = []
        for index, t in enumerate(tensors_to_quantize):
            if len(tensor_quantizers) <= index:
                raise AssertionError("Not enough tensor quantizers (%d) allocated" % len(tensor_quantizers))
            outputs.append(inner(t, index))
        return outputs

    def enable_per_channel_quantization(self):
        """v1/qc_quantize_op.py:899-923."""
        new = {}
        for name, param in self._module_to_wrap.named_parameters():
            new[name] = _per_channel_from_per_tensor(self.param_quantizers[name], self._module_to_wrap, name)
        self.param_quantizers = new


QcPostTrainingWrapper = StaticGridQuantWrapper


class SteGatingFuncForParameters(torch.autograd.Function):
    """v1/qc_quantize_op.py:1314-1366: identity on the inputs; on the way back, gates every
    quantized parameter's gradient with the STE kernel (grad * (min <= w <= max))."""

    @staticmethod
    def forward(ctx, quant_wrapper_ref, *quantized_inputs):
        ctx.quantization_wrapper_ref = quant_wrapper_ref
        return quantized_inputs

    @staticmethod
    def backward(ctx, *output_grad):
        wrapper = ctx.quantization_wrapper_ref
        for name, param in wrapper.get_named_parameters():
            q = wrapper.param_quantizers[name]
            if q.bitwidth == 32 or q.data_type == QuantizationDataType.float:
                continue
            if q.enabled and param.grad is not None and q.encoding is not None:
                if isinstance(q.encoding, list):
                    param.grad = compute_dloss_by_dx(param, param.grad, [e.min for e in q.encoding],
                                                     [e.max for e in q.encoding], q._ch_axis)
                else:
                    param.grad = compute_dloss_by_dx(param, param.grad, q.encoding.min, q.encoding.max)
        return (None, *output_grad)


@contextlib.contextmanager
def _patched_params(module: nn.Module, patches: Dict[str, torch.Tensor]):
    """v1/qc_quantize_op.py:1369-1410 (_patch_param): inside the block ``getattr(module, name)``
    returns the quantized tensor (module.__dict__ is looked up before nn.Module.__getattr__), so
    the wrapped forward differentiates through the QDQ into the parameter and its range."""
    restore = {}
    for name, value in patches.items():
        original = getattr(module, name)
        if original.shape != value.shape:
            raise AssertionError("quantized %s has shape %s, parameter %s" % (name, value.shape, original.shape))
        # DataParallel replicas keep their broadcast parameters in module.__dict__ itself
        restore[name] = module.__dict__[name] if name in module.__dict__ else None
    try:
        module.__dict__.update(patches)
        yield
    finally:
        for name, original in restore.items():
            if original is None:
                module.__dict__.pop(name, None)
            else:
                module.__dict__[name] = original


# fuse autocast's 16-bit cast of a quantized Linear weight into the learned-grid kernels (tests
# switch it off to compare with the unfused chain)
_FUSE_AUTOCAST_CAST = True


class LearnedGridQuantWrapper(QcQuantizeWrapper):
    """v1/qc_quantize_op.py:947-1198: range learning. Every enabled quantizer's range is a pair
    of trainable parameters on the wrapper (``input0_encoding_min``, ``weight_encoding_max``, ...);
    inputs, parameters and outputs are quantize-dequantized by the fused learned-grid kernels
    (aimet_amd.learned_grid) in every mode, with gradients into the tensor and both range ends."""

    def __init__(self, module_to_wrap: nn.Module, weight_bw: int, activation_bw: int, round_mode, quant_scheme,
                 device, is_output_quantized=True, is_symmetric=False, num_inputs=1, num_outputs=1,
                 data_type: QuantizationDataType = QuantizationDataType.int):
        if data_type != QuantizationDataType.int:
            raise ValueError("Only QuantizationDataType.int is supported for LearnedGridQuantWrapper")
        round_mode = MAP_ROUND_MODE_TO_PYMO[round_mode] if isinstance(round_mode, str) else round_mode
        super().__init__(module_to_wrap, weight_bw, activation_bw, round_mode, quant_scheme, is_output_quantized,
                         is_symmetric, num_inputs, num_outputs, data_type)
        self.device = device
        self._initialize_trainable_parameters_and_tensor_quantizers(num_inputs, num_outputs)

    def _initialize_trainable_parameters_and_tensor_quantizers(self, num_inputs, num_outputs):
        """v1/qc_quantize_op.py:981-1017."""
        for kind, quantizers in (("input", self.input_quantizers), ("output", self.output_quantizers)):
            for index, q in enumerate(quantizers):
                self.register_parameter("%s%d_encoding_min" % (kind, index), None)
                self.register_parameter("%s%d_encoding_max" % (kind, index), None)
                q.name, q.wrapper_ref, q.device = "%s%d" % (kind, index), self, self.device
        for name, param in self.get_named_parameters():
            self.register_parameter(name + "_encoding_min", None)
            self.register_parameter(name + "_encoding_max", None)
            q = self.param_quantizers[name]
            q.name, q.wrapper_ref, q.device = name, self, self.device
            q._ch_axis = _param_channel_axis(self._module_to_wrap, param)

    def _ranges(self, q):
        return getattr(self, q.name + "_encoding_min"), getattr(self, q.name + "_encoding_max")

    def apply_gating_logic(self):
        """v1/qc_quantize_op.py:1019-1055."""
        quantizers = list(self.input_quantizers) + list(self.output_quantizers) + \
            [self.param_quantizers[n] for n, _ in self._module_to_wrap.named_parameters()]
        ranges = []
        for q in quantizers:
            if q.enabled and q.bitwidth != 32 and q.data_type != QuantizationDataType.float:
                emin, emax = self._ranges(q)
                if emin is not None and emax is not None:
                    ranges.append((emin, emax))
        # one launch for the wrapper's device ranges (aimet_lg_gate_ranges), the same expressions
        set_encoding_min_max_gating_threshold_many(ranges)

    def forward(self, *inputs, **kwargs):
        """v1/qc_quantize_op.py:1057-1098."""
        self.apply_gating_logic()
        quantized_inputs = self._quantize_activation(list(inputs), self.input_quantizers)
        with self._quantize_params():
            wrapped_output = self._module_to_wrap(*quantized_inputs, **kwargs)
        if not isinstance(wrapped_output, (list, tuple)):
            wrapped_output = [wrapped_output]
        output = self._quantize_activation(list(wrapped_output), self.output_quantizers)
        return output[0] if len(output) == 1 else output

    def _quantize_params(self):
        """v1/qc_quantize_op.py:1100-1127. A Linear's weight under CUDA autocast at 16 bits is
        returned already in that dtype (the cast autocast applies for the matmul, fused into the
        quantizer's kernels: see LearnedGridQuantizeDequantize)."""
        patches = {}
        cast = None
        if isinstance(self._module_to_wrap, torch.nn.Linear) and torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            cast = dt if dt in (torch.float16, torch.bfloat16) else None
        for name, param in self.get_named_parameters():
            q = self.param_quantizers[name]
            if q.enabled:
                emin, emax = self._ranges(q)
                out_dtype = cast if (name == "weight" and _FUSE_AUTOCAST_CAST and param.is_cuda) else None
                patches[name] = q.quantize_dequantize(param, emin, emax, out_dtype) if out_dtype else \
                    q.quantize_dequantize(param, emin, emax)
        return _patched_params(self._module_to_wrap, patches)

    def _quantize_activation(self, tensors_to_quantize, tensor_quantizers):
        """v1/qc_quantize_op.py:1129-1170."""

        def inner(t, index):
            if isinstance(t, (list, tuple)):
                return [inner(x, index) for x in t]
            q = tensor_quantizers[index]
            if not self.should_perform_quant_dequant(t, q):
                return t
            emin, emax = self._ranges(q)
            return q.quantize_dequantize(t, emin, emax)

        outputs = []
        for index, t in enumerate(tensors_to_quantize):
            if len(tensor_quantizers) <= index:
                raise AssertionError("Not enough tensor quantizers (%d) allocated" % len(tensor_quantizers))
            outputs.append(inner(t, index))
        return outputs

    def compute_encoding(self):
        """Range-learning quantizers are initialised from a static-grid calibration (QuantSim
        replaces the wrappers after compute_encodings); they have no statistics of their own."""

    def set_percentile_value(self, percentile_value: float):
        pass


def construct_learned_grid_wrapper(post_training_module: StaticGridQuantWrapper, weight_bw: int,
                                   activation_bw: int, round_mode, quant_scheme, device) -> LearnedGridQuantWrapper:
    """v1/quantsim.py:786-831 (_construct_and_initialize_trainable_wrapper): a LearnedGridQuantWrapper
    around the same module with every quantizer's settings and calibrated encodings copied."""
    trainable = LearnedGridQuantWrapper(post_training_module._module_to_wrap, weight_bw, activation_bw, round_mode,
                                        quant_scheme, device=device,
                                        num_inputs=len(post_training_module.input_quantizers),
                                        num_outputs=len(post_training_module.output_quantizers))
    pairs = list(zip(trainable.output_quantizers, post_training_module.output_quantizers)) + \
        list(zip(trainable.input_quantizers, post_training_module.input_quantizers)) + \
        [(trainable.param_quantizers[n], q) for n, q in post_training_module.param_quantizers.items()]
    for new, old in pairs:
        initialize_learned_grid_quantizer_attributes(new, old)
        if new.encoding_min_max_fixed_vals is not None:
            new.freeze_encoding()
    return trainable
