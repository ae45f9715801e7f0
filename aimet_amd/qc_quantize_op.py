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
from aimet_amd.libpymo import RoundingMode, TfEncoding
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


def _tensor_version(t):
    """t's autograd version counter (bumped by every in-place op on t or on any view of its
    storage), or None for an inference-mode tensor, which keeps none."""
    try:
        return t._version
    except RuntimeError:
        return None


def _default_stats_limit():
    """Elements a StatsBatch may hold: a quarter of the free device memory in float32, between
    2^24 and 2^30 (peak memory of the calibration stays bounded on a large model)."""
    try:
        free, _ = torch.cuda.mem_get_info()
    except Exception:   # noqa: BLE001 -- no device (CPU tests)
        return 1 << 30
    return max(1 << 24, min(1 << 30, free // 16))


class StatsBatch:
    """The activation statistics of QuantizationSimModel.compute_encodings' ANALYSIS forwards,
    batched: a wrapper hands (quantizer, tensor) here instead of launching the quantizer's update
    (aimet_tq_update_stats: ~4 launches and ~25 us of host time each), and flush() updates every
    pending quantizer with one AimetTensorQuantizer.updateStatsMany call per device (one launch per
    phase). Each quantizer still sees its tensors in the order the forward produced them: a second
    tensor for a pending quantizer flushes first. compute_encodings flushes when every forward of
    the model returns (end_forward) and at the end. Shared by DataParallel replicas (their wrappers'
    __dict__ is a shallow copy).

    In-place writes. The statistics must see the values the quantizer was given -- what the
    per-call update, launched at once on the stream, reads -- but the network may overwrite a
    queued tensor before the flush (nn.ReLU(inplace=True) after a folded conv, `out += identity`).
    The first forward (`learning`) therefore queues copies, and watches the originals' version
    counters: a quantizer whose tensor some op wrote in place before the flush is copied in every
    later forward; the others are queued as they are (no copy: one read of each tensor instead of
    three), and their version counters are checked at the flush. A tensor overwritten in a later
    forward but not in the first (control flow that changes between batches) raises instead of
    giving statistics of the overwritten values.

    Sharded (`group` spans several ranks): every rank passes its shard of the
    calibration batch; each flush runs the per-batch exchange of aimet_amd.distributed over the
    flushed quantizers (one all_reduce(MAX) of the packed {-min, max}, one all_reduce(SUM) of the
    packed bin and element counts), so every rank ends with the statistics of one device fed the
    whole batch. Flush points are then rank-invariant: the end of every model forward and a
    quantizer's second tensor within one forward, never an element budget (ranks holding unequal
    shards would reach it at different points); per-channel and 16-bit activations are batched too,
    so no data-dependent statistics bypass the exchange. Held memory is then one forward's queued
    activations (plus their copies in the first)."""

    def __init__(self, limit: Optional[int] = None, group=None, sharded: bool = False):
        self.limit = _default_stats_limit() if limit is None else int(limit)
        self.group = group
        self.sharded = bool(sharded)
        self.lock = threading.Lock()
        self.items = []          # (quantizer, tensor queued, channel axis, watch)
        self.pending = set()
        self.elems = 0
        self.learning = True     # the first forward: copy everything, learn who is written in place
        self.copy_ids = set()    # quantizers whose tensor the network overwrote before a flush
        self.exchange = None     # the packed exchange buffers of the last sharded flush
        self.copied = 0          # elements copied (reported by the tests)

    @staticmethod
    def eligible(q, t) -> bool:
        from aimet_amd.quantizers import StaticGridPerTensorQuantizer
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        return (type(q) is StaticGridPerTensorQuantizer and q.enabled and not q._is_encoding_frozen and
                q.bitwidth != 32 and q.data_type == QuantizationDataType.int and
                q.encoding_min_max_fixed_vals is None and isinstance(t, torch.Tensor) and t.is_cuda and
                t.dtype == torch.float32 and type(q._op()) is AimetTensorQuantizer)

    @staticmethod
    def eligible_sharded(q, t) -> bool:
        """Every quantizer whose statistics depend on this rank's data: per-tensor or per-channel,
        any floating dtype (upcast to float32, as update_encoding_stats does). The operator is
        duck-typed (the phased statistics interface of aimet_amd.distributed)."""
        from aimet_amd.quantizers import StaticGridPerChannelQuantizer, StaticGridPerTensorQuantizer
        if not (type(q) in (StaticGridPerTensorQuantizer, StaticGridPerChannelQuantizer) and q.enabled and
                not q._is_encoding_frozen and q.bitwidth != 32 and q.data_type == QuantizationDataType.int and
                q.encoding_min_max_fixed_vals is None and isinstance(t, torch.Tensor) and t.is_floating_point()):
            return False
        op = q._op()
        if not hasattr(op, "bind_exchange"):
            return False
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        if isinstance(op, AimetTensorQuantizer) and not t.is_cuda:
            raise NotImplementedError("sharded calibration exchanges device statistics: the activations of a "
                                      "QuantizationSimModel calibrated over several ranks must be on the GPU")
        return True

    def accepts(self, q, t) -> bool:
        return self.eligible_sharded(q, t) if self.sharded else self.eligible(q, t)

    def add(self, q, t, owned: bool = False):
        """Queue q's update with t (`owned`: a copy nobody else sees, e.g. the downsampled one)."""
        from aimet_amd.quantizers import StaticGridPerChannelQuantizer
        ch_axis = q.channel_axis if isinstance(q, StaticGridPerChannelQuantizer) else None
        if t.dtype != torch.float32:
            t, owned = t.to(torch.float32), True
        watch = None
        if not owned:
            ver = _tensor_version(t)
            if ver is None or self.learning or id(q) in self.copy_ids:
                if ver is not None and self.learning:
                    watch = (t, ver, True)
                t = t.clone(memory_format=torch.contiguous_format)
                self.copied += t.numel()
            else:
                watch = (t, ver, False)
        if not t.is_contiguous():
            t = t.contiguous()   # a copy of the values as they are now: nothing to watch
            watch = None
        with self.lock:
            held = t.numel() * (2 if watch is not None and watch[2] else 1)
            if id(q) in self.pending or (not self.sharded and self.elems + held > self.limit):
                self._flush_locked()
            self.items.append((q, t, ch_axis, watch))
            self.pending.add(id(q))
            self.elems += held

    def flush(self):
        with self.lock:
            self._flush_locked()

    def end_forward(self):
        """The model's forward returned: flush, and stop copying what the first forward showed
        is not written in place."""
        with self.lock:
            self._flush_locked()
            self.learning = False

    def _flush_locked(self):
        from aimet_amd.tensor_quantizer import AimetTensorQuantizer
        items, self.items, self.pending, self.elems = self.items, [], set(), 0
        overwritten = []
        for q, _, _, watch in items:
            if watch is None:
                continue
            src, ver, learning = watch
            if _tensor_version(src) != ver:
                if learning:
                    self.copy_ids.add(id(q))   # the copy was right; copy it from now on
                else:
                    overwritten.append(q)
        if overwritten:
            raise RuntimeError("compute_encodings: %d activation tensor(s) were written in place before their "
                               "statistics were taken, in a calibration forward after the first (whose in-place "
                               "writes decide which tensors are copied); the model's in-place behaviour must be "
                               "the same in every calibration forward" % len(overwritten))
        if not items:
            return
        if self.sharded:
            from aimet_amd import distributed as D
            self.exchange = D.sharded_update_stats([q._op() for q, _, _, _ in items], [t for _, t, _, _ in items],
                                                   [ax or 0 for _, _, ax, _ in items], group=self.group,
                                                   exchange=self.exchange)
            return
        by_dev = {}
        for q, t, _, _ in items:
            by_dev.setdefault(t.device, []).append((q, t))
        for dev, group in by_dev.items():
            with torch.cuda.device(dev):
                AimetTensorQuantizer.updateStatsMany([q._op() for q, _ in group], [t for _, t in group])

class ParamQdqCache:
    """The QDQ'd parameters of QuantizationSimModel.compute_encodings' ANALYSIS forwards, kept for
    the next forward while the parameter, its encoding and the rounding are unchanged (the same
    values: the reference recomputes them in every forward). Shared by the sim's wrappers and
    bounded (`limit` elements, 2^27 by default): on a model whose quantized weights exceed it --
    Llama-3-8B's 7.5 G -- the cache would hold a second copy of every weight through the whole
    calibration, and the caching allocator would keep those segments reserved afterwards (measured:
    the QAT step after such a calibration took 11 ms more); parameters past the limit are
    recomputed per forward, as the reference does."""

    def __init__(self, limit: int = 1 << 27):
        self.limit = int(limit)
        self.entries = {}
        self.elems = 0

    def get(self, owner, name, key):
        hit = self.entries.get((id(owner), name))
        return hit[1] if hit is not None and hit[0] == key else None

    def put(self, owner, name, key, value):
        self.drop(owner, name)
        if self.elems + value.numel() <= self.limit:
            self.entries[(id(owner), name)] = (key, value)
            self.elems += value.numel()

    def drop(self, owner, name):
        hit = self.entries.pop((id(owner), name), None)
        if hit is not None:
            self.elems -= hit[1].numel()


def _data_dependent(q) -> bool:
    """update_encoding_stats(t) of q reads t (not a fixed range, not a disabled / frozen / 32-bit
    quantizer, which ignore it)."""
    return (q.enabled and not q._is_encoding_frozen and q.bitwidth != 32 and
            getattr(q, "encoding_min_max_fixed_vals", None) is None)


_IGNORED_DTYPES = (torch.int8,torch.uint8, torch.int16, torch.int32, torch.int64, torch.bool)
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
        # QuantizationSimModel.compute_encodings: the QDQ'd parameters of one ANALYSIS forward are
        # reused by the next while the parameter, its encoding and the rounding are unchanged (the
        # same values: the reference recomputes them in every forward)
        cache = None if replica else self.__dict__.get("_param_qdq_cache")
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
                    if cache is not None:
                        cache.drop(self, name)
                    if not q.enabled:
                        continue
                round_mode = q.round_mode if self.training else RoundingMode.ROUND_NEAREST
                shadow_params[name] = param.data
                if cache is None:
                    param.data = q.quantize_dequantize(param.data, round_mode)
                    continue
                # TfEncoding._version moves whenever any encoding is created or assigned
                key = (param.data_ptr(), param._version, tuple(param.shape), param.dtype, id(q._encoding),
                       TfEncoding._version, int(round_mode))
                out = cache.get(self, name, key)
                if out is None:
                    out = q.quantize_dequantize(param.data, round_mode)
                    cache.put(self, name, key, out)
                param.data = out
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
                if batch is not None and batch.accepts(q, x):
                    batch.add(q, x, owned=x is not t and x._base is None)
                elif batch is not None and batch.sharded and _data_dependent(q):
                    raise NotImplementedError("sharded calibration cannot exchange the statistics of %r (tensor "
                                              "%s)" % (type(q).__name__, getattr(x, "dtype", type(x))))
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
