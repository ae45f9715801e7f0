"""QuantizationSimModel for the MI355X core: wraps a model's quantizable layers, calibrates them
(compute_encodings) and exports / loads encodings.

Mirrors aimet_torch/v1/quantsim.py (QuantizationSimModel :170-1043, compute_encodings :381-449,
_export_encodings_to_files :940-1043, load_encodings :1696-1838) for the hot path of §8: the
calibration loop (ANALYSIS mode: every quantizer's updateStats on the device, no host sync), the
encoding computation (batched: one device search launch + one sync per setting instead of one
per quantizer) and the ACTIVE fake-quant forward.

Deliberately narrower than the reference (SURVEY §8 marks the rest out of scope):
  * the quantizable layers are the modules of `quantizable_types` (default: conv / conv-transpose /
    linear), each with an output quantizer, a weight quantizer (bias unquantized) and an input
    quantizer enabled for the first layer only -- the reference's default config
    (aimet_common/quantsim_config/default_config.json) without connected-graph supergroups;
  * `config_file` accepts the defaults section of that JSON schema (params is_symmetric,
    strict_symmetric, unsigned_symmetric, per_channel_quantization) as a path or a dict;
  * export writes the PyTorch-named `<prefix>_torch.encodings` file; the ONNX-named
    `<prefix>.encodings` needs an ONNX export of the model, which is outside this core.
"""
import contextlib
import copy
import json
import os
import pickle
from typing import Any, Callable, Dict, List, Optional, Union

import torch
from torch import nn

from aimet_amd.qc_quantize_op import (QUANTIZER_TYPE_INPUT, QUANTIZER_TYPE_OUTPUT, LearnedGridQuantWrapper,
                                      ParamQdqCache, QcQuantizeOpMode, QcQuantizeWrapper, StaticGridQuantWrapper,
                                      StatsBatch,
                                      construct_learned_grid_wrapper)
from aimet_amd.quantizers import QuantizationDataType, QuantScheme, compute_encodings_batched

ENCODING_VERSION = "0.6.1"
DEFAULT_QUANTIZABLE_TYPES = (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.ConvTranspose1d, nn.ConvTranspose2d,
                             nn.ConvTranspose3d, nn.Linear)

_SCHEME_NAMES = {"tf": QuantScheme.post_training_tf, "tf_enhanced": QuantScheme.post_training_tf_enhanced,
                 "percentile": QuantScheme.post_training_percentile}
_RANGE_LEARNING = (QuantScheme.training_range_learning_with_tf_init,
                   QuantScheme.training_range_learning_with_tf_enhanced_init)


def get_v1_quant_scheme_for_initialization(quant_scheme: QuantScheme) -> QuantScheme:
    """aimet_torch/utils.py:1199-1212: range learning is initialised by a TF / TF-E calibration."""
    if quant_scheme == QuantScheme.training_range_learning_with_tf_init:
        return QuantScheme.post_training_tf
    if quant_scheme == QuantScheme.training_range_learning_with_tf_enhanced_init:
        return QuantScheme.post_training_tf_enhanced
    return quant_scheme


def _model_device(model):
    """aimet_torch/utils.py get_device: the device of the first parameter (CPU without any)."""
    for p in model.parameters():
        return p.device
    return torch.device("cpu")


def _truthy(v):
    return v if isinstance(v, bool) else str(v) == "True"


def _load_config(config_file) -> Dict:
    # no config file: the reference's default_config.json (params symmetric, per-tensor)
    cfg = {"param_symmetric": True, "act_symmetric": False, "strict_symmetric": False,
           "unsigned_symmetric": False, "per_channel_quantization": False, "param_symmetric_given": True}
    if config_file is None:
        return cfg
    cfg["param_symmetric_given"] = False
    if isinstance(config_file, (str, os.PathLike)):
        with open(config_file) as f:
            config_file = json.load(f)
    d = config_file.get("defaults", {})
    if "is_symmetric" in d.get("params", {}):
        cfg["param_symmetric"] = _truthy(d["params"]["is_symmetric"])
        cfg["param_symmetric_given"] = True
    if "is_symmetric" in d.get("ops", {}):
        cfg["act_symmetric"] = _truthy(d["ops"]["is_symmetric"])
    for k in ("strict_symmetric", "unsigned_symmetric", "per_channel_quantization"):
        if k in d:
            cfg[k] = _truthy(d[k])
    return cfg


def _count_inputs(model, dummy_input, types):
    """The positional input count of every module of `types` in a forward on `dummy_input`: the
    wrapper's input quantizer count, from one forward with hooks as the reference does
    (v1/quantsim.py:282-283, 2202-2215; aimet_torch/utils.py:768 get_inout_tensor_shape_per_module).
    Modules the forward does not reach keep one (v1/quantsim.py:1409-1410)."""
    counts = {}

    def pre(m, args):
        counts[id(m)] = max(counts.get(id(m), 1), len(args))
    hooks = [m.register_forward_pre_hook(pre) for m in model.modules() if isinstance(m, types)]
    try:
        with _eval_mode(model), torch.no_grad():
            if isinstance(dummy_input, (list, tuple)):
                model(*dummy_input)
            else:
                model(dummy_input)
    finally:
        for h in hooks:
            h.remove()
    return counts


@contextlib.contextmanager
def _eval_mode(model):
    was = model.training
    model.eval()
    try:
        yield
    finally:
        model.train(was)


class QuantizationSimModel:
    """v1/quantsim.py:170."""

    def __init__(self, model: nn.Module, dummy_input=None,
                 quant_scheme: Union[str, QuantScheme] = QuantScheme.post_training_tf_enhanced,
                 rounding_mode: str = "nearest", default_output_bw: int = 8, default_param_bw: int = 8,
                 in_place: bool = False, config_file=None,
                 default_data_type: QuantizationDataType = QuantizationDataType.int,
                 quantizable_types=DEFAULT_QUANTIZABLE_TYPES):
        if isinstance(quant_scheme, str):
            quant_scheme = _SCHEME_NAMES[quant_scheme]
        if default_data_type != QuantizationDataType.int:
            raise NotImplementedError("float (fp8/fp16) quantization is outside the MI355X integer QDQ core")
        self.model = model if in_place else copy.deepcopy(model)
        self._quant_scheme = quant_scheme
        self._rounding_mode = rounding_mode
        self._default_output_bw = default_output_bw
        self._default_param_bw = default_param_bw
        self._percentile_value = 100
        self._cfg = _load_config(config_file)
        self._excluded_layer_names = []
        self._last_calibration = None
        n_inputs = _count_inputs(self.model, dummy_input, quantizable_types) if dummy_input is not None else {}
        first = True
        for parent_name, parent in list(self.model.named_modules()):
            for child_name, child in list(parent.named_children()):
                if isinstance(child, quantizable_types) and not isinstance(child, QcQuantizeWrapper):
                    w = StaticGridQuantWrapper(child, default_param_bw, default_output_bw, rounding_mode,
                                               get_v1_quant_scheme_for_initialization(quant_scheme),
                                               is_output_quantized=True,
                                               is_symmetric=self._cfg["act_symmetric"],
                                               num_inputs=n_inputs.get(id(child), 1))
                    for pname, pq in w.param_quantizers.items():
                        pq.use_symmetric_encodings = self._cfg["param_symmetric"]
                        if pname == "bias":
                            pq.enabled = False
                    if self._cfg["per_channel_quantization"]:
                        w.enable_per_channel_quantization()
                    for q in self._quantizers_of(w):
                        q.use_strict_symmetric = self._cfg["strict_symmetric"]
                        q.use_unsigned_symmetric = self._cfg["unsigned_symmetric"]
                    if first:
                        w.enable_input_quantizers(True)   # model_input: is_input_quantized
                        first = False
                    setattr(parent, child_name, w)
        if dummy_input is not None:
            self._run_passthrough(dummy_input)

    # -- helpers --------------------------------------------------------------------------------
    @staticmethod
    def _quantizers_of(w):
        return list(w.input_quantizers) + list(w.param_quantizers.values()) + list(w.output_quantizers)

    def quant_wrappers(self):
        for name, m in self.model.named_modules():
            if isinstance(m, QcQuantizeWrapper):
                yield name, m

    def _run_passthrough(self, dummy_input):
        """Checks the wrapped model runs on the dummy input (no statistics are collected)."""
        for _, w in self.quant_wrappers():
            w.set_mode(QcQuantizeOpMode.PASSTHROUGH)
        with _eval_mode(self.model), torch.no_grad():
            if isinstance(dummy_input, (list, tuple)):
                self.model(*dummy_input)
            else:
                self.model(dummy_input)

    def set_percentile_value(self, percentile_value: float):
        """v1/quantsim.py:361-372."""
        if self._quant_scheme != QuantScheme.post_training_percentile:
            raise ValueError("set_percentile_value() can only be called with the percentile quant scheme")
        self._percentile_value = percentile_value

    # -- calibration ------------------------------------------------------------------------------
    def compute_encodings(self, forward_pass_callback: Callable[[nn.Module, Any], Any],
                          forward_pass_callback_args: Any = None, *, process_group=None,
                          sharded: Optional[bool] = None):
        """v1/quantsim.py:381-449: reset, ANALYSIS forward(s), encodings, ACTIVE; range-learning
        schemes then swap in the trainable wrappers (v1/quantsim.py:423, 833-846).

        The resets of every static-grid quantizer are one batched call, the parameter encodings the
        first ANALYSIS forward would compute wrapper by wrapper (a statistics launch, a device search
        and a synchronisation per parameter, v1/qc_quantize_op.py:753-798) are computed for every
        wrapper at once beforehand (_precompute_param_encodings: the same encodings, since the
        parameters do not change during the forwards), the QDQ'd parameters of one forward are
        reused by the next, and the activation statistics of each forward are launched together
        when the model's forward returns (StatsBatch: the same statistics, every quantizer updated
        in its own order).

        Sharded calibration (the reference calibrates on one device only,
        Docs/api_docs/torch_multi_gpu.rst): when torch.distributed is initialised with more than
        one rank in `process_group` (default: the world), every rank runs the callback on ITS
        shard of the calibration data, and each forward's activation statistics are exchanged --
        one all_reduce(MAX) of the packed batch min/max and one all_reduce(SUM) of the packed
        histogram and element counts per forward, over RCCL -- so that every rank ends with the
        encodings of one device fed every rank's samples. Every rank must then call
        compute_encodings and run the same number of model forwards. `sharded=False` keeps the
        reference's behaviour (each rank calibrates on its own data alone), e.g. to calibrate on
        one rank only; `sharded=True` insists on a process group."""
        from aimet_amd import distributed as D
        world = D._world(process_group)
        if sharded is None:
            sharded = world > 1
        elif sharded and not (torch.distributed.is_available() and torch.distributed.is_initialized()):
            raise RuntimeError("sharded calibration needs an initialised torch.distributed process group")
        wrappers = [w for _, w in self.quant_wrappers()]
        _reset_many(wrappers)
        for w in wrappers:
            w.set_mode(QcQuantizeOpMode.ANALYSIS)
            if self._quant_scheme == QuantScheme.post_training_percentile:
                w.set_percentile_value(self._percentile_value)
        with _eval_mode(self.model), torch.no_grad():
            pre = _precompute_param_encodings(wrappers)
            batch = StatsBatch(group=process_group, sharded=bool(sharded))
            static = [w for w in wrappers if isinstance(w, StaticGridQuantWrapper)]
            qdq_cache = ParamQdqCache()
            for w in static:
                w.__dict__["_stats_batch"] = batch
                w.__dict__["_param_qdq_cache"] = qdq_cache
            hook = self.model.register_forward_hook(lambda *_: batch.end_forward())
            try:
                forward_pass_callback(self.model, forward_pass_callback_args)
                batch.flush()
            finally:
                hook.remove()
                for w in static:
                    w.__dict__.pop("_stats_batch", None)
                    w.__dict__.pop("_param_qdq_cache", None)
                _forget_unused_param_encodings(pre)
                # what the calibration copied / exchanged (reported by the tests and bench.py)
                self._last_calibration = {"sharded": batch.sharded, "world": world, "copied_elements": batch.copied,
                                          "copied_quantizers": len(batch.copy_ids)}
        # every activation / param quantizer of the model in one batched native call per setting
        # range-learning wrappers keep their trained ranges (they have no statistics)
        quantizers = [q for _, w in self.quant_wrappers() if not isinstance(w, LearnedGridQuantWrapper)
                      for q in self._quantizers_of(w)]
        compute_encodings_batched(quantizers)
        for _, w in self.quant_wrappers():
            w.set_mode(QcQuantizeOpMode.ACTIVE)
        self.replace_wrappers_for_quantize_dequantize()

    def replace_wrappers_for_quantize_dequantize(self):
        """v1/quantsim.py:833-846, 764-831: every StaticGridQuantWrapper becomes a
        LearnedGridQuantWrapper initialised from its calibrated encodings (range-learning schemes)."""
        if self._quant_scheme not in _RANGE_LEARNING:
            return
        device = _model_device(self.model)
        for parent_name, parent in list(self.model.named_modules()):
            for child_name, child in list(parent.named_children()):
                if isinstance(child, StaticGridQuantWrapper):
                    setattr(parent, child_name, construct_learned_grid_wrapper(
                        child, self._default_param_bw, self._default_output_bw, self._rounding_mode,
                        self._quant_scheme, device))

    def __call__(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    # -- export / import --------------------------------------------------------------------------
    def get_encodings_dict(self) -> Dict:
        """The `<prefix>_torch.encodings` content (v1/quantsim.py:884-938, 1031-1043)."""
        activation, params = {}, {}
        for name, w in self.quant_wrappers():
            for kind, encs in ((QUANTIZER_TYPE_INPUT, w.export_input_encodings()),
                               (QUANTIZER_TYPE_OUTPUT, w.export_output_encodings())):
                for i, e in enumerate(encs):
                    if e is not None:
                        activation.setdefault(name, {}).setdefault(kind, {})[str(i)] = e[0]
            for pname, e in w.export_param_encodings().items():
                if e is not None:
                    params["%s.%s" % (name, pname)] = e
        return {"version": ENCODING_VERSION, "activation_encodings": activation, "param_encodings": params,
                "excluded_layers": list(self._excluded_layer_names),
                "quantizer_args": self.quant_args}

    @property
    def quant_args(self) -> Dict:
        """aimet_common/quantsim.py:280-310 extract_global_quantizer_args (v1/quantsim.py:295): the
        scheme's name (range learning reports its init scheme), default bitwidths, dtype, the
        params' is_symmetric (the per-channel setting when the config does not give it) and
        per_channel_quantization."""
        scheme = self._quant_scheme
        if scheme == QuantScheme.training_range_learning_with_tf_init:
            scheme = QuantScheme.post_training_tf
        elif scheme == QuantScheme.training_range_learning_with_tf_enhanced_init:
            scheme = QuantScheme.post_training_tf_enhanced
        per_channel = self._cfg["per_channel_quantization"]
        return {"quant_scheme": scheme.name, "param_bitwidth": self._default_param_bw,
                "activation_bitwidth": self._default_output_bw, "dtype": "int",
                "is_symmetric": self._cfg["param_symmetric"] if self._cfg["param_symmetric_given"] else per_channel,
                "per_channel_quantization": per_channel}

    def exclude_layers_from_quantization(self, layers_to_exclude: List[nn.Module]):
        """v1/quantsim.py:731-751: every quantization wrapper inside the given layers is replaced by
        its original module; the wrappers' names are recorded as the excluded layers."""
        names = {m: n for n, m in self.model.named_modules()}
        wrappers = []
        for layer in layers_to_exclude:
            for m in layer.modules():
                if isinstance(m, QcQuantizeWrapper):
                    wrappers.append(m)
                    self._excluded_layer_names.append(names.get(m))

        def strip(parent):
            for child_name, child in list(parent.named_children()):
                if any(child is w for w in wrappers):
                    setattr(parent, child_name, child.get_original_module())
                else:
                    strip(child)
        strip(self.model)

    def export(self, path: str, filename_prefix: str, dummy_input=None):
        """Writes `<path>/<prefix>_torch.encodings` (JSON) and the model state dict
        (`<prefix>.pth`, weights unquantized as in v1/quantsim.py:455-520)."""
        os.makedirs(path, exist_ok=True)
        enc_path = os.path.join(path, filename_prefix + "_torch.encodings")
        with open(enc_path, "w") as f:
            json.dump(self.get_encodings_dict(), f, sort_keys=True, indent=4)
        torch.save(self._original_state_dict(), os.path.join(path, filename_prefix + ".pth"))
        return enc_path

    def _original_state_dict(self):
        sd = self.model.state_dict()
        return {k.replace("._module_to_wrap", ""): v for k, v in sd.items()}

    def load_encodings(self, encodings: Union[Dict, str, os.PathLike], strict: bool = True, partial: bool = True,
                       requires_grad: Optional[bool] = None, allow_overwrite: bool = True):
        """v1/quantsim.py:1696-1838."""
        if isinstance(encodings, (str, os.PathLike)):
            with open(encodings) as f:
                encodings = json.load(f)
        if "param_encodings" not in encodings:
            param_encodings, activation_encodings = encodings, {}
        else:
            param_encodings = encodings.get("param_encodings", {})
            activation_encodings = encodings.get("activation_encodings", {})
        if not param_encodings and not activation_encodings:
            raise RuntimeError("the encodings contain neither parameter nor activation encodings")
        if strict:
            keys = set(param_encodings) | set(activation_encodings)
            model_keys = {n.replace("._module_to_wrap", "") for n, _ in self.model.named_modules()} | \
                         {n.replace("._module_to_wrap", "") for n, _ in self.model.named_parameters()}
            missing = keys - model_keys
            if missing:
                raise RuntimeError("Encoding dictionary contains modules/parameters that doesn't exist in the "
                                   "model: " + ", ".join(sorted(missing)))
        for name, w in self.quant_wrappers():
            penc = {p: param_encodings["%s.%s" % (name, p)] for p in w.param_quantizers
                    if "%s.%s" % (name, p) in param_encodings}
            try:
                w.import_param_encodings(penc, strict, partial, requires_grad, allow_overwrite)
                entry = activation_encodings.get(name, {})
                w.import_input_encodings(entry.get(QUANTIZER_TYPE_INPUT, {}), strict, partial, requires_grad,
                                         allow_overwrite)
                w.import_output_encodings(entry.get(QUANTIZER_TYPE_OUTPUT, {}), strict, partial, requires_grad,
                                          allow_overwrite)
            except RuntimeError as e:
                raise RuntimeError("Encoding import failed for module: %s.\n%s" % (name, e)) from e
        for _, w in self.quant_wrappers():
            w.set_mode(QcQuantizeOpMode.ACTIVE)

    def load_and_freeze_encodings(self, encoding_path: str, ignore_when_quantizer_disabled: bool = False):
        self.load_encodings(encoding_path, strict=not ignore_when_quantizer_disabled, partial=True,
                            requires_grad=False, allow_overwrite=False)

    # -- the unwrapped model (v1/quantsim.py:1490-1575) -----------------------------------------
    @classmethod
    def _remove_quantization_wrappers(cls, starting_module: nn.Module, list_of_modules_to_exclude):
        """v1/quantsim.py:1490-1517: every wrapper among `list_of_modules_to_exclude` below
        `starting_module` is replaced by the module it wraps."""
        for name, child in list(starting_module.named_children()):
            if any(child is m for m in list_of_modules_to_exclude) and isinstance(child, QcQuantizeWrapper):
                child = child.get_original_module()
                setattr(starting_module, name, child)
            cls._remove_quantization_wrappers(child, list_of_modules_to_exclude)

    @classmethod
    def get_original_model(cls, model: nn.Module, qdq_weights: bool = False) -> nn.Module:
        """v1/quantsim.py:1519-1534: a deep copy of `model` with every quantization wrapper removed;
        with `qdq_weights` the copy's parameters are first replaced by their quantize-dequantized
        values. `model` itself is not changed."""
        original = copy.deepcopy(model)
        if qdq_weights:
            cls._apply_qdq_to_model_parameters(original)
        cls._remove_quantization_wrappers(original, list(original.modules()))
        return original

    @classmethod
    @torch.no_grad()
    def _apply_qdq_to_model_parameters(cls, model: nn.Module):
        """v1/quantsim.py:1536-1552: every wrapper's parameters become their quantize-dequantized
        values (eval mode: nearest rounding, no recalibration of calibrated weights)."""
        for m in model.modules():
            if isinstance(m, (StaticGridQuantWrapper, LearnedGridQuantWrapper)):
                was = m.training
                m.eval()
                try:
                    if isinstance(m, StaticGridQuantWrapper):
                        m._quantize_dequantize_params()   # leaves the QDQ values in param.data
                    else:
                        with m._quantize_params():
                            patched = {n: m._module_to_wrap.__dict__[n] for n, _ in m.get_named_parameters()
                                       if n in m._module_to_wrap.__dict__}
                        for n, p in m._module_to_wrap.named_parameters():
                            if n in patched:
                                p.data = patched[n].detach().to(p.dtype)
                finally:
                    m.train(was)


def save_checkpoint(quant_sim_model: QuantizationSimModel, file_path: str):
    """v1/quantsim.py:2216-2227: the whole sim pickled. Quantizers travel with their encodings and
    settings; their device statistics do not (as the reference's C++ ops, they are rebuilt empty)."""
    with open(file_path, "wb") as f:
        pickle.dump(quant_sim_model, f)


def load_checkpoint(file_path: str) -> QuantizationSimModel:
    """v1/quantsim.py:2230-2240: a new QuantizationSimModel from a save_checkpoint file. Like the
    reference this unpickles the file, so load only checkpoints you wrote yourself."""
    with open(file_path, "rb") as f:
        return pickle.load(f)


def load_encodings_to_sim(quant_sim_model: QuantizationSimModel, pytorch_encoding_path: str):
    """v1/quantsim.py:2278."""
    quant_sim_model.load_encodings(pytorch_encoding_path, strict=True, partial=False, requires_grad=None,
                                   allow_overwrite=None)


# -- compute_encodings helpers ----------------------------------------------------------------------
def _static_quantizers(w):
    return list(w.input_quantizers) + list(w.param_quantizers.values()) + list(w.output_quantizers)


def _reset_many(wrappers):
    """w.reset_encodings() of every wrapper (StaticGridTensorQuantizer.reset_encoding_stats of each
    quantizer) with the native resets of all static-grid quantizers in one batched call."""
    from aimet_amd.quantizers import StaticGridTensorQuantizer
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    ops = []
    for w in wrappers:
        if not isinstance(w, StaticGridQuantWrapper):
            w.reset_encodings()
            continue
        for q in _static_quantizers(w):
            if type(q).reset_encoding_stats is not StaticGridTensorQuantizer.reset_encoding_stats or \
                    type(q._op()) is not AimetTensorQuantizer:
                q.reset_encoding_stats()
            elif not q._is_encoding_frozen:
                ops.append(q._op())
                q._encoding = None
    if ops:
        AimetTensorQuantizer.resetEncodingStatsMany(ops)


def _precompute_param_encodings(wrappers):
    """What the first ANALYSIS forward does for every parameter of an eval-mode StaticGridQuantWrapper
    whose quantizer has no encoding (v1/qc_quantize_op.py:753-798: reset, statistics of param.data,
    percentile 100 for the percentile scheme, compute_encoding), for all of them at once: the
    per-tensor statistics in one launch per phase, the per-channel ones in two launches, the
    encodings in one search per setting (compute_encodings_batched). The wrapper's forward then
    finds the encodings set and quantizes with them, as after its own computation. Returns what
    was precomputed, so that the encodings of wrappers the forwards never ran can be dropped
    again (_forget_unused_param_encodings): the reference computes them only in a forward."""
    from aimet_amd.quantizers import StaticGridPerChannelQuantizer, StaticGridPerTensorQuantizer
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    items = []
    for w in wrappers:
        if type(w) is not StaticGridQuantWrapper or w._module_to_wrap.training:
            continue
        for name, param in w.get_named_parameters():
            q = w.param_quantizers[name]
            if not (q.enabled and q.bitwidth != 32) or q.encoding is not None or q._is_encoding_frozen:
                continue
            if type(q) not in (StaticGridPerTensorQuantizer, StaticGridPerChannelQuantizer) or \
                    q.data_type != QuantizationDataType.int or q.encoding_min_max_fixed_vals is not None or \
                    not param.is_cuda or param.dtype != torch.float32:
                continue   # the wrapper computes these itself in the forward
            items.append((w, q, param.data))
    if not items:
        return []
    per_tensor = [(q, t) for _, q, t in items if type(q) is StaticGridPerTensorQuantizer]
    per_channel = [(q, t) for _, q, t in items if type(q) is StaticGridPerChannelQuantizer]
    AimetTensorQuantizer.resetEncodingStatsMany([q._op() for _, q, _ in items])
    keep = []
    by_dev = {}
    for q, t in per_tensor:
        by_dev.setdefault(t.device, []).append((q, t))
    for dev, group in by_dev.items():
        with torch.cuda.device(dev):
            keep.append(AimetTensorQuantizer.updateStatsMany([q._op() for q, _ in group],
                                                             [t.contiguous() for _, t in group]))
    by_dev = {}
    for q, t in per_channel:
        by_dev.setdefault(t.device, []).append((q, t))
    for dev, group in by_dev.items():
        with torch.cuda.device(dev):
            keep.append(AimetTensorQuantizer.updateStatsPerChannelMany([q._op() for q, _ in group],
                                                                       [t for _, t in group],
                                                                       [q.channel_axis for q, _ in group]))
    enabled = [q.enabled for _, q, _ in items]
    percentile = [None] * len(items)
    for i, (_, q, _) in enumerate(items):
        if q.quant_scheme == QuantScheme.post_training_percentile:
            percentile[i] = q._op().getPercentileValue()
            q.set_percentile_value(100)
        q._encoding = None
    compute_encodings_batched([q for _, q, _ in items])
    del keep
    # a one-element list: DataParallel replicas copy the wrapper's __dict__ shallowly, so a replica's
    # forward marks the same list
    for w in {id(w): w for w, _, _ in items}.values():
        w.__dict__["_analysis_ran"] = [False]
    return [(w, q, (e, p)) for (w, q, _), e, p in zip(items, enabled, percentile)]


def _forget_unused_param_encodings(pre):
    """The parameter encodings precomputed for wrappers that no ANALYSIS forward ran: back to the
    reset state the reference leaves them in (no statistics, no encoding, enabled and percentile
    as before)."""
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    unused = [(w, q, e) for w, q, e in pre if not w.__dict__.get("_analysis_ran", [True])[0]]
    if unused:
        AimetTensorQuantizer.resetEncodingStatsMany([q._op() for _, q, _ in unused])
        for _, q, (e, p) in unused:
            q._encoding = None
            q.enabled = e
            if p is not None:
                q.set_percentile_value(p)
    for w, _, _ in pre:
        w.__dict__.pop("_analysis_ran", None)
