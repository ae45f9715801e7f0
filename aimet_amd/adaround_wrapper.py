"""AdaroundWrapper: the reference's soft-rounding wrapper around a quantized layer, on the fused
gfx950 AdaRound kernels.

Reference: aimet_torch/v1/adaround/adaround_wrapper.py:55-224 (AdaroundWrapperBase,
AdaroundWrapper). Same constructor (a QcQuantizeWrapper whose weight quantizer holds an encoding),
attributes (module_to_wrap, alpha, broadcasted_delta / broadcasted_offset, bitwidth,
use_soft_rounding, clip_min / clip_max) and methods (forward, get_original_module,
apply_adaround, _generate_alpha_parameter, _get_weight_quantizer_delta_and_offset, ...).

apply_adaround is ONE kernel (aimet_adaround_forward) with ONE backward kernel for d/d(alpha)
(AdaroundFunction), where the reference runs ~6 torch kernels forward and ~10 backward. The
arithmetic is the reference's: Wq bit-exact against its apply_adaround (tests/golden/
golden_adaround.npz), the sigmoid in Sleef expf_u10 form as torch's. A float32 weight is computed
as is; a 16-bit weight is upcast, computed in float32 and cast back (the reference computes in the
weight's dtype: results at least as accurate, documented difference).
"""
import abc
import contextlib
from typing import Tuple

import torch

from aimet_amd.adaround import GAMMA, ZETA, AdaroundFunction
from aimet_amd.quantizers import MAP_QUANT_SCHEME_TO_PYMO, StaticGridPerChannelQuantizer
from aimet_amd.tensor_quantizer import AimetTensorQuantizer


def broadcast_to_tensor(tensor, encoding, ch_axis):
    """quantsim_straight_through_grad.py:66-88: a 1-element encoding stays as is, a per-channel one
    is viewed with `tensor`'s rank, its channels along ch_axis."""
    if not isinstance(encoding, torch.Tensor):
        encoding = torch.tensor(encoding).to(tensor.device)
    assert len(encoding.shape) <= 1
    if encoding.numel() == 1:
        return encoding
    assert encoding.numel() == tensor.shape[ch_axis]
    return encoding.view(tuple(d if a == ch_axis else 1 for a, d in enumerate(tensor.shape)))


@contextlib.contextmanager
def _patch_attr(module, name, value):
    """aimet_torch.v2.utils.patch_attr / _patch_param_or_buffer (v2/utils.py:113-181): for the
    scope, module.__dict__[name] shadows the parameter held in module._parameters."""
    orig = getattr(module, name)
    if orig is not None:
        assert value.shape == orig.shape
    in_dict = name in module.__dict__
    if not in_dict and name not in module._parameters and name not in module._buffers:
        raise RuntimeError("'%s' is not a valid name of parameter of buffer of %s." % (name, type(module)))
    module.__dict__[name] = value
    try:
        yield
    finally:
        if in_dict:
            module.__dict__[name] = orig
        else:
            module.__dict__.pop(name, None)


class AdaroundWrapperBase(abc.ABC, torch.nn.Module):
    """adaround_wrapper.py:55-91."""

    @abc.abstractmethod
    def forward(self, *args, **kwargs):
        """Apply adaround and run forward function of the wrapped module."""

    @abc.abstractmethod
    def get_original_module(self) -> torch.nn.Module:
        """The original module (its type and weight)."""

    @abc.abstractmethod
    def apply_adaround(self, tensor: torch.Tensor) -> torch.Tensor:
        """Apply adaround to the input tensor."""

    @property
    def weight(self) -> torch.Tensor:
        return getattr(self.get_original_module(), self.weight_name)

    @property
    def weight_name(self) -> str:
        return "weight"


class AdaroundWrapper(AdaroundWrapperBase):
    """adaround_wrapper.py:93-224: AdaRound of a QcQuantizeWrapper's weight."""

    def __init__(self, module):
        super().__init__()
        assert self.weight_name in module.param_quantizers
        self.module_to_wrap = module
        self._init_param()

    def forward(self, *args, **kwargs):
        """adaround_wrapper.py:104-117: the wrapped module's forward with the adarounded weight in
        place of its parameter and its weight quantizer disabled."""
        original = self.get_original_module()
        weight = self.weight
        if self._is_weight_quantizer_enabled():
            weight = self.apply_adaround(weight)
        with self._disable_weight_quantizer(), _patch_attr(original, self.weight_name, weight):
            return self.module_to_wrap.forward(*args, **kwargs)

    def get_original_module(self) -> torch.nn.Module:
        return self.module_to_wrap._module_to_wrap

    def apply_adaround(self, tensor: torch.Tensor) -> torch.Tensor:
        """adaround_wrapper.py:124-149 as one fused kernel (soft rounding: the rectified sigmoid of
        alpha; hard rounding: alpha >= 0); differentiable w.r.t. alpha."""
        input_dtype = tensor.dtype
        w = tensor if tensor.dtype == torch.float32 else tensor.float()
        alpha = self.alpha if self.alpha.device == w.device else self.alpha.to(w.device)
        delta, offset = self._delta_vec.to(w.device), self._offset_vec.to(w.device)
        out = AdaroundFunction.apply(w, alpha, delta, offset, self.bitwidth, self._ch_axis, self.use_soft_rounding)
        return out.to(input_dtype)

    @contextlib.contextmanager
    def _disable_weight_quantizer(self):
        q = self.module_to_wrap.param_quantizers[self.weight_name]
        enabled = q.enabled
        q.enabled = False
        try:
            yield
        finally:
            q.enabled = enabled

    def _is_weight_quantizer_enabled(self) -> bool:
        return self.module_to_wrap.param_quantizers[self.weight_name].enabled

    def _get_weight_quantizer_channel_axis(self) -> int:
        q = self.module_to_wrap.param_quantizers[self.weight_name]
        if isinstance(q, StaticGridPerChannelQuantizer):
            return q._ch_axis
        return 0

    def _get_weight_quantizer_delta_and_offset(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """adaround_wrapper.py:179-193: per-channel encodings -> makeDeltaOffsetTensor (float32
        vectors on the weight's device), per-tensor -> the encoding's delta / offset; broadcast
        along the channel axis."""
        q = self.module_to_wrap.param_quantizers[self.weight_name]
        if isinstance(q.encoding, list):
            op = AimetTensorQuantizer(MAP_QUANT_SCHEME_TO_PYMO[q.quant_scheme])
            delta, offset = op.makeDeltaOffsetTensor(self.weight.device, q.encoding)
        else:
            delta, offset = q.encoding.delta, q.encoding.offset
        ch_axis = self._get_weight_quantizer_channel_axis()
        return broadcast_to_tensor(self.weight, delta, ch_axis), broadcast_to_tensor(self.weight, offset, ch_axis)

    def _get_weight_quantizer_bitwidth(self) -> int:
        return self.module_to_wrap.param_quantizers[self.weight_name].bitwidth

    def _init_param(self):
        """adaround_wrapper.py:201-209."""
        self.broadcasted_delta, self.broadcasted_offset = self._get_weight_quantizer_delta_and_offset()
        self.alpha = self._generate_alpha_parameter(self.weight, self.broadcasted_delta)
        self.bitwidth = self._get_weight_quantizer_bitwidth()
        self.use_soft_rounding = True
        self.clip_max = 2 ** self.bitwidth - 1
        self.clip_min = 0
        # the kernel's operands: float32 per-channel vectors (one element: per tensor) + the axis
        self._ch_axis = self._get_weight_quantizer_channel_axis()
        self._delta_vec = torch.as_tensor(self.broadcasted_delta, dtype=torch.float32).reshape(-1)
        self._offset_vec = torch.as_tensor(self.broadcasted_offset, dtype=torch.float32).reshape(-1)

    @staticmethod
    def _generate_alpha_parameter(tensor: torch.Tensor, delta: torch.Tensor) -> torch.nn.Parameter:
        """adaround_wrapper.py:211-224 (the reference's torch ops; alpha kept in float32)."""
        tensor_floor = torch.floor(tensor / delta)
        tensor = (tensor / delta) - tensor_floor
        alpha = -torch.log((ZETA - GAMMA) / (tensor - GAMMA) - 1)
        return torch.nn.Parameter(alpha.float(), requires_grad=True)
