"""Range-learning (LearnedGrid) QAT quantize-dequantize on the fused gfx950 kernels.

Reference: ``QuantizeDequantizeFunc`` (v1/tensor_quantizer.py:896-986) over
``calculate_forward_pass`` / ``asymmetric_gradients`` / ``symmetric_gradients``
(v1/quantsim_straight_through_grad.py:121-347). The reference saves x, an uint8 x_quant and a bool
mask and runs ~10 torch kernels per tensor per step; here the forward is one kernel that saves
nothing but x, and the backward one kernel that recomputes x_round and emits grad_x plus three
per-channel sums, from which the encoding gradients are assembled on C-element vectors.

Inputs are computed in float32 (fp16/bf16 tensors are upcast; the reference keeps bf16/fp16
arithmetic for bitwidth <= 8 -- a documented difference, results are then at least as accurate).
"""
import math

import torch

from aimet_amd import _native
from aimet_amd.tensor_quantizer import _require_gpu, _stream, per_channel_view


def get_computed_encodings(bitwidth, encoding_min, encoding_max, use_symmetric_encodings, use_strict_symmetric,
                           is_unsigned_symmetric):
    """quantsim_straight_through_grad.py:121-160 (torch ops on the C-element encoding vectors)."""
    num_steps = 2 ** bitwidth - 1
    if use_symmetric_encodings and use_strict_symmetric:
        num_steps -= 1
    half_num_steps = num_steps / 2
    num_steps_tensor = torch.full_like(encoding_min, num_steps)
    if use_symmetric_encodings and not is_unsigned_symmetric:
        delta = encoding_max / torch.full_like(encoding_min, math.floor(half_num_steps))
        offset = -torch.full_like(encoding_min, math.ceil(half_num_steps))
    else:
        delta = (encoding_max - encoding_min) / num_steps_tensor
        if use_symmetric_encodings:
            offset = encoding_min / delta
        else:
            zero = torch.full_like(encoding_min, 0.)
            b_zero = torch.round(-encoding_min / delta)
            b_zero = torch.min(num_steps_tensor, torch.max(zero, b_zero))
            offset = -b_zero
    return delta, offset, num_steps_tensor


def _channels(shape, ch_axis, per_channel):
    if not per_channel:
        n = 1
        for s in shape:
            n *= s
        return 1, 1, n
    return per_channel_view(shape, ch_axis)


class LearnedGridQuantizeDequantize(torch.autograd.Function):
    """apply(tensor, encoding_min, encoding_max, bitwidth, use_symmetric, use_strict_symmetric,
    is_unsigned_symmetric, ch_axis)."""

    @staticmethod
    def forward(ctx, tensor, encoding_min, encoding_max, bitwidth, use_symmetric=False, use_strict_symmetric=False,
                is_unsigned_symmetric=False, ch_axis=0):
        if bitwidth >= 32:
            raise RuntimeError("Invalid bitwidth: %d" % bitwidth)
        _require_gpu(tensor.float() if tensor.dtype != torch.float32 else tensor, True, "tensor")
        orig_dtype = tensor.dtype
        x = tensor.to(torch.float32).contiguous()
        emin = encoding_min.detach().to(torch.float32).reshape(-1).contiguous()
        emax = encoding_max.detach().to(torch.float32).reshape(-1).contiguous()
        delta, offset, steps = get_computed_encodings(bitwidth, emin, emax, use_symmetric, use_strict_symmetric,
                                                      is_unsigned_symmetric)
        delta, offset = delta.contiguous(), offset.contiguous()
        outer, C, K = _channels(x.shape, ch_axis, emin.numel() > 1)
        if C != emin.numel():
            raise ValueError("encoding has %d channels, tensor has %d along axis %d" % (emin.numel(), C, ch_axis))
        y = torch.empty_like(x)
        with torch.cuda.device(x.device):
            _native.call("aimet_lg_forward", x.data_ptr(), y.data_ptr(), outer, C, K, delta.data_ptr(),
                         offset.data_ptr(), float(steps[0]), _stream(x))
        ctx.save_for_backward(x, delta, offset, emin, emax)
        ctx.cfg = (outer, C, K, float(steps[0]), use_symmetric, is_unsigned_symmetric, orig_dtype,
                   encoding_min.shape, encoding_max.shape)
        return y.to(orig_dtype)

    @staticmethod
    def backward(ctx, grad):
        x, delta, offset, emin, emax = ctx.saved_tensors
        outer, C, K, steps, sym, unsigned, dtype, min_shape, max_shape = ctx.cfg
        g = grad.to(torch.float32).contiguous()
        gx = torch.empty_like(g) if ctx.needs_input_grad[0] else None
        sums = torch.empty((C, 3), dtype=torch.float32, device=x.device)
        with torch.cuda.device(x.device):
            _native.call("aimet_lg_backward", x.data_ptr(), g.data_ptr(), gx.data_ptr() if gx is not None else None,
                         sums.data_ptr(), outer, C, K, delta.data_ptr(), offset.data_ptr(), steps, _stream(x))
        A, B, D = sums[:, 0], sums[:, 1], sums[:, 2]
        grad_scale_sum = A - B
        if sym:
            # symmetric_gradients: (sum((xq+off)*g) - sum(mask*(x/delta)*g)) / floor(steps/2)
            gmax = grad_scale_sum / math.floor(steps / 2)
            gmin = -gmax
        else:
            term1 = grad_scale_sum / steps
            term2 = steps / (emax - emin) ** 2 * (delta * D)
            gmin = -term1 + emax * term2
            gmax = term1 - emin * term2
        gx_out = gx.to(dtype) if gx is not None else None
        return gx_out, gmin.view(min_shape), gmax.view(max_shape), None, None, None, None, None


class LearnedGridTensorQuantizer:
    """Minimal mirror of v1 LearnedGridTensorQuantizer (v1/tensor_quantizer.py:573-893): learnable
    encoding_min / encoding_max parameters and quantize_dequantize()."""

    def __init__(self, bitwidth, use_symmetric_encodings, enabled_by_default=True, num_channels=1, ch_axis=0,
                 device="cuda"):
        self.bitwidth = bitwidth
        self.use_symmetric_encodings = use_symmetric_encodings
        self.use_strict_symmetric = False
        self.use_unsigned_symmetric = False
        self.is_unsigned_symmetric = False
        self.enabled = enabled_by_default
        self._ch_axis = ch_axis
        shape = (num_channels,) if num_channels > 1 else (1,)
        self.encoding_min = torch.nn.Parameter(torch.zeros(shape, device=device))
        self.encoding_max = torch.nn.Parameter(torch.zeros(shape, device=device))

    @property
    def channel_axis(self):
        return self._ch_axis

    def init_from(self, encodings):
        """Initialise the learnable range from computed TfEncodings (QuantSim's tf/tf-e init)."""
        with torch.no_grad():
            self.encoding_min.copy_(torch.tensor([e.min for e in encodings], dtype=torch.float32))
            self.encoding_max.copy_(torch.tensor([e.max for e in encodings], dtype=torch.float32))

    def quantize_dequantize(self, tensor, round_mode=None):
        if not self.enabled or self.bitwidth == 32:
            return tensor
        return LearnedGridQuantizeDequantize.apply(tensor, self.encoding_min, self.encoding_max, self.bitwidth,
                                                   self.use_symmetric_encodings, self.use_strict_symmetric,
                                                   self.is_unsigned_symmetric, self._ch_axis)
