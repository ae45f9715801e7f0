"""AdaRound soft rounding on the fused gfx950 kernels.

Reference: v1/adaround/adaround_wrapper.py:124-149 (apply_adaround, ~6 torch kernels forward and
~10 backward per iteration) and v1/adaround/adaround_loss.py:83-133 (rounding loss, beta
annealing). Here the forward is one kernel (W, alpha -> Wq) and the backward one kernel
(grad_Wq, W, alpha -> grad_alpha) that also folds in the rounding-loss gradient and value.
"""
import math

import torch

from aimet_amd import _native
from aimet_amd.tensor_quantizer import _require_gpu, _stream, per_channel_view

ZETA = 1.1     # aimet_common/defs.py:305
GAMMA = -0.1   # aimet_common/defs.py:304


def set_exact_pow(exact: bool):
    """The rounding loss's pow for every AdaRound backward launched afterwards (process-wide,
    aimet_adaround_set_exact_pow): False (default) the table-driven f32 pow, within 1 ulp of torch's CPU pow
    (Sleef powf_u10) over every f32 input in (0, 1) and the AdaRound beta schedules
    (profiles/r06/pow_fast_check.txt); True the bit-exact emulation of torch's pow, about 3x the
    arithmetic. Returns the previous setting."""
    prev = get_exact_pow()
    _native.call("aimet_adaround_set_exact_pow", int(bool(exact)))
    return prev


def get_exact_pow() -> bool:
    import ctypes
    v = ctypes.c_int(0)
    _native.call("aimet_adaround_get_exact_pow", ctypes.byref(v))
    return bool(v.value)


def _channel_vec(v, C, device):
    v = torch.as_tensor(v, dtype=torch.float32, device=device).reshape(-1)
    if v.numel() == 1 and C != 1:
        v = v.expand(C)
    if v.numel() != C:
        raise ValueError("expected %d per-channel values, got %d" % (C, v.numel()))
    return v.contiguous()


class AdaroundFunction(torch.autograd.Function):
    """Wq = (clamp(floor(W/delta) + h(alpha) - offset, 0, 2^bw-1) + offset) * delta.

    apply(weight, alpha, delta, offset, bitwidth, ch_axis, use_soft_rounding=True, reg_param=0.0,
          beta=0.0, round_loss_out=None). delta/offset: scalars or per-channel vectors along ch_axis.
    With reg_param != 0 the backward adds d/dalpha of reg*sum(1-|2h-1|^beta) and accumulates that
    loss into round_loss_out (a 1-element float32 tensor)."""

    @staticmethod
    def forward(ctx, weight, alpha, delta, offset, bitwidth, ch_axis=0, use_soft_rounding=True, reg_param=0.0,
                beta=0.0, round_loss_out=None):
        _require_gpu(weight, True, "weight")
        w = weight.contiguous()
        a = alpha.detach().to(torch.float32).contiguous()
        outer, C, K = per_channel_view(w.shape, ch_axis)
        if torch.as_tensor(delta).numel() == 1:
            outer, C, K = 1, 1, w.numel()
        d = _channel_vec(delta, C, w.device)
        o = _channel_vec(offset, C, w.device)
        wq = torch.empty_like(w)
        with torch.cuda.device(w.device):
            _native.call("aimet_adaround_forward", w.data_ptr(), a.data_ptr(), wq.data_ptr(), outer, C, K,
                         d.data_ptr(), o.data_ptr(), int(bitwidth), int(bool(use_soft_rounding)), _stream(w))
        ctx.save_for_backward(w, a, d, o)
        ctx.shape = (outer, C, K)
        ctx.bw = int(bitwidth)
        ctx.reg = float(reg_param)
        ctx.beta = float(beta)
        ctx.loss_out = round_loss_out
        return wq

    @staticmethod
    def backward(ctx, grad):
        w, a, d, o = ctx.saved_tensors
        g = grad.contiguous().to(torch.float32)
        ga = torch.empty_like(a)
        outer, C, K = ctx.shape
        loss = ctx.loss_out
        with torch.cuda.device(w.device):
            _native.call("aimet_adaround_backward", w.data_ptr(), a.data_ptr(), g.data_ptr(), ga.data_ptr(), outer, C,
                         K, d.data_ptr(), o.data_ptr(), ctx.bw, ctx.reg, ctx.beta,
                         loss.data_ptr() if (loss is not None and ctx.reg != 0.0) else None, _stream(w))
        return None, ga, None, None, None, None, None, None, None, None


def round_loss_and_grad(alpha, reg_param, beta):
    """reg * sum(1 - |2h(alpha)-1|^beta) and its gradient w.r.t. alpha (adaround_loss.py:83-110),
    computed by the fused backward kernel with a zero reconstruction gradient."""
    _require_gpu(alpha, True, "alpha")
    a = alpha.contiguous()
    zeros = torch.zeros_like(a)
    ga = torch.empty_like(a)
    loss = torch.zeros(1, dtype=torch.float32, device=a.device)
    one = torch.ones(1, dtype=torch.float32, device=a.device)
    with torch.cuda.device(a.device):
        _native.call("aimet_adaround_backward", zeros.data_ptr(), a.data_ptr(), zeros.data_ptr(), ga.data_ptr(), 1, 1,
                     a.numel(), one.data_ptr(), zeros.data_ptr(), 8, float(reg_param), float(beta),
                     loss.data_ptr(), _stream(a))
    return loss[0], ga


def compute_beta(max_iter, cur_iter, beta_range, warm_start):
    """adaround_loss.py:112-133 (cosine decay)."""
    assert cur_iter < max_iter, "Current iteration should be less than total maximum number of iterations."
    start_beta, end_beta = beta_range
    warm_start_end_iter = warm_start * max_iter
    rel_iter = (cur_iter - warm_start_end_iter) / (max_iter - warm_start_end_iter)
    return end_beta + 0.5 * (start_beta - end_beta) * (1 + math.cos(rel_iter * math.pi))


def init_alpha(weight, delta):
    """adaround_wrapper.py:211-224 _generate_alpha_parameter (torch float32 ops)."""
    floor = torch.floor(weight / delta)
    rest = (weight / delta) - floor
    alpha = -torch.log((ZETA - GAMMA) / (rest - GAMMA) - 1)
    return torch.nn.Parameter(alpha.float(), requires_grad=True)
