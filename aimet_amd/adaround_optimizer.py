"""AdaRound per-layer rounding optimisation on the fused soft-quant kernels.

Mirrors aimet_torch/v1/adaround/adaround_optimizer.py:115-222 (AdaroundOptimizer._optimize_rounding)
with the loss of adaround_loss.py:70-133 and the hyper-parameters of AdaroundParameters
(adaround_weight.py: 10000 iterations, reg 0.01, beta 20 -> 2, warm start 0.2): Adam on alpha,
batches of 32 cached (input, fp output) pairs drawn by randperm, reconstruction loss
||q_out - fp_out||_F^2 over dim 1 averaged, rounding loss reg * sum(1 - |2h(alpha) - 1|^beta) after
the warm start with cosine-annealed beta.

MI355X-first: the soft-quantized weight is ONE kernel (aimet_adaround_forward) and its backward ONE
kernel (aimet_adaround_backward) that also adds the rounding-loss gradient -- the reference builds
both from ~16 torch ops per iteration (adaround_wrapper.py:124-149 + compute_round_loss) and runs
the rounding loss as a separate autograd graph. The rounding-loss VALUE is accumulated on the device
(no host sync per iteration) and read back only when asked.
"""
from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import ctypes

import torch
import torch.nn.functional as F

from aimet_amd import _native
from aimet_amd.adaround import AdaroundFunction, compute_beta, init_alpha
from aimet_amd.tensor_quantizer import per_channel_view

BATCH_SIZE = 32   # adaround_optimizer.py:58


@dataclass
class AdaroundHyperParameters:
    """adaround_loss.py:46-63 (defaults of AdaroundParameters, adaround_weight.py)."""
    num_iterations: int = 10000
    reg_param: float = 0.01
    beta_range: Tuple[float, float] = (20, 2)
    warm_start: float = 0.2


def layer_forward(module: torch.nn.Module, inp: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """The wrapped layer's forward with `weight` in place of its parameter
    (adaround_optimizer.py:257-286 _compute_output_with_adarounded_weights)."""
    if isinstance(module, torch.nn.Conv2d):
        return F.conv2d(inp, weight, module.bias, module.stride, module.padding, module.dilation, module.groups)
    if isinstance(module, torch.nn.Conv1d):
        return F.conv1d(inp, weight, module.bias, module.stride, module.padding, module.dilation, module.groups)
    if isinstance(module, torch.nn.Linear):
        return F.linear(inp, weight, module.bias)
    if isinstance(module, torch.nn.ConvTranspose2d):
        return F.conv_transpose2d(inp, weight, module.bias, module.stride, module.padding, module.output_padding,
                                  module.groups, module.dilation)
    raise NotImplementedError("AdaRound supports Conv1d / Conv2d / ConvTranspose2d / Linear (got %s)"
                              % type(module).__name__)


def recon_loss(quant_out: torch.Tensor, orig_out: torch.Tensor) -> torch.Tensor:
    """adaround_loss.py:70-80."""
    return (torch.norm(quant_out - orig_out, p="fro", dim=1) ** 2).mean()


class _BoundSoftQuant:
    """The per-iteration soft quantization of ONE layer with every kernel argument bound once
    (weight, alpha, delta, offset and the Wq / grad-alpha buffers keep their addresses for the
    whole optimisation): a forward and a backward are one direct library call each, no per-call
    Python argument marshalling (the loop is launch-bound for MobileNet-sized weights)."""

    def __init__(self, w, alpha, d, o, bitwidth, ch_axis, round_loss_out):
        lib = _native.load()
        self.fwd, self.bwd = lib.aimet_adaround_forward, lib.aimet_adaround_backward
        self.w, self.alpha = w.contiguous(), alpha
        outer, C, K = per_channel_view(self.w.shape, ch_axis) if d.numel() > 1 else (1, 1, self.w.numel())
        self.shape = (outer, C, K)
        self.d, self.o = d.contiguous(), o.contiguous()
        self.bw = int(bitwidth)
        self.loss = round_loss_out
        P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
        self.pw, self.pa = P(self.w), P(alpha)
        self.pd, self.po = P(self.d), P(self.o)
        self.pl = P(round_loss_out) if round_loss_out is not None else None
        self.stream = ctypes.c_void_p(torch.cuda.current_stream(self.w.device).cuda_stream)
        self.reg = self.beta = 0.0

    def forward(self):
        wq = torch.empty_like(self.w)    # fresh outputs: autograd may keep / steal them
        rc = self.fwd(self.pw, self.pa, ctypes.c_void_p(wq.data_ptr()), *self.shape, self.pd, self.po, self.bw, 1,
                      self.stream)
        if rc:
            _native.check(rc)
        return wq

    def backward(self, grad):
        g = grad if grad.is_contiguous() else grad.contiguous()
        ga = torch.empty_like(self.w)
        rc = self.bwd(self.pw, self.pa, ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(ga.data_ptr()), *self.shape,
                      self.pd, self.po, self.bw, ctypes.c_float(self.reg), ctypes.c_float(self.beta),
                      self.pl if self.reg != 0.0 else None, self.stream)
        if rc:
            _native.check(rc)
        return ga


class _SoftQuantFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, alpha, bound):
        ctx.bound = bound
        return bound.forward()

    @staticmethod
    def backward(ctx, grad):
        return ctx.bound.backward(grad), None


class AdaroundOptimizer:
    """v1/adaround/adaround_optimizer.py."""

    @staticmethod
    def optimize_rounding(module: torch.nn.Module, inp_data: torch.Tensor, out_data: torch.Tensor,
                          delta: torch.Tensor, offset: torch.Tensor, bitwidth: int, ch_axis: int = 0,
                          opt_params: AdaroundHyperParameters = AdaroundHyperParameters(),
                          act_func: Optional[Callable] = None, generator: Optional[torch.Generator] = None,
                          round_loss_out: Optional[torch.Tensor] = None) -> torch.nn.Parameter:
        """Optimises alpha for `module` on the cached activations (inp_data / out_data: [N, ...] on
        the device); returns alpha. delta / offset: the weight quantizer's (per-channel) encoding."""
        w = module.weight.detach()
        dev = w.device
        shape = [1] * w.dim()
        shape[ch_axis] = -1
        d = torch.as_tensor(delta, dtype=torch.float32, device=dev).reshape(-1)
        o = torch.as_tensor(offset, dtype=torch.float32, device=dev).reshape(-1)
        alpha = init_alpha(w, d.view(shape) if d.numel() > 1 else d)
        # one Adam kernel per step (the reference's default multi-tensor Adam: same update rule)
        try:
            optimizer = torch.optim.Adam([alpha], fused=True)
        except (RuntimeError, TypeError):
            optimizer = torch.optim.Adam([alpha])
        sq = _BoundSoftQuant(w, alpha, d, o, bitwidth, ch_axis, round_loss_out)
        n = inp_data.shape[0]
        warm = opt_params.num_iterations * opt_params.warm_start
        for it in range(opt_params.num_iterations):
            idx = torch.randperm(n, generator=generator)[:BATCH_SIZE].to(dev, non_blocking=True)
            inp = inp_data.index_select(0, idx)
            target = out_data.index_select(0, idx)
            optimizer.zero_grad()
            if it < warm:
                sq.reg, sq.beta = 0.0, 0.0
            else:
                sq.reg = opt_params.reg_param
                sq.beta = compute_beta(opt_params.num_iterations, it, opt_params.beta_range, opt_params.warm_start)
            wq = _SoftQuantFn.apply(alpha, sq)
            q_out = layer_forward(module, inp, wq)
            if act_func is not None:
                q_out, target = act_func(q_out), act_func(target)
            recon_loss(q_out, target).backward()   # + the rounding-loss gradient, fused in the kernel
            optimizer.step()
        return alpha

    @staticmethod
    def hard_rounded_weight(module: torch.nn.Module, alpha: torch.Tensor, delta, offset, bitwidth: int,
                            ch_axis: int = 0) -> torch.Tensor:
        """The adarounded weight: hard rounding h = (alpha >= 0) (adaround_wrapper.py:124-149 with
        use_soft_rounding False)."""
        w = module.weight.detach()
        d = torch.as_tensor(delta, dtype=torch.float32, device=w.device).reshape(-1)
        o = torch.as_tensor(offset, dtype=torch.float32, device=w.device).reshape(-1)
        with torch.no_grad():
            return AdaroundFunction.apply(w, alpha.detach(), d, o, bitwidth, ch_axis, False)
