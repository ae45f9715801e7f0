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
(no host sync per iteration) and read back only when asked. The reconstruction loss and its backward
(~12 torch kernels over the layer output) are one pass too (aimet_adaround_recon_grad).

The loop is launch-bound for MobileNet-sized layers, so by default one iteration is captured in a
HIP graph and replayed (batch indices drawn up front in the eager loop's order, the annealed beta
read from device memory, Adam capturable); depthwise convolutions run on PyTorch's native kernels
(3-5x faster than MIOpen's here). MobileNet-v2, 53 layers: 0.47 ms -> 0.19 ms per iteration.

Data parallel (adaround_optimizer.py:139-160,214-216), when torch.distributed is initialised (or a
group is given): the cached samples are sharded rank::world, Adam's learning rate is multiplied by
the world size, each rank runs num_iterations // world iterations on batches from its shard, and
alpha.grad is all-reduced (SUM) and divided by the world size before every Adam step. As in the
reference, the rounding-loss schedule keeps num_iterations as its horizon (so with world > 1 the
iterations run are the first 1/world of it). In the HIP-graph form the iteration is two graphs with
the collective between them: [forward + backward] -> all_reduce(alpha.grad) -> [/ world + Adam].
"""
import contextlib
import logging
import warnings
from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import ctypes

import torch
import torch.distributed as dist
import torch.nn.functional as F

from aimet_amd import _native
from aimet_amd.adaround import AdaroundFunction, compute_beta, init_alpha
from aimet_amd.tensor_quantizer import per_channel_view

BATCH_SIZE = 32   # adaround_optimizer.py:58
_log = logging.getLogger("aimet_amd.adaround")


@dataclass
class AdaroundHyperParameters:
    """adaround_loss.py:46-63 (defaults of AdaroundParameters, adaround_weight.py)."""
    num_iterations: int = 10000
    reg_param: float = 0.01
    beta_range: Tuple[float, float] = (20, 2)
    warm_start: float = 0.2


def layer_forward(module: torch.nn.Module, inp: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """The wrapped layer's forward with `weight` in place of its parameter
    (adaround_optimizer.py:257-286 _compute_output_with_adarounded_weights). The bias enters
    detached: only alpha is optimised, so its gradient (a reduction over the whole layer output
    per iteration) is never needed."""
    bias = module.bias.detach() if module.bias is not None else None
    if isinstance(module, torch.nn.Conv2d):
        return F.conv2d(inp, weight, bias, module.stride, module.padding, module.dilation, module.groups)
    if isinstance(module, torch.nn.Conv1d):
        return F.conv1d(inp, weight, bias, module.stride, module.padding, module.dilation, module.groups)
    if isinstance(module, torch.nn.Linear):
        return F.linear(inp, weight, bias)
    if isinstance(module, torch.nn.ConvTranspose2d):
        return F.conv_transpose2d(inp, weight, bias, module.stride, module.padding, module.output_padding,
                                  module.groups, module.dilation)
    raise NotImplementedError("AdaRound supports Conv1d / Conv2d / ConvTranspose2d / Linear (got %s)"
                              % type(module).__name__)


@contextlib.contextmanager
def conv_backend(module: torch.nn.Module):
    """Context for a layer's whole iteration (forward AND autograd backward, which picks its
    backend when it runs): depthwise convolutions on PyTorch's native depthwise kernels, 3-5x
    faster than MIOpen's for the forward + weight gradient at MobileNet-v2 shapes on MI355X
    (tools/studies/dw_conv_time.py); MIOpen restricted to deterministic solutions (its weight-gradient
    kernels may add partial sums atomically: the optimised alpha of two runs with one seed then
    differed, tools/studies/adaround_loop_divergence.py)."""
    depthwise = isinstance(module, torch.nn.Conv2d) and 1 < module.groups == module.in_channels
    prev, prev_det = torch.backends.cudnn.enabled, torch.backends.cudnn.deterministic
    torch.backends.cudnn.enabled = prev and not depthwise
    torch.backends.cudnn.deterministic = True
    try:
        yield
    finally:
        torch.backends.cudnn.enabled = prev
        torch.backends.cudnn.deterministic = prev_det


# The loop's forms are fixed rules by layer shape, never timings, so two runs with the same seed give
# the same alpha. The module-level switches below select between forms that the tests compare
# (tests/test_adaround_wrapper.py patches them); none is read from the environment.

# 1x1 convolutions and linear layers of the fused AdaRound loop as direct GEMMs (torch.matmul /
# hipBLASLt) instead of MIOpen convolutions through autograd
_GEMM_LAYERS = True
# 1x1 / linear layers have two loop forms that sum the weight gradient in different orders (GEMM or
# MIOpen convolution through autograd), so the optimised alpha depends on the form: "gemm" (the
# rule) or "autograd" (the convolution form, the GEMM form's fallback when it cannot be captured)
_LOOP_FORM = "gemm"
# the pointwise / im2col weight gradient: "bmm" (per-sample GEMMs + a sum over the batch) or "mm"
# (one GEMM over (n, hw) from channel-major copies); "auto" takes mm for spatial sizes <= 64
# (MobileNet-v2's 7x7 layers: up to 0.047 ms per iteration less) and bmm above
# (profiles/r03/adaround_pw_grad_forms.txt)
_PW_GRAD = "auto"
# depthwise layers: the whole iteration up to dL/dWq as one pass over the cached rows
# (aimet_adaround_dw_step, bit-identical to gather + forward + reconstruction gradient + weight
# gradient); False runs those four launches instead (the tests' comparison)
_DW_FUSED = True
# the depthwise / 1x1 one-pass steps' weight-gradient slices folded by the Adam step
# (aimet_adaround_backward_adam_parts with part_kk: the folds' sums, one launch fewer per iteration)
_DW_FOLD_ADAM = True
# 1x1 layers / the unfolded stem with few input channels (Cin <= 192, HW % 4 == 0)
# can run the iteration up to dL/dWq as one pass too (aimet_adaround_pw_step: q, g and the gradient
# partials on chip; sums in a fixed order, not a library GEMM's). "auto" (default) takes it for every
# eligible layer with >= 28 x 28 positions except the projecting ones (C_in > C_out) below 56 x 56,
# where the GEMM form measured faster (MobileNet-v2 per iteration: 0.24 -> 0.16 ms at 16 -> 96 x
# 112^2, 0.127 -> 0.088 at 24 -> 144 x 56^2, the stem 0.172 -> 0.133; 192 -> 32 x 28^2: 0.074 vs
# 0.092; 64 -> 384 x 14^2: 0.064 vs 0.076; profiles/r03/adaround_pw_fused_forms.txt). Since the step
# runs on the matrix cores for C_in >= 32 (round 4), the projecting layers at 28 x 28 with C_in >= 32
# take it too (144 -> 32: 0.073 -> 0.056 ms, 192 -> 32: 0.070 -> 0.067; profiles/r04/
# adaround_pw_fused_all.txt) when the step does run them on the matrix cores
# (aimet_adaround_pw_step_uses_mfma; the VALU form is slower than the GEMM form there); below 28 x 28
# the channel-major GEMMs stay faster. "all": every eligible layer, "0": none.
_PW_FUSED = "auto"
# the GEMM form of 1x1 layers with channel-major batches (aimet_adaround_gather_cm: x as [C_in][nb hw],
# so q = W x and dL/dW = g x^T are ONE GEMM each, no per-sample GEMMs, batch sum or transposes), for
# layers of <= 14 x 14 positions (MobileNet-v2: 0.117 -> 0.063 ms per iteration at 576 -> 96 x 14^2;
# slower at 28^2: 0.071 -> 0.09); False: the [nb][C][hw] batches with per-sample GEMMs (_PW_GRAD)
# everywhere. (The same form on the f32 matrix cores in two kernels of our own, and the weight
# gradient as split-K GEMM slices, measured slower and are not in the library:
# tools/studies/pw_cm_mfma.hip, profiles/r04/pw_cm_*.jsonl.)
_PW_CM = True
# iterations per captured HIP graph in the single-process loop: one hipGraphLaunch per iteration
# left the GPU waiting on the host between replays for small layers (a depthwise layer's ~10 us of
# kernels per iteration in a ~100 us window, profiles/r04/adaround_loop_summary.txt); the counters and
# the batch table live on the device, so k consecutive iterations are one graph. Results are those
# of one iteration per graph, bit for bit.
_GRAPH_ITERS = 10


def _pw_step_uses_mfma(cin: int, cout: int) -> bool:
    """aimet_adaround_pw_step runs (cin, cout) on the matrix cores (else its VALU form)."""
    uses = ctypes.c_int()
    _native.call("aimet_adaround_pw_step_uses_mfma", int(cin), int(cout), ctypes.byref(uses))
    return bool(uses.value)


def _is_pointwise(module: torch.nn.Module) -> bool:
    return isinstance(module, torch.nn.Conv2d) and module.kernel_size == (1, 1) and module.stride == (1, 1) \
        and module.padding in ((0, 0), "valid") and module.dilation == (1, 1) and module.groups == 1


# im2col form of small-Cin convolutions (the stem): C_in * k * k at most this, and the unfolded
# input cache at most this many bytes
_IM2COL_MAX_K = 64
_IM2COL_MAX_BYTES = 8 << 30


def _im2col_ok(module: torch.nn.Module, inp_data: torch.Tensor) -> bool:
    """A groups-1 Conv2d (not 1x1 / stride 1, which _is_pointwise runs directly) whose
    C_in * kh * kw <= _IM2COL_MAX_K and whose unfolded input cache fits _IM2COL_MAX_BYTES: its
    loop runs as the pointwise form on the unfolded cache (deterministic GEMMs; MIOpen's
    deterministic stem solutions were 4x slower than its default ones)."""
    if not isinstance(module, torch.nn.Conv2d) or module.groups != 1 or _is_pointwise(module) \
            or module.padding_mode != "zeros" or isinstance(module.padding, str) or inp_data.dim() != 4:
        return False
    kdim = module.in_channels * module.kernel_size[0] * module.kernel_size[1]
    if kdim > _IM2COL_MAX_K:
        return False
    h, w = inp_data.shape[2], inp_data.shape[3]
    oh = (h + 2 * module.padding[0] - module.dilation[0] * (module.kernel_size[0] - 1) - 1) // module.stride[0] + 1
    ow = (w + 2 * module.padding[1] - module.dilation[1] * (module.kernel_size[1] - 1) - 1) // module.stride[1] + 1
    return inp_data.shape[0] * kdim * oh * ow * inp_data.element_size() <= _IM2COL_MAX_BYTES


def depthwise_spec(module: torch.nn.Module):
    """(K, stride, padding, dilation) when `module` is a depthwise Conv2d the native depthwise
    kernels (aimet_dwconv2d_*) run: groups == in == out channels, square K in {3, 5}, square
    stride / padding / dilation, zero padding; else None."""
    if not isinstance(module, torch.nn.Conv2d) or not (module.groups == module.in_channels == module.out_channels) \
            or module.groups == 1 or module.padding_mode != "zeros" or isinstance(module.padding, str):
        return None
    (kh, kw), (sh, sw), (ph, pw), (dh, dw) = module.kernel_size, module.stride, module.padding, module.dilation
    if kh != kw or kh not in (3, 5) or sh != sw or ph != pw or dh != dw:
        return None
    return kh, sh, ph, dh


def recon_loss(quant_out: torch.Tensor, orig_out: torch.Tensor) -> torch.Tensor:
    """adaround_loss.py:70-80."""
    return (torch.norm(quant_out - orig_out, p="fro", dim=1) ** 2).mean()


def _act_code(act_func) -> Optional[int]:
    """The fused reconstruction-loss kernel's activation code, None when it has no fused form."""
    if act_func is None:
        return 0
    if isinstance(act_func, torch.nn.ReLU6) or act_func is F.relu6:
        return 2
    if isinstance(act_func, torch.nn.ReLU) or act_func in (F.relu, torch.relu):
        return 1
    return None


def recon_loss_backward(quant_out: torch.Tensor, orig_out: torch.Tensor, act_func=None):
    """recon_loss(act(quant_out), act(orig_out)).backward() as ONE kernel (aimet_adaround_recon_grad:
    the gradient 2 (act(q) - act(t)) act'(q) / count, then autograd from quant_out on); other
    activations take the torch-op form."""
    code = _act_code(act_func)
    if code is None or quant_out.dtype != torch.float32 or quant_out.dim() < 2:
        q, t = (act_func(quant_out), act_func(orig_out)) if act_func is not None else (quant_out, orig_out)
        recon_loss(q, t).backward()
        return
    q = quant_out.detach()
    q = q if q.is_contiguous() else q.contiguous()
    t = orig_out if orig_out.is_contiguous() else orig_out.contiguous()
    g = torch.empty_like(q)
    _native.call("aimet_adaround_recon_grad", q.data_ptr(), t.data_ptr(), g.data_ptr(), q.numel(), q.shape[1], code,
                 torch.cuda.current_stream(q.device).cuda_stream)
    quant_out.backward(g)


class _BoundSoftQuant:
    """The per-iteration soft quantization of ONE layer with every kernel argument bound once
    (weight, alpha, delta, offset and the Wq / grad-alpha buffers keep their addresses for the
    whole optimisation): a forward and a backward are one direct library call each, no per-call
    Python argument marshalling (the loop is launch-bound for MobileNet-sized weights)."""

    def __init__(self, w, alpha, d, o, bitwidth, ch_axis, round_loss_out):
        lib = _native.load()
        self.fwd, self.bwd = lib.aimet_adaround_forward, lib.aimet_adaround_backward
        self.bwd_dev = lib.aimet_adaround_backward_dev
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
        self.reg = self.beta = 0.0
        self.reg_beta = None   # graph mode: device tensor [reg, beta, beta - 1] read by the backward kernel

    def _stream(self):
        # the current stream at call time: a HIP-graph capture runs on torch's capture stream
        return ctypes.c_void_p(torch.cuda.current_stream(self.w.device).cuda_stream)

    def forward(self):
        wq = torch.empty_like(self.w)    # fresh outputs: autograd may keep / steal them
        rc = self.fwd(self.pw, self.pa, ctypes.c_void_p(wq.data_ptr()), *self.shape, self.pd, self.po, self.bw, 1,
                      self._stream())
        if rc:
            _native.check(rc)
        return wq

    def backward(self, grad):
        g = grad if grad.is_contiguous() else grad.contiguous()
        ga = torch.empty_like(self.w)
        if self.reg_beta is not None:
            rc = self.bwd_dev(self.pw, self.pa, ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(ga.data_ptr()),
                              *self.shape, self.pd, self.po, self.bw, ctypes.c_void_p(self.reg_beta.data_ptr()),
                              self.pl, self._stream())
        else:
            rc = self.bwd(self.pw, self.pa, ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(ga.data_ptr()),
                          *self.shape, self.pd, self.po, self.bw, ctypes.c_double(self.reg), ctypes.c_double(self.beta),
                          self.pl if self.reg != 0.0 else None, self._stream())
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


def _group_world(group):
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _reduce_grad(grad, world, group, divide=True):
    """adaround_optimizer.py:214-216: all_reduce(alpha.grad) (SUM), then / world_size."""
    if world > 1:
        if grad.is_cuda and dist.get_backend(group) == "gloo":
            h = grad.cpu()
            dist.all_reduce(h, group=group)
            grad.copy_(h)
        else:
            dist.all_reduce(grad, group=group)
    if divide:
        grad.div_(world)


def _starting_alpha(w, d, shape, alpha_init):
    """The optimised alpha: a float32 copy of the caller's (an AdaroundWrapper's parameter) or
    init_alpha of the weight (_generate_alpha_parameter, adaround_wrapper.py:211-224)."""
    if alpha_init is not None:
        if alpha_init.shape != w.shape:
            raise ValueError("alpha has shape %s, the weight %s" % (tuple(alpha_init.shape), tuple(w.shape)))
        return torch.nn.Parameter(alpha_init.detach().to(w.device, torch.float32).contiguous().clone(),
                                  requires_grad=True)
    return init_alpha(w, d.view(shape) if d.numel() > 1 else d)


def _finish_alpha(alpha, alpha_init):
    """The optimised values written back into the caller's alpha (returned), else alpha."""
    if alpha_init is None:
        return alpha
    with torch.no_grad():
        alpha_init.copy_(alpha.detach())
    return alpha_init


class AdaroundOptimizer:
    """v1/adaround/adaround_optimizer.py."""

    last_loop_form = None   # the layer form the last fused loop ran (dw / pointwise / im2col / linear / autograd)
    is_activation_caching_enabled = True

    # ---- the reference's caller surface (v1/adaround/adaround_optimizer.py:69-260) -------------
    @classmethod
    def adaround_module(cls, module: torch.nn.Module, quant_module, orig_model: torch.nn.Module,
                        quant_model: torch.nn.Module, act_func, cached_dataset, forward_fn,
                        opt_params: AdaroundHyperParameters, cached_quant_dataset=None):
        """adaround_optimizer.py:69-113: the reconstruction metrics before / after (debug log),
        the rounding optimisation of `quant_module` (an AdaroundWrapper), then hard rounding."""
        from aimet_amd.activation_sampler import ActivationSampler
        from aimet_amd.adaround_wrapper import AdaroundWrapper
        assert isinstance(quant_module, AdaroundWrapper), "%s is not adaround wrapper module." % quant_module
        sampler = ActivationSampler(module, quant_module, orig_model, quant_model, forward_fn)
        if cached_quant_dataset:
            inp_data, _ = sampler.sample_acts(cached_quant_dataset[0], collect_input=True, collect_output=False)
            _, out_data = sampler.sample_acts(cached_dataset[0], collect_input=False, collect_output=True)
        else:
            inp_data, out_data = sampler.sample_acts(cached_dataset[0])
        hard, soft = cls._compute_recons_metrics(quant_module, act_func, inp_data, out_data)
        _log.debug("Before opt, Recons. error metrics using soft rounding=%f and hard rounding=%f", soft, hard)
        cls._optimize_rounding(module, quant_module, orig_model, quant_model, act_func, cached_dataset, forward_fn,
                               opt_params, cached_quant_dataset)
        hard, soft = cls._compute_recons_metrics(quant_module, act_func, inp_data, out_data)
        _log.debug("After opt, Recons. error metrics using soft rounding=%f and hard rounding=%f", soft, hard)
        quant_module.use_soft_rounding = False

    @classmethod
    def _optimize_rounding(cls, module: torch.nn.Module, quant_module, orig_model: torch.nn.Module,
                           quant_model: torch.nn.Module, act_func, cached_dataset, forward_fn,
                           opt_params: AdaroundHyperParameters, cached_quant_dataset=None):
        """adaround_optimizer.py:115-221 over the fused loop (optimize_rounding): the cached
        dataset sharded by batch rank::world as the reference's Subset, every batch's layer input
        (QuantSim model) and output (original model) sampled into HBM, then num_iterations // world
        iterations of Adam (lr 1e-3 x world) on quant_module.alpha with batches of 32 drawn by
        torch.randperm from the global generator, alpha.grad all-reduced / world."""
        from aimet_amd.activation_sampler import ActivationSampler
        from aimet_amd.adaround_wrapper import AdaroundWrapper
        rank, world = _group_world(None)
        indices = range(rank, len(cached_dataset), world)
        shard = [cached_dataset[i] for i in indices]
        shard_q = [cached_quant_dataset[i] for i in indices] if cached_quant_dataset is not None else None
        assert isinstance(quant_module, AdaroundWrapper), "%s is not adaround wrapper module." % quant_module
        assert quant_module.use_soft_rounding, "optimization should use soft rounding only."
        assert quant_module.alpha is not None, "alpha parameter should be initialized."
        original = quant_module.get_original_module()
        device = original.weight.device
        sampler = ActivationSampler(module, quant_module, orig_model, quant_model, forward_fn)
        inp_data, out_data = sampler.sample_all_acts(shard, shard_q, device=device)
        cls.optimize_rounding(original, inp_data, out_data, quant_module._delta_vec.to(device),
                              quant_module._offset_vec.to(device), quant_module.bitwidth, quant_module._ch_axis,
                              opt_params, act_func, generator=None, alpha=quant_module.alpha, presharded=True)

    @classmethod
    def _compute_recons_metrics(cls, quant_module, act_func, inp_data: torch.Tensor,
                                out_data: torch.Tensor) -> Tuple[float, float]:
        """adaround_optimizer.py:223-255: (MSE with hard rounding, MSE with soft rounding)."""
        with torch.no_grad():
            quant_module.use_soft_rounding = False
            out_hard = cls._compute_output_with_adarounded_weights(quant_module, inp_data)
            quant_module.use_soft_rounding = True
            out_soft = cls._compute_output_with_adarounded_weights(quant_module, inp_data)
            if act_func is not None:
                out_data, out_soft, out_hard = act_func(out_data), act_func(out_soft), act_func(out_hard)
            return float(F.mse_loss(out_hard, out_data)), float(F.mse_loss(out_soft, out_data))

    @staticmethod
    def _compute_output_with_adarounded_weights(quant_module, inp_data: torch.Tensor):
        """adaround_optimizer.py:257-286."""
        module = quant_module.get_original_module()
        quant_module.to(inp_data.device)
        if not isinstance(module, (torch.nn.Conv2d, torch.nn.ConvTranspose2d, torch.nn.Linear)):
            raise ValueError("AdaRound is not supported for the module: ", module)
        weight = quant_module.apply_adaround(quant_module.weight)
        if isinstance(module, torch.nn.Conv2d):
            return F.conv2d(inp_data, weight, bias=module.bias, stride=module.stride, dilation=module.dilation,
                            padding=module.padding, groups=module.groups)
        if isinstance(module, torch.nn.ConvTranspose2d):
            return F.conv_transpose2d(inp_data, weight, bias=module.bias, stride=module.stride,
                                      padding=module.padding, output_padding=module.output_padding,
                                      groups=module.groups, dilation=module.dilation)
        return F.linear(inp_data, weight, bias=module.bias)

    @staticmethod
    def enable_caching_acts_data() -> bool:
        """adaround_optimizer.py:340-349: the samples are always cached here (in HBM)."""
        return AdaroundOptimizer.is_activation_caching_enabled

    @staticmethod
    def optimize_rounding(module: torch.nn.Module, inp_data: torch.Tensor, out_data: torch.Tensor,
                          delta: torch.Tensor, offset: torch.Tensor, bitwidth: int, ch_axis: int = 0,
                          opt_params: AdaroundHyperParameters = AdaroundHyperParameters(),
                          act_func: Optional[Callable] = None, generator: Optional[torch.Generator] = None,
                          round_loss_out: Optional[torch.Tensor] = None, use_graph: bool = True,
                          group=None, alpha: Optional[torch.Tensor] = None,
                          presharded: bool = False) -> torch.nn.Parameter:
        """Optimises alpha for `module` on the cached activations (inp_data / out_data: [N, ...] on
        the device); returns alpha. delta / offset: the weight quantizer's (per-channel) encoding.

        use_graph: the iteration is captured once in a HIP graph and replayed num_iterations times
        (the batch indices of every iteration drawn up front from `generator` in the same order as
        the eager loop, the annealed beta read from device memory by the backward kernel, Adam in
        its capturable form); the loop is launch-bound for MobileNet-sized layers.

        group: the process group to run data parallel over (default: the default group when
        torch.distributed is initialised); see the module docstring.

        alpha: the starting alpha (an AdaroundWrapper's parameter, adaround_wrapper.py:211-224);
        it is updated in place and returned. Default: init_alpha of the weight.
        presharded: inp_data / out_data already hold only this rank's samples (adaround_module
        shards the cached dataset by batch, as the reference does)"""
        rank, world = _group_world(group)
        if world > 1 and not presharded:
            # adaround_optimizer.py:147-150: this rank's shard of the cached samples
            shard = torch.arange(rank, inp_data.shape[0], world, device=inp_data.device)
            inp_data, out_data = inp_data.index_select(0, shard), out_data.index_select(0, shard)
        args = (module, inp_data, out_data, delta, offset, bitwidth, ch_axis, opt_params, act_func, generator,
                round_loss_out, world, group, alpha)
        if opt_params.num_iterations // world == 0:
            # fewer iterations than ranks (or none): the loop runs zero times and alpha keeps its
            # initial value, as the reference's range() loop does -- no batch draw, no capture
            use_graph = False
        with conv_backend(module):
            if use_graph:
                rng = generator.get_state() if generator is not None else torch.get_rng_state()
                loss0 = round_loss_out.clone() if round_loss_out is not None else None
                try:
                    return AdaroundOptimizer._optimize_graphed(*args)
                except RuntimeError as e:   # a layer whose iteration cannot be captured: same loop, eager
                    warnings.warn("AdaRound: HIP-graph capture failed for %s (%s); running the loop eagerly"
                                  % (type(module).__name__, e))
                    torch.cuda.synchronize()
                    if generator is not None:
                        generator.set_state(rng)
                    else:
                        torch.set_rng_state(rng)
                    if round_loss_out is not None:
                        round_loss_out.copy_(loss0)
            return AdaroundOptimizer._optimize_eager(*args)

    @staticmethod
    def _optimize_eager(module, inp_data, out_data, delta, offset, bitwidth, ch_axis, opt_params, act_func,
                        generator, round_loss_out, world=1, group=None, alpha_init=None):
        w = module.weight.detach()
        dev = w.device
        shape = [1] * w.dim()
        shape[ch_axis] = -1
        d = torch.as_tensor(delta, dtype=torch.float32, device=dev).reshape(-1)
        o = torch.as_tensor(offset, dtype=torch.float32, device=dev).reshape(-1)
        alpha = _starting_alpha(w, d, shape, alpha_init)
        # one Adam kernel per step (the reference's default multi-tensor Adam: same update rule); the
        # learning rate scaled by the world size (adaround_optimizer.py:155-158)
        lr = 1e-3 * world
        try:
            optimizer = torch.optim.Adam([alpha], lr=lr, fused=True)
        except (RuntimeError, TypeError):
            optimizer = torch.optim.Adam([alpha], lr=lr)
        sq = _BoundSoftQuant(w, alpha, d, o, bitwidth, ch_axis, round_loss_out)
        n = inp_data.shape[0]
        warm = opt_params.num_iterations * opt_params.warm_start
        for it in range(opt_params.num_iterations // world):
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
            # fused reconstruction-loss gradient; + the rounding-loss gradient, fused in the soft-quant kernel
            recon_loss_backward(q_out, target, act_func)
            if world > 1:
                _reduce_grad(alpha.grad, world, group)
            optimizer.step()
        return _finish_alpha(alpha, alpha_init)

    @staticmethod
    def _drawer(generator, n, iters, dev):
        """The eager loop's batch draws, in its order: idx_all [iters, nb] int64 on the device and
        draw(a, b), which fills rows [a, b) from the host generator through a pinned buffer
        (stream-ordered copy; the host buffers stay alive in `staged` until the caller
        synchronises), so chunk k + 1 is drawn while the GPU replays chunk k."""
        nb = min(n, BATCH_SIZE)
        idx_all = torch.empty((max(iters, 1), nb), dtype=torch.long, device=dev)
        staged = []

        def draw(a, b):
            h = torch.stack([torch.randperm(n, generator=generator)[:BATCH_SIZE] for _ in range(a, b)]).pin_memory()
            idx_all[a:b].copy_(h, non_blocking=True)
            staged.append(h)
        return idx_all, draw, staged

    @staticmethod
    def _reg_beta_all(opt_params, iters, dev):
        """{reg, beta, beta - 1} of every iteration, formed in double as the reference's python /
        ATen pow_backward do, then stored as float32 (the kernel's arithmetic type)."""
        warm = opt_params.num_iterations * opt_params.warm_start
        return torch.tensor([(0.0, 0.0, 0.0) if it < warm else
                             (lambda b: (opt_params.reg_param, b, b - 1.0))(
                                 compute_beta(opt_params.num_iterations, it, opt_params.beta_range,
                                              opt_params.warm_start))
                             for it in range(max(iters, 1))], dtype=torch.float64).to(torch.float32).to(dev)

    @staticmethod
    def _optimize_fused_graph(module, inp_data, out_data, delta, offset, bitwidth, ch_axis, opt_params, act_func,
                              generator, round_loss_out, alpha_init=None):
        """Single-process HIP-graph loop with the iteration's bookkeeping fused into two kernels:
        aimet_adaround_gather (the batch draw: index lookup + both row gathers, for the four
        index_select kernels) and aimet_adaround_backward_adam (dL/dalpha + torch's fused-Adam
        update of alpha in place, for the backward + gradient zero / accumulate + three Adam
        kernels). The iteration counter and Adam moments live in device memory; the weight
        gradient comes from torch.autograd.grad (no accumulation into a .grad)."""
        w = module.weight.detach()
        dev = w.device
        shape = [1] * w.dim()
        shape[ch_axis] = -1
        d = torch.as_tensor(delta, dtype=torch.float32, device=dev).reshape(-1).contiguous()
        o = torch.as_tensor(offset, dtype=torch.float32, device=dev).reshape(-1).contiguous()
        alpha = _starting_alpha(w, d, shape, alpha_init)
        sq = _BoundSoftQuant(w, alpha, d, o, bitwidth, ch_axis, round_loss_out)
        iters, n = opt_params.num_iterations, inp_data.shape[0]
        nb = min(n, BATCH_SIZE)
        idx_all, draw, staged = AdaroundOptimizer._drawer(generator, n, iters, dev)
        chunk = 500
        draw(0, min(chunk, iters))
        rb_all = AdaroundOptimizer._reg_beta_all(opt_params, iters, dev)
        im2col = (_GEMM_LAYERS and _LOOP_FORM != "autograd" and out_data.dim() == 4
                  and out_data.dtype == torch.float32 and _act_code(act_func) is not None
                  and _im2col_ok(module, inp_data))
        if im2col:
            # the cached inputs unfolded once ([N, C_in k k, OH OW]): each iteration's batch is then
            # a pointwise GEMM problem, gathered by rows like any other cache
            inp_data = torch.nn.functional.unfold(inp_data, module.kernel_size, module.dilation, module.padding,
                                                  module.stride)
        inp_data = inp_data.contiguous()
        out_data = out_data.contiguous()
        inp = torch.empty((nb,) + tuple(inp_data.shape[1:]), dtype=inp_data.dtype, device=dev)
        target = torch.empty((nb,) + tuple(out_data.shape[1:]), dtype=out_data.dtype, device=dev)
        row_in, row_out = inp[0].numel(), target[0].numel()
        exp_avg, exp_avg_sq = torch.zeros_like(alpha), torch.zeros_like(alpha)
        counters = torch.zeros(2, dtype=torch.long, device=dev)   # [it_cur, it_next]
        wq = torch.empty_like(sq.w).requires_grad_(True)
        lib = _native.load()
        P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
        it_cur, it_next = ctypes.c_void_p(counters.data_ptr()), ctypes.c_void_p(counters.data_ptr() + 8)
        adam = (ctypes.c_double(1e-3), ctypes.c_double(0.9), ctypes.c_double(0.999), ctypes.c_double(1e-8))
        # Adam's bias corrections for every step of the loop, computed once (the same device
        # arithmetic the step would run per wave: same bits)
        bias_corr = torch.empty(iters, 2, dtype=torch.float32, device=dev)
        _native.check(lib.aimet_adaround_adam_bias_corrections(adam[1], adam[2], iters, P(bias_corr),
                                                               ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
        loss_ptr = P(round_loss_out) if round_loss_out is not None else None
        code = _act_code(act_func)
        out_shape = tuple(out_data.shape[1:])
        # the fused reconstruction gradient reads the fp target in place (no gathered copy) when it
        # has a fused form: [N, C, ...] outputs, ReLU / ReLU6 / no activation
        indexed = code is not None and out_data.dim() >= 2 and out_data.dtype == torch.float32
        C_out = out_shape[0] if out_data.dim() >= 2 else 1
        hw = row_out // C_out if indexed else 1
        bias = module.bias.detach().contiguous() if module.bias is not None else None
        mode = "autograd"
        if im2col and indexed:
            mode = "im2col"
        elif indexed and depthwise_spec(module) is not None and inp.dim() == 4:
            mode = "dw"
        elif indexed and _GEMM_LAYERS and _is_pointwise(module) and inp.dim() == 4:
            mode = "pointwise"
        elif indexed and _GEMM_LAYERS and isinstance(module, torch.nn.Linear) and inp.dim() == 2:
            mode = "linear"
        q_buf = torch.empty((nb,) + out_shape, dtype=torch.float32, device=dev)
        g_buf = torch.empty_like(q_buf)
        dw_slices = 0
        if mode == "dw":
            # depthwise layers: native forward + weight gradient, no autograd (aimet_dwconv2d_*)
            K, stride, pad, dil = depthwise_spec(module)
            Nb, C, H, W = inp.shape
            gw_dw = torch.empty_like(sq.w)
            ws_n = ctypes.c_int64()
            _native.check(lib.aimet_dwconv2d_grad_weight_workspace(Nb, C, out_shape[1], out_shape[2], K,
                                                                   ctypes.byref(ws_n)))
            ws = torch.empty(ws_n.value, dtype=torch.float32, device=dev)
            dims = (Nb, C, H, W, out_shape[1], out_shape[2], K, stride, pad, dil)
            if _DW_FOLD_ADAM and _DW_FUSED and sq.shape[0] * sq.shape[1] * sq.shape[2] == C * K * K:
                sl = ctypes.c_int64()
                _native.check(lib.aimet_adaround_dw_step_slices(P(out_data), Nb, C, out_shape[1], out_shape[2], K,
                                                                stride, dil, ctypes.byref(sl)))
                dw_slices = sl.value
        pbias = P(bias) if bias is not None else None
        pw_dims, cm, pw_slices = None, None, None
        if mode in ("pointwise", "im2col") and _PW_FUSED != "0" and _LOOP_FORM != "autograd":
            cin, cout, hw_in = inp_data.shape[1], C_out, inp_data[0, 0].numel()
            wanted = _PW_FUSED == "all" or (hw >= 28 * 28 and (not (cin > cout and hw < 56 * 56) or
                                                              (cin >= 32 and _pw_step_uses_mfma(cin, cout))))
            if (wanted and cin <= 192 and hw_in == hw and hw % 4 == 0
                    and inp_data.data_ptr() % 16 == 0 and out_data.data_ptr() % 16 == 0 and wq.is_contiguous()):
                pw_dims = (nb, cin, cout, hw)
                gw_pw = torch.empty_like(sq.w)
                ws_n = ctypes.c_int64()
                _native.check(lib.aimet_adaround_pw_step_workspace(*pw_dims, ctypes.byref(ws_n)))
                ws_pw = torch.empty(ws_n.value, dtype=torch.float32, device=dev)
                if _DW_FOLD_ADAM and sq.w.numel() == cin * cout:
                    # the step's slices added by the Adam step (pw_fold_final's sum, one launch fewer)
                    off, nsl = ctypes.c_int64(), ctypes.c_int64()
                    _native.check(lib.aimet_adaround_pw_step_slices(*pw_dims, ctypes.byref(off), ctypes.byref(nsl)))
                    pw_slices = (off.value, nsl.value)
        if (mode in ("pointwise", "im2col") and pw_dims is None and _PW_CM and hw <= 14 * 14
                and inp_data[0].numel() % hw == 0):
            cin_cm = inp_data[0].numel() // hw
            x_cm = torch.empty((cin_cm, nb * hw), dtype=torch.float32, device=dev)
            q_cm = torch.empty((C_out, nb * hw), dtype=torch.float32, device=dev)
            cm = (cin_cm, x_cm, q_cm, torch.empty_like(q_cm))

        def recon(q, with_bias, s):
            _native.check(lib.aimet_adaround_recon_grad_indexed(P(q), P(out_data), P(idx_all), it_cur, P(g_buf), nb,
                                                                C_out, hw, pbias if with_bias else None, code, s))

        def adam_step(gw, s):
            # the Adam step also writes the next iteration's soft-quantized weight into wq (it reads
            # W and the new alpha anyway): no separate forward launch per iteration
            _native.check(lib.aimet_adaround_backward_adam_parts(sq.pw, sq.pa, P(gw), 1, 0, P(exp_avg), P(exp_avg_sq),
                                                                 *sq.shape, sq.pd, sq.po, sq.bw, P(rb_all), it_next,
                                                                 it_cur, *adam, loss_ptr, P(wq), P(bias_corr), s))

        def soft_weight():   # wq from the current alpha (before the first iteration)
            s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            _native.check(sq.fwd(sq.pw, sq.pa, P(wq), *sq.shape, sq.pd, sq.po, sq.bw, 1, s))

        def step():
            s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            if mode == "dw" and _DW_FUSED:
                # the batch read in place from the caches, q and g never stored; it_next moves here
                if dw_slices:
                    # the per-channel slices folded by the Adam step (one launch fewer; the same sum)
                    _native.check(lib.aimet_adaround_dw_step(P(inp_data), P(out_data), P(idx_all), it_cur, it_next,
                                                             P(wq), pbias, None, P(ws), *dims, code, s))
                    _native.check(lib.aimet_adaround_backward_adam_parts(
                        sq.pw, sq.pa, P(ws), dw_slices, dims[6] * dims[6], P(exp_avg), P(exp_avg_sq), *sq.shape,
                        sq.pd, sq.po, sq.bw, P(rb_all), it_next, it_cur, *adam, loss_ptr, P(wq),
                        P(bias_corr), s))
                    return
                _native.check(lib.aimet_adaround_dw_step(P(inp_data), P(out_data), P(idx_all), it_cur, it_next,
                                                         P(wq), pbias, P(gw_dw), P(ws), *dims, code, s))
                adam_step(gw_dw, s)
                return
            if mode in ("pointwise", "im2col") and pw_dims is not None:
                # 1x1 / unfolded stem with few channels: one pass, the batch read in place
                if pw_slices:
                    _native.check(lib.aimet_adaround_pw_step(P(inp_data), P(out_data), P(idx_all), it_cur, it_next,
                                                             P(wq), pbias, None, P(ws_pw), *pw_dims, code, s))
                    _native.check(lib.aimet_adaround_backward_adam_parts(
                        sq.pw, sq.pa, ctypes.c_void_p(ws_pw.data_ptr() + 4 * pw_slices[0]), pw_slices[1],
                        sq.w.numel(), P(exp_avg), P(exp_avg_sq), *sq.shape, sq.pd, sq.po, sq.bw, P(rb_all), it_next,
                        it_cur, *adam, loss_ptr, P(wq), P(bias_corr), s))
                    return
                _native.check(lib.aimet_adaround_pw_step(P(inp_data), P(out_data), P(idx_all), it_cur, it_next,
                                                         P(wq), pbias, P(gw_pw), P(ws_pw), *pw_dims, code, s))
                adam_step(gw_pw, s)
                return
            if mode in ("pointwise", "im2col") and cm is not None:
                # channel-major batch: one GEMM per direction over all nb * hw positions
                cin_cm, x_cm, q_cm, g_cm = cm
                _native.check(lib.aimet_adaround_gather_cm(P(inp_data), P(x_cm), P(idx_all), it_cur, it_next, nb,
                                                           cin_cm, hw, s))
                w2 = wq.detach().view(wq.shape[0], -1)
                torch.mm(w2, x_cm, out=q_cm)
                _native.check(lib.aimet_adaround_recon_grad_indexed_cm(P(q_cm), P(out_data), P(idx_all), it_cur,
                                                                       P(g_cm), nb, C_out, hw, pbias, code, s))
                adam_step(torch.mm(g_cm, x_cm.t()).view_as(wq), s)
                return
            _native.check(lib.aimet_adaround_gather(P(inp_data), P(out_data), P(inp),
                                                    None if indexed else P(target), P(idx_all), it_cur, it_next, nb,
                                                    row_in, row_out, s))
            if mode == "dw":
                _native.check(lib.aimet_dwconv2d_forward(P(inp), P(wq), pbias, P(q_buf), *dims, s))
                recon(q_buf, False, s)
                _native.check(lib.aimet_dwconv2d_grad_weight(P(inp), P(g_buf), P(gw_dw), P(ws), *dims, s))
                adam_step(gw_dw, s)
                return
            if mode in ("pointwise", "im2col"):
                # 1x1 convolution (or the unfolded stem) as one batched GEMM per direction
                # (hipBLASLt, no NCHW<->NHWC transposes): q[n] = Wq @ x[n]; the bias is added inside
                # the reconstruction kernel
                x3 = inp.view(nb, inp.shape[1], -1)
                w2 = wq.detach().view(wq.shape[0], -1)
                torch.matmul(w2, x3, out=q_buf.view(nb, w2.shape[0], -1))
                recon(q_buf, True, s)
                g3 = g_buf.view(nb, w2.shape[0], -1)
                if _PW_GRAD == "mm" or (_PW_GRAD == "auto" and g3.shape[2] <= 64):
                    # one GEMM over (n, hw): [C_out, nb * hw] @ [nb * hw, C_in] from channel-major copies
                    gw = torch.mm(g3.transpose(0, 1).reshape(w2.shape[0], -1),
                                  x3.transpose(0, 1).reshape(w2.shape[1], -1).t())
                else:
                    gw = torch.matmul(g3, x3.transpose(1, 2)).sum(0)
                adam_step(gw.contiguous().view_as(wq), s)
                return
            if mode == "linear":
                torch.mm(inp, wq.detach().t(), out=q_buf)
                recon(q_buf, True, s)
                adam_step(torch.mm(g_buf.t(), inp), s)
                return
            q_out = layer_forward(module, inp, wq)
            if indexed:
                recon(q_out, False, s)
                (gw,) = torch.autograd.grad(q_out, wq, grad_outputs=g_buf)
            else:
                qa, ta = (act_func(q_out), act_func(target)) if act_func is not None else (q_out, target)
                (gw,) = torch.autograd.grad(recon_loss(qa, ta), wq)
            adam_step(gw if gw.is_contiguous() else gw.contiguous(), s)

        alpha0 = alpha.detach().clone()
        loss0 = round_loss_out.clone() if round_loss_out is not None else None

        def restart():   # back to iteration 0
            with torch.no_grad():
                alpha.copy_(alpha0)
                exp_avg.zero_()
                exp_avg_sq.zero_()
                counters.zero_()
                if round_loss_out is not None:
                    round_loss_out.copy_(loss0)
            soft_weight()

        def capture(m, k=1):
            nonlocal mode
            mode = m
            # warm-up on a side stream (library handles, allocator, autograd), then capture
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side), torch.enable_grad():
                soft_weight()
                for _ in range(min(2, iters)):
                    step()
            torch.cuda.current_stream(dev).wait_stream(side)
            restart()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), torch.enable_grad():
                for _ in range(k):   # k consecutive iterations (the counters advance on the device)
                    step()
            return g

        # layers with two forms (GEMM or MIOpen convolution through autograd): the form is fixed by
        # _LOOP_FORM (deterministic results); the convolution form only when the GEMM form cannot be
        # captured
        two_forms = mode in ("pointwise", "linear")
        if two_forms and _LOOP_FORM == "autograd":
            mode = "autograd"
        candidates = [mode] + (["autograd"] if two_forms and mode != "autograd" else [])
        graph = None
        for m in candidates:
            try:
                graph = capture(m)
            except RuntimeError:
                if m == candidates[0] and len(candidates) > 1:
                    continue   # the GEMM form could not be captured: the convolution form
                raise
            mode = m
            break
        AdaroundOptimizer.last_loop_form = mode + ("_fused" if mode in ("pointwise", "im2col") and pw_dims else
                                                   "_cm" if mode in ("pointwise", "im2col") and cm else "")
        k = min(_GRAPH_ITERS, chunk)
        graph_k = None
        if k > 1 and iters >= k:
            try:
                graph_k = capture(mode, k)
            except RuntimeError:
                # k iterations could not be captured (graph-pool memory, an autograd form): the
                # one-iteration graph runs them, the same results
                graph_k = None
            restart()
        for a in range(0, iters, chunk):
            b = min(a + chunk, iters)
            if b < iters:
                draw(b, min(b + chunk, iters))
            i = a
            while graph_k is not None and i + k <= b:
                graph_k.replay()
                i += k
            for _ in range(i, b):
                graph.replay()
        torch.cuda.current_stream(dev).synchronize()
        del staged
        return _finish_alpha(alpha, alpha_init)

    @staticmethod
    def _optimize_graphed(module, inp_data, out_data, delta, offset, bitwidth, ch_axis, opt_params, act_func,
                          generator, round_loss_out, world=1, group=None, alpha_init=None, fused_step=True):
        if world == 1 and fused_step:
            return AdaroundOptimizer._optimize_fused_graph(module, inp_data, out_data, delta, offset, bitwidth,
                                                           ch_axis, opt_params, act_func, generator, round_loss_out,
                                                           alpha_init)
        w = module.weight.detach()
        dev = w.device
        shape = [1] * w.dim()
        shape[ch_axis] = -1
        d = torch.as_tensor(delta, dtype=torch.float32, device=dev).reshape(-1)
        o = torch.as_tensor(offset, dtype=torch.float32, device=dev).reshape(-1)
        alpha = _starting_alpha(w, d, shape, alpha_init)
        lr = 1e-3 * world
        try:
            optimizer = torch.optim.Adam([alpha], lr=lr, capturable=True, fused=True)
        except (RuntimeError, TypeError):
            optimizer = torch.optim.Adam([alpha], lr=lr, capturable=True)
        sq = _BoundSoftQuant(w, alpha, d, o, bitwidth, ch_axis, round_loss_out)
        iters, n = opt_params.num_iterations // world, inp_data.shape[0]
        warm = opt_params.num_iterations * opt_params.warm_start
        # the eager loop's draws, in its order: drawn on the host chunk by chunk while the GPU replays
        # the previous chunk (stream-ordered pinned copies into idx_all)
        nb = min(n, BATCH_SIZE)
        idx_all = torch.empty((iters, nb), dtype=torch.long, device=dev)
        chunk = 500
        staged = []

        def draw(a, b):
            h = torch.stack([torch.randperm(n, generator=generator)[:BATCH_SIZE] for _ in range(a, b)]).pin_memory()
            idx_all[a:b].copy_(h, non_blocking=True)
            staged.append(h)   # alive until the copies have run (synchronised below)

        draw(0, min(chunk, iters))
        # {reg, beta, beta - 1} of every iteration, formed in double as the reference's python / ATen
        # pow_backward do, then stored as float32 (the kernel's arithmetic type)
        rb_all = torch.tensor([(0.0, 0.0, 0.0) if it < warm else
                               (lambda b: (opt_params.reg_param, b, b - 1.0))(
                                   compute_beta(opt_params.num_iterations, it, opt_params.beta_range,
                                                opt_params.warm_start))
                               for it in range(max(iters, 1))], dtype=torch.float64).to(torch.float32).to(dev)
        it_buf = torch.zeros(1, dtype=torch.long, device=dev)
        alpha.grad = torch.zeros_like(alpha)

        def grad_step():
            idx = idx_all.index_select(0, it_buf).view(-1)
            inp = inp_data.index_select(0, idx)
            target = out_data.index_select(0, idx)
            sq.reg_beta = rb_all.index_select(0, it_buf).view(-1)
            optimizer.zero_grad(set_to_none=False)
            wq = _SoftQuantFn.apply(alpha, sq)
            q_out = layer_forward(module, inp, wq)
            recon_loss_backward(q_out, target, act_func)

        def update_step():
            if world > 1:
                alpha.grad.div_(world)
            optimizer.step()
            it_buf.add_(1)

        def step():
            grad_step()
            if world > 1:
                _reduce_grad(alpha.grad, world, group, divide=False)   # the SUM; / world in update_step
            update_step()

        # warm-up on a side stream (library handles, allocator, autograd), then back to iteration 0
        alpha0 = alpha.detach().clone()
        loss0 = round_loss_out.clone() if round_loss_out is not None else None
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(min(3, iters)):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        with torch.no_grad():
            alpha.copy_(alpha0)
            it_buf.zero_()
            for st in optimizer.state.values():
                for v in st.values():
                    if torch.is_tensor(v):
                        v.zero_()
            if round_loss_out is not None:
                round_loss_out.copy_(loss0)
        if world == 1:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                step()
            replay = graph.replay
        else:
            # the collective between two graphs (any backend; gloo stages through the host)
            g_grad, g_upd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_grad):
                grad_step()
            with torch.cuda.graph(g_upd):
                update_step()

            def replay():
                g_grad.replay()
                _reduce_grad(alpha.grad, world, group, divide=False)
                g_upd.replay()
        for a in range(0, iters, chunk):
            b = min(a + chunk, iters)
            if b < iters:
                draw(b, min(b + chunk, iters))
            for _ in range(a, b):
                replay()
        torch.cuda.current_stream(dev).synchronize()
        sq.reg_beta = None
        return _finish_alpha(alpha, alpha_init)

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
