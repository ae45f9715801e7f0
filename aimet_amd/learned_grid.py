"""Range-learning (LearnedGrid) QAT quantize-dequantize on the fused gfx950 kernels.

Reference: ``QuantizeDequantizeFunc`` (v1/tensor_quantizer.py:896-986) over
``calculate_forward_pass`` / ``asymmetric_gradients`` / ``symmetric_gradients``
(v1/quantsim_straight_through_grad.py:121-347). The reference saves x, an uint8 x_quant and a bool
mask and runs ~10 torch kernels per tensor per step; here the forward is one kernel that saves
nothing but x, and the backward one kernel that recomputes x_round and emits grad_x plus three
per-channel sums, from which the encoding gradients are assembled on C-element vectors.

Inputs are computed in float32: fp16 / bf16 tensors with a per-tensor range run the 16-bit I/O
kernels (aimet_lg_forward_16 / _backward_16: the casts in registers, results identical to the
upcast -> fp32 -> downcast chain), other 16-bit cases are upcast. The reference keeps bf16/fp16
arithmetic for bitwidth <= 8 -- a documented difference, results are then at least as accurate.
"""
import ctypes
import math

import numpy as np

import torch

from aimet_amd import _native
from aimet_amd.libpymo import TfEncoding, encodings_to_c
from aimet_amd.tensor_quantizer import IO_DTYPES, _stage, _stream, per_channel_view


class _RangeSpec(ctypes.Structure):
    """aimet_lg_range_spec (include/aimet_amd.h)."""
    _fields_ = [("encoding_min", ctypes.c_void_p), ("encoding_max", ctypes.c_void_p), ("delta", ctypes.c_void_p),
                ("grad_min", ctypes.c_void_p), ("grad_max", ctypes.c_void_p), ("use_symmetric", ctypes.c_int)]


_CONSTS = {}


def _const(value: float, like: torch.Tensor) -> torch.Tensor:
    """A cached 0-dim tensor holding `value` (no fill launch per call)."""
    key = (value, like.dtype, like.device)
    t = _CONSTS.get(key)
    if t is None:
        t = _CONSTS[key] = torch.full((), value, dtype=like.dtype, device=like.device)
    return t


def num_steps_of(bitwidth, use_symmetric_encodings, use_strict_symmetric) -> float:
    """The quantisation grid's step count (host side: no device read-back per call)."""
    num_steps = 2 ** bitwidth - 1
    if use_symmetric_encodings and use_strict_symmetric:
        num_steps -= 1
    return float(num_steps)


def _delta_offset(bitwidth, encoding_min, encoding_max, use_symmetric_encodings, use_strict_symmetric,
                  is_unsigned_symmetric):
    """quantsim_straight_through_grad.py:121-160 with the reference's torch.full_like constant
    tensors replaced by cached 0-dim device tensors of the same values: identical results (a
    divisor stays a device tensor -- torch multiplies by the reciprocal of a host scalar divisor),
    2-7 launches per call instead of 4-10 and no fill."""
    num_steps = num_steps_of(bitwidth, use_symmetric_encodings, use_strict_symmetric)
    half_num_steps = num_steps / 2
    if use_symmetric_encodings and not is_unsigned_symmetric:
        delta = encoding_max / _const(float(math.floor(half_num_steps)), encoding_max)
        offset = torch.full_like(encoding_min, -float(math.ceil(half_num_steps)))
    else:
        delta = (encoding_max - encoding_min) / _const(num_steps, encoding_min)
        if use_symmetric_encodings:
            offset = encoding_min / delta
        else:
            # torch.min(steps, torch.max(zero, b)) with cached 0-dim operands in the same argument
            # order (the sign of a zero b_zero, hence of a zero offset, follows the reference)
            b_zero = torch.round(-encoding_min / delta)
            b_zero = torch.minimum(_const(num_steps, b_zero), torch.maximum(_const(0.0, b_zero), b_zero))
            offset = b_zero.neg_()
    return delta, offset, num_steps


def get_computed_encodings(bitwidth, encoding_min, encoding_max, use_symmetric_encodings, use_strict_symmetric,
                           is_unsigned_symmetric):
    """quantsim_straight_through_grad.py:121-160 (torch ops on the C-element encoding vectors):
    (delta, offset, num_steps tensor)."""
    delta, offset, num_steps = _delta_offset(bitwidth, encoding_min, encoding_max, use_symmetric_encodings,
                                             use_strict_symmetric, is_unsigned_symmetric)
    return delta, offset, torch.full_like(encoding_min, num_steps)


def _device_delta_offset(bitwidth, emin, emax, use_symmetric, use_strict_symmetric, is_unsigned_symmetric):
    """_delta_offset in ONE launch (aimet_lg_encodings, the same float32 expressions element by
    element) for contiguous float32 device vectors."""
    delta = torch.empty_like(emin)
    offset = torch.empty_like(emin)
    _native.call("aimet_lg_encodings", emin.data_ptr(), emax.data_ptr(), emin.numel(), int(bitwidth),
                 int(bool(use_symmetric)), int(bool(use_strict_symmetric)), int(bool(is_unsigned_symmetric)),
                 delta.data_ptr(), offset.data_ptr(), _stream(emin))
    return delta, offset, num_steps_of(bitwidth, use_symmetric, use_strict_symmetric)


def _saved_encoding(emin):
    """[4][C] float32: rows delta, offset, encoding_min, encoding_max, filled by the forward kernel.
    The range rows are the reference's encoding_min/max.clone().detach() saved for the backward
    (v1/tensor_quantizer.py:940-951): not aliases of the Parameters, which the wrapper's gate updates
    in place on every call (a module run twice before backward keeps the range it saw)."""
    return torch.empty((4, emin.numel()), dtype=torch.float32, device=emin.device)


def _channels(shape, ch_axis, per_channel):
    if not per_channel:
        n = 1
        for s in shape:
            n *= s
        return 1, 1, n
    return per_channel_view(shape, ch_axis)


class LearnedGridQuantizeDequantize(torch.autograd.Function):
    """apply(tensor, encoding_min, encoding_max, bitwidth, use_symmetric, use_strict_symmetric,
    is_unsigned_symmetric, ch_axis, out_dtype=None).

    out_dtype (fp16 / bf16, float32 per-channel tensors only): return the result already cast to
    it -- for a weight that autocast would cast anyway for its matmul (LearnedGridQuantWrapper
    passes it for a Linear's weight under autocast); the cast happens in the kernel's store and
    the 16-bit gradient is upcast in the backward kernel's loads. Results == the float32 op
    followed by .to(out_dtype), gradients == the float32 op's on grad.to(float32)."""

    @staticmethod
    def forward(ctx, tensor, encoding_min, encoding_max, bitwidth, use_symmetric=False, use_strict_symmetric=False,
                is_unsigned_symmetric=False, ch_axis=0, out_dtype=None):
        if bitwidth >= 32:
            raise RuntimeError("Invalid bitwidth: %d" % bitwidth)
        orig_dtype = tensor.dtype
        if out_dtype in IO_DTYPES and orig_dtype == torch.float32 and tensor.is_cuda and encoding_min.numel() > 1:
            return LearnedGridQuantizeDequantize._forward_cast(ctx, tensor, encoding_min, encoding_max, bitwidth,
                                                               use_symmetric, use_strict_symmetric,
                                                               is_unsigned_symmetric, ch_axis, out_dtype)
        if tensor.is_cuda and orig_dtype in IO_DTYPES and encoding_min.numel() == 1:
            return LearnedGridQuantizeDequantize._forward_16(ctx, tensor, encoding_min, encoding_max, bitwidth,
                                                             use_symmetric, use_strict_symmetric,
                                                             is_unsigned_symmetric)
        # a CPU tensor (and its CPU range) is staged through HBM; results go back to the host
        x, staged = _stage(tensor.to(torch.float32), "tensor")
        x = x.contiguous()
        emin = encoding_min.detach().to(x.device, torch.float32).reshape(-1).contiguous()
        emax = encoding_max.detach().to(x.device, torch.float32).reshape(-1).contiguous()
        outer, C, K = _channels(x.shape, ch_axis, emin.numel() > 1)
        if C != emin.numel():
            raise ValueError("encoding has %d channels, tensor has %d along axis %d" % (emin.numel(), C, ch_axis))
        y = torch.empty_like(x)
        # get_computed_encodings inside the forward kernel (delta / offset stored for the backward,
        # with a copy of the range as the kernel read it)
        enc = _saved_encoding(emin)
        steps = num_steps_of(bitwidth, use_symmetric, use_strict_symmetric)
        with torch.cuda.device(x.device):
            _native.call("aimet_lg_forward_range", x.data_ptr(), y.data_ptr(), outer, C, K, 0, emin.data_ptr(),
                         emax.data_ptr(), int(bitwidth), int(bool(use_symmetric)), int(bool(use_strict_symmetric)),
                         int(bool(is_unsigned_symmetric)), enc[0].data_ptr(), enc[1].data_ptr(), enc[2].data_ptr(),
                         _stream(x))
        ctx.save_for_backward(x, enc)
        ctx.cfg = (outer, C, K, steps, use_symmetric, is_unsigned_symmetric, orig_dtype,
                   encoding_min.shape, encoding_max.shape, staged)
        return y.to(orig_dtype).cpu() if staged else y.to(orig_dtype)

    @staticmethod
    def _forward_cast(ctx, tensor, encoding_min, encoding_max, bitwidth, use_symmetric, use_strict_symmetric,
                      is_unsigned_symmetric, ch_axis, out_dtype):
        """float32 per-channel tensor, 16-bit result (aimet_lg_forward_cast). Saves the float32 input."""
        x = tensor.contiguous()
        emin = encoding_min.detach().to(x.device, torch.float32).reshape(-1).contiguous()
        emax = encoding_max.detach().to(x.device, torch.float32).reshape(-1).contiguous()
        outer, C, K = _channels(x.shape, ch_axis, True)
        if C != emin.numel():
            raise ValueError("encoding has %d channels, tensor has %d along axis %d" % (emin.numel(), C, ch_axis))
        y = torch.empty(x.shape, dtype=out_dtype, device=x.device)
        enc = _saved_encoding(emin)
        steps = num_steps_of(bitwidth, use_symmetric, use_strict_symmetric)
        with torch.cuda.device(x.device):
            _native.call("aimet_lg_forward_range", x.data_ptr(), y.data_ptr(), outer, C, K, IO_DTYPES[out_dtype],
                         emin.data_ptr(), emax.data_ptr(), int(bitwidth), int(bool(use_symmetric)),
                         int(bool(use_strict_symmetric)), int(bool(is_unsigned_symmetric)), enc[0].data_ptr(),
                         enc[1].data_ptr(), enc[2].data_ptr(), _stream(x))
        ctx.save_for_backward(x, enc)
        ctx.cfg = (outer, C, K, steps, use_symmetric, is_unsigned_symmetric, torch.float32,
                   encoding_min.shape, encoding_max.shape, False)
        return y

    @staticmethod
    def _forward_16(ctx, tensor, encoding_min, encoding_max, bitwidth, use_symmetric, use_strict_symmetric,
                    is_unsigned_symmetric):
        """fp16 / bf16 tensor, per-tensor range: aimet_lg_forward_16 (the casts in registers;
        identical to the upcast -> fp32 kernel -> downcast chain). Saves the 16-bit input."""
        x = tensor.contiguous()
        emin = encoding_min.detach().to(x.device, torch.float32).reshape(-1).contiguous()
        emax = encoding_max.detach().to(x.device, torch.float32).reshape(-1).contiguous()
        y = torch.empty_like(x)
        enc = _saved_encoding(emin)
        steps = num_steps_of(bitwidth, use_symmetric, use_strict_symmetric)
        with torch.cuda.device(x.device):
            _native.call("aimet_lg_forward_16_range", x.data_ptr(), y.data_ptr(), x.numel(), IO_DTYPES[x.dtype],
                         emin.data_ptr(), emax.data_ptr(), int(bitwidth), int(bool(use_symmetric)),
                         int(bool(use_strict_symmetric)), int(bool(is_unsigned_symmetric)), enc[0].data_ptr(),
                         enc[1].data_ptr(), enc[2].data_ptr(), _stream(x))
        ctx.save_for_backward(x, enc)
        ctx.cfg = (1, 1, x.numel(), steps, use_symmetric, is_unsigned_symmetric, x.dtype,
                   encoding_min.shape, encoding_max.shape, False)
        return y

    @staticmethod
    def backward(ctx, grad):
        x, enc = ctx.saved_tensors
        delta, offset, emin, emax = enc[0], enc[1], enc[2], enc[3]
        outer, C, K, steps, sym, unsigned, dtype, min_shape, max_shape, staged = ctx.cfg
        sums = torch.empty((C, 3), dtype=torch.float32, device=x.device)
        # symmetric_gradients: gmax = (A - B) / floor(steps/2), gmin = -gmax; asymmetric_gradients:
        # term1 = (A - B) / steps, term2 = steps / (max - min)^2 * (delta * D), gmin = -term1 + max *
        # term2, gmax = term1 - min * term2 -- the torch expressions, evaluated by the kernel that
        # folds the sums (aimet_lg_range_spec)
        gmin = torch.empty_like(emin)
        gmax = torch.empty_like(emax)
        spec = ctypes.byref(_RangeSpec(emin.data_ptr(), emax.data_ptr(), delta.data_ptr(), gmin.data_ptr(),
                                       gmax.data_ptr(), int(bool(sym))))
        g16 = grad.contiguous() if (x.dtype == torch.float32 and grad.dtype in IO_DTYPES and grad.is_cuda
                                    and C > 1) else None
        gx = torch.empty_like(x) if (g16 is not None and ctx.needs_input_grad[0]) else None
        if g16 is not None and _native.load().aimet_lg_backward_grad16_supported(
                outer, C, K, x.data_ptr(), g16.data_ptr(), gx.data_ptr() if gx is not None else None):
            # the 16-bit weight gradient of a cast-fused forward, upcast in the kernel's loads
            with torch.cuda.device(x.device):
                _native.call("aimet_lg_backward_grad16", x.data_ptr(), g16.data_ptr(),
                             gx.data_ptr() if gx is not None else None, sums.data_ptr(), outer, C, K,
                             IO_DTYPES[g16.dtype], delta.data_ptr(), offset.data_ptr(), steps, spec, _stream(x))
        elif x.dtype in IO_DTYPES and grad.dtype == x.dtype and grad.is_cuda:
            g = grad.contiguous()
            gx = torch.empty_like(g) if ctx.needs_input_grad[0] else None
            with torch.cuda.device(x.device):
                _native.call("aimet_lg_backward_16", x.data_ptr(), g.data_ptr(),
                             gx.data_ptr() if gx is not None else None, sums.data_ptr(), x.numel(), IO_DTYPES[x.dtype],
                             delta.data_ptr(), offset.data_ptr(), steps, spec, _stream(x))
        else:
            x = x.to(torch.float32)   # a 16-bit input with a gradient of another dtype
            g = grad.to(x.device, torch.float32).contiguous()
            gx = torch.empty_like(g) if ctx.needs_input_grad[0] else None
            with torch.cuda.device(x.device):
                _native.call("aimet_lg_backward", x.data_ptr(), g.data_ptr(), gx.data_ptr() if gx is not None else None,
                             sums.data_ptr(), outer, C, K, delta.data_ptr(), offset.data_ptr(), steps, spec,
                             _stream(x))
        gx_out = gx.to(dtype) if gx is not None else None
        gmin, gmax = gmin.view(min_shape), gmax.view(max_shape)
        if staged:
            gx_out = gx_out.cpu() if gx_out is not None else None
            gmin, gmax = gmin.cpu(), gmax.cpu()
        return gx_out, gmin, gmax, None, None, None, None, None, None


def _gate_fusable(encoding_min, encoding_max):
    return (encoding_min.is_cuda and encoding_max.is_cuda and encoding_min.dtype == torch.float32
            and encoding_max.dtype == torch.float32 and encoding_min.is_contiguous() and encoding_max.is_contiguous()
            and encoding_min.numel() == encoding_max.numel() and encoding_min.device == encoding_max.device)


def set_encoding_min_max_gating_threshold_many(ranges):
    """set_encoding_min_max_gating_threshold over a wrapper's (encoding_min, encoding_max) pairs:
    the device float32 ones of one device in launches of up to 8 ranges (aimet_lg_gate_ranges,
    element by element the single-range gate), any other pair through the single-range call."""
    fused = []
    for emin, emax in ranges:
        if _gate_fusable(emin, emax) and (not fused or fused[0][0].device == emin.device):
            fused.append((emin, emax))
        else:
            set_encoding_min_max_gating_threshold(emin, emax)
    for i in range(0, len(fused), 8):
        chunk = fused[i:i + 8]
        n = len(chunk)
        mins = (ctypes.c_void_p * n)(*[a.data_ptr() for a, _ in chunk])
        maxs = (ctypes.c_void_p * n)(*[b.data_ptr() for _, b in chunk])
        counts = (ctypes.c_int64 * n)(*[a.numel() for a, _ in chunk])
        with torch.cuda.device(chunk[0][0].device):
            _native.call("aimet_lg_gate_ranges", mins, maxs, counts, n, _stream(chunk[0][0]))
        for a, b in chunk:
            torch.autograd.graph.increment_version(a)
            torch.autograd.graph.increment_version(b)


def set_encoding_min_max_gating_threshold(encoding_min, encoding_max):
    """v1/tensor_quantizer.py:1347-1359: keep a trainable range ordered and around zero
    (min <= 0 <= max, max >= min + 1e-5), in place."""
    if _gate_fusable(encoding_min, encoding_max):
        # one launch, the same expressions element by element (aimet_lg_gate_range)
        with torch.cuda.device(encoding_min.device):
            _native.call("aimet_lg_gate_range", encoding_min.data_ptr(), encoding_max.data_ptr(),
                         encoding_min.numel(), _stream(encoding_min))
        # an in-place update, as the reference's clamp_ / copy_: bump the autograd version counters
        torch.autograd.graph.increment_version(encoding_min)
        torch.autograd.graph.increment_version(encoding_max)
        return
    with torch.no_grad():
        encoding_min.clamp_(max=0.0)
        encoding_max.clamp_(min=0.0)
        # min + 1e-5 with the scalar rounded to float32, as the reference's full_like tensor
        torch.maximum(encoding_max, encoding_min + 1e-5, out=encoding_max)


class LearnedGridTensorQuantizer:
    """v1/tensor_quantizer.py:573-893. The learnable range lives in the owning wrapper's
    ``<name>_encoding_min`` / ``<name>_encoding_max`` parameters (one element per channel);
    ``encoding`` is computed from them on every read, and setting it re-creates them."""

    def __init__(self, bitwidth, round_mode, quant_scheme, use_symmetric_encodings, enabled_by_default,
                 data_type=None):
        from aimet_amd.quantizers import QuantizationDataType, _round_mode
        data_type = QuantizationDataType.int if data_type is None else data_type
        if data_type != QuantizationDataType.int:
            raise ValueError("Only QuantizationDataType.int is supported for LearnedGridTensorQuantizer")
        self.round_mode = _round_mode(round_mode)
        self.quant_scheme = quant_scheme
        self.use_symmetric_encodings = use_symmetric_encodings
        self.use_strict_symmetric = False
        self.use_unsigned_symmetric = False
        self.is_unsigned_symmetric = False
        self.bitwidth = bitwidth
        self.enabled = enabled_by_default
        self.data_type = data_type
        self.is_const = False
        self._encoding_min_max_fixed_vals = None
        self._is_encoding_frozen = False
        self.wrapper_ref = None
        self.name = None
        self.device = None
        self._ch_axis = 0

    def __str__(self):
        s = ["LearnedGrid TensorQuantizer:\n",
             "    quant-scheme:{}, round_mode={}, bitwidth={}, enabled={}\n".format(
                 self.quant_scheme, self.round_mode, self.bitwidth, self.enabled)]
        enc = self.get_effective_encoding() if self.encoding else None
        if enc is None:
            s.append("    no encoding\n")
        else:
            for e in (enc if isinstance(enc, list) else [enc]):
                s.append("    min:{}, max={}, delta={}, offset={}\n".format(e.min, e.max, e.delta, e.offset))
        return "".join(s)

    @property
    def is_encoding_frozen(self):
        return self._is_encoding_frozen

    @property
    def channel_axis(self):
        return self._ch_axis

    @property
    def encoding_min_max_fixed_vals(self):
        return self._encoding_min_max_fixed_vals

    @encoding_min_max_fixed_vals.setter
    def encoding_min_max_fixed_vals(self, vals):
        self._encoding_min_max_fixed_vals = vals

    def _params(self):
        if self.wrapper_ref is None or self.name is None:
            return None, None
        return getattr(self.wrapper_ref, self.name + "_encoding_min"), \
            getattr(self.wrapper_ref, self.name + "_encoding_max")

    def n(self, device=None):
        return torch.tensor([0.0], device=device or self.device)

    def p(self, device=None):
        # the reference passes use_strict_symmetric for both flags (v1/tensor_quantizer.py:631-639)
        p = 2 ** self.bitwidth - 1 - (1 if self.use_strict_symmetric else 0)
        return torch.tensor([float(p)], device=device or self.device)

    def compute_scaling_offset(self, encoding_min, encoding_max):
        """v1/tensor_quantizer.py:744-758."""
        if encoding_min is None or encoding_max is None:
            return None, None
        scaling, offset, _ = get_computed_encodings(self.bitwidth, encoding_min, encoding_max,
                                                    self.use_symmetric_encodings, self.use_strict_symmetric,
                                                    self.is_unsigned_symmetric)
        return scaling, offset

    @property
    def encoding(self):
        """v1/tensor_quantizer.py:687-702: the learned encoding(s), computed from the parameters."""
        from aimet_amd.quantizers import QuantizationDataType
        if not self.enabled or self.bitwidth == 32 or self.data_type == QuantizationDataType.float:
            return None
        return self._compute_updated_encoding()

    @encoding.setter
    def encoding(self, encoding):
        """v1/tensor_quantizer.py:704-729."""
        from aimet_amd.quantizers import QuantizationDataType
        if not self.enabled or self.bitwidth == 32 or self.data_type == QuantizationDataType.float:
            return
        if encoding is None:
            raise RuntimeError("Encodings cannot be None if Quantizer is enabled.")
        bw = encoding[0].bw if isinstance(encoding, list) else encoding.bw
        if bw != self.bitwidth:
            raise RuntimeError("Bitwidth mismatched. The bitwidth for quantizer is %d, but the bitwidth in encodings "
                               "is %d. If the intent is to change the bitwidth, please set quantizer bitwidth to %d "
                               "first." % (self.bitwidth, bw, bw))
        if self._is_encoding_frozen:
            raise RuntimeError("Encoding can be set only when it is not frozen.")
        self._set_encoding_min_max_parameters(encoding)

    def _compute_updated_encoding(self):
        """v1/tensor_quantizer.py:775-819: delta / offset from the parameters with the forward's
        torch float32 arithmetic; asymmetric ranges are moved onto the grid (min = delta * offset)."""
        emin, emax = self._params()
        if emin is None or emax is None:
            return None
        emin, emax = emin.detach().float(), emax.detach().float()
        scale, offset = self.compute_scaling_offset(emin, emax)
        scale, offset = scale.expand_as(emin), offset.expand_as(emin)
        if not self.use_symmetric_encodings or self.is_unsigned_symmetric:
            adjusted_min = scale * offset
            emax = emax - emin + adjusted_min
            emin = adjusted_min
        rows = torch.stack([emin, emax, scale, offset]).cpu().tolist()   # one device->host copy
        encodings = []
        for mn, mx, dl, off in zip(*rows):
            e = TfEncoding()
            e.min, e.max, e.delta, e.offset, e.bw = mn, mx, dl, off, self.bitwidth
            encodings.append(e)
        return encodings[0] if len(encodings) == 1 else encodings

    def get_effective_encoding(self):
        """v1/tensor_quantizer.py:642-685: non-strict symmetric quantizers learn a strictly
        symmetric range; the effective (exported) min carries the extra bin."""
        if not self.enabled:
            return None
        encodings = self.encoding
        if not encodings:
            return None
        if isinstance(encodings, TfEncoding):
            encodings = [encodings]
        out = []
        for e in encodings:
            if self.use_symmetric_encodings and not self.use_strict_symmetric and not self.is_unsigned_symmetric:
                f = TfEncoding()
                f.min, f.max, f.offset, f.delta, f.bw = e.min - e.delta, e.max, e.offset, e.delta, e.bw
                out.append(f)
            else:
                out.append(e)
        return out[0] if len(out) == 1 else out

    def _set_encoding_min_max_parameters(self, encodings):
        """v1/tensor_quantizer.py:821-852 (float32 parameters on the wrapper's device)."""
        encs = encodings if isinstance(encodings, list) else [encodings]
        if len(encs) > 1:
            arr = _encoding_array(encs)
            self._set_min_max_arrays(arr["min"], arr["max"])
            return
        self._set_min_max_arrays(np.array([float(e.min) for e in encs]), np.array([float(e.max) for e in encs]))

    def _set_min_max_arrays(self, mins, maxs):
        """The encoding-min / -max Parameters from float64 arrays (rounded to float32 as
        torch.tensor([python floats], dtype=float32) rounds them)."""
        params = self.wrapper_ref._parameters
        dev = self.wrapper_ref.device
        params[self.name + "_encoding_min"] = torch.nn.Parameter(
            torch.from_numpy(np.ascontiguousarray(mins, dtype=np.float64)).to(torch.float32).to(dev),
            requires_grad=True)
        params[self.name + "_encoding_max"] = torch.nn.Parameter(
            torch.from_numpy(np.ascontiguousarray(maxs, dtype=np.float64)).to(torch.float32).to(dev),
            requires_grad=True)

    def freeze_encoding(self):
        """v1/tensor_quantizer.py:854-869."""
        params = self.wrapper_ref._parameters
        pmin, pmax = params.get(self.name + "_encoding_min"), params.get(self.name + "_encoding_max")
        if pmin is None and pmax is None:
            raise RuntimeError("Encoding can be frozen only when it is not None.")
        self._is_encoding_frozen = True
        pmin.requires_grad = False
        pmax.requires_grad = False

    def reset_encoding_stats(self):
        """Range-learning quantizers hold no statistics."""

    def quantize_dequantize(self, tensor, encoding_min, encoding_max, out_dtype=None):
        """v1/tensor_quantizer.py:760-773 over the fused forward / backward kernels (out_dtype: see
        LearnedGridQuantizeDequantize)."""
        if not self.enabled or self.bitwidth == 32:
            return tensor
        if encoding_min is None or encoding_max is None:
            raise RuntimeError("Forward pass used for compute_encodings differs from forward pass used during "
                               "training")
        return LearnedGridQuantizeDequantize.apply(tensor, encoding_min, encoding_max, self.bitwidth,
                                                   self.use_symmetric_encodings, self.use_strict_symmetric,
                                                   self.is_unsigned_symmetric, self._ch_axis, out_dtype)


_TF_ENCODING_DTYPE = np.dtype({"names": ["min", "max", "delta", "offset", "bw"],
                               "formats": ["<f8", "<f8", "<f8", "<f8", "<i4"],
                               "offsets": [_native.TfEncodingC.min.offset, _native.TfEncodingC.max.offset,
                                           _native.TfEncodingC.delta.offset, _native.TfEncodingC.offset.offset,
                                           _native.TfEncodingC.bw.offset],
                               "itemsize": ctypes.sizeof(_native.TfEncodingC)})


def _encoding_array(encodings):
    """A numpy structured array (min, max, delta, offset, bw) of a sequence of TfEncoding: one
    C-level copy."""
    return np.frombuffer(encodings_to_c(encodings), dtype=_TF_ENCODING_DTYPE)


def initialize_learned_grid_quantizer_attributes(new_quantizer, old_quantizer):
    """v1/tensor_quantizer.py:1285-1344: copy a static-grid quantizer's settings and encodings;
    symmetric ranges become strictly symmetric (min = -max), unsigned-symmetric ones signed."""
    from aimet_amd.quantizers import QuantizationDataType
    new_quantizer.enabled = old_quantizer.enabled
    new_quantizer.bitwidth = old_quantizer.bitwidth
    new_quantizer.data_type = old_quantizer.data_type
    new_quantizer.use_symmetric_encodings = old_quantizer.use_symmetric_encodings
    new_quantizer.use_strict_symmetric = old_quantizer.use_strict_symmetric
    new_quantizer.use_unsigned_symmetric = old_quantizer.use_unsigned_symmetric
    new_quantizer.is_unsigned_symmetric = False
    new_quantizer.encoding_min_max_fixed_vals = old_quantizer.encoding_min_max_fixed_vals
    new_quantizer.is_const = old_quantizer.is_const
    if new_quantizer.data_type == QuantizationDataType.float or new_quantizer.bitwidth == 32:
        return
    encoding = old_quantizer.encoding
    encs = encoding if isinstance(encoding, list) else ([encoding] if encoding is not None else [])
    if len(encs) > 1 and new_quantizer.enabled and not new_quantizer._is_encoding_frozen:
        # per-channel (Llama-3-8B: 1.5 M channels): the same values from arrays, without a Python
        # assignment per channel; the static-grid quantizer being replaced keeps its encodings
        arr = _encoding_array(encs)
        if int(arr["bw"][0]) != new_quantizer.bitwidth:
            new_quantizer.encoding = encoding   # the setter's bitwidth error
        maxs = arr["max"]
        mins = -maxs if old_quantizer.enabled and (
            (old_quantizer.use_symmetric_encodings and not old_quantizer.is_unsigned_symmetric) or
            old_quantizer.is_unsigned_symmetric) else arr["min"]
        new_quantizer._set_min_max_arrays(mins, maxs)
        return
    if old_quantizer.enabled and old_quantizer.use_symmetric_encodings and not old_quantizer.is_unsigned_symmetric:
        for e in encs:
            e.min = -e.max
    if old_quantizer.enabled and old_quantizer.is_unsigned_symmetric:
        half = (2 ** old_quantizer.bitwidth - 1) / 2
        for e in encs:
            e.min = -e.max
            e.delta = e.max / math.floor(half)
            e.offset = -math.ceil(half)
    new_quantizer.encoding = encoding
