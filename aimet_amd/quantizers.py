"""Static-grid tensor quantizers and their autograd functions on the MI355X core.

Mirrors the aimet_torch v1 surface that owns ``AimetTensorQuantizer`` objects
(TrainingExtensions/torch/src/python/aimet_torch/v1/tensor_quantizer.py) and the STE gradient
(v1/quantsim_straight_through_grad.py:66-118): same class names, properties and methods, same
encoding/validity behaviour. MI355X-first changes:

* a per-channel quantizer holds ONE native object with C analyzers (one stats launch per
  tensor instead of C Python-level ``select().contiguous()`` + ``updateStats`` calls);
* per-channel QDQ tables are built once per encoding change and kept in HBM;
* the STE backward is one fused kernel (``grad * (min <= x <= max)``) instead of 3-4 torch
  kernels plus a host->device copy of the per-channel bounds on every backward.
"""
import enum
import io

import torch

from aimet_amd import _native
from aimet_amd.libpymo import QuantizationMode, RoundingMode, TfEncoding
from aimet_amd.tensor_quantizer import (IO_DTYPES, AimetTensorQuantizer, PerChannelTable, _require_gpu, _stage,
                                        _stream, per_channel_view, qdq_per_channel_table)


class QuantScheme(enum.Enum):
    """aimet_common/defs.py:50-71."""
    post_training_tf = 1
    post_training_tf_enhanced = 2
    training_range_learning_with_tf_init = 3
    training_range_learning_with_tf_enhanced_init = 4
    training_range_learning = 5
    post_training_percentile = 6


class QuantizationDataType(enum.Enum):
    """aimet_common/defs.py:309-314."""
    undefined = 0
    int = 1
    float = 2


MAP_QUANT_SCHEME_TO_PYMO = {   # aimet_common/defs.py:70-78
    QuantScheme.post_training_tf: QuantizationMode.QUANTIZATION_TF,
    QuantScheme.post_training_tf_enhanced: QuantizationMode.QUANTIZATION_TF_ENHANCED,
    QuantScheme.training_range_learning_with_tf_init: QuantizationMode.QUANTIZATION_TF,
    QuantScheme.training_range_learning_with_tf_enhanced_init: QuantizationMode.QUANTIZATION_TF_ENHANCED,
    QuantScheme.post_training_percentile: QuantizationMode.QUANTIZATION_PERCENTILE,
}
MAP_ROUND_MODE_TO_PYMO = {"nearest": RoundingMode.ROUND_NEAREST,   # aimet_common/defs.py:79-80
                          "stochastic": RoundingMode.ROUND_STOCHASTIC}


def _pymo_mode(quant_scheme):
    if isinstance(quant_scheme, QuantScheme):
        return MAP_QUANT_SCHEME_TO_PYMO[quant_scheme]
    return QuantizationMode(int(quant_scheme))


def _round_mode(rm):
    if isinstance(rm, str):
        return MAP_ROUND_MODE_TO_PYMO[rm]
    return RoundingMode(int(rm))


class StaticGridTensorQuantizer:
    """v1/tensor_quantizer.py:132-401."""

    def __init__(self, bitwidth, round_mode, quant_scheme, use_symmetric_encodings, enabled_by_default,
                 data_type=QuantizationDataType.int):
        self.round_mode = _round_mode(round_mode)
        self._quant_scheme = quant_scheme
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
        self._encoding = None
        self._cppOp = None

    def __str__(self):
        s = io.StringIO()
        s.write("StaticGrid TensorQuantizer:\n")
        s.write("    quant-scheme:{}, round_mode={}, bitwidth={}, enabled={}\n".format(
            self._quant_scheme, self.round_mode, self.bitwidth, self.enabled))
        if self._encoding:
            for e in self._encoding:
                s.write("    min:{}, max={}, delta={}, offset={}\n".format(e.min, e.max, e.delta, e.offset))
        else:
            s.write("    no encoding\n")
        return s.getvalue()

    @property
    def quant_scheme(self):
        return self._quant_scheme

    @quant_scheme.setter
    def quant_scheme(self, quant_scheme):
        self._quant_scheme = quant_scheme
        self._make_op()

    @property
    def is_encoding_frozen(self):
        return self._is_encoding_frozen

    @property
    def channel_axis(self):
        return None

    @property
    def encoding_min_max_fixed_vals(self):
        return self._encoding_min_max_fixed_vals

    @encoding_min_max_fixed_vals.setter
    def encoding_min_max_fixed_vals(self, vals):
        if not (isinstance(vals, tuple) and len(vals) == 2 and vals[0] < vals[1]):
            raise AssertionError("Min max vals must be a tuple of two increasing values")
        if self.quant_scheme != QuantScheme.post_training_tf:
            self.quant_scheme = QuantScheme.post_training_tf
        self._encoding_min_max_fixed_vals = vals

    def __getstate__(self):
        """v1/tensor_quantizer.py:182-192 (PickableState :128-140): every attribute but the native
        op travels; the encodings as (min, max, delta, offset, bw) tuples, and none when the
        quantizer has no (or an empty) encoding list. The device caches (STE bounds) stay behind."""
        state = self.__dict__.copy()
        state.pop("_cppOp", None)
        state.pop("_ste_cache", None)
        encodings = state.pop("_encoding", None)
        state["_pickled_encodings"] = [e.to_tuple() for e in encodings] if encodings else None
        return state

    def __setstate__(self, state):
        """v1/tensor_quantizer.py:194-220: a fresh native op (empty statistics, created on the device
        of first use) and new TfEncoding objects carrying the saved values."""
        state = dict(state)
        encodings = state.pop("_pickled_encodings", None)
        self.__dict__.update(state)
        self._make_op()
        if encodings is None:
            self._encoding = None
        else:
            self._encoding = []
            for mn, mx, delta, offset, bw in encodings:
                e = TfEncoding()
                e.bw, e.max, e.min, e.delta, e.offset = bw, mx, mn, delta, offset
                self._encoding.append(e)

    def _make_op(self):
        raise NotImplementedError

    def _encodings_from_op(self):
        """(encodings, valid) from the native analyzers."""
        raise NotImplementedError

    def compute_encoding(self):
        """v1/tensor_quantizer.py:280-321."""
        if not self.enabled or self._is_encoding_frozen:
            return
        if self.bitwidth == 32:
            self._encoding = None
            return
        if self.data_type == QuantizationDataType.float:
            if self.bitwidth == 16:
                self._encoding = None
            elif self.bitwidth == 8:
                self._encoding = [TfEncoding()]
            else:
                raise ValueError("Only bitwidths [8, 16] allowed for float data type, not ", str(self.bitwidth))
            return
        encodings, valid = self._encodings_from_op()
        self._encoding = []
        if not valid:
            self.enabled = False
        else:
            self._encoding = encodings
        self.is_unsigned_symmetric = (self.use_symmetric_encodings and self.use_unsigned_symmetric and
                                      all(e.min >= 0 and e.max >= 0 for e in self._encoding))

    def quantize_dequantize(self, tensor, round_mode):
        if not (torch.is_grad_enabled() and isinstance(tensor, torch.Tensor) and tensor.requires_grad):
            # no graph would be recorded: the forward's values without the autograd call
            return _qdq_values(tensor, self, _round_mode(round_mode))
        return QuantizeDequantize.apply(tensor, self, _round_mode(round_mode))

    def quantize(self, tensor, round_mode):
        return Quantize.apply(tensor, self, _round_mode(round_mode))

    def reset_encoding_stats(self):
        if not self._is_encoding_frozen:
            self._op().resetEncodingStats()
            self._encoding = None

    def get_stats_histogram(self):
        if self._quant_scheme != QuantScheme.post_training_tf_enhanced:
            raise RuntimeError("get_stats_histogram() can be invoked only when quantization scheme is TF-Enhanced.")
        if not self._encoding:
            raise RuntimeError("get_stats_histogram() can be invoked only when encoding is computed.")
        op = self._op()
        return [op.getStatsHistogram(c) for c in range(op.num_channels)]

    def freeze_encoding(self):
        if not self._encoding:
            raise RuntimeError("Encoding can be frozen only when it is not None.")
        self._is_encoding_frozen = True

    def set_percentile_value(self, percentile_value):
        self._op().setPercentileValue(percentile_value)

    def _op(self) -> AimetTensorQuantizer:
        return self._cppOp[0]


class StaticGridPerTensorQuantizer(StaticGridTensorQuantizer):
    """v1/tensor_quantizer.py:403-481."""

    def __init__(self, bitwidth, round_mode, quant_scheme, use_symmetric_encodings, enabled_by_default,
                 data_type=QuantizationDataType.int):
        super().__init__(bitwidth, round_mode, quant_scheme, use_symmetric_encodings, enabled_by_default, data_type)
        self._make_op()

    def _make_op(self):
        self._cppOp = [AimetTensorQuantizer(_pymo_mode(self._quant_scheme))]

    @property
    def encoding(self):
        return self._encoding[0] if self._encoding else None

    @encoding.setter
    def encoding(self, encoding):
        if self._is_encoding_frozen:
            raise RuntimeError("Encoding can be set only when it is not frozen.")
        if isinstance(encoding, list) and len(encoding) == 1:
            self._encoding = encoding
        else:
            self._encoding = [encoding]

    def update_encoding_stats(self, tensor):
        """v1/tensor_quantizer.py:452-481."""
        if not self.enabled or self._is_encoding_frozen or self.bitwidth == 32:
            return
        if self.data_type == QuantizationDataType.float:
            raise NotImplementedError("float (fp8/fp16) quantization is outside the MI355X integer QDQ core")
        if self.encoding_min_max_fixed_vals is not None:
            tensor = torch.tensor(list(self.encoding_min_max_fixed_vals), device=tensor.device)
        if tensor.dtype in (torch.float16, torch.bfloat16):
            tensor = tensor.to(torch.float32)
        self._op().updateStats(tensor, tensor.is_cuda)

    def _encodings_from_op(self):
        enc, valid = self._op().getEncoding(self.bitwidth, self.use_symmetric_encodings, self.use_strict_symmetric,
                                            self.use_unsigned_symmetric)
        return [enc], valid


class StaticGridPerChannelQuantizer(StaticGridTensorQuantizer):
    """v1/tensor_quantizer.py:483-571."""

    def __init__(self, bitwidth, round_mode, quant_scheme, use_symmetric_encodings, num_channels,
                 enabled_by_default, ch_axis=0, data_type=QuantizationDataType.int):
        super().__init__(bitwidth, round_mode, quant_scheme, use_symmetric_encodings, enabled_by_default, data_type)
        self._num_channels = int(num_channels)
        self._ch_axis = ch_axis
        self._make_op()

    def _make_op(self):
        self._cppOp = [AimetTensorQuantizer(_pymo_mode(self._quant_scheme), num_channels=self._num_channels)]

    @property
    def encoding(self):
        return self._encoding

    @encoding.setter
    def encoding(self, encoding):
        if self._is_encoding_frozen:
            raise RuntimeError("Encoding can be set only when it is not frozen.")
        self._encoding = encoding

    @property
    def channel_axis(self):
        return self._ch_axis

    def update_encoding_stats(self, tensor):
        """v1/tensor_quantizer.py:535-571, all channels in one launch."""
        if not self.enabled or self._is_encoding_frozen or self.bitwidth == 32:
            return
        if self.data_type == QuantizationDataType.float:
            raise NotImplementedError("float (fp8/fp16) quantization is outside the MI355X integer QDQ core")
        if tensor.dtype in (torch.float16, torch.bfloat16):
            tensor = tensor.to(torch.float32)
        if self.encoding_min_max_fixed_vals is not None:
            # every channel analyzer sees the same 2-element tensor (v1/tensor_quantizer.py:556-561)
            fixed = torch.tensor(list(self.encoding_min_max_fixed_vals), device=tensor.device)
            tensor = fixed.view(1, 2).expand(self._num_channels, 2).contiguous()
            self._op().updateStatsPerChannel(tensor, 0)
            return
        self._op().updateStatsPerChannel(tensor, self._ch_axis)

    def _encodings_from_op(self):
        return self._op()._get_encodings(self.bitwidth, self.use_symmetric_encodings, self.use_strict_symmetric,
                                         self.use_unsigned_symmetric)

    def channel_table(self, device):
        return self._op().channelTable(self._encoding, device)


# ---------------------------------------------------------------------------------------------
# autograd
# ---------------------------------------------------------------------------------------------
def _is_scalar_bound(v):
    """A bound the reference's broadcast_to_tensor turns into a 0-dim tensor (a python number or a
    0-dim tensor). A list or a 1-D tensor, even of one element, stays 1-D
    (quantsim_straight_through_grad.py:66-88)."""
    return isinstance(v, (int, float)) or (torch.is_tensor(v) and v.dim() == 0)


def _scalar_bound(v, dtype):
    """The value the reference compares x with for a scalar bound: broadcast_to_tensor makes a
    python number a 0-dim tensor (torch.tensor(float) is float32), and a 0-dim tensor takes no part
    in type promotion, so `encoding_min <= x` runs in x's dtype with the bound rounded to it
    (float32 -> fp16/bf16 for a python float: two roundings)."""
    t = v.detach().cpu() if torch.is_tensor(v) else torch.tensor(v)
    return float(t.to(dtype))


def compute_dloss_by_dx(x, grad, encoding_min, encoding_max, ch_axis=0):
    """quantsim_straight_through_grad.py:91-118 as one kernel: grad * (min <= x <= max).

    encoding_min/max: python floats / 0-dim tensors (per-tensor: compared in x's dtype, as the
    reference's 0-dim bound is) or sequences / 1-D tensors of C values (compared in float32, the
    promoted type of the reference's 1-D float32 bound tensor)."""
    if not (x.is_cuda and grad.is_cuda):   # CPU tensors: staged through HBM, result back on grad's device
        xd, _ = _stage(x, "x", allow_16bit=True)
        gd, _ = _stage(grad, "grad", device=xd.device.index, allow_16bit=True)
        return compute_dloss_by_dx(xd, gd, encoding_min, encoding_max, ch_axis).to(grad.device)
    _require_gpu(x, True, "x", allow_16bit=True)
    _require_gpu(grad, True, "grad", allow_16bit=True)
    x = x.contiguous()
    grad = grad.contiguous()
    if _is_scalar_bound(encoding_min) and x.dtype in IO_DTYPES:
        # rounded to x's dtype before any upcast: the mask is the reference's 16-bit compare
        encoding_min, encoding_max = _scalar_bound(encoding_min, x.dtype), _scalar_bound(encoding_max, x.dtype)
    if x.dtype in IO_DTYPES and grad.dtype == x.dtype:
        return _ste_16(x, grad, encoding_min, encoding_max, ch_axis)
    if x.dtype != torch.float32 or grad.dtype != torch.float32:
        return compute_dloss_by_dx(x.float(), grad.float(), encoding_min, encoding_max, ch_axis).to(grad.dtype)
    out = torch.empty_like(grad)
    if _is_scalar_bound(encoding_min):
        mn = _scalar_bound(encoding_min, torch.float32)
        mx = _scalar_bound(encoding_max, torch.float32)
        # torch.tensor(python float) is float32: the comparison bounds are rounded to float
        with torch.cuda.device(x.device):
            _native.call("aimet_ste_backward_per_tensor", x.data_ptr(), grad.data_ptr(), out.data_ptr(), x.numel(),
                         mn, mx, _stream(x))
        return out
    mins = torch.as_tensor(encoding_min, dtype=torch.float32).to(x.device).contiguous()
    maxs = torch.as_tensor(encoding_max, dtype=torch.float32).to(x.device).contiguous()
    outer, C, K = per_channel_view(x.shape, ch_axis)
    if mins.numel() != C:
        raise ValueError("expected %d per-channel bounds, got %d" % (C, mins.numel()))
    with torch.cuda.device(x.device):
        _native.call("aimet_ste_backward", x.data_ptr(), grad.data_ptr(), out.data_ptr(), outer, C, K,
                     mins.data_ptr(), maxs.data_ptr(), _stream(x))
    return out


def _ste_16(x, grad, encoding_min, encoding_max, ch_axis):
    """fp16 / bf16 STE in one pass (aimet_ste_backward_16): float(x) vs float32 bounds. Scalar
    bounds arrive already rounded to x's dtype (compute_dloss_by_dx), so the float32 compare is
    the reference's 16-bit one; per-channel bounds are float32, as the reference's promoted ones."""
    out = torch.empty_like(grad)
    code = IO_DTYPES[x.dtype]
    with torch.cuda.device(x.device):
        if _is_scalar_bound(encoding_min):
            _native.call("aimet_ste_backward_16", x.data_ptr(), grad.data_ptr(), out.data_ptr(), 1, 1, x.numel(), code,
                         None, None, float(encoding_min), float(encoding_max), _stream(x))
            return out
        mins = torch.as_tensor(encoding_min, dtype=torch.float32).to(x.device).contiguous()
        maxs = torch.as_tensor(encoding_max, dtype=torch.float32).to(x.device).contiguous()
        outer, C, K = per_channel_view(x.shape, ch_axis)
        if mins.numel() != C:
            raise ValueError("expected %d per-channel bounds, got %d" % (C, mins.numel()))
        _native.call("aimet_ste_backward_16", x.data_ptr(), grad.data_ptr(), out.data_ptr(), outer, C, K, code,
                     mins.data_ptr(), maxs.data_ptr(), 0.0, 0.0, _stream(x))
    return out


def _ste_bounds(tq, device):
    """float32 per-channel STE bounds = the raw encoding min/max (the QDQ table holds the gated
    ones), cached until any encoding changes (the reference re-uploads them every backward,
    quantsim_straight_through_grad.py:75-76)."""
    key = PerChannelTable.key(tq._encoding)
    cache = tq.__dict__.setdefault("_ste_cache", {})   # device -> (key, mins, maxs)
    hit = cache.get(device)
    if hit is None or hit[0] != key:
        mins = torch.tensor([e.min for e in tq._encoding], dtype=torch.float32, device=device)
        maxs = torch.tensor([e.max for e in tq._encoding], dtype=torch.float32, device=device)
        cache[device] = hit = (key, mins, maxs)
    return hit[1], hit[2]


def _qdq_values(tensor, tq, round_mode):
    """QuantizeDequantize's forward values (v1/tensor_quantizer.py:1098-1168)."""
    if not tq.enabled or tq.bitwidth == 32:
        return tensor
    if tq.data_type == QuantizationDataType.float:
        if tq.bitwidth == 16:
            return tensor.half().float()
        raise NotImplementedError("fp8 quantization is outside the MI355X integer QDQ core")
    dtype = tensor.dtype
    # a CPU tensor is staged through HBM (the same kernels; the result goes back to the host)
    if tensor.is_cuda:
        t, staged = tensor, False
    else:
        t, staged = _stage(tensor if dtype in IO_DTYPES else tensor.to(torch.float32), "tensor", allow_16bit=True)
    # fp16 / bf16 go through the fused 16-bit I/O kernels (identical to the reference's
    # upcast -> fp32 QDQ -> downcast, v1/tensor_quantizer.py:1116-1168); others upcast
    t = t if dtype in IO_DTYPES else t.to(torch.float32)
    if isinstance(tq, StaticGridPerChannelQuantizer):
        t = t.contiguous()
        outer, C, K = per_channel_view(t.shape, tq.channel_axis)
        table = tq.channel_table(t.device)
        out = qdq_per_channel_table(t, table, outer, C, K, round_mode)
    else:
        out = AimetTensorQuantizer.quantize_dequantize_tensor(t, tq.encoding, round_mode)
    return out.to(dtype).cpu() if staged else out.to(dtype)


class QuantizeDequantize(torch.autograd.Function):
    """v1/tensor_quantizer.py:1098-1213."""

    @staticmethod
    def forward(ctx, tensor, tensor_quantizer, round_mode):
        tq = tensor_quantizer
        ctx.tensor_quantizer = tq
        out = _qdq_values(tensor, tq, round_mode)
        if out is not tensor:
            ctx.save_for_backward(tensor)
        return out

    @staticmethod
    def backward(ctx, grad):
        tq = ctx.tensor_quantizer
        if tq.enabled and tq.data_type == QuantizationDataType.int and tq.bitwidth != 32:
            (x,) = ctx.saved_tensors
            dtype = grad.dtype
            # fp16 / bf16 x stays in its dtype: a scalar bound is compared in x's dtype, as in the
            # reference (compute_dloss_by_dx rounds it, then fuses or upcasts)
            xf = x if x.dtype in IO_DTYPES else x.to(torch.float32)
            gf = grad if grad.dtype in IO_DTYPES else grad.to(torch.float32)
            if isinstance(tq, StaticGridPerChannelQuantizer):
                mins, maxs = _ste_bounds(tq, x.device)
                g = compute_dloss_by_dx(xf, gf, mins, maxs, tq.channel_axis)
            else:
                g = compute_dloss_by_dx(xf, gf, tq.encoding.min, tq.encoding.max)
            return g.to(dtype), None, None
        return grad, None, None


class Quantize(torch.autograd.Function):
    """v1/tensor_quantizer.py:1216-1264 (quantize-only, STE gradient)."""

    @staticmethod
    def forward(ctx, tensor, tensor_quantizer, round_mode):
        tq = tensor_quantizer
        ctx.tensor_quantizer = tq
        shift_to_signed = not (tq.use_symmetric_encodings and tq.use_unsigned_symmetric)
        if isinstance(tq, StaticGridPerChannelQuantizer):
            outs = []
            for c, enc in enumerate(tq.encoding):
                sl = tensor.select(tq.channel_axis, c).contiguous()
                outs.append(tq._op().quantize(sl, enc, round_mode, True, shift_to_signed))
            out = torch.stack(outs, dim=tq.channel_axis)
        else:
            out = tq._op().quantize(tensor.to(torch.float32), tq.encoding, round_mode, True, shift_to_signed)
        ctx.save_for_backward(tensor)
        return out

    @staticmethod
    def backward(ctx, grad):
        return QuantizeDequantize.backward(ctx, grad)


# ---------------------------------------------------------------------------------------------
# batched compute_encoding (QuantizationSimModel.compute_encodings' per-quantizer loop)
# ---------------------------------------------------------------------------------------------
def compute_encodings_batched(quantizers):
    """``q.compute_encoding()`` for every quantizer (v1/tensor_quantizer.py:280-321 semantics) with
    one native call -- one device search launch + one stream sync -- per distinct
    (bitwidth, symmetric, strict, unsigned) setting instead of one sync per quantizer."""
    groups = {}
    for q in quantizers:
        if not q.enabled or q._is_encoding_frozen or q.bitwidth == 32 or \
                q.data_type == QuantizationDataType.float:
            q.compute_encoding()           # the non-native branches
            continue
        key = (int(q.bitwidth), bool(q.use_symmetric_encodings), bool(q.use_strict_symmetric),
               bool(q.use_unsigned_symmetric), str(q._op()._device))
        groups.setdefault(key, []).append(q)
    for (bw, sym, strict, unsign, _), qs in groups.items():
        results = AimetTensorQuantizer.getEncodings([q._op() for q in qs], bw, sym, strict, unsign)
        for q, (enc, valid) in zip(qs, results):
            q._encoding = []
            if not valid:
                q.enabled = False
            else:
                q._encoding = enc if isinstance(enc, list) else [enc]
            q.is_unsigned_symmetric = (q.use_symmetric_encodings and q.use_unsigned_symmetric and
                                       all(e.min >= 0 and e.max >= 0 for e in q._encoding))
