"""Drop-in for the ``AimetTensorQuantizer`` torch extension
(TrainingExtensions/torch/src/AimetTensorQuantizer.cpp:79-331).

Same class name, method names and argument meaning. Differences, all MI355X-first:

* statistics stay in HBM (no host synchronisation in ``updateStats``);
* kernels run on torch's *current* HIP stream of the tensor's device (the reference used the
  legacy default stream);
* one object may hold the analyzers of C channels (``num_channels``), updated in one launch by
  ``updateStatsPerChannel`` -- the reference needed C objects and a Python loop;
* there is no CPU compute path: a CPU tensor (the reference's ``use_cuda=False``,
  COMP_MODE_CPU) is staged through HBM -- copied to the device, computed by the same HIP
  kernels, results copied back -- and a process without a HIP device raises ``RuntimeError``.
"""
import array
import ctypes
import gc
import itertools

import torch

from aimet_amd import _native
from aimet_amd.libpymo import QuantizationMode, RoundingMode, TfEncoding, encodings_to_c

_seed_counter = itertools.count(1)
# calibrateResidentAsync: activations and parameters in two native calls (False: one; the tests
# compare the two forms)
_CAL_SPLIT = True


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _require_gpu(t: torch.Tensor, use_cuda: bool = True, what: str = "input", allow_16bit: bool = False):
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor" % what)
    if not t.is_cuda or not use_cuda:
        raise RuntimeError("aimet_amd: %s must be a HIP (cuda) tensor with use_cuda=True; the MI355X core has no "
                           "CPU path" % what)
    if allow_16bit and t.dtype in (torch.float16, torch.bfloat16):
        return
    if t.dtype != torch.float32:
        raise TypeError("aimet_amd: %s must be float32 (got %s); upcast as the reference callers do "
                        "(v1/tensor_quantizer.py:1124)" % (what, t.dtype))


def _stage(t: torch.Tensor, what: str = "input", device=None, allow_16bit: bool = False):
    """(HIP tensor, staged) for a tensor given to a public entry point: a CPU tensor is copied to
    `device` (default: the current HIP device) and `staged` is True, so the caller copies its
    result back. Nothing is computed on the host."""
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor" % what)
    staged = False
    if not t.is_cuda:
        if not torch.cuda.is_available():
            raise RuntimeError("aimet_amd: %s is a CPU tensor and no HIP device is visible; the MI355X core "
                               "stages CPU tensors through HBM and has no CPU compute path" % what)
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        t, staged = t.to(dev), True
    _require_gpu(t, True, what, allow_16bit)
    return t, staged


def per_channel_view(shape, ch_axis):
    """[outer][C][K] triple of a tensor quantized along ch_axis (v1/tensor_quantizer.py:1150-1153)."""
    sizes = list(shape)
    if ch_axis < 0:
        ch_axis += len(sizes)
    outer = 1
    for s in sizes[:ch_axis]:
        outer *= s
    K = 1
    for s in sizes[ch_axis + 1:]:
        K *= s
    return outer, sizes[ch_axis], K


class PerChannelTable:
    """Device table [4][C] {min, max, delta, offset} built once per encoding change
    (AimetTensorQuantizer.cpp:262-299 rebuilt and re-uploaded it on every call)."""

    def __init__(self):
        self._tables = {}   # device -> (key, table): DataParallel replicas read it on every device

    @staticmethod
    def key(encodings):
        """Changes when any encoding field is assigned (TfEncoding._version) or any list element is
        replaced, even by an older TfEncoding (the element identities)."""
        return (TfEncoding._version, tuple(map(id, encodings)))

    def get(self, encodings, device):
        key = PerChannelTable.key(encodings)
        hit = self._tables.get(device)
        if hit is None or hit[0] != key:
            C = len(encodings)
            table = torch.empty((4, C), dtype=torch.float32, device=device)
            _native.call("aimet_per_channel_table", encodings_to_c(encodings), C, table.data_ptr(),
                         torch.cuda.current_stream(device).cuda_stream)
            self._tables[device] = hit = (key, table)
        return hit[1]


class AimetTensorQuantizer:
    """AimetTensorQuantizer(quant_scheme[, num_channels]) -- AimetTensorQuantizer.cpp:82-87."""

    def __init__(self, quant_scheme, num_channels: int = 1, device=None):
        self._scheme = QuantizationMode(int(quant_scheme))
        self._num_channels = int(num_channels)
        self._device = device
        self._handle = None
        self._is_encoding_valid = False
        self._pc_table = PerChannelTable()
        self._pending_percentile = None

    # -- lifetime ------------------------------------------------------------------------------
    def _ensure(self, device: torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
        if self._handle is not None and self._device == idx:
            return self._handle
        if self._handle is not None:
            # statistics live on one device; moving devices starts from empty statistics
            self._release()
        h = ctypes.c_void_p()
        _native.call("aimet_tq_create", int(self._scheme), self._num_channels, idx, ctypes.byref(h))
        self._handle, self._device = h, idx
        if self._pending_percentile is not None:
            _native.call("aimet_tq_set_percentile_value", self._handle, float(self._pending_percentile))
        return h

    @staticmethod
    def _ensure_many(quantizers, device: torch.device):
        """_ensure for many quantizers: the ones without device state on `device` get it from one
        aimet_tq_create_many call (one allocation + one initialisation launch for all)."""
        idx = device.index if device.index is not None else torch.cuda.current_device()
        handles = [q._handle if q._device == idx else None for q in quantizers]
        if None not in handles:   # every quantizer already has its state on this device
            return handles
        fresh = [q for q in quantizers if q._handle is None or q._device != idx]
        if len(fresh) > 1:
            for q in fresh:
                q._release()
            n = len(fresh)
            out = (ctypes.c_void_p * n)()
            _native.call("aimet_tq_create_many", (ctypes.c_int * n)(*[int(q._scheme) for q in fresh]),
                         (ctypes.c_int64 * n)(*[q._num_channels for q in fresh]), n, idx, out)
            for q, h in zip(fresh, out):
                q._handle, q._device = ctypes.c_void_p(h), idx
                if q._pending_percentile is not None:
                    _native.call("aimet_tq_set_percentile_value", q._handle, float(q._pending_percentile))
        return [q._handle if q._handle is not None and q._device == idx else q._ensure(device) for q in quantizers]

    def _release(self):
        if self._handle is not None:
            try:
                _native.call("aimet_tq_destroy", self._handle)
            finally:
                self._handle = None

    def __del__(self):
        try:
            self._release()
        except Exception:  # interpreter shutdown
            pass

    def __getstate__(self):
        """Pickle / deepcopy: the analyzer settings travel, the device statistics do not (the
        reference never pickles its op: StaticGridTensorQuantizer.__getstate__ drops it and
        __setstate__ builds a fresh one, v1/tensor_quantizer.py:182-220). The copy starts with
        empty statistics and creates its native object on first use."""
        return {"scheme": int(self._scheme), "num_channels": self._num_channels}

    def __setstate__(self, state):
        self.__init__(state["scheme"], state["num_channels"])

    @property
    def num_channels(self):
        return self._num_channels

    @property
    def quant_scheme(self):
        return self._scheme

    # -- statistics --------------------------------------------------------------------------
    def resetEncodingStats(self):
        """AimetTensorQuantizer.cpp:89-96."""
        self._is_encoding_valid = False
        self._pending_percentile = None
        if self._handle is not None:
            with torch.cuda.device(self._device):
                _native.call("aimet_tq_reset_encoding_stats", self._handle,
                             torch.cuda.current_stream(self._device).cuda_stream)

    @staticmethod
    def resetEncodingStatsMany(quantizers):
        """resetEncodingStats of many quantizers: two launches on the current stream of their device
        (aimet_tq_reset_encoding_stats_many), no host synchronisation."""
        qs = list(quantizers)
        for q in qs:
            q._is_encoding_valid = False
            q._pending_percentile = None
        live = [q for q in qs if q._handle is not None]
        by_dev = {}
        for q in live:
            by_dev.setdefault(q._device, []).append(q)
        for dev, group in by_dev.items():
            handles = (ctypes.c_void_p * len(group))(*[q._handle for q in group])
            with torch.cuda.device(dev):
                _native.call("aimet_tq_reset_encoding_stats_many", handles, len(group),
                             torch.cuda.current_stream(dev).cuda_stream)

    def updateStats(self, tensor: torch.Tensor, use_cuda: bool = True):
        """AimetTensorQuantizer.cpp:98-127 (per-tensor; the whole tensor feeds one analyzer)."""
        if self._num_channels != 1:
            raise ValueError("updateStats on a %d-channel quantizer: use updateStatsPerChannel" % self._num_channels)
        t, _ = _stage(tensor, device=self._device)
        t = t if t.is_contiguous() else t.contiguous()
        h = self._ensure(t.device)
        with torch.cuda.device(t.device):
            _native.call("aimet_tq_update_stats", h, t.data_ptr(), 1, 1, t.numel(), _stream(t))
        self._is_encoding_valid = True

    def updateStatsPerChannel(self, tensor: torch.Tensor, ch_axis: int = 0, use_cuda: bool = True):
        """All C channel analyzers in one pass: replaces the loop of
        v1/tensor_quantizer.py:567-570 (select(ch_axis, c).contiguous() + updateStats per channel)."""
        t, _ = _stage(tensor, device=self._device)
        t = t if t.is_contiguous() else t.contiguous()
        outer, C, K = per_channel_view(t.shape, ch_axis)
        if C != self._num_channels:
            raise ValueError("tensor has %d channels along axis %d, quantizer has %d" % (C, ch_axis,
                                                                                         self._num_channels))
        h = self._ensure(t.device)
        with torch.cuda.device(t.device):
            _native.call("aimet_tq_update_stats", h, t.data_ptr(), outer, C, K, _stream(t))
        self._is_encoding_valid = True

    # -- phased statistics (sharded calibration, aimet_amd.distributed) ------------------------
    @property
    def uses_histogram(self):
        return self._scheme != QuantizationMode.QUANTIZATION_TF

    def _view(self, tensor, ch_axis):
        _require_gpu(tensor)
        t = tensor if tensor.is_contiguous() else tensor.contiguous()
        if self._num_channels == 1:
            return t, (1, 1, t.numel())
        outer, C, K = per_channel_view(t.shape, ch_axis)
        if C != self._num_channels:
            raise ValueError("tensor has %d channels, quantizer has %d" % (C, self._num_channels))
        return t, (outer, C, K)

    def bind_exchange(self, minmax: torch.Tensor, counts: torch.Tensor = None):
        """Keep this quantizer's exchanged statistics in slices of caller-owned packed buffers:
        minmax float32[2*C], counts int64[512*C] (zeroed)."""
        h = self._ensure(minmax.device)
        _native.call("aimet_tq_bind_exchange", h, minmax.data_ptr(),
                     counts.data_ptr() if counts is not None else None)
        self._bound = (minmax, counts)   # keep the memory alive

    def batch_minmax(self, tensor, ch_axis=0):
        t, (outer, C, K) = self._view(tensor, ch_axis)
        h = self._ensure(t.device)
        _native.call("aimet_tq_batch_minmax", h, t.data_ptr(), outer, C, K, _stream(t))
        self._is_encoding_valid = True

    def fold_minmax(self):
        _native.call("aimet_tq_fold_minmax", self._handle, torch.cuda.current_stream(self._device).cuda_stream)

    def batch_histogram(self, tensor, ch_axis=0):
        t, (outer, C, K) = self._view(tensor, ch_axis)
        _native.call("aimet_tq_batch_histogram", self._ensure(t.device), t.data_ptr(), outer, C, K, _stream(t))

    def fold_histogram(self, count_per_channel: int):
        _native.call("aimet_tq_fold_histogram", self._handle, int(count_per_channel),
                     torch.cuda.current_stream(self._device).cuda_stream)

    def getEncoding(self, bitwidth, use_symmetric_encodings, use_strict_symmetric, use_unsigned_symmetric):
        """AimetTensorQuantizer.cpp:180-192 -> (TfEncoding, is_valid). Per-channel objects return a
        list of C encodings."""
        encs, valid = self._get_encodings(bitwidth, use_symmetric_encodings, use_strict_symmetric,
                                          use_unsigned_symmetric)
        if self._num_channels == 1:
            return encs[0], valid
        return encs, valid

    def _get_encodings(self, bw, sym, strict, unsign):
        C = self._num_channels
        if self._handle is None or not self._is_encoding_valid:
            return [TfEncoding() for _ in range(C)], False
        out = TfEncoding.array(C)
        valid = ctypes.c_int(0)
        with torch.cuda.device(self._device):
            _native.call("aimet_tq_get_encoding", self._handle, int(bw), int(bool(sym)), int(bool(strict)),
                         int(bool(unsign)), out, ctypes.byref(valid),
                         torch.cuda.current_stream(self._device).cuda_stream)
        return list(out), bool(valid.value)

    # -- many per-tensor quantizers at once (aimet_tq_*_many: one launch per phase) ------------
    @staticmethod
    def _many(name, quantizers, tensors=None, counts=None):
        """One batched entry point over many per-tensor quantizers. The argument tables are built
        from array.array buffers (no per-element ctypes conversion): for ViT-L/16's 318
        quantizers the host side of a calibration batch is on the critical path (the GPU waits for
        the first launch)."""
        qs = quantizers if type(quantizers) is list else list(quantizers)
        if not qs:
            return
        n = len(qs)
        ts = None
        if tensors is not None:
            ts = tensors if type(tensors) is list else list(tensors)
            f32 = torch.float32
            ptrs, sizes = array.array("Q"), array.array("q")
            for i, t in enumerate(ts):   # one pass: layout, device, dtype, pointer, size
                if not t.is_contiguous():
                    if ts is tensors:
                        ts = list(ts)
                    t = ts[i] = t.contiguous()
                if not (t.is_cuda and t.dtype is f32):
                    _require_gpu(t)
                ptrs.append(t.data_ptr())
                sizes.append(t.numel())
            dev = ts[0].device
            idx = dev.index if dev.index is not None else torch.cuda.current_device()
        else:
            idx = qs[0]._device
            dev = torch.device("cuda", idx)
        hv = array.array("Q")
        for q in qs:
            h = q._handle
            if q._num_channels != 1:
                raise ValueError("the batched statistics entry points take per-tensor quantizers")
            if h is None or q._device != idx:
                if tensors is None:
                    raise RuntimeError("aimet_amd: quantizer has no device state")
                AimetTensorQuantizer._ensure_many(qs, dev)
                hv = array.array("Q", [q._handle.value for q in qs])
                break
            hv.append(h.value)
        args = [(ctypes.c_void_p * n).from_buffer(hv)]
        keep = [hv]
        if ts is not None:
            keep += [ptrs, sizes]
            args += [(ctypes.c_void_p * n).from_buffer(ptrs), (ctypes.c_int64 * n).from_buffer(sizes)]
        if counts is not None:
            cnt = array.array("q", [int(c) for c in counts])
            keep.append(cnt)
            args.append((ctypes.c_int64 * n).from_buffer(cnt))
        with torch.cuda.device(dev):
            _native.call(name, *args, n, torch.cuda.current_stream(dev).cuda_stream)
        if name in ("aimet_tq_update_stats_many", "aimet_tq_batch_minmax_many"):
            for q in qs:
                q._is_encoding_valid = True
        del keep
        return ts   # keep the contiguous copies alive until the caller synchronises

    @staticmethod
    def updateStatsMany(quantizers, tensors):
        """updateStats(tensors[i]) for every (per-tensor) quantizer with one launch per phase."""
        return AimetTensorQuantizer._many("aimet_tq_update_stats_many", quantizers, tensors)

    @staticmethod
    def updateStatsPerChannelMany(quantizers, tensors, ch_axes=None):
        """updateStatsPerChannel(tensors[i], ch_axes[i]) for every quantizer in two launches (one
        workgroup per channel; the fold runs in the workgroup that reduced the channel). Returns
        the contiguous inputs, to be kept alive until the stream is synchronised."""
        qs = list(quantizers)
        if not qs:
            return []
        ch_axes = list(ch_axes) if ch_axes is not None else [0] * len(qs)
        ts, outers, Cs, Ks = [], [], [], []
        for q, t, ax in zip(qs, tensors, ch_axes):
            _require_gpu(t)
            t = t if t.is_contiguous() else t.contiguous()
            outer, C, K = per_channel_view(t.shape, ax) if q._num_channels != 1 else (1, 1, t.numel())
            if C != q._num_channels:
                raise ValueError("tensor has %d channels along axis %d, quantizer has %d" % (C, ax, q._num_channels))
            ts.append(t)
            outers.append(outer)
            Cs.append(C)
            Ks.append(K)
        dev = ts[0].device
        n = len(qs)
        handles = AimetTensorQuantizer._ensure_many(qs, dev)
        with torch.cuda.device(dev):
            _native.call("aimet_tq_update_stats_channels_many", (ctypes.c_void_p * n)(*handles),
                         (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]), (ctypes.c_int64 * n)(*outers),
                         (ctypes.c_int64 * n)(*Cs), (ctypes.c_int64 * n)(*Ks), n,
                         torch.cuda.current_stream(dev).cuda_stream)
        for q in qs:
            q._is_encoding_valid = True
        return ts

    @staticmethod
    def batch_minmax_many(quantizers, tensors):
        return AimetTensorQuantizer._many("aimet_tq_batch_minmax_many", quantizers, tensors)

    @staticmethod
    def fold_minmax_many(quantizers):
        return AimetTensorQuantizer._many("aimet_tq_fold_minmax_many", quantizers)

    @staticmethod
    def batch_histogram_many(quantizers, tensors):
        return AimetTensorQuantizer._many("aimet_tq_batch_histogram_many", quantizers, tensors)

    @staticmethod
    def fold_histogram_many(quantizers, counts):
        """counts: per-quantizer element counts, a host sequence, or an int64 device tensor read by
        the fold kernel itself (no host round trip: aimet_tq_fold_histogram_many_dev)."""
        if isinstance(counts, torch.Tensor):
            qs = list(quantizers)
            if not qs:
                return
            if counts.dtype != torch.int64 or not counts.is_cuda or counts.numel() < len(qs) \
                    or not counts.is_contiguous():
                raise ValueError("device element counts: a contiguous int64 HIP tensor of >= %d entries" % len(qs))
            dev = counts.device
            n = len(qs)
            with torch.cuda.device(dev):
                _native.call("aimet_tq_fold_histogram_many_dev", (ctypes.c_void_p * n)(*[q._handle for q in qs]),
                             counts.data_ptr(), n, torch.cuda.current_stream(dev).cuda_stream)
            return
        return AimetTensorQuantizer._many("aimet_tq_fold_histogram_many", quantizers, counts=counts)

    @staticmethod
    def getEncodings(quantizers, bitwidth, use_symmetric_encodings, use_strict_symmetric,
                     use_unsigned_symmetric):
        """getEncoding of many quantizers with ONE stream synchronisation (every device-side
        encoding search is enqueued first): the per-quantizer loop of
        QuantizationSimModel.compute_encodings (v1/quantsim.py:425-449), batched.
        Returns [(encoding or list of encodings, is_valid)] in input order."""
        return AimetTensorQuantizer.getEncodingsAsync(quantizers, bitwidth, use_symmetric_encodings,
                                                      use_strict_symmetric, use_unsigned_symmetric).result()

    @staticmethod
    def getEncodingsAsync(quantizers, bitwidth, use_symmetric_encodings, use_strict_symmetric,
                          use_unsigned_symmetric) -> "PendingEncodings":
        """getEncodings in two halves: the device searches and the copies of their results are
        enqueued on the current stream now (aimet_tq_get_encodings_launch); .result() waits for
        them and builds the encodings. Between the two the host may enqueue other work."""
        return PendingEncodings(list(quantizers), bitwidth, use_symmetric_encodings, use_strict_symmetric,
                                use_unsigned_symmetric)

    @staticmethod
    def calibrateResidentAsync(act_quantizers, activations, param_quantizers, params, param_ch_axes=None,
                               act_settings=(8, False, False, False), param_settings=(8, True, False, False),
                               reset=False, main_stream=None, side_stream=None):
        """One calibration batch in two native calls (aimet_calibrate_launch; one when `side_stream`
        is `main_stream` or _CAL_SPLIT is False): the activations' call first, so their min/max pass
        runs while the parameters' call is prepared. Optionally
        resetEncodingStats of every quantizer, the activations' statistics (one launch per phase for
        all per-tensor quantizers) + search on `main_stream`, the parameters' per-channel statistics
        + search on `side_stream` (after everything queued on main so far). Returns
        (PendingEncodings of the activations, PendingEncodings of the parameters) and the
        contiguous inputs, to be kept alive until both are finished."""
        aq, pq = list(act_quantizers), list(param_quantizers)
        if any(q._num_channels != 1 for q in aq):
            raise ValueError("calibrateResidentAsync: the activation quantizers are per-tensor")
        dev = (activations[0] if aq else params[0]).device
        ch_axes = list(param_ch_axes) if param_ch_axes is not None else [0] * len(pq)
        # every check runs before anything is launched or any quantizer changes: a refused call
        # leaves all state as it was (only native failures reach the request-discard path below)
        # host preparation is on the critical path of a ~4 ms call (the first launch waits for it):
        # one pass over the activations (checks, pointers, sizes) with the fewest torch attribute
        # calls, then the parameters' checks; a non-contiguous input's copy is queued only after
        # every check passed, on `main`, the stream the activations' kernels run on (the caller's
        # current stream may be another one)
        f32 = torch.float32
        keep, a_ptr, a_n, copies = list(activations), [], [], []
        for i, t in enumerate(keep):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == f32):
                _require_gpu(t)
                raise TypeError("calibrateResidentAsync takes float32 tensors (got %s)" % t.dtype)
            if t.is_contiguous():
                a_ptr.append(t.data_ptr())
            else:
                copies.append(i)
                a_ptr.append(0)
            a_n.append(t.numel())
        p_specs = _param_specs(pq, params, ch_axes)
        main = main_stream if main_stream is not None else torch.cuda.current_stream(dev)
        side = side_stream if side_stream is not None else main
        if copies:
            with torch.cuda.stream(main):
                for i in copies:
                    keep[i] = keep[i].contiguous()
                    a_ptr[i] = keep[i].data_ptr()
        na, np_ = len(aq), len(pq)
        i32x4 = ctypes.c_int32 * 4
        a_set, p_set = i32x4(*[int(v) for v in act_settings]), i32x4(*[int(v) for v in param_settings])
        split = _CAL_SPLIT and na > 0 and np_ > 0 and side is not main
        ra, rp = ctypes.c_void_p(), ctypes.c_void_p()
        if split:
            # two native calls: the activations' HBM passes are enqueued before the parameters'
            # host preparation runs, which then overlaps the min/max pass instead of delaying it.
            # The side stream starts after the inputs (everything on `main` so far); the first
            # call resets the activation quantizers there, the second adds the parameters' work.
            side.wait_stream(main)
            ha = AimetTensorQuantizer._ensure_many(aq, dev)
            nul = ctypes.c_void_p * 1
            with torch.cuda.device(dev):
                _native.call("aimet_calibrate_launch", (ctypes.c_void_p * na)(*ha), (ctypes.c_void_p * na)(*a_ptr),
                             (ctypes.c_int64 * na)(*a_n), na, nul(), nul(), (ctypes.c_int64 * 1)(),
                             (ctypes.c_int64 * 1)(), (ctypes.c_int64 * 1)(), 0, a_set, p_set, int(bool(reset)),
                             main.cuda_stream, side.cuda_stream, ctypes.byref(ra), ctypes.byref(ctypes.c_void_p()))
            for q in aq:
                q._is_encoding_valid = True
            if reset:
                for q in aq + pq:
                    q._pending_percentile = None
            try:
                # a non-contiguous parameter's copy goes on the side stream, after its wait for
                # `main` above and before the parameters' kernels (the second call runs every
                # operation on `side`, so no join would order a copy queued on `main`)
                with torch.cuda.stream(side):
                    p_ptr = _param_pointers(p_specs, keep)
                hp = AimetTensorQuantizer._ensure_many(pq, dev)
                nul, empty = ctypes.c_void_p * 1, ctypes.c_void_p()
                outers, Cs, Ks = ([s[i] for s in p_specs] for i in (1, 2, 3))
                with torch.cuda.device(dev):
                    # the parameters alone, every operation on the side stream; the main stream
                    # then waits for it (later work there sees the parameters' state, as in one call)
                    _native.call("aimet_calibrate_launch", nul(), nul(), (ctypes.c_int64 * 1)(), 0,
                                 (ctypes.c_void_p * np_)(*hp), (ctypes.c_void_p * np_)(*p_ptr),
                                 (ctypes.c_int64 * np_)(*outers), (ctypes.c_int64 * np_)(*Cs),
                                 (ctypes.c_int64 * np_)(*Ks), np_, a_set, p_set, int(bool(reset)),
                                 side.cuda_stream, side.cuda_stream, ctypes.byref(empty), ctypes.byref(rp))
            except BaseException:
                # the activations' call is in flight: discard its request (waits for its result copy)
                _native.call("aimet_tq_get_encodings_finish", ra, None, None)
                raise
            main.wait_stream(side)
            if empty.value:   # the second call's (empty) activation request
                _native.call("aimet_tq_get_encodings_finish", empty, None, None)
            for q in pq:
                q._is_encoding_valid = True
        else:
            if reset:
                for q in aq + pq:
                    q._pending_percentile = None
            # the copies on `main`: the native call starts `side` after everything queued there
            with torch.cuda.stream(main):
                p_ptr = _param_pointers(p_specs, keep)
            outers, Cs, Ks = ([s[i] for s in p_specs] for i in (1, 2, 3))
            handles = AimetTensorQuantizer._ensure_many(aq + pq, dev)
            with torch.cuda.device(dev):
                _native.call("aimet_calibrate_launch", (ctypes.c_void_p * max(na, 1))(*handles[:na]),
                             (ctypes.c_void_p * max(na, 1))(*a_ptr), (ctypes.c_int64 * max(na, 1))(*a_n), na,
                             (ctypes.c_void_p * max(np_, 1))(*handles[na:]), (ctypes.c_void_p * max(np_, 1))(*p_ptr),
                             (ctypes.c_int64 * max(np_, 1))(*outers), (ctypes.c_int64 * max(np_, 1))(*Cs),
                             (ctypes.c_int64 * max(np_, 1))(*Ks), np_, a_set, p_set, int(bool(reset)),
                             main.cuda_stream, side.cuda_stream, ctypes.byref(ra), ctypes.byref(rp))
            for q in aq + pq:
                q._is_encoding_valid = True
        return (PendingEncodings(aq, *act_settings, request=ra), PendingEncodings(pq, *param_settings, request=rp),
                keep)

    def getStatsHistogram(self, channel: int = 0):
        """AimetTensorQuantizer.cpp:194-198 -> list of (xLeft, pdf)."""
        import numpy as np
        if self._handle is None:
            if self._scheme == QuantizationMode.QUANTIZATION_TF:
                raise RuntimeError("the TF encoding analyzer keeps no histogram (TfEncodingAnalyzer.cpp:53-57)")
            return []
        xl = np.zeros(512, dtype=np.float64)
        pdf = np.zeros(512, dtype=np.float64)
        n = ctypes.c_int(0)
        with torch.cuda.device(self._device):
            _native.call("aimet_tq_get_stats_histogram", self._handle, int(channel),
                         xl.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                         pdf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(n),
                         torch.cuda.current_stream(self._device).cuda_stream)
        return [(float(xl[i]), float(pdf[i])) for i in range(n.value)]

    def entropy_state(self, channel: int = 0):
        """The entropy analyzer's TensorProfilingParams (math_functions.hpp:71-77) of `channel`:
        dict(has_hist, min, max, hist[512] bin counts, iterations)."""
        import numpy as np
        if self._scheme != QuantizationMode.QUANTIZATION_ENTROPY:
            raise RuntimeError("entropy_state() exists for the entropy quant scheme only")
        mm = np.zeros(2, dtype=np.float64)
        hist = np.zeros(512, dtype=np.float64)
        if self._handle is None:
            return dict(has_hist=0, min=0.0, max=0.0, hist=hist, iterations=0)
        has, it = ctypes.c_int(0), ctypes.c_int(0)
        with torch.cuda.device(self._device):
            _native.call("aimet_tq_get_entropy_state", self._handle, int(channel),
                         mm.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                         hist.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(has), ctypes.byref(it),
                         torch.cuda.current_stream(self._device).cuda_stream)
        return dict(has_hist=has.value, min=float(mm[0]), max=float(mm[1]), hist=hist, iterations=it.value)

    def setPercentileValue(self, percentile: float):
        """AimetTensorQuantizer.cpp:200-207 (percentile scheme only)."""
        if self._scheme != QuantizationMode.QUANTIZATION_PERCENTILE:
            return
        self._pending_percentile = float(percentile)
        if self._handle is not None:
            _native.call("aimet_tq_set_percentile_value", self._handle, float(percentile))

    def getPercentileValue(self) -> float:
        if self._scheme != QuantizationMode.QUANTIZATION_PERCENTILE:
            raise RuntimeError("Percentile Value only exists in case of percentile quant scheme.")
        return 100.0 if self._pending_percentile is None else self._pending_percentile

    # -- quantize-dequantize -----------------------------------------------------------------
    @staticmethod
    def quantize_dequantize_tensor(tensor, encoding, round_mode=RoundingMode.ROUND_NEAREST, out=None):
        _require_gpu(tensor, allow_16bit=True)
        t = tensor.contiguous(memory_format=_suggest_memory_format(tensor))
        if out is None:
            out = torch.empty_like(t)
        seed = next(_seed_counter) if int(round_mode) == RoundingMode.ROUND_STOCHASTIC else 0
        with torch.cuda.device(t.device):
            if t.dtype in IO_DTYPES:   # fp16 / bf16 I/O fused (aimet_qdq_per_tensor_16)
                _native.call("aimet_qdq_per_tensor_16", t.data_ptr(), out.data_ptr(), t.numel(), IO_DTYPES[t.dtype],
                             encoding.to_c(), int(round_mode), seed, _stream(t))
            else:
                _native.call("aimet_qdq_per_tensor", t.data_ptr(), out.data_ptr(), t.numel(), encoding.to_c(),
                             int(round_mode), seed, _stream(t))
        return out

    def quantizeDequantize(self, tensor, encoding, round_mode, use_cuda=True):
        """AimetTensorQuantizer.cpp:129-155: new output tensor, uses encoding.min/max/bw."""
        t, staged = _stage(tensor)
        t = t.contiguous(memory_format=_suggest_memory_format(t))
        out = AimetTensorQuantizer.quantize_dequantize_tensor(t, encoding, round_mode)
        return out.cpu() if staged else out

    def quantize(self, tensor, encoding, round_mode, use_cuda=True, shift_to_signed=False):
        """AimetTensorQuantizer.cpp:157-178: float tensor of integer codes."""
        t, staged = _stage(tensor)
        t = t.contiguous(memory_format=_suggest_memory_format(t))
        out = torch.empty_like(t)
        seed = next(_seed_counter) if int(round_mode) == RoundingMode.ROUND_STOCHASTIC else 0
        with torch.cuda.device(t.device):
            _native.call("aimet_quantize_per_tensor", t.data_ptr(), out.data_ptr(), t.numel(), encoding.to_c(),
                         int(round_mode), int(bool(shift_to_signed)), seed, _stream(t))
        return out.cpu() if staged else out

    def makeDeltaOffsetTensor(self, device, encodings):
        """AimetTensorQuantizer.cpp:209-231 -> (delta[C], offset[C]) float32 on `device`."""
        device = torch.device(device)
        C = len(encodings)
        if device.type != "cuda":
            raise RuntimeError("aimet_amd: makeDeltaOffsetTensor needs a HIP device")
        table = torch.empty((2, C), dtype=torch.float32, device=device)
        with torch.cuda.device(device):
            _native.call("aimet_make_delta_offset", encodings_to_c(encodings), C, table.data_ptr(),
                         torch.cuda.current_stream(device).cuda_stream)
        return table[0], table[1]

    def channelTable(self, encodings, device):
        """Device table [4][C] for per-channel QDQ/STE, cached until any encoding changes."""
        return self._pc_table.get(encodings, torch.device(device))

    def quantizeDequantizePerChannel(self, tensor, encodings, num_channel, num_element, num_element_per_channel,
                                     round_mode, use_cuda=True):
        """AimetTensorQuantizer.cpp:233-307 (numChannel, numElement, numElementPerChannel)."""
        t, staged = _stage(tensor)
        t = t.contiguous()
        C, N, K = int(num_channel), int(num_element), int(num_element_per_channel)
        if len(encodings) != C:
            raise ValueError("expected %d encodings, got %d" % (C, len(encodings)))
        if C * K == 0 or N % (C * K) != 0 or N != t.numel():
            raise ValueError("inconsistent per-channel shape: numElement=%d numChannel=%d "
                             "numElementPerChannel=%d" % (N, C, K))
        table = self.channelTable(encodings, t.device)
        out = qdq_per_channel_table(t, table, N // (C * K), C, K, round_mode)
        return out.cpu() if staged else out


# (shape, channel axis, channels) -> per_channel_view (calibrateResidentAsync)
_PER_CHANNEL_VIEWS = {}


def _param_specs(pq, params, ch_axes):
    """calibrateResidentAsync's parameter checks, before anything is launched: [(tensor, outer, C,
    K)] of the float32 HIP tensors, the per-channel views (from the shape alone, no copy) cached by
    (shape, axis, channels)."""
    f32 = torch.float32
    specs = []
    views = _PER_CHANNEL_VIEWS
    for q, t, ax in zip(pq, params, ch_axes):
        if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == f32):
            _require_gpu(t)
            raise TypeError("calibrateResidentAsync takes float32 tensors (got %s)" % t.dtype)
        nc = q._num_channels
        key = (t.shape, ax, nc)
        v = views.get(key)
        if v is None:
            v = views[key] = per_channel_view(t.shape, ax) if nc != 1 else (1, 1, t.numel())
        outer, C, K = v
        if C != nc:
            raise ValueError("tensor has %d channels along axis %d, quantizer has %d" % (C, ax, nc))
        specs.append((t, outer, C, K))
    return specs


def _param_pointers(specs, keep):
    """The parameters' device pointers; a non-contiguous tensor is copied on the current stream
    (the caller picks it) and every tensor is kept alive in `keep`."""
    ptrs = []
    for t, _, _, _ in specs:
        if not t.is_contiguous():
            t = t.contiguous()
        keep.append(t)
        ptrs.append(t.data_ptr())
    return ptrs


class PendingEncodings:
    """A batched getEncoding in flight (AimetTensorQuantizer.getEncodingsAsync)."""

    def __init__(self, quantizers, bitwidth, sym, strict, unsign, request=None):
        self.quantizers = quantizers
        self.live = [q for q in quantizers if q._handle is not None and q._is_encoding_valid]
        self.req = None
        if request is not None:
            # a request launched for exactly these quantizers (aimet_calibrate_launch)
            if len(self.live) != len(quantizers):
                raise RuntimeError("a launched request covers every quantizer")
            self.req = request if request.value else None
        elif self.live:
            dev = self.live[0]._device
            handles = (ctypes.c_void_p * len(self.live))(*[q._handle for q in self.live])
            req = ctypes.c_void_p()
            with torch.cuda.device(dev):
                _native.call("aimet_tq_get_encodings_launch", handles, len(self.live), int(bitwidth), int(bool(sym)),
                             int(bool(strict)), int(bool(unsign)), torch.cuda.current_stream(dev).cuda_stream,
                             ctypes.byref(req))
            self.req = req
        self._views = self._encoding_views() if self.live and self.req is not None else None

    def _encoding_views(self):
        """The result block and its per-quantizer TfEncoding objects, built while the searches run
        on the device: ctypes array items (and slices) are views into the array's buffer, so
        aimet_tq_get_encodings_finish filling the block fills them (about 1.3 ms of Python for
        ResNet-50's 27,560 weight channels, hidden behind the device's ~5 ms)."""
        total = sum(q._num_channels for q in self.live)
        out = TfEncoding.array(total)
        valid = (ctypes.c_int * len(self.live))()
        views = []
        # tens of thousands of small objects: keep the cyclic GC from firing mid-list
        gc_was_enabled = gc.isenabled()
        gc.disable()
        try:
            # ctypes array slicing builds the element objects in one C-level pass (about 2x faster
            # than list(out) + list slicing)
            off = 0
            for q in self.live:
                C = q._num_channels
                views.append(out[off] if C == 1 else out[off:off + C])
                off += C
        finally:
            if gc_was_enabled:
                gc.enable()
        return out, valid, views

    def result(self):
        results = {}
        if not self.live and self.req is not None:
            # a launched request over no live quantizer (an empty activation list of a plan): free it
            req, self.req = self.req, None
            _native.call("aimet_tq_get_encodings_finish", req, None, None)
        if self.live:
            if self.req is None:
                raise RuntimeError("PendingEncodings.result() called twice")
            out, valid, views = self._views
            self._views = None
            req, self.req = self.req, None
            _native.call("aimet_tq_get_encodings_finish", req, out, valid)
            for i, q in enumerate(self.live):
                results[id(q)] = (views[i], bool(valid[i]))
        res = []
        for q in self.quantizers:
            if id(q) in results:
                res.append(results[id(q)])
            else:
                e = [TfEncoding() for _ in range(q._num_channels)]
                res.append((e[0] if q._num_channels == 1 else e, False))
        return res

    def __del__(self):
        if getattr(self, "req", None) is not None:   # never finished: release it (waits for the searches)
            try:
                _native.call("aimet_tq_get_encodings_finish", self.req, None, None)
            except Exception:
                pass


IO_DTYPES = {torch.float16: 1, torch.bfloat16: 2}   # aimet_*_16 io_dtype codes


def qdq_per_channel_table(t, table, outer, C, K, round_mode=RoundingMode.ROUND_NEAREST, out=None):
    """Per-channel QDQ of a contiguous fp32 / fp16 / bf16 tensor (16-bit I/O fused, see
    aimet_qdq_per_channel_16), output in the input dtype."""
    if out is None:
        out = torch.empty_like(t)
    seed = next(_seed_counter) if int(round_mode) == RoundingMode.ROUND_STOCHASTIC else 0
    with torch.cuda.device(t.device):
        if t.dtype in IO_DTYPES:
            _native.call("aimet_qdq_per_channel_16", t.data_ptr(), out.data_ptr(), outer, C, K, IO_DTYPES[t.dtype],
                         table.data_ptr(), int(round_mode), seed, _stream(t))
        else:
            _native.call("aimet_qdq_per_channel", t.data_ptr(), out.data_ptr(), outer, C, K, table.data_ptr(),
                         int(round_mode), seed, _stream(t))
    return out


def _suggest_memory_format(t):
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last) and not t.is_contiguous():
        return torch.channels_last
    return torch.contiguous_format


class ChannelQdqPlan:
    """Every per-channel parameter QDQ of a forward in ONE launch (aimet_qdq_channel_plan_*).

    entries: list of (input, output, ch_axis, table) with device fp32 tensors and [4][C] tables
    from ``AimetTensorQuantizer.channelTable``. The tensors must stay alive (and not move) while
    the plan is used; the plan is graph-capturable."""

    def __init__(self, entries):
        from aimet_amd._native import ChannelDescC
        if not entries:
            raise ValueError("empty plan")
        descs = (ChannelDescC * len(entries))()
        self._keep = []
        device = None
        for i, (x, y, ax, table) in enumerate(entries):
            _require_gpu(x)
            _require_gpu(y, True, "output")
            if not (x.is_contiguous() and y.is_contiguous() and x.shape == y.shape):
                raise ValueError("plan tensors must be contiguous and of equal shape")
            outer, C, K = per_channel_view(x.shape, ax)
            descs[i] = ChannelDescC(x.data_ptr(), y.data_ptr(), outer, C, K, table.data_ptr())
            self._keep += [x, y, table]
            device = x.device
        self.device = device
        h = ctypes.c_void_p()
        _native.call("aimet_qdq_channel_plan_create", descs, len(entries), device.index, ctypes.byref(h))
        self._handle = h

    def run(self, round_mode=RoundingMode.ROUND_NEAREST, stream=None):
        seed = next(_seed_counter) if int(round_mode) == RoundingMode.ROUND_STOCHASTIC else 0
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        _native.call("aimet_qdq_channel_plan_run", self._handle, int(round_mode), seed, s)

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None:
            try:
                _native.call("aimet_qdq_channel_plan_destroy", h)
            except Exception:
                pass
            self._handle = None
