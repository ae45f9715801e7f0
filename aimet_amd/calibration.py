"""One calibration pass over tensors that are already resident in HBM: every quantizer's statistics
and encodings with a handful of launches and two stream synchronisations.

This is QuantizationSimModel.compute_encodings' work (v1/quantsim.py:381-449: updateStats of every
activation quantizer for the batch, then getEncoding of every activation and parameter quantizer)
for callers that hold the activations and parameters themselves (a captured forward, a serving
stack, bench.py), scheduled for the MI355X:

* activations: one launch per phase for all per-tensor quantizers (aimet_tq_*_many), sharded across
  ranks with one packed collective per phase when a process group is given (aimet_amd.distributed);
* parameters: on a second stream, per-channel statistics in two launches (one workgroup per
  channel), the TF-Enhanced / MSE searches in one launch, and the host building the parameter
  encodings while the activation passes still stream;
* activation encodings: one search launch + one synchronisation.
"""
import ctypes
import weakref
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from aimet_amd import _native
from aimet_amd import distributed as D
from aimet_amd.tensor_quantizer import AimetTensorQuantizer, PendingEncodings, _param_specs

_SIDE = {}
# the path of compute_encodings_resident: "plan" (a cached CalibrationPlan: every job table prepared
# once), "native" (aimet_calibrate_launch, the tables built per call) or "phased" (one launch per
# phase from Python). The last two are what the tests compare the plan with; none is read from the
# environment. (Other schedules -- the activations' passes first, the parameters serial on one
# stream, a normal-priority side stream -- measured slower: tools/studies/enc_schedule_tune.py,
# profiles/r02/compute_encodings_study.txt.)
_SCHEDULE = "plan"
_SIDE_PRIORITY = -1   # the side stream's priority: high, so the parameters' work is dispatched first


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    """One high-priority stream per device, created once (stream creation is not free). The
    parameters' short statistics launches and their compute-bound encoding search run on it: at high
    priority their workgroups are dispatched ahead of the HBM-bound activation passes queued on the
    main stream, so the parameter encodings are ready (and built on the host) while the activation
    passes still stream."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(torch.device("cuda", key), priority=_SIDE_PRIORITY)
    return _SIDE[key]


class CalibrationPlan:
    """compute_encodings of a FIXED set of quantizers over resident tensors, prepared once and run
    many times (aimet_calib_plan_*, calib_plan.cpp): v1/quantsim.py:381-449's reset + updateStats +
    getEncoding of every quantizer for one batch, with every job table built and uploaded at
    creation, so ``run`` is one native call that only launches kernels.

    act_quantizers[i] (per-tensor AimetTensorQuantizer) sees activations[i] (this rank's shard when
    `group` spans several ranks); param_quantizers[j] (per-tensor or per-channel along
    param_ch_axes[j]) sees params[j] (replicated). Tensors: float32, on one HIP device. The plan
    reads the tensors' memory at every run, so it keeps them (and the quantizers) alive; refill
    them in place between runs for a new batch.

    Sharded (`group` of several ranks, or `force_exchange`): the activation quantizers are bound
    to packed exchange buffers (aimet_amd.distributed.PackedExchange) and every run is the three
    plan stages with ONE all_reduce(MAX) of the packed {-min, max} and ONE all_reduce(SUM) of the
    packed bin and element counts between them, all on the current stream: no host
    round trip, the element counts formed on the device."""

    def __init__(self, act_quantizers, activations, param_quantizers=(), params=(), param_ch_axes=None,
                 act_settings=(8, False, False, False), param_settings=(8, True, False, False), group=None,
                 force_exchange=False):
        aq, pq = list(act_quantizers), list(param_quantizers)
        acts, params = list(activations), list(params)
        if len(aq) != len(acts) or len(pq) != len(params):
            raise ValueError("one tensor per quantizer")
        if not aq and not pq:
            raise ValueError("an empty calibration plan")
        for q in aq + pq:
            if type(q) is not AimetTensorQuantizer:
                raise TypeError("a calibration plan takes AimetTensorQuantizer objects")
        if any(q._num_channels != 1 for q in aq):
            raise ValueError("the activation quantizers of a calibration plan are per-tensor")
        f32 = torch.float32
        for t in acts:
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == f32):
                raise TypeError("a calibration plan takes float32 HIP tensors")
        self.dev = (acts[0] if acts else params[0]).device
        ch_axes = list(param_ch_axes) if param_ch_axes is not None else [0] * len(pq)
        p_specs = _param_specs(pq, params, ch_axes)
        self.act_quantizers, self.param_quantizers = aq, pq
        self.act_settings = tuple(int(v) for v in act_settings)
        self.param_settings = tuple(int(v) for v in param_settings)
        self.group = group
        self.world = D._world(group)
        self.exchanging = self.world > 1 or bool(force_exchange)
        # contiguous tensors the plan reads at every run (a non-contiguous input is copied ONCE here,
        # so a caller refilling the original would not be seen: such inputs are refused instead)
        for t in acts + [sp[0] for sp in p_specs]:
            if not t.is_contiguous():
                raise ValueError("a calibration plan reads its tensors in place: pass contiguous tensors")
            if t.device != self.dev:
                raise ValueError("the tensors of a calibration plan share one device")
        self._tensors = acts + [sp[0] for sp in p_specs]
        with torch.cuda.device(self.dev):
            handles = AimetTensorQuantizer._ensure_many(aq + pq, self.dev)
            self.exchange = None
            elem = None
            if self.exchanging and aq:
                ex = D.PackedExchange(aq, self.dev)   # binds the activation quantizers
                self.exchange = (ex.minmax, ex.counts)
                elem = ex.elem_counts
            na, np_ = len(aq), len(pq)
            i32x4 = ctypes.c_int32 * 4
            h = ctypes.c_void_p()
            _native.call("aimet_calib_plan_create", (ctypes.c_void_p * max(na, 1))(*handles[:na]),
                         (ctypes.c_void_p * max(na, 1))(*[t.data_ptr() for t in acts]),
                         (ctypes.c_int64 * max(na, 1))(*[t.numel() for t in acts]), na,
                         (ctypes.c_void_p * max(np_, 1))(*handles[na:]),
                         (ctypes.c_void_p * max(np_, 1))(*[sp[0].data_ptr() for sp in p_specs]),
                         (ctypes.c_int64 * max(np_, 1))(*[sp[1] for sp in p_specs]),
                         (ctypes.c_int64 * max(np_, 1))(*[sp[2] for sp in p_specs]),
                         (ctypes.c_int64 * max(np_, 1))(*[sp[3] for sp in p_specs]), np_,
                         i32x4(*self.act_settings), i32x4(*self.param_settings),
                         elem.data_ptr() if elem is not None else None, ctypes.byref(h))
        self._handle = h
        self._native_handles = [hh.value if isinstance(hh, ctypes.c_void_p) else hh for hh in handles]
        self._ra, self._rp = ctypes.c_void_p(), ctypes.c_void_p()

    def launch(self, reset=False, main_stream=None, side_stream=None):
        """Enqueue one batch; returns (PendingEncodings of the activations, of the parameters).
        One device: one native call (the activations on `main_stream`, default the current stream;
        the parameters on `side_stream`, default a high-priority stream of the device). Sharded:
        stage 1, all_reduce(MAX), stage 2, all_reduce(SUM), stage 4, each collective on the
        current stream between the stages (the host waits for nothing)."""
        return self._launch(reset, self.act_quantizers, self.param_quantizers, main_stream, side_stream)

    def _launch(self, reset, aq, pq, main_stream=None, side_stream=None):
        if self._handle is None:
            raise RuntimeError("calibration plan already closed")
        main = main_stream if main_stream is not None else torch.cuda.current_stream(self.dev)
        side = side_stream if side_stream is not None else (_side_stream(self.dev) if pq else main)
        ra, rp = self._ra, self._rp
        launch = _native.load().aimet_calib_plan_launch
        with torch.cuda.device(self.dev):
            if not self.exchanging:
                _native.check(launch(self._handle, 7, int(bool(reset)), main.cuda_stream, side.cuda_stream,
                                     ctypes.byref(ra), ctypes.byref(rp)))
            else:
                empty = ctypes.c_void_p()
                _native.check(launch(self._handle, 1, int(bool(reset)), main.cuda_stream, side.cuda_stream,
                                     ctypes.byref(empty), ctypes.byref(rp)))
                try:
                    ex = self.exchange
                    with torch.cuda.stream(main):
                        if ex is not None:
                            # {-min, max}: a single MAX reduces both ends exactly
                            D._all_reduce(ex[0], dist.ReduceOp.MAX, self.group)
                        _native.check(launch(self._handle, 2, 0, main.cuda_stream, side.cuda_stream,
                                             ctypes.byref(empty), ctypes.byref(empty)))
                        if ex is not None:
                            # bin counts + element counts of every histogram quantizer in one SUM
                            D._all_reduce(ex[1], dist.ReduceOp.SUM, self.group)
                        _native.check(launch(self._handle, 4, 0, main.cuda_stream, side.cuda_stream,
                                             ctypes.byref(ra), ctypes.byref(empty)))
                except BaseException:
                    if rp.value:   # the parameters' request is in flight: discard it
                        _native.call("aimet_tq_get_encodings_finish", rp, None, None)
                        rp.value = None
                    raise
        if reset:
            for q in aq + pq:
                q._pending_percentile = None
        for q in aq + pq:
            q._is_encoding_valid = True
        a = PendingEncodings(aq, *self.act_settings, request=ctypes.c_void_p(ra.value))
        p = PendingEncodings(pq, *self.param_settings, request=ctypes.c_void_p(rp.value))
        ra.value = rp.value = None
        return a, p

    def run(self, reset=False):
        """launch + both results: ([(encoding, valid)] of the activations, [(encodings, valid)] of
        the parameters); the parameters' (ready first) are built while the activations stream."""
        a, p = self.launch(reset)
        p_res = p.result()
        return a.result(), p_res

    def close(self):
        h, self._handle = getattr(self, "_handle", None), None
        if h is not None:
            _native.call("aimet_calib_plan_destroy", h)

    def __del__(self):
        try:
            self.close()
        except Exception:   # interpreter shutdown
            pass


# the plan of the last compute_encodings_resident call, reused while the same quantizers see the
# same tensors. The cache holds the plan's own tables only: the tensors and quantizers are checked
# by identity through weak references (and the tensors' addresses, shapes and strides, which the
# plan's tables hold), so nothing is kept alive. A plan is built only when a call sees the tensors
# of the previous call again: a calibration loop passing new activation tensors every batch takes
# the per-call native path instead of building (and dropping) a plan per call.
_PLAN_CACHE = {}


def _identity(aq, acts, pq, params, ch_axes, act_settings, param_settings, group):
    ts, qs = list(acts) + list(params), list(aq) + list(pq)
    key = (tuple(map(id, qs)), len(aq), tuple(act_settings), tuple(param_settings),
           tuple(ch_axes) if ch_axes is not None else None, id(group) if group is not None else None,
           tuple((t.data_ptr(), tuple(t.shape), tuple(t.stride())) for t in ts))
    return key, ts, qs


def _same(entry, key, ts, qs):
    return (entry is not None and entry[0] == key and len(ts) == len(entry[1])
            and all(r() is t for r, t in zip(entry[1], ts)) and all(r() is q for r, q in zip(entry[2], qs)))


def _cached_plan(aq, acts, pq, params, ch_axes, act_settings, param_settings, group):
    """The cached plan for exactly these quantizers and tensors; a new one (which replaces it) when
    the previous call passed the same ones; else None (the caller takes the per-call path)."""
    key, ts, qs = _identity(aq, acts, pq, params, ch_axes, act_settings, param_settings, group)
    hit = _PLAN_CACHE.get("plan")
    if _same(hit, key, ts, qs):
        plan = hit[3]
        if [q._handle.value if q._handle is not None else None for q in qs] == plan._native_handles:
            return plan
    seen = _PLAN_CACHE.get("seen")
    _PLAN_CACHE["seen"] = (key, [weakref.ref(t) for t in ts], [weakref.ref(q) for q in qs])
    if not _same(seen, key, ts, qs):
        return None
    _PLAN_CACHE.pop("plan", None)
    plan = CalibrationPlan(aq, acts, pq, params, ch_axes, act_settings, param_settings, group=group)
    plan._tensors = plan.act_quantizers = plan.param_quantizers = None   # see above
    _PLAN_CACHE["plan"] = (key, [weakref.ref(t) for t in ts], [weakref.ref(q) for q in qs], plan)
    return plan


def compute_encodings_resident(act_quantizers: Sequence[AimetTensorQuantizer], activations: Sequence[torch.Tensor],
                               param_quantizers: Sequence[AimetTensorQuantizer], params: Sequence[torch.Tensor],
                               act_settings: Tuple[int, bool, bool, bool] = (8, False, False, False),
                               param_settings: Tuple[int, bool, bool, bool] = (8, True, False, False),
                               param_ch_axes: Optional[Sequence[int]] = None, group=None, reset: bool = False
                               ) -> Tuple[List, List]:
    """Statistics + encodings of every quantizer for one batch.

    act_quantizers[i] (per-tensor) sees activations[i] (this rank's shard when `group` spans several
    ranks); param_quantizers[j] (per-tensor or per-channel along param_ch_axes[j]) sees params[j]
    (replicated). *_settings = (bitwidth, symmetric, strict symmetric, unsigned symmetric).
    Returns ([(encoding, valid)] of the activations, [(encodings, valid)] of the parameters).

    Everything is enqueued before the host waits for anything: both streams' statistics and both
    streams' encoding searches (with the copies of their results) -- the activations' search
    launch does not wait for the parameters' host work -- then the parameter encodings are built
    (their stream finishes first) while the activation passes still stream.

    reset=True: resetEncodingStats of every quantizer first (QuantizationSimModel.compute_encodings
    on quantizers that already hold statistics, v1/quantsim.py:387-399).

    With AimetTensorQuantizers (per-tensor activations) and contiguous float32 device tensors, a
    call that sees the quantizers and tensors of the previous call again runs a calibration plan
    (CalibrationPlan, aimet_calib_plan_*: every job table prepared once and cached for the next call
    on the same quantizers and tensors): one native launch of about fifteen HIP calls on one rank;
    on several ranks its three stages with the packed all_reduce(MAX) and all_reduce(SUM) between
    them. Other calls take the per-call native path (one rank: aimet_calibrate_launch) or enqueue
    the phases from here (sharded with the same collectives when `group` spans several ranks)."""
    if not activations and not params:
        if reset:
            AimetTensorQuantizer.resetEncodingStatsMany(list(act_quantizers) + list(param_quantizers))
        return [], []
    dev = (activations[0] if activations else params[0]).device
    planned = (_SCHEDULE == "plan"
               and all(type(q) is AimetTensorQuantizer and q.num_channels == 1 for q in act_quantizers)
               and all(type(q) is AimetTensorQuantizer for q in param_quantizers)
               and all(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                       and t.device == dev for t in list(activations) + list(params)))
    plan = None
    if planned:
        # a calibration plan (every job table prepared once, cached for the next call on the same
        # quantizers and tensors): one native call on one device; the three stages with the two
        # packed collectives between them when `group` spans several ranks
        plan = _cached_plan(act_quantizers, activations, param_quantizers, params, param_ch_axes, act_settings,
                            param_settings, group)
    if plan is not None:
        a_pending, p_pending = plan._launch(reset, list(act_quantizers), list(param_quantizers))
        p_res = p_pending.result()
        return a_pending.result(), p_res
    native = (D._world(group) == 1 and _SCHEDULE in ("plan", "native")
              and all(type(q) is AimetTensorQuantizer and q.num_channels == 1 for q in act_quantizers)
              and all(type(q) is AimetTensorQuantizer for q in param_quantizers)
              and all(t.dtype == torch.float32 for t in list(activations) + list(params)))
    if native:
        cur = torch.cuda.current_stream(dev)
        main, side = cur, _side_stream(dev)
        a_pending, p_pending, keep = AimetTensorQuantizer.calibrateResidentAsync(
            act_quantizers, activations, param_quantizers, params, param_ch_axes, act_settings, param_settings,
            reset=reset, main_stream=main, side_stream=side)
        p_res = p_pending.result()
        a_res = a_pending.result()
        del keep
        return a_res, p_res
    if reset:
        AimetTensorQuantizer.resetEncodingStatsMany(list(act_quantizers) + list(param_quantizers))
    AimetTensorQuantizer._ensure_many(list(act_quantizers) + list(param_quantizers), dev)
    cur = torch.cuda.current_stream(dev)
    main, side = cur, _side_stream(dev)
    # the inputs are ordered on the current stream (torch's stream semantics); the side stream
    # starts after everything queued there so far (a device-side dependency, no host wait)
    side.wait_stream(cur)
    keep, p_pending = None, None
    if param_quantizers:
        # enqueued first: the parameters' statistics take the CUs before the activation passes
        with torch.cuda.stream(side):
            keep = AimetTensorQuantizer.updateStatsPerChannelMany(param_quantizers, params, param_ch_axes)
            p_pending = AimetTensorQuantizer.getEncodingsAsync(param_quantizers, *param_settings)
    with torch.cuda.stream(main):
        if act_quantizers:
            D.sharded_update_stats(list(act_quantizers), list(activations), group=group)
        a_pending = AimetTensorQuantizer.getEncodingsAsync(act_quantizers, *act_settings) if act_quantizers else None
    p_res = p_pending.result() if p_pending is not None else []
    del keep
    a_res = a_pending.result() if a_pending is not None else []
    torch.cuda.synchronize(dev)
    return a_res, p_res
