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
import os
from typing import List, Optional, Sequence, Tuple

import torch

from aimet_amd import distributed as D
from aimet_amd.tensor_quantizer import AimetTensorQuantizer

_SIDE = {}
# tuning knobs (tools/studies/enc_schedule_tune.py): launch order and the side stream's priority
_SCHEDULE = os.environ.get("AIMET_CAL_SCHEDULE", "params_first")
_SIDE_PRIORITY = int(os.environ.get("AIMET_CAL_SIDE_PRIORITY", "-1"))
# the parameters' statistics + search on the activations' stream, ahead of the passes (no overlap)
_PARAMS_SERIAL = os.environ.get("AIMET_CAL_PARAMS_SERIAL", "0") == "1"


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

    On one rank, with AimetTensorQuantizers and float32 tensors, all of it is two native calls
    (aimet_calibrate_launch for the activations, then for the parameters while the activations'
    min/max pass runs: about a dozen HIP launches from C++, no Python per phase); otherwise
    the phases are enqueued from here (sharded with collectives when `group` spans several ranks)."""
    if not activations and not params:
        if reset:
            AimetTensorQuantizer.resetEncodingStatsMany(list(act_quantizers) + list(param_quantizers))
        return [], []
    dev = (activations[0] if activations else params[0]).device
    native = (D._world(group) == 1 and _SCHEDULE == "params_first"
              and all(type(q) is AimetTensorQuantizer and q.num_channels == 1 for q in act_quantizers)
              and all(type(q) is AimetTensorQuantizer for q in param_quantizers)
              and all(t.dtype == torch.float32 for t in list(activations) + list(params)))
    if native:
        cur = torch.cuda.current_stream(dev)
        main, side = cur, (cur if _PARAMS_SERIAL else _side_stream(dev))
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
    acts_first = _SCHEDULE == "acts_first"
    if act_quantizers and acts_first:
        # the HBM-bound activation passes start first; the parameters' short statistics and their
        # compute-bound searches run beside them on the side stream
        with torch.cuda.stream(main):
            D.sharded_update_stats(list(act_quantizers), list(activations), group=group)
    if param_quantizers:
        # enqueued first: the parameters' statistics take the CUs before the activation passes
        with torch.cuda.stream(side):
            keep = AimetTensorQuantizer.updateStatsPerChannelMany(param_quantizers, params, param_ch_axes)
            p_pending = AimetTensorQuantizer.getEncodingsAsync(param_quantizers, *param_settings)
    with torch.cuda.stream(main):
        if act_quantizers and not acts_first:
            D.sharded_update_stats(list(act_quantizers), list(activations), group=group)
        a_pending = AimetTensorQuantizer.getEncodingsAsync(act_quantizers, *act_settings) if act_quantizers else None
    p_res = p_pending.result() if p_pending is not None else []
    del keep
    a_res = a_pending.result() if a_pending is not None else []
    torch.cuda.synchronize(dev)
    return a_res, p_res
