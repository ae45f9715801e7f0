"""TEST INFRASTRUCTURE ONLY: float32 torch restatements of the reference's Python-side arithmetic
on the path (only tests/ import this):

* learned-grid forward / gradients -- quantsim_straight_through_grad.py:121-328
  (pinned against the reference module itself: tests/golden/golden_lg.npz, make_golden.py)
* AdaRound soft rounding -- adaround_wrapper.py:124-149, adaround_loss.py:83-110
  (pinned by the reference KATs in tests/golden/kat.json)
"""
import json
import math
import os

import torch


def _bcast(tensor, v, ch_axis):
    if v.numel() == 1:
        return v.reshape(())
    shape = tuple(d if a == ch_axis else 1 for a, d in enumerate(tensor.shape))
    return v.view(shape)


def lg_encodings(bw, emin, emax, sym, strict, unsigned):
    """quantsim_straight_through_grad.py:121-160 get_computed_encodings."""
    steps = 2 ** bw - 1
    if sym and strict:
        steps -= 1
    half = steps / 2
    steps_t = torch.full_like(emin, steps)
    if sym and not unsigned:
        delta = emax / torch.full_like(emin, math.floor(half))
        offset = -torch.full_like(emin, math.ceil(half))
    else:
        delta = (emax - emin) / steps_t
        if sym:
            offset = emin / delta
        else:
            b0 = torch.round(-emin / delta)
            b0 = torch.min(steps_t, torch.max(torch.full_like(emin, 0.), b0))
            offset = -b0
    return delta, offset, steps_t


def lg_forward(x, emin, emax, bw, sym=False, strict=False, unsigned=False, ch_axis=0):
    """calculate_forward_pass (:191-249), float32: returns (y, mask, x_quant, delta_b, offset_b, steps)."""
    delta, offset, steps = lg_encodings(bw, emin, emax, sym, strict, unsigned)
    delta_b, offset_b = _bcast(x, delta, ch_axis), _bcast(x, offset, ch_axis)
    zero = torch.zeros_like(steps)
    x_round = torch.round(x / delta_b) - offset_b
    x_quant = x_round.clamp(zero[0], steps[0])
    y = (x_quant + offset_b) * delta_b
    mask = x_round.ge(zero[0]) * x_round.le(steps[0])
    return y, mask, x_quant, delta_b, offset_b, steps[0]


def lg_gradients(x, grad, emin, emax, bw, sym=False, strict=False, unsigned=False, ch_axis=0):
    """(grad_x, grad_min, grad_max): QuantizeDequantizeFunc.backward + asymmetric/symmetric_gradients."""
    y, mask, x_quant, delta, offset, steps = lg_forward(x, emin, emax, bw, sym, strict, unsigned, ch_axis)
    grad_x = mask * grad
    dims = list(range(x.dim()))
    if emin.numel() > 1:
        dims.pop(ch_axis)
    if sym:
        gmax = ((x_quant + offset) * grad).sum(dim=dims) - (mask * (x / delta) * grad).sum(dim=dims)
        gmax = gmax / torch.div(steps, 2, rounding_mode="floor")
        return grad_x, (-gmax).view_as(emin), gmax.view_as(emax)
    grad_xq = delta * grad
    grad_scale = (x_quant + offset - x * mask / delta) * grad
    grad_offset = grad_xq * (~mask)
    t1 = grad_scale.sum(dim=dims) / steps
    t2 = steps / (emax - emin) ** 2 * grad_offset.sum(dim=dims)
    return grad_x, (-t1 + emax * t2).view_as(emin), (t1 - emin * t2).view_as(emax)


def lg_encoding_grads_bound(x, grad, emin, emax, bw, sym=False, strict=False, unsigned=False, ch_axis=0):
    """The encoding gradients of lg_gradients with its float32 terms summed exactly (float64) and
    combined in float64, and the magnitude each one is summed from: returns (gmin, gmax, bmin,
    bmax) where b = sum of |terms| carried through the same linear combination. The terms are the
    reference's float32 expressions element by element (which the kernels reproduce bit for bit),
    so an fp32 result whose error is at most c * eps * b differs from the exact sum of those very
    terms by summation order (and the combination's few roundings) only; tests state c."""
    _, mask, x_quant, delta, offset, steps = lg_forward(x, emin, emax, bw, sym, strict, unsigned, ch_axis)
    dims = list(range(x.dim()))
    if emin.numel() > 1:
        dims.pop(ch_axis)
    st = float(steps)
    if sym:
        t1 = ((x_quant + offset) * grad).double()
        t2 = (mask * (x / delta) * grad).double()
        half = math.floor(st / 2)
        gmax = (t1.sum(dim=dims) - t2.sum(dim=dims)) / half
        b = (t1.abs().sum(dim=dims) + t2.abs().sum(dim=dims)) / half
        return (-gmax).view_as(emin), gmax.view_as(emax), b.view_as(emin), b.view_as(emax)
    gs = ((x_quant + offset - x * mask / delta) * grad).double()
    go = ((delta * grad) * (~mask)).double()
    lo, hi = emin.double().reshape(-1), emax.double().reshape(-1)
    k = st / (hi - lo) ** 2
    t1, b1 = gs.sum(dim=dims).reshape(-1) / st, gs.abs().sum(dim=dims).reshape(-1) / st
    s2, b2 = go.sum(dim=dims).reshape(-1), go.abs().sum(dim=dims).reshape(-1)
    gmin, gmax = -t1 + hi * k * s2, t1 - lo * k * s2
    bmin, bmax = b1 + hi.abs() * k * b2, b1 + lo.abs() * k * b2
    return gmin.view_as(emin), gmax.view_as(emax), bmin.view_as(emin), bmax.view_as(emax)


def lg_range_grads_rounded_sums(x, grad, emin, emax, bw, sym=False, strict=False, unsigned=False, ch_axis=0):
    """The reference's float32 range-gradient expressions (lg_gradients) applied to the exact
    (float64) sums of its float32 terms, each rounded once to float32: the closest any float32
    evaluation of the reference's formula can come, i.e. the part of the error that is the
    formula's, not the sums'."""
    _, mask, x_quant, delta, offset, steps = lg_forward(x, emin, emax, bw, sym, strict, unsigned, ch_axis)
    dims = list(range(x.dim()))
    if emin.numel() > 1:
        dims.pop(ch_axis)
    if sym:
        s1 = ((x_quant + offset) * grad).double().sum(dim=dims).float()
        s2 = (mask * (x / delta) * grad).double().sum(dim=dims).float()
        gmax = (s1 - s2) / torch.div(steps, 2, rounding_mode="floor")
        return (-gmax).view_as(emin), gmax.view_as(emax)
    gs = ((x_quant + offset - x * mask / delta) * grad).double().sum(dim=dims).float()
    go = ((delta * grad) * (~mask)).double().sum(dim=dims).float()
    t1 = gs / steps
    t2 = steps / (emax - emin) ** 2 * go.view_as(emax)
    return (-t1.view_as(emin) + emax * t2).view_as(emin), (t1.view_as(emax) - emin * t2).view_as(emax)


def sum_bound_units(got, exact, bound):
    """The worst |got - exact| / (2^-24 * bound) over the elements: the error in the unit the
    learned-grid tests bound (an fp32 sum of n terms in any order is within ~log2(n) of it)."""
    err = (got.double().reshape(-1).cpu() - exact.reshape(-1).cpu()).abs()
    unit = 2.0 ** -24 * bound.reshape(-1).cpu() + 1.2e-38
    return float((err / unit).max()) if err.numel() else 0.0


def report_sum_bound_units(got, exact, bound, what):
    """sum_bound_units, appended to AIMET_BOUND_REPORT when set (figures reported beside a bound)."""
    units = sum_bound_units(got, exact, bound)
    report = os.environ.get("AIMET_BOUND_REPORT")
    if report:
        with open(report, "a") as f:
            f.write(json.dumps({"what": what, "units": round(units, 4), "c": None}) + "\n")
    return units


def assert_within_sum_bound(got, exact, bound, c, what=""):
    """|got - exact| <= c * 2^-24 * bound elementwise (+ the smallest normal, for all-zero sums).
    Returns the measured worst error in that unit; with AIMET_BOUND_REPORT=<path> every check
    appends {what, units, c} to that JSON-lines file (the figures behind the stated bound)."""
    worst = sum_bound_units(got, exact, bound)
    report = os.environ.get("AIMET_BOUND_REPORT")
    if report:
        with open(report, "a") as f:
            f.write(json.dumps({"what": what, "units": round(worst, 4), "c": c}) + "\n")
    assert worst <= c, "%s: error %.3g units of the bound (c = %g)" % (what, worst, c)
    return worst


ZETA, GAMMA = 1.1, -0.1   # aimet_common/defs.py:302-306


def adaround_forward(w, alpha, delta, offset, bw):
    """AdaroundWrapper.apply_adaround (adaround_wrapper.py:124-149), soft rounding."""
    t = torch.floor(w / delta)
    h = torch.clamp(torch.sigmoid(alpha) * (ZETA - GAMMA) + GAMMA, 0, 1)
    q = torch.clamp(t + h - offset, 0, 2 ** bw - 1)
    return (q + offset) * delta


def adaround_round_loss(alpha, reg, beta):
    """AdaroundLoss.compute_round_loss after warm start (adaround_loss.py:97-110)."""
    h = torch.clamp(torch.sigmoid(alpha) * (ZETA - GAMMA) + GAMMA, 0, 1)
    return reg * torch.add(1, -(torch.add(2 * h, -1).abs()).pow(beta)).sum()
