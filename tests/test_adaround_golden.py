"""AdaRound soft rounding against the reference's own arithmetic (tests/golden/golden_adaround.npz:
AdaroundWrapper.apply_adaround / _generate_alpha_parameter and AdaroundLoss.compute_round_loss
executed by make_golden.py on torch CPU float32, one thread) on MobileNet-v2 weight shapes
(conv, depthwise [C,1,3,3], pointwise, classifier, a ragged [7,5,3,3]), 4 and 8 bits, alpha from
the reference's initialisation, N(0, 4) and U(-110, 110) (the sigmoid's saturated tails and the
exp underflow / overflow range).

Bars (north_star "within 1 ULP on the dequantized float tensor"):
* Wq (soft and hard rounding): bit-exact;
* dL/dalpha of the reconstruction term (warm start, no rounding loss): bit-exact;
* dL/dalpha with the rounding loss: with the exact pow (aimet_amd.adaround.set_exact_pow(True):
  torch's CPU pow restated, Sleef powf_u10 in the vectorized part, the correctly rounded value in
  the scalar tail of the last n mod 32 elements -- cases 7 and 8 have such tails;
  tools/studies/sleef_powf_check.py) bit-exact; with the default fast pow (within 1 ulp of torch's
  pow, profiles/r06/pow_fast_check.txt) the reference's own float32 chain after the pow evaluated
  at a pow within 1 ulp of torch's, bit for bit (_fast_pow_gradient_ok);
* the rounding loss value: rtol 1e-5 (float32 sums in a different order)."""
import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

DEV = "cuda"


@pytest.fixture(scope="module")
def gad(golden_dir):
    import os
    return dict(np.load(os.path.join(golden_dir, "golden_adaround.npz")))


def _case(z, i):
    k = "c%d_" % i
    return {n: z[k + n] for n in ("w", "alpha", "delta", "offset", "grad", "wq", "wq_hard", "ga_recon", "ga_total",
                                  "round_loss", "beta")} | {"bw": int(z[k + "bw"])}


def _ulps(a, b):
    a = np.asarray(a, np.float32).ravel().view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).ravel().view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7FFFFFFF), a)
    b = np.where(b < 0, -(b & 0x7FFFFFFF), b)
    return np.abs(a - b)


def test_adaround_forward_bit_exact_vs_reference(gad):
    from aimet_amd.adaround import AdaroundFunction
    worst = 0
    for i in range(int(gad["count"])):
        c = _case(gad, i)
        w, a = torch.from_numpy(c["w"]).to(DEV), torch.from_numpy(c["alpha"]).to(DEV)
        d, o = torch.from_numpy(c["delta"]).to(DEV), torch.from_numpy(c["offset"]).to(DEV)
        with torch.no_grad():
            wq = AdaroundFunction.apply(w, a, d, o, c["bw"], 0).cpu().numpy()
            wh = AdaroundFunction.apply(w, a, d, o, c["bw"], 0, False).cpu().numpy()
        u = _ulps(wq, c["wq"])
        worst = max(worst, int(u.max()))
        assert u.max() == 0, (i, c["w"].shape, int((u != 0).sum()), int(u.max()))
        assert np.array_equal(wh.view(np.int32), c["wq_hard"].view(np.int32)), i
    print("adaround Wq: max ulp vs reference = %d" % worst)


def _f32_step(p, k):
    """p (float32 >= 0) moved by k ulps, clamped at +0"""
    b = p.view(np.int32).astype(np.int64) + k
    return np.maximum(b, 0).astype(np.int32).view(np.float32)


def _fast_pow_gradient_ok(c, reg, got):
    """dL/dalpha with the rounding loss is recon + T(p) with p = |2h - 1|^(beta - 1) and T the
    reference's autograd chain after the pow (pow_backward: grad * (beta * p); abs; 2*h; clamp;
    * (zeta - gamma); sigmoid_backward), every step a float32 op. Restated here (numpy float32,
    sigmoid from torch's CPU op, as the kernel's, and the golden reconstruction gradient): for each
    element, the pow values within 3 ulp of the correctly rounded x^(beta - 1) whose T reproduces
    the golden dL/dalpha bit for bit are torch's pow (`pinned`: at least one must); the kernel's
    result must then be T(p') for a p' within 1 ulp of one of them -- the bar the fast pow is
    proven to (profiles/r06/pow_fast_check.txt), carried through the reference's own chain. A
    difference of 1 ulp in p can move dL/dalpha by more than 1 ulp of its value: the loss term
    and the reconstruction gradient cancel in part (tests/golden, case 6: up to 64 ulp)."""
    f = np.float32
    beta = float(c["beta"])
    sg = torch.sigmoid(torch.from_numpy(c["alpha"])).numpy()
    pre = sg * f(1.2) + f(-0.1)
    h = np.clip(pre, f(0), f(1))
    in_h = (pre >= 0) & (pre <= 1)
    x = f(2) * h + f(-1)
    sgn = np.sign(x).astype(f)

    def chain(p):
        dpw = f(-reg) * (f(beta) * p)
        dh = (dpw * sgn) * f(2)
        return c["ga_recon"] + ((np.where(in_h, dh, f(0)) * f(1.2)) * (f(1) - sg)) * sg

    p_cr = np.power(np.abs(x).astype(np.float64), np.float64(f(beta - 1.0))).astype(f)
    want = c["ga_total"].view(np.int32)
    got = got.view(np.int32)
    outs = {k: chain(_f32_step(p_cr, k)).view(np.int32) for k in range(-4, 5)}
    sleef = {k: outs[k] == want for k in range(-3, 4)}
    pinned = np.zeros(want.shape, bool)
    ok = np.zeros(want.shape, bool)
    for k, m in sleef.items():
        pinned |= m
        for d in (-1, 0, 1):
            ok |= m & (outs[k + d] == got)
    return ok, pinned


def test_adaround_backward_vs_reference(gad, exact_pow):
    from aimet_amd.adaround import AdaroundFunction
    reg = float(gad["reg_param"])
    worst, differ, total = 0, 0, 0
    for i in range(int(gad["count"])):
        c = _case(gad, i)
        w, alpha = torch.from_numpy(c["w"]).to(DEV), torch.from_numpy(c["alpha"]).to(DEV)
        d, o = torch.from_numpy(c["delta"]).to(DEV), torch.from_numpy(c["offset"]).to(DEV)
        g = torch.from_numpy(c["grad"]).to(DEV)
        # warm start: reconstruction gradient only -> bit-exact
        a = alpha.clone().requires_grad_(True)
        (AdaroundFunction.apply(w, a, d, o, c["bw"], 0) * g).sum().backward()
        got = a.grad.cpu().numpy()
        assert np.array_equal(got.view(np.int32), c["ga_recon"].view(np.int32)), \
            (i, int((_ulps(got, c["ga_recon"]) != 0).sum()))
        # after warm start: + the rounding loss (fused in the same kernel)
        a = alpha.clone().requires_grad_(True)
        loss = torch.zeros(1, device=DEV)
        (AdaroundFunction.apply(w, a, d, o, c["bw"], 0, True, reg, float(c["beta"]), loss) * g).sum().backward()
        got = a.grad.cpu().numpy()
        u = _ulps(got, c["ga_total"])
        worst, differ, total = max(worst, int(u.max())), differ + int((u != 0).sum()), total + u.size
        if exact_pow:
            assert u.max() == 0, (i, int((u != 0).sum()), int(u.max()))
        else:
            ok, pinned = _fast_pow_gradient_ok(c, reg, got)
            assert pinned.all(), (i, "the restated chain does not reproduce the golden", int((~pinned).sum()))
            assert ok.all(), (i, int((~ok).sum()), int(u.max()))
        want_loss = float(c["round_loss"])
        assert abs(loss.item() - want_loss) <= 1e-5 * abs(want_loss), (i, loss.item(), want_loss)
        # the loss value not requested: the kernel skips pow(x, beta) (the loss term), the gradient's
        # pow(x, beta - 1) is the same
        a2 = alpha.clone().requires_grad_(True)
        (AdaroundFunction.apply(w, a2, d, o, c["bw"], 0, True, reg, float(c["beta"]), None) * g).sum().backward()
        assert np.array_equal(a2.grad.cpu().numpy().view(np.int32), got.view(np.int32)), i
    print("adaround dL/dalpha (%s): %d of %d elements differ from the reference, max %d ulp"
          % ("exact pow" if exact_pow else "fast pow", differ, total, worst))


def test_adaround_alpha_init_vs_reference(gad):
    """aimet_amd.adaround.init_alpha (torch ops on the device) vs the reference's
    _generate_alpha_parameter on the CPU: the device log differs from torch's CPU log by <= 2 ulp,
    so alpha0 is within a few ulp (stated bound: 8 ulp, relative to |alpha0| >= 2^-20)."""
    from aimet_amd.adaround import init_alpha
    for i in range(int(gad["count"])):
        k = "c%d_alpha_init" % i
        if k not in gad:
            continue
        c = _case(gad, i)
        w = torch.from_numpy(c["w"]).to(DEV)
        shape = (-1,) + (1,) * (w.dim() - 1)
        d = torch.from_numpy(c["delta"]).to(DEV).view(shape)
        got = init_alpha(w, d).detach().cpu().numpy()
        want = gad[k]
        fin = np.isfinite(want)
        assert np.array_equal(np.isfinite(got), fin)
        u = _ulps(got[fin], want[fin])
        big = np.abs(want[fin]).ravel() >= 2.0 ** -20
        assert u[big].max() <= 8, (i, int(u.max()))


# ------------------------------------------------------------------------------------------
# fp16 / bf16 STE against the reference's compute_dloss_by_dx (golden_ste16.npz)
# ------------------------------------------------------------------------------------------
def _t16(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a)).view(dt)


def test_ste_16bit_bounds_vs_reference(golden_dir):
    """Per-tensor python-float bounds that fp16 / bf16 cannot represent: the reference compares in
    x's dtype with the bound rounded (0-dim float32 tensor -> x's dtype); per-channel lists (C = 1
    included) compare in float32. x sits exactly on and beside the rounded bounds."""
    import os
    from aimet_amd.quantizers import compute_dloss_by_dx
    z = dict(np.load(os.path.join(golden_dir, "golden_ste16.npz")))
    dts = {"torch.float16": torch.float16, "torch.bfloat16": torch.bfloat16, "torch.float32": torch.float32}
    for i in range(int(z["count"])):
        xd, gd = (dts[str(v)] for v in z["t%d_dtypes" % i])
        x = _t16(z["t%d_x" % i], xd).to(DEV)
        g = (_t16(z["t%d_grad" % i], gd) if gd != torch.float32 else torch.from_numpy(z["t%d_grad" % i])).to(DEV)
        mn, mx = (float(v) for v in z["t%d_bounds" % i])
        got = compute_dloss_by_dx(x, g, mn, mx).cpu()
        want = z["t%d_pt" % i]
        got = got.view(torch.int16).numpy() if got.dtype != torch.float32 else got.numpy().view(np.int32)
        want = want if want.dtype == np.int16 else want.view(np.int32)
        assert np.array_equal(got, want), (i, xd, gd, int((got != want).sum()))
    for C in (1, 8):
        for name, dt in (("float16", torch.float16), ("bfloat16", torch.bfloat16)):
            k = "p%d_%s_" % (C, name)
            x, g = _t16(z[k + "x"], dt).to(DEV), _t16(z[k + "grad"], dt).to(DEV)
            got = compute_dloss_by_dx(x, g, z[k + "mins"].tolist(), z[k + "maxs"].tolist(), 0)
            assert np.array_equal(got.cpu().view(torch.int16).numpy(), z[k + "out"]), (C, name)


def test_ste_16bit_autograd_bounds_vs_reference():
    """QuantizeDequantize.backward with a bf16 / fp16 input (v1/tensor_quantizer.py:1197-1213):
    the mask uses the encoding bounds rounded to x's dtype, as the reference's torch expression."""
    from aimet_amd.quantizers import QuantScheme, StaticGridPerTensorQuantizer
    g = torch.Generator(device=DEV).manual_seed(12)
    for dt in (torch.float16, torch.bfloat16):
        tq = StaticGridPerTensorQuantizer(8, "nearest", QuantScheme.post_training_tf, False, True)
        src = torch.randn(4096, device=DEV, generator=g) * 0.3
        tq.update_encoding_stats(src)
        tq.compute_encoding()
        x = src.to(dt)
        rmn, rmx = torch.tensor(tq.encoding.min).to(dt), torch.tensor(tq.encoding.max).to(dt)
        x[:4] = rmn.to(DEV)
        x[4:8] = rmx.to(DEV)
        a = x.clone().requires_grad_(True)
        y = tq.quantize_dequantize(a, "nearest")
        up = torch.randn(4096, device=DEV, generator=g).to(dt)
        y.backward(up)
        # the reference's expression on the CPU (quantsim_straight_through_grad.py:66-118)
        emin, emax = torch.tensor(tq.encoding.min), torch.tensor(tq.encoding.max)
        xc = x.cpu()
        want = up.cpu() * (emin <= xc).logical_and(xc <= emax)
        assert torch.equal(a.grad.cpu().view(torch.int16), want.view(torch.int16)), dt


def _same_bits_or_nan(got, want):
    got, want = np.asarray(got, np.float32).ravel(), np.asarray(want, np.float32).ravel()
    nan = np.isnan(want)
    return np.array_equal(np.isnan(got), nan) and np.array_equal(got[~nan].view(np.int32), want[~nan].view(np.int32))


def test_adaround_special_values_vs_torch_cpu():
    """Inputs the golden vectors do not hold, against torch's CPU ops on the reference's expressions
    (oracle/torch_ref.py: apply_adaround, compute_round_loss; autograd for dL/dalpha): alpha NaN,
    +-inf, +-0, at and beside the sigmoid's range clamps (+-100, -104, 88.7) and +-1e30; weights
    NaN, +-inf, +-0, tiny negatives (the floor guard's fract near 1) and multiples of delta one ulp
    off. With the exact pow Wq and dL/dalpha (rounding loss included) are bit-exact, NaN for NaN;
    with the default pow Wq and the reconstruction gradient are. n = 1024: no scalar pow tail."""
    from aimet_amd.adaround import AdaroundFunction, set_exact_pow
    from oracle import torch_ref as T
    f32 = np.float32
    alphas = f32([np.nan, np.inf, -np.inf, 0.0, -0.0, 100.0, 100.5, 99.99, -100.0, -103.9, -104.0, -104.5, 88.7,
                  87.3, -88.7, 1e30, -1e30, 3e38, -3e38, 1e-30, -1e-30, 2.3, -2.3, 0.125])
    rng = np.random.default_rng(21)
    C, K = 4, 256
    a = rng.standard_normal(C * K).astype(f32) * f32(3)
    a[:alphas.size] = alphas
    a[512:512 + alphas.size] = alphas[::-1]
    delta = f32([0.01, 0.0037, 0.25, 1e-3])
    k = rng.integers(-140, 140, (C, K)).astype(f32)
    w = (k * delta[:, None]).astype(f32)
    w[:, 1::3] = np.nextafter(w[:, 1::3], f32(np.inf))
    w[:, 2::3] = np.nextafter(w[:, 2::3], f32(-np.inf))
    wspecial = f32([np.nan, np.inf, -np.inf, 0.0, -0.0, -1e-40, -1e-30, 1e-40, -1e-8, -0.0049999])
    w[0, 100:100 + wspecial.size] = wspecial
    w[3, 7:7 + wspecial.size] = wspecial
    a = a.reshape(C, K)
    off = f32([-128.0, -100.0, -3.0, 0.0])
    g = rng.standard_normal((C, K)).astype(f32)
    reg, beta, bw = 0.01, 7.5, 8
    # torch CPU: the reference's expressions, autograd for dL/dalpha
    at = torch.from_numpy(a.copy()).requires_grad_(True)
    dt, ot = torch.from_numpy(delta).view(C, 1), torch.from_numpy(off).view(C, 1)
    wq_ref = T.adaround_forward(torch.from_numpy(w), at, dt, ot, bw)
    (wq_ref * torch.from_numpy(g)).sum().backward()
    ga_recon = at.grad.numpy().copy()
    at.grad = None
    wq_ref2 = T.adaround_forward(torch.from_numpy(w), at, dt, ot, bw)
    ((wq_ref2 * torch.from_numpy(g)).sum() + T.adaround_round_loss(at, reg, beta)).backward()
    ga_total = at.grad.numpy().copy()
    wq_ref = wq_ref.detach().numpy()
    wd, dd, od, gd = (torch.from_numpy(v).to(DEV) for v in (w, delta, off, g))
    for exact in (True, False):
        prev = set_exact_pow(exact)
        try:
            ad = torch.from_numpy(a).to(DEV).requires_grad_(True)
            wq = AdaroundFunction.apply(wd, ad, dd, od, bw, 0)
            (wq * gd).sum().backward()
            assert _same_bits_or_nan(wq.detach().cpu().numpy(), wq_ref), exact
            assert _same_bits_or_nan(ad.grad.cpu().numpy(), ga_recon), exact
            if exact:
                ad = torch.from_numpy(a).to(DEV).requires_grad_(True)
                (AdaroundFunction.apply(wd, ad, dd, od, bw, 0, True, reg, beta, None) * gd).sum().backward()
                assert _same_bits_or_nan(ad.grad.cpu().numpy(), ga_total)
        finally:
            set_exact_pow(prev)
