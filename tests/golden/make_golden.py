"""Generate the committed golden fixtures of tests/golden from the REFERENCE itself.

Run in the build container only (it needs /root/reference):

    python tests/golden/make_golden.py

Sources of truth, in order:
  * oracle/_ref/libdlq_ref.so -- the reference DlQuantization C++ compiled in place from
    /root/reference (oracle/build_ref.sh). Produces every integer encoding, QDQ output,
    histogram/PDF and analyzer encoding stored here.
  * the reference's own known-answer tests (values copied with file:line into kat.json).
  * the reference's Python (aimet_torch.v1.quantsim_straight_through_grad,
    aimet_torch.v1.adaround.adaround_loss), imported read-only with bytecode writing off,
    for the STE mask and the AdaRound round-loss/beta.
  * torch CPU float32 ops in exactly the sequence of AimetTensorQuantizer.cpp:236-299 for the
    per-channel encoding tables (that is what the reference executes on that path).
  * AdaroundWrapper.apply_adaround / _generate_alpha_parameter (adaround_wrapper.py:124-149,
    211-224): the module cannot be imported here (its import chain needs bokeh, jsonschema,
    torchvision, spconv and the aimet_torch.v1.nn package the reference snapshot lacks), so the
    generator parses the reference file, takes those two function definitions as they stand and
    executes them (torch CPU, one thread) with the attributes they read. Nothing of that source is
    written anywhere; only inputs and outputs are stored (golden_adaround.npz).

The fixtures are data (inputs + expected outputs); no reference source text is stored.
"""
import json
import os
import subprocess
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
REF_ROOT = os.environ.get("AIMET_REFERENCE", "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import ref as R  # noqa: E402

EDGE = np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 1e30, -1e30, 1e-40, -1e-40, 0.5, -0.5, 1.5, -2.5],
                dtype=np.float32)


def per_tensor_cases(rng):
    xs, encs = [], []
    for t in range(40):
        x = (rng.standard_normal(2048) * rng.uniform(0.01, 30) + rng.uniform(-3, 3)).astype(np.float32)
        x[:EDGE.size] = EDGE
        mn, mx = sorted(rng.uniform(-8, 8, 2))
        bw = int([8, 8, 8, 4, 16, 31, 32][t % 7])
        if t % 5 == 0:
            mn = -mx            # strict-symmetric detection branch (TensorQuantizationSim.cpp:70-73)
        if t % 9 == 0:
            mn = 0.0            # ReLU-like encodings
        if t % 13 == 0:
            mx = mn             # gated min == max
        xs.append(x)
        encs.append((mn, mx, bw))
    # ties: values exactly on .5 quantization boundaries of a 1/255 grid
    e = R.fill_encoding_info(8, -1.0, 1.0)
    k = np.arange(-300, 300, dtype=np.float64)
    xs.append(((k + 0.5) * e.delta).astype(np.float32)[:2048] if k.size >= 2048 else
              np.resize(((k + 0.5) * e.delta).astype(np.float32), 2048))
    encs.append((-1.0, 1.0, 8))
    return np.stack(xs), np.array(encs, dtype=np.float64)


def torch_channel_table(encs):
    """AimetTensorQuantizer.cpp:236-299, CPU torch float32 ops, literally."""
    C = len(encs)
    ev = torch.tensor([e[0] for e in encs] + [e[1] for e in encs], dtype=torch.float32).view(2, C)
    emin, emax = ev[0], ev[1]
    steps = 2 ** int(encs[0][4]) - 1
    if encs[0][0] == -encs[0][1]:
        steps -= 1
    zero = torch.zeros(1)
    emin = torch.minimum(emin, zero)
    emax = torch.maximum(emax, zero)
    emax = torch.maximum(emax, emin + 1e-5)
    delta = (emax - emin) / float(steps)
    off = torch.round(emin / delta)
    return torch.stack([emin, emax, delta, off]).numpy()


def per_channel_cases(rng):
    out = []
    shapes = [(1, 64, 27), (1, 16, 9), (1, 3, 1), (2, 8, 33), (1, 300, 4), (4, 5, 6)]   # (outer, C, K)
    for si, (outer, C, K) in enumerate(shapes):
        x = (rng.standard_normal(outer * C * K) * rng.uniform(0.1, 3)).astype(np.float32)
        x[:min(EDGE.size, x.size)] = EDGE[:min(EDGE.size, x.size)]
        bw = 8 if si % 2 == 0 else 4
        sym = si % 3 == 0
        encs = []
        for c in range(C):
            a = R.Analyzer(0)
            a.update(rng.standard_normal(64).astype(np.float32) * (c + 1) / C)
            e = a.compute(bw, sym, False, False)
            encs.append(e.as_tuple())
        table = torch_channel_table(encs)
        y = R.qdq_per_channel(x, C, K, table)
        out.append(dict(x=x, outer=outer, C=C, K=K, encs=np.array(encs), table=table, y=y))
    return out


def analyzer_cases(rng):
    cases = []
    flagsets = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 1)]
    for scheme, ncase in ((0, 6), (1, 6), (3, 5), (4, 3)):
        for t in range(ncase):
            nb = 3
            batches = []
            for k in range(nb):
                n = int(rng.integers(500, 1500))
                x = (rng.standard_normal(n) * rng.uniform(0.05, 5) + rng.uniform(-2, 2)).astype(np.float32)
                if t == 1:
                    x = np.maximum(x, 0)                     # ReLU output: min == 0
                if t == 2 and k == 0:
                    x[:] = 0                                 # all-zero first batch (math_functions.cpp:254-259)
                if t == 3:
                    x[:7] = EDGE[2:9]                        # nan/inf/huge/denormal
                batches.append(x)
            a = R.Analyzer(scheme)
            pct = 99.0 if (scheme == 3 and t % 2) else 100.0
            if scheme == 3:
                a.set_percentile(pct)
            for x in batches:
                a.update(x)
            encs = {}
            for bw in (8, 4, 16):
                for fl in flagsets:
                    encs["%d_%d%d%d" % ((bw,) + fl)] = a.compute(bw, *fl).as_tuple()
            xl, pdf = a.histogram() if scheme != 0 else (np.zeros(0), np.zeros(0))
            cases.append(dict(scheme=scheme, percentile=pct, batches=batches, encs=encs, xleft=xl, pdf=pdf))
    return cases


def tfe_kat_data(count=6000):
    exe = os.path.join(tempfile.mkdtemp(), "gen")
    subprocess.run(["g++", "-O2", "-o", exe, os.path.join(HERE, "gen_mt19937_normal.cpp")], check=True)
    path = exe + ".f32"
    subprocess.run([exe, path, str(count)], check=True)
    return np.fromfile(path, dtype=np.float32)


ENTROPY_FLAGS = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 1), (0, 1, 0)]


def entropy_cases(rng):
    """Entropy analyzer (EntropyEncodingAnalyzer.cpp + updateTensorHistogram_cpu): batch sequences
    that initialise, widen (rescale) and skip the histogram. Per case: the TensorProfilingParams
    after the last batch (reference updateTensorHistogram_cpu) and the analyzer's encodings."""
    cases = []
    for t in range(12):
        nb = 5 if t in (6, 9) else 3
        batches = []
        for k in range(nb):
            n = int(rng.integers(300, 3000)) if t != 7 else 20000
            mu, s = rng.uniform(-2, 2), rng.uniform(0.05, 5) * (1 + k)      # ranges grow: rescales
            x = (rng.standard_normal(n) * s + mu).astype(np.float32)
            if t == 1:
                x = np.maximum(x, 0)                                      # ReLU output
            elif t == 2 and k != 1:
                x[:] = 0                                                  # all-zero batches (skipped)
            elif t == 3:
                x[:5] = [np.nan, 1e30, -1e30, 1e-40, -1e-40]              # no inf: the reference asserts
            elif t == 4 and k == 0:
                x[:] = 1.25                                               # min == max (+0.01)
            elif t == 5:
                x = -np.abs(x)                                            # one-sided negative
            elif t == 6:
                x = (rng.laplace(0, 1, n) * rng.uniform(0.1, 10)).astype(np.float32)
            elif t == 8:
                x = (np.abs(x) + 3).astype(np.float32)                    # positive, away from 0
            elif t == 9 and k % 2:
                x = x[::-1].copy() * 0.01                                 # narrower batch: no rescale
            elif t == 10:
                x = np.round(x * 4).astype(np.float32) / 4                # values on a lattice
            elif t == 11:
                x[:] = rng.uniform(-1, 1) * np.float32(1e-3) * (1 + k)    # constant batches
            batches.append(x.astype(np.float32))
        cases.append(batches)
    out = []
    for batches in cases:
        a, tpp = R.Analyzer(5), R.TensorProfilingParams()
        for x in batches:
            a.update(x)
            tpp.update(x)
        encs = {}
        for bw in (8, 4, 16):
            for fl in ENTROPY_FLAGS:
                encs["%d_%d%d%d" % ((bw,) + fl)] = a.compute(bw, *fl).as_tuple()
        out.append(dict(batches=batches, encs=encs, tpp=tpp.state()))
    return out


def entropy_golden():
    """golden_entropy.npz: entropy analyzer cases + the TestEntropyEncodingAnalyzer KAT input."""
    rng = np.random.default_rng(20251016)
    en = {}
    cases = entropy_cases(rng)
    for i, c in enumerate(cases):
        en["e%d_nb" % i] = np.array(len(c["batches"]))
        for k, b in enumerate(c["batches"]):
            en["e%d_b%d" % (i, k)] = b
        st = c["tpp"]
        en["e%d_tpp" % i] = np.array([st["has_hist"], st["min"], st["max"], st["iterations"]], dtype=np.float64)
        en["e%d_hist" % i] = st["hist"]
        keys = sorted(c["encs"])
        en["e%d_enc_keys" % i] = np.array(keys)
        en["e%d_enc_vals" % i] = np.array([c["encs"][k] for k in keys], dtype=np.float64)
    en["count"] = np.array(len(cases))
    kx = tfe_kat_data(100000)
    a = R.Analyzer(5)
    a.update(kx)
    en["kat_x"] = kx
    en["kat_enc_keys"] = np.array(["8_%d%d%d" % fl for fl in ENTROPY_FLAGS])
    en["kat_enc_vals"] = np.array([a.compute(8, *fl).as_tuple() for fl in ENTROPY_FLAGS], dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "golden_entropy.npz"), **en)


def reference_python():
    """Import the reference's pure-Python STE and AdaRound-loss modules (read-only)."""
    for p in ("TrainingExtensions/torch/src/python", "TrainingExtensions/common/src/python"):
        sys.path.insert(0, os.path.join(REF_ROOT, p))
    import aimet_torch.v1.quantsim_straight_through_grad as ste  # noqa
    from aimet_torch.v1.adaround.adaround_loss import AdaroundLoss, AdaroundHyperParameters  # noqa
    return ste, AdaroundLoss, AdaroundHyperParameters


BROADCAST_CASES = [   # (input shape, channel axis, block axis, block size)
    ((2, 3, 4), 1, 0, 1), ((4, 2, 2), 2, 0, 2), ((4, 4), 0, 1, 2), ((10, 4, 10), 1, 0, 2),
    ((16, 64), 0, 1, 16), ((64, 32), 1, 0, 8), ((8, 6, 3, 3), 0, 1, 3), ((3, 5, 7), -1, 2, 7),
    ((4, 2, 2), 1, -1, 0), ((6, 2), 1, 0, 2), ((2, 6), 0, 1, 3), ((5, 12, 4), 2, 1, 4),
]


def broadcast_golden():
    """golden_broadcast.npz: blockwise QDQ (quantizeDequantizeBroadcastCpu, trim_functions.cpp:633-660)
    of random tensors under random per-block encodings, views from BroadcastShapeInfo."""
    from oracle import oracle as O
    rng = np.random.default_rng(20251017)
    g = {}
    for i, (shape, ch, ba, bs) in enumerate(BROADCAST_CASES):
        info = O.broadcast_shape_info(shape, ch, ba, bs)
        E = info["num_encodings"]
        x = (rng.standard_normal(int(np.prod(shape))) * rng.uniform(0.5, 4)).astype(np.float32)
        x[: min(4, x.size)] = EDGE[[2, 5, 7, 10]][: min(4, x.size)]     # nan, 1e30, denormal, -0.5
        bw = 4 if i % 3 == 0 else 8
        encs = []
        for e in range(E):
            lo, hi = -rng.uniform(0.1, 3), rng.uniform(0.1, 3)
            sym = bool(e % 2)
            encs.append(R.get_computed_encodings(bw, lo, hi, sym, False, False).as_tuple())
        encs = np.array(encs, dtype=np.float64)
        f = encs[:, :4].astype(np.float32)
        y = R.qdq_broadcast(x, info["tensor_strides"], info["encoding_strides"], f[:, 0], f[:, 1], f[:, 2], f[:, 3])
        g["b%d_cfg" % i] = np.array([ch, ba, bs], dtype=np.int64)
        g["b%d_shape" % i] = np.array(shape, dtype=np.int64)
        g["b%d_x" % i], g["b%d_encs" % i], g["b%d_y" % i] = x, encs, y
    g["count"] = np.array(len(BROADCAST_CASES))
    np.savez_compressed(os.path.join(HERE, "golden_broadcast.npz"), **g)


def _reference_adaround_functions():
    """apply_adaround and _generate_alpha_parameter exactly as the reference defines them
    (adaround_wrapper.py), compiled from the reference file at generation time."""
    import ast
    for p in ("TrainingExtensions/torch/src/python", "TrainingExtensions/common/src/python"):
        sys.path.insert(0, os.path.join(REF_ROOT, p))
    from aimet_common.defs import AdaroundConstants
    path = os.path.join(REF_ROOT, "TrainingExtensions/torch/src/python/aimet_torch/v1/adaround/adaround_wrapper.py")
    tree = ast.parse(open(path).read(), path)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "AdaroundWrapper")
    fns = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name in ("apply_adaround",
                                                                                "_generate_alpha_parameter")]
    for f in fns:
        f.decorator_list = []
    mod = ast.Module(body=fns, type_ignores=[])
    ns = {"torch": torch, "AdaroundConstants": AdaroundConstants, "Tuple": tuple}
    exec(compile(mod, path, "exec"), ns)
    return ns["apply_adaround"], ns["_generate_alpha_parameter"]


# MobileNet-v2 weight shapes (conv / depthwise / pointwise / classifier) + a ragged one
ADAROUND_CASES = [   # (shape, bitwidth, alpha source)
    ((32, 3, 3, 3), 8, "init"), ((32, 1, 3, 3), 8, "init"), ((96, 1, 3, 3), 4, "init"),
    ((16, 32, 1, 1), 4, "wide"), ((64, 24, 1, 1), 8, "wide"), ((160, 320, 1, 1), 8, "init"),
    ((100, 1280), 4, "wide"), ((24, 1, 3, 3), 8, "tails"), ((7, 5, 3, 3), 4, "wide"),
]


def adaround_golden():
    """golden_adaround.npz: forward Wq of the reference's apply_adaround and d(loss)/d(alpha)
    through torch autograd of the reference expressions, for (a) a reconstruction-like loss
    sum(Wq * g) alone (warm start: no rounding loss) and (b) plus the reference's
    AdaroundLoss.compute_round_loss after warm start. Per-channel symmetric delta / offset along
    axis 0 (broadcast_to_tensor form), torch CPU float32 on ONE thread, so every element except a
    tensor's last numel % 32 takes torch's vectorized sigmoid (Sleef expf_u10 + IEEE divide)."""
    from types import SimpleNamespace
    apply_adaround, gen_alpha = _reference_adaround_functions()
    _, AdaroundLoss, AdaroundHyperParameters = reference_python()
    torch.set_num_threads(1)
    g = torch.Generator().manual_seed(20251107)
    hp = AdaroundHyperParameters(num_iterations=10000, reg_param=0.01, beta_range=(20, 2), warm_start=0.2)
    out = {}
    for i, (shape, bw, src) in enumerate(ADAROUND_CASES):
        C = shape[0]
        w = torch.randn(shape, generator=g) * (0.05 + 0.3 * torch.rand(C, *[1] * (len(shape) - 1), generator=g))
        steps = 2 ** bw - 1
        absmax = w.reshape(C, -1).abs().amax(1)
        # symmetric encodings (quantization_utils.cpp:83-93 form), float32 as makeDeltaOffsetTensor gives them
        delta = (absmax / float(steps // 2)).float()
        offset = torch.full((C,), -float((steps + 1) // 2))
        bshape = (C,) + (1,) * (len(shape) - 1)
        bd, bo = delta.view(bshape), offset.view(bshape)
        if src == "init":
            alpha = gen_alpha(w, bd).detach()
        elif src == "wide":
            alpha = torch.randn(shape, generator=g) * 4.0
        else:   # sigmoid's saturated tails and |alpha| near the exp under/overflow range
            alpha = (torch.rand(shape, generator=g) * 2 - 1) * 110.0
        mod = SimpleNamespace(alpha=alpha.clone().requires_grad_(True), broadcasted_delta=bd, broadcasted_offset=bo,
                              use_soft_rounding=True, clip_min=0, clip_max=steps)
        wq = apply_adaround(mod, w)
        grad = torch.randn(shape, generator=g) * 1e-3
        (wq * grad).sum().backward()
        ga_recon = mod.alpha.grad.detach().clone()
        # + the rounding loss at iteration 6000 of 10000 (after the 20% warm start)
        mod.alpha.grad = None
        wq2 = apply_adaround(mod, w)
        loss = (wq2 * grad).sum() + AdaroundLoss.compute_round_loss(mod.alpha, hp, 6000)
        loss.backward()
        ga_total = mod.alpha.grad.detach().clone()
        round_loss = float(AdaroundLoss.compute_round_loss(mod.alpha.detach(), hp, 6000))
        beta = float(AdaroundLoss._compute_beta(10000, 6000, (20, 2), 0.2))
        # hard rounding (use_soft_rounding False)
        mod.use_soft_rounding = False
        wq_hard = apply_adaround(mod, w).detach()
        k = "c%d_" % i
        out[k + "w"], out[k + "alpha"], out[k + "delta"], out[k + "offset"] = (w.numpy(), alpha.numpy(),
                                                                             delta.numpy(), offset.numpy())
        out[k + "bw"] = np.array(bw)
        out[k + "grad"], out[k + "wq"], out[k + "wq_hard"] = grad.numpy(), wq.detach().numpy(), wq_hard.numpy()
        out[k + "ga_recon"], out[k + "ga_total"] = ga_recon.numpy(), ga_total.numpy()
        out[k + "round_loss"], out[k + "beta"] = np.array(round_loss), np.array(beta)
        if src == "init":
            out[k + "alpha_init"] = alpha.numpy()   # _generate_alpha_parameter(w, delta)
    out["count"] = np.array(len(ADAROUND_CASES))
    out["reg_param"], out["cur_iter"] = np.array(0.01), np.array(6000)
    np.savez_compressed(os.path.join(HERE, "golden_adaround.npz"), **out)


def ste16_golden():
    """golden_ste16.npz: the reference compute_dloss_by_dx with fp16 / bf16 x and grad, per-tensor
    python-float bounds that are NOT representable in the 16-bit type (broadcast_to_tensor makes
    them 0-dim float32 tensors: compared in x's dtype) and per-channel lists (1-D float32: compared
    in float32), with x values placed exactly on and next to the rounded bounds; plus bf16 x with
    an fp32 grad (mixed dtypes)."""
    ste, _, _ = reference_python()
    g = torch.Generator().manual_seed(77)
    out = {}
    cases = []
    for dt in (torch.float16, torch.bfloat16):
        for mn, mx in ((-0.1, 0.1), (-1.2345678, 2.7182818), (0.30000001, 0.7), (-3.1415926, -0.01)):
            cases.append((dt, dt, mn, mx))
    cases.append((torch.bfloat16, torch.float32, -0.1, 0.1))
    cases.append((torch.float16, torch.float32, -1.2345678, 2.7182818))
    for i, (xd, gd, mn, mx) in enumerate(cases):
        x = (torch.randn(4096, generator=g) * max(abs(mn), abs(mx)) * 1.3).to(xd)
        # the rounded bounds and their 16-bit neighbours
        for j, b in enumerate((mn, mx)):
            rb = torch.tensor(b).to(xd)
            nb = torch.stack([rb, torch.nextafter(rb.float(), torch.tensor(1e9)).to(xd),
                              torch.nextafter(rb.float(), torch.tensor(-1e9)).to(xd)])
            x[100 * j:100 * j + 60] = nb.repeat(20)
        grad = torch.randn(4096, generator=g).to(gd)
        out["t%d_x" % i] = x.view(torch.int16).numpy()
        out["t%d_grad" % i] = grad.view(torch.int16).numpy() if gd != torch.float32 else grad.numpy()
        out["t%d_dtypes" % i] = np.array([str(xd), str(gd)])
        out["t%d_bounds" % i] = np.array([mn, mx])
        out["t%d_pt" % i] = _as_bits(ste.compute_dloss_by_dx(x, grad, mn, mx))
    # per-channel lists (C = 1 included: a 1-D bound, compared in float32)
    for C in (1, 8):
        for dt in (torch.float16, torch.bfloat16):
            x = (torch.randn(C, 256, generator=g) * 0.2).to(dt)
            grad = torch.randn(C, 256, generator=g).to(dt)
            mins = [-0.1 - 0.013 * c for c in range(C)]
            maxs = [0.1 + 0.017 * c for c in range(C)]
            for c in range(C):
                x[c, :3] = torch.tensor(mins[c]).to(dt)
                x[c, 3:6] = torch.tensor(maxs[c]).to(dt)
            k = "p%d_%s_" % (C, str(dt).split(".")[1])
            out[k + "x"] = x.view(torch.int16).numpy()
            out[k + "grad"] = grad.view(torch.int16).numpy()
            out[k + "mins"], out[k + "maxs"] = np.array(mins), np.array(maxs)
            out[k + "out"] = _as_bits(ste.compute_dloss_by_dx(x, grad, mins, maxs, ch_axis=0))
    out["count"] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, "golden_ste16.npz"), **out)


# ---- encoding export (the `<prefix>_torch.encodings` file) -----------------------------------
# One layer spec per wrapper of the stand-in sim model: (name, module kind, quantizer settings).
# Encodings are exact binary fractions and small integers so the JSON carries them unrounded.
ENCODING_LAYERS = [
    # name, module, input quantizers, output quantizers, params {name: quantizer}
    ("conv1", "conv", [{"enabled": True, "bw": 8, "sym": False, "enc": [-1.0, 2.984375, 0.015625, -64]}],
     [{"enabled": True, "bw": 8, "sym": False, "enc": [-0.25, 3.734375, 0.015625, -16]}],
     {"weight": {"enabled": True, "bw": 4, "sym": True,
                 "enc": [[-0.5, 0.4375, 0.0625, -8], [-1.0, 0.875, 0.125, -8], [-0.25, 0.21875, 0.03125, -8]]},
      "bias": {"enabled": False, "bw": 8, "sym": True, "enc": None}}),
    ("conv2", "conv", [{"enabled": False, "bw": 8, "sym": False, "enc": None}],
     [{"enabled": True, "bw": 16, "sym": True, "enc": [-4.0, 3.9998779296875, 0.0001220703125, -32768]}],
     {"weight": {"enabled": True, "bw": 8, "sym": True, "enc": [-0.5, 0.49609375, 0.00390625, -128]},
      "bias": {"enabled": False, "bw": 8, "sym": True, "enc": None}}),
    ("head.fc", "linear", [{"enabled": False, "bw": 8, "sym": False, "enc": None}],
     [{"enabled": True, "bw": 8, "sym": False, "enc": [-8.0, 7.9375, 0.0625, -128]}],
     {"weight": {"enabled": True, "bw": 4, "sym": False, "enc": [-0.75, 1.125, 0.125, -6]},
      "bias": {"enabled": True, "bw": 8, "sym": True, "enc": [-2.0, 1.984375, 0.015625, -128]}}),
    ("head.quiet", "linear", [{"enabled": False, "bw": 8, "sym": False, "enc": None}],
     [{"enabled": False, "bw": 8, "sym": False, "enc": None}],
     {"weight": {"enabled": False, "bw": 8, "sym": True, "enc": None},
      "bias": {"enabled": False, "bw": 8, "sym": True, "enc": None}}),
]
ENCODING_SETTINGS = {"quant_scheme": "post_training_tf_enhanced", "default_param_bw": 4, "default_output_bw": 8,
                     "config": {"defaults": {"params": {"is_symmetric": True}, "per_channel_quantization": True}},
                     "excluded_layers": ["head.dropout"]}


def _ast_functions(rel, names, cls=None, keep_decorators=False):
    import ast
    path = os.path.join(REF_ROOT, rel)
    tree = ast.parse(open(path).read(), path)
    body = tree.body
    if cls is not None:
        body = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls).body
    fns = [n for n in body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert {f.name for f in fns} == set(names), (rel, names)
    if not keep_decorators:
        for f in fns:
            f.decorator_list = []
    return ast.Module(body=fns, type_ignores=[]), path


def encodings_golden():
    """golden_encodings.json: the `<prefix>_torch.encodings` content that the reference's own export
    code writes -- QuantizationSimModel._export_encodings_to_files (v1/quantsim.py:940-1043) with
    _get_torch_encodings_for_missing_layers (:884-938), has_valid_encodings (:2302-2323),
    QcQuantizeWrapper.export_*_encodings and export_quantizer_encoding / get_encoding_by_quantizer
    (v1/qc_quantize_op.py:481-497, 1514-1545), create_encoding_dict (aimet_torch/utils.py:1156-1186),
    extract_global_quantizer_args (aimet_common/quantsim.py:280-310) and save_json_yaml
    (aimet_common/utils.py:347-360), compiled from the reference files at generation time -- run
    over stand-in wrappers / quantizers holding ENCODING_LAYERS (the modules cannot be imported
    here: their import chains need the compiled libpymo). With no ONNX graph every layer takes the
    torch-only path, as the torch encodings file is built. Stored with the layer specs it came from."""
    import logging
    import types
    for p in ("TrainingExtensions/torch/src/python", "TrainingExtensions/common/src/python"):
        if os.path.join(REF_ROOT, p) not in sys.path:
            sys.path.insert(0, os.path.join(REF_ROOT, p))
    from typing import Dict, List, Optional, Union
    from aimet_common.defs import QuantizationDataType, QuantScheme

    class LearnedGridTensorQuantizer:   # none of the stand-in quantizers is one
        pass

    class QcQuantizeRecurrent:
        pass

    class TfEncoding:   # libpymo.TfEncoding's fields
        def __init__(self, mn, mx, delta, offset, bw):
            self.min, self.max, self.delta, self.offset, self.bw = mn, mx, delta, offset, bw

    ns = {"QuantizationDataType": QuantizationDataType, "QuantScheme": QuantScheme, "Dict": Dict, "List": List,
          "Optional": Optional, "Union": Union, "LearnedGridTensorQuantizer": LearnedGridTensorQuantizer,
          "QcQuantizeRecurrent": QcQuantizeRecurrent, "logger": logging.getLogger("golden"), "os": os,
          "json": json, "SAVE_TO_YAML": False, "QUANTIZER_TYPE_INPUT": "input", "QUANTIZER_TYPE_OUTPUT": "output",
          "libpymo": types.SimpleNamespace(TfEncoding=TfEncoding), "StaticGridTensorQuantizer": object,
          "QuantizedModuleProtocol": object, "QuantSimConfigurator": object, "TensorQuantizer": object,
          "torch": torch, "Tuple": tuple, "Any": object}
    for rel, names, cls in (
            ("TrainingExtensions/torch/src/python/aimet_torch/utils.py", ["create_encoding_dict"], None),
            ("TrainingExtensions/torch/src/python/aimet_torch/v1/qc_quantize_op.py",
             ["get_encoding_by_quantizer", "export_quantizer_encoding"], None),
            ("TrainingExtensions/common/src/python/aimet_common/quantsim.py", ["extract_global_quantizer_args"], None),
            ("TrainingExtensions/common/src/python/aimet_common/utils.py", ["save_json_yaml"], None),
            ("TrainingExtensions/torch/src/python/aimet_torch/v1/quantsim.py", ["has_valid_encodings"], None)):
        mod, path = _ast_functions(rel, names, cls)
        exec(compile(mod, path, "exec"), ns)
    ns["utils"] = types.SimpleNamespace(create_encoding_dict=ns["create_encoding_dict"],
                                        DROPOUT_TYPES=(torch.nn.Dropout, torch.nn.Dropout2d, torch.nn.Dropout3d))
    wmod, wpath = _ast_functions("TrainingExtensions/torch/src/python/aimet_torch/v1/qc_quantize_op.py",
                                 ["export_param_encodings", "export_output_encodings", "export_input_encodings",
                                  "get_original_module"], cls="QcQuantizeWrapper")
    wns = dict(ns)
    exec(compile(wmod, wpath, "exec"), wns)

    class Wrapper(torch.nn.Module):   # the reference wrapper's export surface over stand-in quantizers
        export_param_encodings = wns["export_param_encodings"]
        export_output_encodings = wns["export_output_encodings"]
        export_input_encodings = wns["export_input_encodings"]
        get_original_module = wns["get_original_module"]

        def __init__(self, module, ins, outs, params):
            super().__init__()
            self._module_to_wrap = module
            self.input_quantizers, self.output_quantizers, self.param_quantizers = ins, outs, params
    ns["QuantizedModuleProtocol"] = Wrapper
    # QuantizationSimModel's export methods with their static / class method decorators, on a class
    # of their own; the ONNX map is synthetic (one op per layer, torch's pre-1.13 naming,
    # EXPORT_TO_ONNX_DIRECT off) so every layer takes the path a real export takes
    from packaging import version
    ns["version"] = version
    omod, opath = _ast_functions("TrainingExtensions/torch/src/python/aimet_torch/onnx_utils.py",
                                 ["get_layers_in_io_tensor_map", "get_tensor_to_consumer_map"])
    ons = dict(ns, EXPORT_TO_ONNX_DIRECT=False)
    exec(compile(omod, opath, "exec"), ons)
    ns["onnx_utils"] = types.SimpleNamespace(EXPORT_TO_ONNX_DIRECT=False,
                                             get_layers_in_io_tensor_map=ons["get_layers_in_io_tensor_map"],
                                             get_tensor_to_consumer_map=ons["get_tensor_to_consumer_map"])
    ns["quantsim"] = types.SimpleNamespace(encoding_version="0.6.1")
    qsm_methods = ["_get_torch_encodings_for_missing_layers", "_update_encoding_dicts_for_layer",
                   "_export_encodings_to_files", "_update_param_encodings_dict_for_layer",
                   "_update_encoding_dict_for_input_activations", "_update_encoding_dict_for_output_activations",
                   "_get_layer_input_tensors", "_get_layer_activation_tensors", "find_op_names_for_layer",
                   "_get_output_map_str"]
    smod, spath = _ast_functions("TrainingExtensions/torch/src/python/aimet_torch/v1/quantsim.py", qsm_methods,
                                 cls="QuantizationSimModel", keep_decorators=True)
    exec(compile(smod, spath, "exec"), ns)

    class QuantizationSimModel:
        pass
    for k in qsm_methods:
        setattr(QuantizationSimModel, k, ns.pop(k))
    ns["QuantizationSimModel"] = QuantizationSimModel

    def quantizer(spec):
        enc = spec["enc"]
        if enc is not None:
            enc = [TfEncoding(*e, spec["bw"]) for e in enc] if isinstance(enc[0], list) else \
                TfEncoding(*enc, spec["bw"])
        return types.SimpleNamespace(enabled=spec["enabled"], bitwidth=spec["bw"], use_symmetric_encodings=spec["sym"],
                                     data_type=QuantizationDataType.int, encoding=enc)

    model = torch.nn.Module()
    model.head = torch.nn.Module()
    valid = set()
    for name, kind, ins, outs, params in ENCODING_LAYERS:
        m = torch.nn.Conv2d(3, 3, 3) if kind == "conv" else torch.nn.Linear(4, 4)
        w = Wrapper(m, [quantizer(q) for q in ins], [quantizer(q) for q in outs],
                    {p: quantizer(q) for p, q in params.items()})
        parent, leaf = (model.head, name.split(".")[1]) if "." in name else (model, name)
        setattr(parent, leaf, w)
        valid |= {name + "." + p for p in params}
    cfg = ENCODING_SETTINGS
    configurator = types.SimpleNamespace(quantsim_configs=cfg["config"], default_param_bw=cfg["default_param_bw"],
                                         default_output_bw=cfg["default_output_bw"],
                                         default_data_type=QuantizationDataType.int)
    qargs = ns["extract_global_quantizer_args"](QuantScheme[cfg["quant_scheme"]], configurator)
    io_map = {}
    for name, kind, ins, outs, params in ENCODING_LAYERS:
        io_map[name] = types.SimpleNamespace(inputs=[name + ".in"] + [name + "." + p for p in params],
                                             outputs=[name + ".out"])
    with tempfile.TemporaryDirectory() as d:
        QuantizationSimModel._export_encodings_to_files(model, d, "golden", io_map, valid, cfg["excluded_layers"],
                                                        False, qargs)
        with open(os.path.join(d, "golden_torch.encodings")) as f:
            torch_encodings = json.load(f)
    out = {"source": "the reference's own export functions (tests/golden/make_golden.py: encodings_golden)",
           "layers": ENCODING_LAYERS, "settings": ENCODING_SETTINGS, "torch_encodings": torch_encodings}
    with open(os.path.join(HERE, "golden_encodings.json"), "w") as f:
        json.dump(out, f, indent=1)


def _as_bits(t):
    return t.view(torch.int16).numpy() if t.dtype in (torch.float16, torch.bfloat16) else t.numpy()


def main():
    if "--adaround-only" in sys.argv:
        adaround_golden()
        return
    if "--ste16-only" in sys.argv:
        ste16_golden()
        return
    if "--broadcast-only" in sys.argv:
        broadcast_golden()
        return
    entropy_golden()
    if "--entropy-only" in sys.argv:
        return
    broadcast_golden()
    rng = np.random.default_rng(20251015)
    R.lib()

    # ---- per-tensor QDQ / quantize-only / encoding math -------------------------------
    xs, encs = per_tensor_cases(rng)
    qdq = np.stack([R.qdq_per_tensor(x, e[0], e[1], int(e[2])) for x, e in zip(xs, encs)])
    q_u = np.stack([R.quantize_per_tensor(x, e[0], e[1], int(e[2]), False) for x, e in zip(xs, encs)])
    q_s = np.stack([R.quantize_per_tensor(x, e[0], e[1], int(e[2]), True) for x, e in zip(xs, encs)])
    fei = np.array([R.fill_encoding_info(int(e[2]), e[0], e[1]).as_tuple() for e in encs])

    gce_in, gce_out = [], []
    for _ in range(200):
        mn, mx = rng.uniform(-50, 50, 2)
        if rng.uniform() < 0.2:
            mn = 0.0
        if rng.uniform() < 0.1:
            mx = np.inf
        if rng.uniform() < 0.1:
            mn = -np.inf
        bw = int(rng.choice([4, 8, 16, 32]))
        for sym, strict, un in [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 1)]:
            gce_in.append((bw, mn, mx, sym, strict, un))
            gce_out.append(R.get_computed_encodings(bw, mn, mx, sym, strict, un).as_tuple())

    pc = per_channel_cases(rng)
    core = dict(pt_x=xs, pt_enc=encs, pt_qdq=qdq, pt_q_unsigned=q_u, pt_q_signed=q_s, pt_fill=fei,
                gce_in=np.array(gce_in, dtype=np.float64), gce_out=np.array(gce_out, dtype=np.float64))
    for i, c in enumerate(pc):
        for k, v in c.items():
            core["pc%d_%s" % (i, k)] = np.asarray(v)
    core["pc_count"] = np.array(len(pc))
    np.savez_compressed(os.path.join(HERE, "golden_core.npz"), **core)

    # ---- analyzers (TF, TF-E, percentile, MSE) ------------------------------------------
    an = {}
    cases = analyzer_cases(rng)
    for i, c in enumerate(cases):
        an["a%d_scheme" % i] = np.array(c["scheme"])
        an["a%d_percentile" % i] = np.array(c["percentile"], dtype=np.float32)
        an["a%d_nb" % i] = np.array(len(c["batches"]))
        for k, b in enumerate(c["batches"]):
            an["a%d_b%d" % (i, k)] = b
        an["a%d_xleft" % i] = c["xleft"]
        an["a%d_pdf" % i] = c["pdf"]
        keys = sorted(c["encs"])
        an["a%d_enc_keys" % i] = np.array(keys)
        an["a%d_enc_vals" % i] = np.array([c["encs"][k] for k in keys], dtype=np.float64)
    an["count"] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, "golden_analyzers.npz"), **an)

    # ---- KATs from the reference test-suites ----------------------------------------------
    kdata = tfe_kat_data()
    a = R.Analyzer(1)
    a.update(kdata)
    kenc = a.compute(8, False, False, False)
    kqdq = R.qdq_per_tensor(np.full(4, 5.0, np.float32), kenc.min, kenc.max, 8)[0]

    ste, AdaroundLoss, AdaroundHyperParameters = reference_python()
    g = torch.Generator().manual_seed(3)
    sx = torch.randn(6, 5, generator=g) * 2
    sg = torch.randn(6, 5, generator=g)
    mins = torch.tensor([-1.0, -0.5, -2.0, -1.5, 0.0, -0.25]).tolist()
    maxs = torch.tensor([1.0, 0.5, 2.0, 0.75, 1.0, 3.0]).tolist()
    ste_pc = ste.compute_dloss_by_dx(sx, sg, mins, maxs, ch_axis=0)
    ste_pt = ste.compute_dloss_by_dx(sx, sg, -1.25, 0.8, ch_axis=0)
    np.savez_compressed(os.path.join(HERE, "golden_torch.npz"), ste_x=sx.numpy(), ste_g=sg.numpy(),
                        ste_mins=np.array(mins, np.float32), ste_maxs=np.array(maxs, np.float32),
                        ste_pc=ste_pc.numpy(), ste_pt=ste_pt.numpy(), tfe_kat_x=kdata)

    # learned-grid forward/backward straight from the reference module (float32)
    from types import SimpleNamespace
    lg = {}
    cases = [((4, 6, 5, 5), 1, 8, False), ((4, 6, 5, 5), 1, 8, True), ((8, 16, 3, 3), 8, 4, True),
             ((16, 8, 3, 3), 16, 8, False), ((300,), 1, 8, False)]
    gl = torch.Generator().manual_seed(9)
    for i, (shape, C, bw, sym) in enumerate(cases):
        x = torch.randn(shape, generator=gl) * 1.5
        grad = torch.randn(shape, generator=gl)
        if C == 1:
            emin = torch.tensor([-2.0]) if not sym else torch.tensor([-2.5])
            emax = torch.tensor([2.5])
        else:
            emax = torch.rand(C, generator=gl) + 0.5
            emin = -emax if sym else -(torch.rand(C, generator=gl) + 0.3)
        emin = emin.clone().requires_grad_(True)
        emax = emax.clone().requires_grad_(True)
        tq = SimpleNamespace(bitwidth=bw, use_symmetric_encodings=sym, is_unsigned_symmetric=False,
                             use_strict_symmetric=False, channel_axis=0)
        y, ir = ste.calculate_forward_pass(x, tq, emin, emax)
        gmin, gmax = ste.calculate_gradients(x, grad, ir, 0)
        lg["c%d_x" % i], lg["c%d_grad" % i] = x.numpy(), grad.numpy()
        lg["c%d_emin" % i], lg["c%d_emax" % i] = emin.detach().numpy(), emax.detach().numpy()
        lg["c%d_cfg" % i] = np.array([bw, int(sym)])
        lg["c%d_y" % i], lg["c%d_gx" % i] = y.detach().numpy(), (ir.mask_tensor * grad).numpy()
        lg["c%d_gmin" % i], lg["c%d_gmax" % i] = gmin.detach().numpy(), gmax.detach().numpy()
    lg["count"] = np.array(len(cases))
    np.savez_compressed(os.path.join(HERE, "golden_lg.npz"), **lg)

    np.random.seed(0)
    alpha = torch.from_numpy(np.random.rand(1, 3, 12, 12))
    hp = AdaroundHyperParameters(num_iterations=10000, reg_param=0.01, beta_range=(20, 2), warm_start=0.2)
    rl = float(AdaroundLoss.compute_round_loss(alpha, hp, 8000))
    beta = float(AdaroundLoss._compute_beta(10000, 8000, (20, 2), 0.2))

    kat = {
        "_sources": "values quoted from the reference test-suites (file:line per entry) plus the reference "
                    "C++/Python re-run in the build container (make_golden.py)",
        "qdq_sanity": {"src": "DlQuantization/test/TestTensorQuantizationSim.cpp:51-75",
                       "x": [-0.5, -0.25, 0.0, 0.25, 0.5, 0.75], "min": -0.46, "max": 0.72, "bw": 8,
                       "expected": [-0.45811754, -0.2498823, 0.0, 0.2498823, 0.49976459, 0.72188222],
                       "tol": "EXPECT_FLOAT_EQ (4 ulp)"},
        "qdq_gated_min": {"src": "TestTensorQuantizationSim.cpp:77-104", "x": [-0.5, -0.25, 0.0, 0.25, 0.5, 0.75],
                          "min": 0.5, "max": 1.0, "bw": 8,
                          "expected": [0.0, 0.0, 0.0, 0.25098041, 0.49803925, 0.74901962]},
        "qdq_gated_equal": {"src": "TestTensorQuantizationSim.cpp:106-132",
                            "x": [-0.5, -0.25, 0.0, 0.25, 0.5, 0.75], "min": 0.5, "max": 0.5, "bw": 8,
                            "expected": [0.0, 0.0, 0.0, 0.24901962, 0.5, 0.5]},
        "qdq_gated_max": {"src": "TestTensorQuantizationSim.cpp:134-159", "x": [-0.5, -0.25, 0.0, 0.25, 0.5, 0.75],
                          "min": -0.5, "max": -0.1, "bw": 8,
                          "expected": [-0.5, -0.24901962, 0.0, 0.0, 0.0, 0.0]},
        "quantize_unsigned": {"src": "TestTensorQuantizationSim.cpp:161-185",
                              "x": [-0.5, -0.25, 0.0, 0.25, 0.5, 0.75], "min": -0.46, "max": 0.72, "bw": 8,
                              "shift": False, "expected": [0, 45, 99, 153, 207, 255]},
        "quantize_signed": {"src": "TestTensorQuantizationSim.cpp:212-236",
                            "x": [-0.5, -0.25, 0.0, 0.25, 0.5, 0.75], "min": -0.46, "max": 0.72, "bw": 8,
                            "shift": True, "expected": [-128, -83, -29, 25, 79, 127]},
        "tfe_normal": {"src": "DlQuantization/test/TestTensorQuantizer.cpp:89-134 (data: golden_torch.npz tfe_kat_x)",
                       "expected_min": -6.52711, "expected_max": 8.88412, "expected_qdq5": 5.0162, "tol": 0.001,
                       "ref_encoding": list(kenc.as_tuple()), "ref_qdq5": float(kqdq)},
        "tfe_all_zero": {"src": "DlQuantization/test/TestTfEnhancedEncodingAnalyzer.cpp:176-196",
                         "n": 6000, "expected_min": -1.00392, "expected_max": 0.996078, "expected_offset": -128,
                         "tol": 0.0001},
        "per_channel_symmetric": {
            "src": "TrainingExtensions/torch/test/python/test_per_channel_quantization.py:66-102",
            "encodings": [[-3.84, 3.81, 0.03, -128, 8]] * 3 + [[-6.4, 6.35, 0.05, -128, 8]],
            "x": [[-7, -5, -3, 0, .1, 2.5]] * 4,
            "expected": [[-3.84, -3.84, -3, 0, .089999996, 2.49]] * 3 + [[-6.4, -5, -3, 0, .1, 2.5]],
            "atol": 1e-5},
        "per_channel_asymmetric": {
            "src": "TrainingExtensions/torch/test/python/test_per_channel_quantization.py:104-141",
            "encodings": [[-2.9999934, 1.9999956, 0.0196078, -153, 8]] * 3 + [[-5.995262, 2.404693, 0.032941, -182, 8]],
            "x": [[-7, -5, -3, 0, .1, 2.5]] * 4,
            "expected": [[-3.0, -3.0, -3.0, 0, .098, 2.0]] * 3 + [[-5.9953, -5.0070, -2.9976, 0, .09888, 2.4047]],
            "atol": 1e-4},
        "adaround_round_loss": {"src": "TrainingExtensions/torch/test/python/test_adaround_loss.py:83-100",
                                "seed": 0, "shape": [1, 3, 12, 12], "reg_param": 0.01, "beta_range": [20, 2],
                                "warm_start": 0.2, "num_iterations": 10000, "cur_iter": 8000,
                                "expected": 4.266156963161077, "places": 5, "ref_value": rl},
        "adaround_beta": {"src": "TrainingExtensions/torch/test/python/test_adaround_loss.py:102-110",
                          "expected": 4.636038969321072, "ref_value": beta},
    }
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    adaround_golden()
    ste16_golden()
    encodings_golden()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "encodings":
        encodings_golden()
    else:
        main()
