"""QuantizationSimModel / StaticGridQuantWrapper (the Python callers of the core, SURVEY §8 a16 and
§8(f) rank 2: encoding export / import).

CPU tests: wrapping, configuration and the encoding JSON contract (no kernel runs).
GPU tests: compute_encodings == the oracle's analyzers fed the same tensors (bit-exact), the ACTIVE
forward == oracle QDQ of every layer's output, export -> load round trip, STE-gated QAT step."""
import json

import numpy as np
import pytest
import torch
from torch import nn

from conftest import bits, gpu_available
from oracle import oracle as O

from aimet_amd.encodings_io import compute_partial_encoding, create_encoding_dict, create_encoding_from_dict
from aimet_amd.qc_quantize_op import QcQuantizeOpMode, StaticGridQuantWrapper
from aimet_amd.quantizers import QuantScheme, StaticGridPerChannelQuantizer
from aimet_amd.quantsim import QuantizationSimModel

PER_CHANNEL_CFG = {"defaults": {"ops": {"is_output_quantized": "True"},
                                "params": {"is_quantized": "True", "is_symmetric": "True"},
                                "strict_symmetric": "False", "per_channel_quantization": "True"}}


class SmallNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 8, 3, padding=1)
        self.bn = nn.BatchNorm2d(8)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2d(8, 16, 3, stride=2, padding=1)
        self.up = nn.ConvTranspose2d(16, 4, 2, stride=2)
        self.fc = nn.Linear(4 * 32 * 32, 10)

    def forward(self, x):
        x = self.relu(self.bn(self.conv1(x)))
        x = self.relu(self.conv2(x))
        x = self.up(x)
        return self.fc(x.flatten(1))


def make_net(seed=0):
    torch.manual_seed(seed)
    net = SmallNet()
    net.eval()
    return net


# ------------------------------------------------------------------------------------------
# CPU
# ------------------------------------------------------------------------------------------
def test_wrapping_and_config():
    sim = QuantizationSimModel(make_net(), quant_scheme="tf_enhanced", config_file=PER_CHANNEL_CFG)
    names = [n for n, _ in sim.quant_wrappers()]
    assert names == ["conv1", "conv2", "up", "fc"]
    conv1 = sim.model.conv1
    assert isinstance(conv1, StaticGridQuantWrapper)
    assert conv1.input_quantizers[0].enabled and not sim.model.conv2.input_quantizers[0].enabled
    assert not conv1.param_quantizers["bias"].enabled
    w = conv1.param_quantizers["weight"]
    assert isinstance(w, StaticGridPerChannelQuantizer) and w.use_symmetric_encodings and w.channel_axis == 0
    up = sim.model.up.param_quantizers["weight"]
    assert up.channel_axis == 1 and up._num_channels == 4        # ConvTranspose: axis 1
    assert not conv1.output_quantizers[0].use_symmetric_encodings
    assert conv1.weight is conv1._module_to_wrap.weight             # attribute passthrough


def test_encoding_dict_helpers():
    class Q:
        use_symmetric_encodings = True
        use_unsigned_symmetric = False
        use_strict_symmetric = False
        round_mode = 0
    d = compute_partial_encoding(Q(), {"bitwidth": 8, "min": -2.0, "max": 2.0, "dtype": "int", "is_symmetric": "True"})
    e = create_encoding_from_dict(d)
    ref = O.partial_encoding(8, O.Encoding(-2.0, 2.0, 0.0, 0.0, 8), sym=True)
    assert (e.min, e.max, e.delta, e.offset) == ref.as_tuple()[:4]

    class Q2(Q):
        data_type = None
        bitwidth = 8
    from aimet_amd.quantizers import QuantizationDataType
    Q2.data_type = QuantizationDataType.int
    out = create_encoding_dict(e, Q2(), False)
    assert out == {"min": e.min, "max": e.max, "scale": e.delta, "offset": int(e.offset), "bitwidth": 8,
                   "is_symmetric": "True", "dtype": "int"}
    with pytest.raises(AssertionError):
        create_encoding_from_dict({"bitwidth": 8, "min": 0, "max": 1, "scale": 1, "offset": 0, "is_symmetric": "x"})


def test_load_encodings_cpu_roundtrip(tmp_path):
    """Hand-written (partly partial) encodings load into the quantizers and export back unchanged."""
    sim = QuantizationSimModel(make_net(), quant_scheme="tf_enhanced")
    enc = {"activation_encodings": {
        "conv1": {"input": {"0": {"bitwidth": 8, "dtype": "int", "is_symmetric": "False", "min": -1.0, "max": 1.0,
                                  "offset": -128, "scale": 2.0 / 255}},
                  "output": {"0": {"bitwidth": 8, "dtype": "int", "is_symmetric": "False", "min": 0.0, "max": 6.0}}}},
        "param_encodings": {"conv2.weight": [{"bitwidth": 4, "dtype": "int", "is_symmetric": "True",
                                              "min": -0.5, "max": 0.5}]}}
    sim.load_encodings(enc, strict=True, partial=True)
    q_out = sim.model.conv1.output_quantizers[0]
    ref = O.partial_encoding(8, O.Encoding(0.0, 6.0, 0.0, 0.0, 8))
    assert (q_out.encoding.min, q_out.encoding.max, q_out.encoding.delta, q_out.encoding.offset) == ref.as_tuple()[:4]
    pq = sim.model.conv2.param_quantizers["weight"]
    assert pq.bitwidth == 4 and pq.encoding.bw == 4
    d = sim.get_encodings_dict()
    assert d["activation_encodings"]["conv1"]["input"]["0"]["offset"] == -128
    assert d["param_encodings"]["conv2.weight"][0]["is_symmetric"] == "True"
    json.dumps(d)
    with pytest.raises(RuntimeError):
        sim.load_encodings({"param_encodings": {"nope.weight": [{}]}, "activation_encodings": {}}, strict=True)


# ------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------
gpu = pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")


def _calib(seed, n=2):
    g = torch.Generator().manual_seed(seed)
    return [torch.rand(4, 3, 32, 32, generator=g).cuda() for _ in range(n)]


def _record(model):
    """inputs / outputs of every wrapped module, in call order, per module name."""
    rec = {}
    hooks = []
    for name, m in model.named_modules():
        if isinstance(m, StaticGridQuantWrapper):
            hooks.append(m.register_forward_hook(
                lambda mod, i, o, name=name: rec.setdefault(name, []).append(
                    (i[0].detach().clone(), o.detach().clone()))))
            # the wrapped layer's own output (before the output quantizer)
            hooks.append(m._module_to_wrap.register_forward_hook(
                lambda mod, i, o, name=name: rec.setdefault(name + ".raw", []).append(
                    (i[0].detach().clone(), o.detach().clone()))))
    return rec, hooks


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("scheme", ["tf_enhanced", "tf"])
def test_compute_encodings_bit_exact_vs_oracle(scheme):
    net = make_net().cuda()
    sim = QuantizationSimModel(net, quant_scheme=scheme, config_file=PER_CHANNEL_CFG)
    batches = _calib(1)
    rec, hooks = _record(sim.model)

    def fwd(model, data):
        for x in data:
            model(x)
    sim.compute_encodings(fwd, batches)
    for h in hooks:
        h.remove()
    mode = O.QUANTIZATION_TF_ENHANCED if scheme == "tf_enhanced" else O.QUANTIZATION_TF
    for name, w in sim.quant_wrappers():
        # output quantizer: analyzer fed the wrapped layer's raw output of every calibration batch
        a = O.Analyzer(mode)
        for _, out in rec[name + ".raw"]:
            a.update(out.cpu().numpy().ravel())
        got = w.output_quantizers[0].encoding
        assert (got.min, got.max, got.delta, got.offset, got.bw) == a.compute(8).as_tuple(), name
        if name == "conv1":
            a = O.Analyzer(mode)
            for inp, _ in rec[name]:
                a.update(inp.cpu().numpy().ravel())
            gi = w.input_quantizers[0].encoding
            assert (gi.min, gi.max, gi.delta, gi.offset, gi.bw) == a.compute(8).as_tuple()
        # weight quantizer: per-channel, symmetric (computed from the weights themselves)
        pq = w.param_quantizers["weight"]
        wt = w._module_to_wrap.weight.detach().cpu().numpy()
        for c, e in enumerate(pq.encoding):
            a = O.Analyzer(mode)
            a.update(np.ascontiguousarray(np.take(wt, c, axis=pq.channel_axis)).ravel())
            assert (e.min, e.max, e.delta, e.offset, e.bw) == a.compute(8, True, False, False).as_tuple(), (name, c)


@pytest.mark.gpu
@gpu
def test_active_forward_equals_oracle_qdq_per_layer(tmp_path):
    net = make_net().cuda()
    sim = QuantizationSimModel(net, quant_scheme="tf_enhanced", config_file=PER_CHANNEL_CFG)
    sim.compute_encodings(lambda m, d: [m(x) for x in d], _calib(2))
    x = _calib(3, 1)[0]
    rec, hooks = _record(sim.model)
    with torch.no_grad():
        y = sim(x)
    for h in hooks:
        h.remove()
    for name, w in sim.quant_wrappers():
        (qin, qout), = rec[name]
        (raw_in, raw_out), = rec[name + ".raw"]
        e = w.output_quantizers[0].encoding
        want = O.qdq_per_tensor(raw_out.cpu().numpy().ravel(), e.min, e.max, 8)
        np.testing.assert_array_equal(bits(qout.cpu().numpy().ravel()), bits(want), err_msg=name)
        if name == "conv1":
            ei = w.input_quantizers[0].encoding
            want_in = O.qdq_per_tensor(x.cpu().numpy().ravel(), ei.min, ei.max, 8)
            np.testing.assert_array_equal(bits(raw_in.cpu().numpy().ravel()), bits(want_in))
        # the wrapped layer ran with QDQ'd weights, and the fp32 weights are restored afterwards
        pq = w.param_quantizers["weight"]
        wt = w._module_to_wrap.weight.detach()
        shape = wt.shape
        ax = pq.channel_axis
        perm = wt.movedim(ax, 0).contiguous() if ax else wt
        table = O.per_channel_table([e.to_tuple() for e in pq.encoding])
        C = shape[ax]
        wq = O.qdq_per_channel(perm.cpu().numpy().ravel(), C, perm[0].numel(), table).reshape(perm.shape)
        wq = torch.from_numpy(wq).cuda()
        wq = wq.movedim(0, ax).contiguous() if ax else wq
        orig = w._module_to_wrap.weight.data
        w._module_to_wrap.weight.data = wq
        with torch.no_grad():
            ref = w._module_to_wrap(raw_in)
        w._module_to_wrap.weight.data = orig
        torch.testing.assert_close(raw_out, ref, rtol=0, atol=0)
    assert y.shape == (1 * 4, 10)

    # export -> load into a fresh sim: identical encodings and identical output
    path = sim.export(str(tmp_path), "small")
    sim2 = QuantizationSimModel(make_net().cuda(), quant_scheme="tf_enhanced", config_file=PER_CHANNEL_CFG)
    sim2.load_encodings(path, strict=True, partial=False)
    assert sim2.get_encodings_dict() == json.loads(json.dumps(sim.get_encodings_dict()))
    with torch.no_grad():
        y2 = sim2(x)
    torch.testing.assert_close(y2, y, rtol=0, atol=0)


@pytest.mark.gpu
@gpu
def test_qat_step_gates_parameter_gradients():
    net = make_net().cuda()
    sim = QuantizationSimModel(net, quant_scheme="tf_enhanced", config_file=PER_CHANNEL_CFG)
    sim.compute_encodings(lambda m, d: [m(x) for x in d], _calib(4))
    sim.model.train()
    # SteGatingFuncForParameters runs in the backward of the wrapper inputs (as in the reference),
    # so the first layer's gating needs an input that requires grad
    x = _calib(5, 1)[0].requires_grad_(True)
    loss = sim(x).square().mean()
    loss.backward()
    for name, w in sim.quant_wrappers():
        wt = w._module_to_wrap.weight
        g = wt.grad
        assert g is not None and torch.isfinite(g).all()
        pq = w.param_quantizers["weight"]
        shape = [1] * wt.dim()
        shape[pq.channel_axis] = -1
        mins = torch.tensor([e.min for e in pq.encoding], dtype=torch.float32, device="cuda").view(shape)
        maxs = torch.tensor([e.max for e in pq.encoding], dtype=torch.float32, device="cuda").view(shape)
        outside = (wt.detach() < mins) | (wt.detach() > maxs)
        assert (g[outside] == 0).all(), name


class BranchNet(nn.Module):
    """Two layers the forward runs -- the first twice per forward, so its quantizers see two tensors
    per batch, and its first output is then overwritten in place (as nn.ReLU(inplace=True) and
    `out += identity` do in torchvision's ResNet) -- and one it never calls."""

    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(64, 32)
        self.fc2 = nn.Linear(32, 10)
        self.unused = nn.Linear(64, 10)

    def forward(self, x):
        a = self.fc1(x)
        a.relu_()
        b = self.fc1(x * 0.5)
        b += a
        return self.fc2(b)


def _quantizer_state(sim):
    out = {}
    for name, w in sim.quant_wrappers():
        for kind, qs in (("in", list(w.input_quantizers)), ("out", list(w.output_quantizers)),
                         ("param", [w.param_quantizers[k] for k in sorted(w.param_quantizers)])):
            for i, q in enumerate(qs):
                enc = q.encoding
                encs = enc if isinstance(enc, list) else ([] if enc is None else [enc])
                pct = q._op().getPercentileValue() if q.quant_scheme == QuantScheme.post_training_percentile else None
                out[(name, kind, i)] = (bool(q.enabled), [(e.min, e.max, e.delta, e.offset, e.bw) for e in encs], pct)
    return out


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("scheme", ["tf_enhanced", "tf", "percentile"])
@pytest.mark.parametrize("per_channel", [False, True])
def test_compute_encodings_precomputed_parameter_encodings_equal_per_wrapper(monkeypatch, scheme, per_channel):
    """compute_encodings computes the executed wrappers' parameter encodings up front in batched
    calls (quantsim._precompute_param_encodings) instead of one at a time inside the first ANALYSIS
    forward, and launches each forward's activation statistics together (qc_quantize_op.StatsBatch)
    instead of one update per quantizer: every quantizer of the sim -- parameters, inputs, outputs,
    enabled flags -- ends as with the per-wrapper, per-call computation, a layer run twice per
    forward and a wrapper no forward runs included (no encoding and its percentile as before, as
    the reference leaves it), over two calibrations of the same sim."""
    import aimet_amd.qc_quantize_op as QO
    import aimet_amd.quantsim as QS
    data = [torch.randn(16, 64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(i))
            for i in range(2)]

    def run(precompute):
        torch.manual_seed(3)
        net = BranchNet().cuda().eval()
        sim = QuantizationSimModel(net, torch.randn(1, 64, device="cuda"), quant_scheme=scheme,
                                   config_file=PER_CHANNEL_CFG if per_channel else None)
        if scheme == "percentile":
            sim.set_percentile_value(99.9)
        if not precompute:
            monkeypatch.setattr(QS, "_precompute_param_encodings", lambda wrappers: [])
            monkeypatch.setattr(QO.StatsBatch, "eligible", staticmethod(lambda q, t: False))
        states = []
        for _ in range(2):
            sim.compute_encodings(lambda m, d: [m(x) for x in d], data)
            states.append(_quantizer_state(sim))
        monkeypatch.undo()
        return states

    per_wrapper = run(False)
    batched = run(True)
    assert batched == per_wrapper
    assert per_wrapper[0][("unused", "param", sorted(["weight", "bias"]).index("weight"))][1] == []
