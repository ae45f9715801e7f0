"""Range learning through QuantizationSimModel (SURVEY §8 a14 at the caller level, config 5):
``training_range_learning_with_tf_init`` / ``_tf_enhanced_init`` calibrate with static-grid
wrappers, then swap in LearnedGridQuantWrapper (v1/quantsim.py:423, 764-846;
v1/qc_quantize_op.py:947-1198) whose ranges are trainable parameters.

CPU tests: the swap, parameter names, the reference's encoding conversions
(initialize_learned_grid_quantizer_attributes, v1/tensor_quantizer.py:1285-1344), the computed /
effective encodings (v1/tensor_quantizer.py:642-819), gating (:1347-1359) and export -- all torch
CPU arithmetic on the range parameters, no kernel.
GPU tests: a QAT step through QuantSim equals the op-level learned-grid path bit for bit, and its
forward equals the reference's torch-op restatement (oracle/torch_ref.py, pinned by golden_lg.npz)."""
import copy
import math

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from conftest import gpu_available
from oracle import torch_ref as T

from aimet_amd.learned_grid import LearnedGridQuantizeDequantize, LearnedGridTensorQuantizer
from aimet_amd.libpymo import TfEncoding
from aimet_amd.qc_quantize_op import LearnedGridQuantWrapper, StaticGridQuantWrapper
from aimet_amd.quantizers import QuantScheme
from aimet_amd.quantsim import QuantizationSimModel

PER_CHANNEL_CFG = {"defaults": {"ops": {"is_output_quantized": "True"},
                                "params": {"is_quantized": "True", "is_symmetric": "True"},
                                "strict_symmetric": "False", "per_channel_quantization": "True"}}
RL_TF = QuantScheme.training_range_learning_with_tf_init


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 8, 3, padding=1)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2d(8, 16, 3, stride=2, padding=1)
        self.fc = nn.Linear(16 * 8 * 8, 10)

    def forward(self, x):
        x = self.relu(self.conv1(x))
        x = self.relu(self.conv2(x))
        return self.fc(x.flatten(1))


def make_net(seed=0):
    torch.manual_seed(seed)
    return Net().eval()


def _enc(mn, mx, bw=8):
    e = TfEncoding()
    e.min, e.max, e.bw = mn, mx, bw
    e.delta = (mx - mn) / (2 ** bw - 1)
    e.offset = round(mn / e.delta) if e.delta else 0
    return e


def _calibrated_by_hand(sim):
    """Static encodings set directly (CPU: no statistics kernels), as compute_encodings would."""
    for _, w in sim.quant_wrappers():
        for q in list(w.input_quantizers) + list(w.output_quantizers):
            if q.enabled:
                q.encoding = _enc(-0.25, 3.5)
        pq = w.param_quantizers["weight"]
        if hasattr(pq, "_num_channels"):
            pq.encoding = [_enc(-0.1 - 0.01 * c, 0.1 + 0.01 * c, pq.bitwidth) for c in range(pq._num_channels)]
        else:
            pq.encoding = _enc(-0.1, 0.1, pq.bitwidth)


# ------------------------------------------------------------------------------------------
# CPU
# ------------------------------------------------------------------------------------------
def test_wrappers_calibrate_with_the_init_scheme():
    sim = QuantizationSimModel(make_net(), quant_scheme=RL_TF, config_file=PER_CHANNEL_CFG)
    for _, w in sim.quant_wrappers():
        assert isinstance(w, StaticGridQuantWrapper)
        assert w.output_quantizers[0].quant_scheme == QuantScheme.post_training_tf
    sim2 = QuantizationSimModel(make_net(), quant_scheme=QuantScheme.training_range_learning_with_tf_enhanced_init)
    assert sim2.model.conv1.output_quantizers[0].quant_scheme == QuantScheme.post_training_tf_enhanced


def test_swap_parameters_and_encodings():
    sim = QuantizationSimModel(make_net(), quant_scheme=RL_TF, config_file=PER_CHANNEL_CFG, default_param_bw=4)
    _calibrated_by_hand(sim)
    sim.replace_wrappers_for_quantize_dequantize()
    names = dict(sim.model.named_parameters())
    for layer in ("conv1", "conv2", "fc"):
        w = getattr(sim.model, layer)
        assert isinstance(w, LearnedGridQuantWrapper)
        for p in ("output0_encoding_min", "output0_encoding_max", "weight_encoding_min", "weight_encoding_max"):
            assert layer + "." + p in names and names[layer + "." + p].requires_grad
        assert w.bias_encoding_min is None                         # bias stays unquantized
        C = w._module_to_wrap.weight.shape[0]
        assert w.weight_encoding_min.shape == (C,)
        # symmetric weights learn a strictly symmetric range: min = -max (tensor_quantizer.py:1319-1325)
        torch.testing.assert_close(w.weight_encoding_min, -w.weight_encoding_max, rtol=0, atol=0)
        torch.testing.assert_close(w.weight_encoding_max,
                                   torch.tensor([0.1 + 0.01 * c for c in range(C)], dtype=torch.float32),
                                   rtol=0, atol=0)
    assert "conv1.input0_encoding_min" in names and sim.model.conv2.input0_encoding_min is None
    # an optimizer over the model trains the ranges
    opt = torch.optim.SGD(sim.model.parameters(), lr=0.1)
    assert sum(p.numel() for g in opt.param_groups for p in g["params"]) == \
        sum(p.numel() for p in sim.model.parameters())


def test_learned_encodings_follow_the_reference_arithmetic():
    """v1/tensor_quantizer.py:775-819 and :642-685, restated with the reference's torch ops."""
    sim = QuantizationSimModel(make_net(), quant_scheme=RL_TF, config_file=PER_CHANNEL_CFG, default_param_bw=4)
    _calibrated_by_hand(sim)
    sim.replace_wrappers_for_quantize_dequantize()
    w = sim.model.conv1
    with torch.no_grad():
        w.output0_encoding_min.fill_(-0.3)
        w.output0_encoding_max.fill_(2.9)
    # asymmetric: delta = (max-min)/steps, offset = -clamp(round(-min/delta)), min moved onto the grid
    q = w.output_quantizers[0]
    emin, emax = torch.tensor([-0.3]), torch.tensor([2.9])
    delta = (emax - emin) / torch.full_like(emin, 255.0)
    offset = -torch.clamp(torch.round(-emin / delta), 0.0, 255.0)
    adj_min = delta * offset
    e = q.encoding
    assert (e.min, e.max, e.delta, e.offset, e.bw) == (float(adj_min), float(emax - emin + adj_min), float(delta),
                                                       float(offset), 8)
    assert q.get_effective_encoding() == e
    # non-strict symmetric: the exported min carries one more bin
    pq = w.param_quantizers["weight"]
    encs, eff = pq.encoding, pq.get_effective_encoding()
    for c, (a, b) in enumerate(zip(encs, eff)):
        mx = torch.tensor([0.1 + 0.01 * c], dtype=torch.float32)
        d = mx / torch.full_like(mx, math.floor(15 / 2))
        assert (a.min, a.max, a.delta, a.offset) == (float(-mx), float(mx), float(d), -8.0)
        assert (b.min, b.max, b.delta) == (a.min - a.delta, a.max, a.delta)
    d = sim.get_encodings_dict()
    assert d["param_encodings"]["conv1.weight"][0]["min"] == eff[0].min
    assert d["activation_encodings"]["conv1"]["output"]["0"]["offset"] == int(e.offset)


def test_gating_keeps_ranges_ordered_around_zero():
    sim = QuantizationSimModel(make_net(), quant_scheme=RL_TF)
    _calibrated_by_hand(sim)
    sim.replace_wrappers_for_quantize_dequantize()
    w = sim.model.fc
    with torch.no_grad():
        w.output0_encoding_min.fill_(0.5)     # min > 0
        w.output0_encoding_max.fill_(-0.2)    # max < 0
    w.apply_gating_logic()
    assert float(w.output0_encoding_min.detach()) == 0.0
    assert float(w.output0_encoding_max.detach()) == float(torch.tensor(0.0) + torch.tensor(1e-5))


def test_set_encoding_checks_and_freeze():
    sim = QuantizationSimModel(make_net(), quant_scheme=RL_TF)
    _calibrated_by_hand(sim)
    sim.replace_wrappers_for_quantize_dequantize()
    w = sim.model.conv2
    q = w.output_quantizers[0]
    assert isinstance(q, LearnedGridTensorQuantizer)
    with pytest.raises(RuntimeError, match="Bitwidth mismatched"):
        q.encoding = _enc(-1.0, 1.0, 4)
    q.encoding = _enc(-1.0, 1.0, 8)
    assert float(w.output0_encoding_min.detach()) == -1.0 and w.output0_encoding_min.requires_grad
    q.freeze_encoding()
    assert not w.output0_encoding_min.requires_grad and not w.output0_encoding_max.requires_grad
    with pytest.raises(RuntimeError, match="frozen"):
        q.encoding = _enc(-2.0, 2.0, 8)


def test_load_encodings_into_learned_wrappers():
    sim = QuantizationSimModel(make_net(), quant_scheme=RL_TF, config_file=PER_CHANNEL_CFG, default_param_bw=4)
    _calibrated_by_hand(sim)
    sim.replace_wrappers_for_quantize_dequantize()
    exported = sim.get_encodings_dict()
    sim2 = QuantizationSimModel(make_net(), quant_scheme=RL_TF, config_file=PER_CHANNEL_CFG, default_param_bw=4)
    _calibrated_by_hand(sim2)
    sim2.replace_wrappers_for_quantize_dequantize()
    with torch.no_grad():
        for p in sim2.model.parameters():
            p.add_(0.01)
    sim2.load_encodings(exported, strict=True, partial=True)
    assert sim2.model.conv1.weight_encoding_min.shape == sim.model.conv1.weight_encoding_min.shape
    got = sim2.get_encodings_dict()
    for k, v in exported["param_encodings"].items():
        assert [e["max"] for e in got["param_encodings"][k]] == [e["max"] for e in v], k


# ------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------
gpu = pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")


def _calib(seed, n=2, dev="cuda"):
    g = torch.Generator().manual_seed(seed)
    return [torch.rand(4, 3, 16, 16, generator=g).to(dev) for _ in range(n)]


def _op_level_forward(m, x):
    """The same network through LearnedGridQuantizeDequantize calls on model m's parameters
    (conv1's input quantizer on, bias unquantized, every output quantized)."""
    def lg(t, w, name, q):
        return LearnedGridQuantizeDequantize.apply(t, getattr(w, name + "_encoding_min"),
                                                   getattr(w, name + "_encoding_max"), q.bitwidth,
                                                   q.use_symmetric_encodings, q.use_strict_symmetric,
                                                   q.is_unsigned_symmetric, q.channel_axis)

    def layer(w, t, fn):
        if w.input_quantizers[0].enabled:
            t = lg(t, w, "input0", w.input_quantizers[0])
        m_ = w._module_to_wrap
        wq = lg(m_.weight, w, "weight", w.param_quantizers["weight"])
        return lg(fn(t, wq, m_), w, "output0", w.output_quantizers[0])

    t = layer(m.conv1, x, lambda t, wq, mm: F.conv2d(t, wq, mm.bias, padding=1))
    t = layer(m.conv2, F.relu(t), lambda t, wq, mm: F.conv2d(t, wq, mm.bias, stride=2, padding=1))
    return layer(m.fc, F.relu(t).flatten(1), lambda t, wq, mm: F.linear(t, wq, mm.bias))


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("scheme", [RL_TF, QuantScheme.training_range_learning_with_tf_enhanced_init])
def test_qat_step_through_quantsim_equals_op_level(scheme, monkeypatch):
    # MIOpen's weight-gradient convolutions may add partial sums atomically: pick deterministic ones
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    monkeypatch.setattr(torch.backends.cudnn, "benchmark", False)
    sim = QuantizationSimModel(make_net().cuda(), quant_scheme=scheme, config_file=PER_CHANNEL_CFG,
                               default_param_bw=4, default_output_bw=8)
    sim.compute_encodings(lambda m, d: [m(x) for x in d], _calib(1))
    assert all(isinstance(w, LearnedGridQuantWrapper) for _, w in sim.quant_wrappers())
    ref_model = copy.deepcopy(sim.model)
    x = _calib(2, 1)[0]
    opt = torch.optim.SGD(sim.model.parameters(), lr=0.05)
    opt_ref = torch.optim.SGD(ref_model.parameters(), lr=0.05)
    for step in range(2):
        sim.model.train()
        loss = sim(x).square().mean()
        loss.backward()
        ref_model.train()
        for _, w in ref_model.named_modules():
            if isinstance(w, LearnedGridQuantWrapper):
                w.apply_gating_logic()
        loss_ref = _op_level_forward(ref_model, x).square().mean()
        loss_ref.backward()
        assert float(loss.detach()) == float(loss_ref.detach()), step
        got = dict(sim.model.named_parameters())
        for name, p in ref_model.named_parameters():
            assert got[name].grad is not None, name
            torch.testing.assert_close(got[name].grad, p.grad, rtol=0, atol=0, msg=name)
        opt.step()
        opt_ref.step()
        opt.zero_grad()
        opt_ref.zero_grad()


@pytest.mark.gpu
@gpu
def test_quantsim_forward_equals_reference_torch_ops():
    """Every quantized tensor of the QuantSim forward equals the reference's calculate_forward_pass
    (quantsim_straight_through_grad.py:191-249) restated in torch ops, bit for bit."""
    sim = QuantizationSimModel(make_net().cuda(), quant_scheme=RL_TF, config_file=PER_CHANNEL_CFG,
                               default_param_bw=4)
    sim.compute_encodings(lambda m, d: [m(x) for x in d], _calib(3))
    rec, outs = {}, {}

    def raw_hook(mod, i, o, n):   # a forward hook that returns a value replaces the output
        rec[n] = (i[0].detach().clone(), o.detach().clone(), mod.weight.detach().clone())

    def out_hook(mod, i, o, n):
        outs[n] = o.detach().clone()
    hooks = [w._module_to_wrap.register_forward_hook(lambda mod, i, o, n=n: raw_hook(mod, i, o, n))
             for n, w in sim.quant_wrappers()]
    hooks += [w.register_forward_hook(lambda mod, i, o, n=n: out_hook(mod, i, o, n)) for n, w in sim.quant_wrappers()]
    with torch.no_grad():
        sim(_calib(4, 1)[0])
    for h in hooks:
        h.remove()
    for n, w in sim.quant_wrappers():
        raw_in, raw_out, wq = rec[n]
        pq = w.param_quantizers["weight"]
        want_w = T.lg_forward(w._module_to_wrap.weight.detach(), w.weight_encoding_min.detach(),
                              w.weight_encoding_max.detach(), 4, True, False, False, pq.channel_axis)[0]
        torch.testing.assert_close(wq, want_w, rtol=0, atol=0, msg=n)
        want_o = T.lg_forward(raw_out, w.output0_encoding_min.detach(), w.output0_encoding_max.detach(), 8)[0]
        torch.testing.assert_close(outs[n], want_o, rtol=0, atol=0, msg=n)


class SharedNet(nn.Module):
    """One Linear called twice per forward (a reused module, as torchvision ResNet's shared relu)."""
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(32, 32)

    def forward(self, x):
        return self.fc(F.relu(self.fc(x)))


@pytest.mark.gpu
@gpu
def test_learned_grid_wrapper_called_twice_before_backward():
    """A LearnedGridQuantWrapper run twice before loss.backward(): its gate updates the range
    Parameters in place on every call, so the forward must save a copy of the range (the reference
    saves encoding_min/max.clone(), v1/tensor_quantizer.py:940-951) -- else backward fails with
    'modified by an inplace operation'. Gradients == the op-level path on the same parameters, and
    the output range's gradient == the sum of the reference's torch-op gradients of both calls
    (oracle/torch_ref.lg_gradients; rtol 1e-4: fp32 summation order)."""
    torch.manual_seed(5)
    sim = QuantizationSimModel(SharedNet().cuda().eval(), quant_scheme=RL_TF, dummy_input=torch.rand(8, 32).cuda())
    sim.compute_encodings(lambda m, d: [m(x) for x in d], [torch.randn(8, 32).cuda() for _ in range(2)])
    assert isinstance(sim.model.fc, LearnedGridQuantWrapper)
    ref = copy.deepcopy(sim.model)
    x = torch.randn(8, 32).cuda()
    sim.model.train()
    loss = sim(x).square().mean()
    loss.backward()                                    # raised before the saved range was a copy

    rw = ref.fc
    rw.apply_gating_logic()
    m = rw._module_to_wrap
    qi, qo, qw = rw.input_quantizers[0], rw.output_quantizers[0], rw.param_quantizers["weight"]
    calls = []   # (pre-quantization output, its quantized tensor) per call

    def lg(t, name, q):
        return LearnedGridQuantizeDequantize.apply(t, getattr(rw, name + "_encoding_min"),
                                                   getattr(rw, name + "_encoding_max"), q.bitwidth,
                                                   q.use_symmetric_encodings, q.use_strict_symmetric,
                                                   q.is_unsigned_symmetric, q.channel_axis)

    def call(t):
        if qi.enabled:
            t = lg(t, "input0", qi)
        out = F.linear(t, lg(m.weight, "weight", qw), m.bias)
        y = lg(out, "output0", qo)
        y.retain_grad()
        calls.append((out.detach(), y))
        return y
    loss_ref = call(F.relu(call(x))).square().mean()
    loss_ref.backward()
    assert float(loss.detach()) == float(loss_ref.detach())
    got = dict(sim.model.named_parameters())
    for name, p in ref.named_parameters():
        if p.grad is None:
            assert got[name].grad is None, name
        else:
            torch.testing.assert_close(got[name].grad, p.grad, rtol=0, atol=0, msg=name)
    emin, emax = rw.output0_encoding_min.detach(), rw.output0_encoding_max.detach()
    want_min, want_max = torch.zeros_like(emin), torch.zeros_like(emax)
    for out, y in calls:
        _, gmin, gmax = T.lg_gradients(out, y.grad, emin, emax, qo.bitwidth, qo.use_symmetric_encodings)
        want_min, want_max = want_min + gmin, want_max + gmax
    torch.testing.assert_close(got["fc.output0_encoding_min"].grad, want_min, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(got["fc.output0_encoding_max"].grad, want_max, rtol=1e-4, atol=1e-7)
