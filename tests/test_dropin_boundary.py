"""Drop-in fidelity at the torch boundary:

* CPU tensors -- the reference's ``AimetTensorQuantizer(..., use_cuda=False)`` / COMP_MODE_CPU and a
  QuantizationSimModel of a CPU model (config 1, "aimet_torch CPU path") -- are staged through HBM
  and computed by the same HIP kernels; results come back as CPU tensors and equal the oracle.
* ``torch.nn.DataParallel`` replicas (v1/qc_quantize_op.py:257-269, 785-796;
  Docs/api_docs/torch_multi_gpu.rst): a replica quantizes its broadcast parameters
  (``_former_parameters``) on its own device and thread.
* The per-channel table / STE-bound caches notice an encoding list whose element was replaced by an
  older TfEncoding.

Without a GPU only the loud failure is checked: a CPU tensor needs a HIP device to be staged to."""
import numpy as np
import pytest
import torch
from torch import nn

from conftest import bits, gpu_available
from oracle import oracle as O

from aimet_amd.libpymo import QuantizationMode, RoundingMode, TfEncoding
from aimet_amd.qc_quantize_op import StaticGridQuantWrapper
from aimet_amd.quantsim import QuantizationSimModel
from aimet_amd.tensor_quantizer import AimetTensorQuantizer, PerChannelTable

PER_CHANNEL_CFG = {"defaults": {"ops": {"is_output_quantized": "True"},
                                "params": {"is_quantized": "True", "is_symmetric": "True"},
                                "strict_symmetric": "False", "per_channel_quantization": "True"}}
gpu = pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")


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


def _calib(seed, n=2, dev="cpu"):
    g = torch.Generator().manual_seed(seed)
    return [torch.rand(4, 3, 16, 16, generator=g).to(dev) for _ in range(n)]


# ------------------------------------------------------------------------------------------
# CPU
# ------------------------------------------------------------------------------------------
@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure")
def test_cpu_tensor_without_a_gpu_fails_loudly():
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
    with pytest.raises(RuntimeError, match="no HIP device"):
        q.updateStats(torch.randn(16), False)
    e = TfEncoding()
    e.min, e.max, e.bw = -1.0, 1.0, 8
    with pytest.raises(RuntimeError, match="no HIP device"):
        q.quantizeDequantize(torch.randn(16), e, RoundingMode.ROUND_NEAREST, False)


def test_per_channel_table_key_sees_replaced_elements():
    a, b, c = TfEncoding(), TfEncoding(), TfEncoding()   # c is older than the list change below
    encs = [a, b]
    k0 = PerChannelTable.key(encs)
    assert PerChannelTable.key(encs) == k0
    encs[1] = c                                          # list __setitem__ bumps no version
    assert PerChannelTable.key(encs) != k0
    k1 = PerChannelTable.key(encs)
    c.max = 2.0
    assert PerChannelTable.key(encs) != k1


# ------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------
@pytest.mark.gpu
@gpu
def test_tensor_quantizer_use_cuda_false_stages_through_hbm():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal((8, 16, 9, 9)) * 1.3).astype(np.float32)
    xt = torch.from_numpy(x)
    for scheme in (QuantizationMode.QUANTIZATION_TF, QuantizationMode.QUANTIZATION_TF_ENHANCED):
        q = AimetTensorQuantizer(scheme)
        q.updateStats(xt, False)
        enc, valid = q.getEncoding(8, False, False, False)
        o = O.Analyzer(int(scheme))
        o.update(x.ravel())
        assert valid and enc.to_tuple() == o.compute(8).as_tuple()
        y = q.quantizeDequantize(xt, enc, RoundingMode.ROUND_NEAREST, False)
        assert y.device.type == "cpu"
        np.testing.assert_array_equal(bits(y.numpy().ravel()), bits(O.qdq_per_tensor(x.ravel(), enc.min, enc.max, 8)))
    # per channel
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF, num_channels=8)
    q.updateStatsPerChannel(xt, 0, False)
    encs, valid = q.getEncoding(8, True, False, False)
    K = x[0].size
    for c in (0, 5):
        o = O.Analyzer(O.QUANTIZATION_TF)
        o.update(x[c].ravel())
        assert encs[c].to_tuple() == o.compute(8, True).as_tuple()
    y = q.quantizeDequantizePerChannel(xt, encs, 8, x.size, K, RoundingMode.ROUND_NEAREST, False)
    assert y.device.type == "cpu"
    table = O.per_channel_table([e.to_tuple() for e in encs])
    np.testing.assert_array_equal(bits(y.numpy().ravel()), bits(O.qdq_per_channel(x.ravel(), 8, K, table)))


@pytest.mark.gpu
@gpu
def test_quantsim_on_a_cpu_model():
    """Config 1 plumbing: the model stays on the host; every statistic and QDQ runs on the device;
    encodings equal the oracle fed the CPU model's own layer outputs; a QAT step's gradients
    come back on the host."""
    sim = QuantizationSimModel(make_net(), quant_scheme="tf_enhanced", config_file=PER_CHANNEL_CFG)
    raw = {}
    hooks = [w._module_to_wrap.register_forward_hook(
        lambda mod, i, o, n=n: raw.setdefault(n, []).append(o.detach().clone())) for n, w in sim.quant_wrappers()]
    sim.compute_encodings(lambda m, d: [m(x) for x in d], _calib(1))
    for h in hooks:
        h.remove()
    for n, w in sim.quant_wrappers():
        a = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
        for t in raw[n]:
            assert t.device.type == "cpu"
            a.update(t.numpy().ravel())
        e = w.output_quantizers[0].encoding
        assert e.to_tuple() == a.compute(8).as_tuple(), n
    x = _calib(2, 1)[0].requires_grad_(True)
    sim.model.train()
    y = sim(x)
    assert y.device.type == "cpu"
    y.square().mean().backward()
    assert sim.model.conv1._module_to_wrap.weight.grad.device.type == "cpu"
    assert x.grad is not None and torch.isfinite(x.grad).all()


@pytest.mark.gpu
@gpu
def test_learned_grid_on_cpu_tensors_equals_device():
    from aimet_amd.learned_grid import LearnedGridQuantizeDequantize
    g = torch.Generator().manual_seed(3)
    x = torch.randn(16, 33, generator=g)
    emin = torch.full((16,), -1.1, requires_grad=True)
    emax = torch.full((16,), 1.3, requires_grad=True)
    y = LearnedGridQuantizeDequantize.apply(x.requires_grad_(True), emin, emax, 4, False, False, False, 0)
    assert y.device.type == "cpu"
    y.sum().backward()
    xd = x.detach().cuda().requires_grad_(True)
    emind = emin.detach().cuda().requires_grad_(True)
    emaxd = emax.detach().cuda().requires_grad_(True)
    yd = LearnedGridQuantizeDequantize.apply(xd, emind, emaxd, 4, False, False, False, 0)
    yd.sum().backward()
    torch.testing.assert_close(y, yd.cpu(), rtol=0, atol=0)
    torch.testing.assert_close(x.grad, xd.grad.cpu(), rtol=0, atol=0)
    torch.testing.assert_close(emin.grad, emind.grad.cpu(), rtol=0, atol=0)
    torch.testing.assert_close(emax.grad, emaxd.grad.cpu(), rtol=0, atol=0)


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("train", [False, True])
def test_dataparallel_replicas(train):
    """torch.nn.parallel.replicate + parallel_apply (what nn.DataParallel runs) over two replicas
    (both on cuda:0 on a one-GPU box; the code path is the multi-device one: replicas hold broadcast
    parameters outside _parameters, share their quantizers and run in one thread each)."""
    from torch.nn.parallel import parallel_apply, replicate
    sim = QuantizationSimModel(make_net().cuda(), quant_scheme="tf_enhanced", config_file=PER_CHANNEL_CFG)
    sim.compute_encodings(lambda m, d: [m(x) for x in d], _calib(4, dev="cuda"))
    sim.model.train(train)
    xs = _calib(5, 2, dev="cuda")
    with torch.no_grad():
        want = [sim(x) for x in xs]
    reps = replicate(sim.model, [0, 0], detach=True)
    for r in reps:
        wr = r.conv1
        assert isinstance(wr, StaticGridQuantWrapper) and wr._is_replica
        assert [n for n, _ in wr.get_named_parameters()] == ["weight", "bias"]
    with torch.no_grad():
        got = parallel_apply(reps, [(x,) for x in xs], devices=[0, 0])
    for g, w in zip(got, want):
        torch.testing.assert_close(g, w, rtol=0, atol=0)
    # the replicas' weights were quantized (not the raw fp32 weights)
    with torch.no_grad():
        plain = make_net().cuda()
        plain.load_state_dict({k.replace("._module_to_wrap", ""): v for k, v in sim.model.state_dict().items()})
        assert not torch.equal(plain(xs[0]), want[0])
