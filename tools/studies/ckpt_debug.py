"""Round 4 debug: where a deep-copied / reloaded QuantizationSimModel first differs from the original."""
import copy
import pickle
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from tests.test_checkpoint import PER_CHANNEL_CFG, _Net  # noqa: E402
from aimet_amd.qc_quantize_op import StaticGridQuantWrapper  # noqa: E402
from aimet_amd.quantizers import QuantScheme  # noqa: E402
from aimet_amd.quantsim import QuantizationSimModel  # noqa: E402
from workloads.resnet import resnet50  # noqa: E402


def bits(t):
    return t.detach().contiguous().view(torch.int32)


def record(model):
    rec, hooks = {}, []
    for n, m in model.named_modules():
        if isinstance(m, StaticGridQuantWrapper):
            hooks.append(m.register_forward_hook(lambda mod, i, o, n=n: rec.__setitem__(n, (i[0].clone(), o.clone()))))
    return rec, hooks


dev = torch.device("cuda", 0)
images = torch.rand(8, 3, 224, 224, generator=torch.Generator().manual_seed(1234)).to(dev)
sim = QuantizationSimModel(resnet50(seed=0, device=dev), images[:1], quant_scheme="tf_enhanced",
                           config_file=PER_CHANNEL_CFG)
sim.compute_encodings(lambda m, _: m(images), None)
with torch.no_grad():
    r0, h0 = record(sim.model)
    y0 = sim.model(images)
    y0b = sim.model(images)
print("repeat equal", torch.equal(bits(y0), bits(y0b)))
for h in h0:
    h.remove()
cp = copy.deepcopy(sim.model)
pk = pickle.loads(pickle.dumps(sim.model))
for name, m in (("deepcopy", cp), ("pickle", pk)):
    r1, h1 = record(m)
    with torch.no_grad():
        y = m(images)
    for h in h1:
        h.remove()
    print(name, "equal", torch.equal(bits(y0), bits(y)))
    for n in r0:
        i0, o0 = r0[n]
        i1, o1 = r1[n]
        if not torch.equal(bits(i0), bits(i1)) or not torch.equal(bits(o0), bits(o1)):
            w0, w1 = dict(sim.model.named_modules())[n], dict(m.named_modules())[n]
            print("  first diff at", n, "in equal", torch.equal(bits(i0), bits(i1)), "out equal",
                  torch.equal(bits(o0), bits(o1)), "frac out diff", (bits(o0) != bits(o1)).float().mean().item())
            for kind in ("input_quantizers", "output_quantizers"):
                for q0, q1 in zip(getattr(w0, kind), getattr(w1, kind)):
                    print("   ", kind, q0.enabled, q1.enabled, q0.encoding, q1.encoding)
            p0, p1 = w0.param_quantizers["weight"], w1.param_quantizers["weight"]
            print("    weight enc equal", [e.to_tuple() for e in p0.encoding] == [e.to_tuple() for e in p1.encoding])
            print("    raw weight equal", torch.equal(w0._module_to_wrap.weight, w1._module_to_wrap.weight))
            print("    types", type(w0._module_to_wrap), w0._mode, w1._mode, w0.training, w1.training)
            break

# range learning: run-to-run determinism of one step on the same sim
torch.manual_seed(0)
net = _Net().to(dev)
x = torch.randn(4, 3, 8, 8, device=dev)
lsim = QuantizationSimModel(net, x[:1], quant_scheme=QuantScheme.training_range_learning_with_tf_init,
                            config_file=PER_CHANNEL_CFG)
lsim.compute_encodings(lambda m, _: m(x), None)


def step(model):
    model.zero_grad(set_to_none=True)
    y = model(x)
    y.square().sum().backward()
    return y, {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}


ya, ga = step(lsim.model)
yb, gb = step(lsim.model)
lcp = pickle.loads(pickle.dumps(lsim.model))
yc, gc = step(lcp)
for n in ga:
    print("LG", n, "repeat", torch.equal(ga[n], gb[n]), "reloaded", torch.equal(ga[n], gc[n]),
          (ga[n] - gc[n]).abs().max().item() if ga[n].shape == gc[n].shape else "shape")
