"""Sharded calibration through the drop-in QuantizationSimModel on the gfx950 operators (SURVEY
§8(e), v1/quantsim.py:381-449), and the copies StatsBatch makes (or does not) of what it queues.

* config 1 (ResNet-50 W8A8 per-tensor, 8 x 32 images, TF-Enhanced and TF), every batch split
  16 + 16 over two gloo ranks on cuda:0 (tests/quantsim_dist_worker.py): every encoding of both
  ranks == one process fed the whole batches (one statistics batch of 32 images each, its tensors
  from the ranks' 16-image forwards: MIOpen's convolutions are not batch-size invariant bit for
  bit), whose encodings == the CPU oracle fed the same tensors. The CPU form, with the oracle as
  the single process, is tests/test_quantsim_sharded.py.
* in-place writes: on a network that overwrites quantized outputs in place, the batched statistics
  equal the per-call updates (the reference's behaviour) in every forward; only the first forward
  copies what it queues unless a tensor was seen overwritten; a network whose in-place writes start
  after the first forward raises instead of calibrating on overwritten values."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
from torch import nn

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]
WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "quantsim_dist_worker.py")


def _run(world, out, scheme):
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, WORKER], env=dict(
        os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
        OUT=out, SCHEME=scheme)) for r in range(world)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    return [json.load(open(out + ".%d" % r)) for r in range(world)]


@pytest.mark.parametrize("scheme", ["post_training_tf_enhanced", "post_training_tf"])
def test_config1_sharded_quantsim_equals_single_process(tmp_path, scheme):
    single, = _run(1, str(tmp_path / "single"), scheme)
    assert single["calibration"]["sharded"] is False
    # the single process (one statistics batch per 32 images) == the oracle fed the same tensors
    assert single["oracle"]["checked"] >= 100 and not single["oracle"]["mismatches"], single["oracle"]
    n_act = sum(len(v) for e in single["encodings"]["activation"].values() for v in e.values())
    assert n_act == 55 and len(single["encodings"]["param"]) == 54
    for r, res in enumerate(_run(2, str(tmp_path / "sharded"), scheme)):
        assert res["calibration"]["sharded"] is True and res["calibration"]["world"] == 2
        same_fwd = len(res["digests"]) == len(single["digests"]) and \
            all(d[0] == s[r] for d, s in zip(res["digests"], single["digests"]))
        assert same_fwd, "rank %d: the 16-image forwards differ from the halves of the 32-image ones" % r
        assert res["encodings"]["param"] == single["encodings"]["param"], r
        bad = [k for k in single["encodings"]["activation"]
               if res["encodings"]["activation"].get(k) != single["encodings"]["activation"][k]]
        assert not bad, "rank %d: %d layers' activation encodings differ (first %s)" % (r, len(bad), bad[:3])


class InplaceNet(nn.Module):
    """fc1's and fc2's quantized outputs are overwritten in place (relu_, +=) before the forward
    returns; in `late` mode only from the second calibration forward on."""

    def __init__(self, late=False):
        super().__init__()
        self.fc1 = nn.Linear(64, 64)
        self.fc2 = nn.Linear(64, 64)
        self.fc3 = nn.Linear(64, 32)
        self.late = late
        self.calls = 0

    def forward(self, x):
        self.calls += 1
        a = self.fc1(x)
        b = self.fc2(a)
        # calls 1, 2: QuantizationSimModel's input count and pass-through check on the dummy input
        if not self.late or self.calls > 3:
            a.relu_()
            b += a
        return self.fc3(b)


def _state(sim):
    out = {}
    for name, w in sim.quant_wrappers():
        for kind, qs in (("in", w.input_quantizers), ("out", w.output_quantizers),
                         ("param", [w.param_quantizers[k] for k in sorted(w.param_quantizers)])):
            for i, q in enumerate(qs):
                e = q.encoding
                encs = e if isinstance(e, list) else ([] if e is None else [e])
                out[(name, kind, i)] = (bool(q.enabled), [x.to_tuple() for x in encs])
    return out


@pytest.mark.parametrize("scheme", ["tf_enhanced", "tf"])
def test_statsbatch_inplace_writes_equal_per_call(monkeypatch, scheme):
    import aimet_amd.qc_quantize_op as QO
    from aimet_amd.quantsim import QuantizationSimModel
    data = [torch.randn(16, 64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(i))
            for i in range(4)]

    def run(per_call):
        torch.manual_seed(3)
        sim = QuantizationSimModel(InplaceNet().cuda().eval(), torch.randn(1, 64, device="cuda"),
                                   quant_scheme=scheme)
        if per_call:
            monkeypatch.setattr(QO.StatsBatch, "eligible", staticmethod(lambda q, t: False))
        sim.compute_encodings(lambda m, d: [m(x) for x in d], data)
        monkeypatch.undo()
        return _state(sim), sim._last_calibration

    ref, _ = run(True)
    got, info = run(False)
    assert got == ref
    # fc1's output (relu_) and fc2's (+=) are copied in every forward, seen overwritten in the
    # first; fc3's output and the model input only in the first
    first = 16 * (64 + 64 + 64 + 32)
    assert info["copied_quantizers"] == 2
    assert info["copied_elements"] == first + 3 * 2 * 16 * 64, info


def test_statsbatch_inplace_after_first_forward_raises():
    from aimet_amd.quantsim import QuantizationSimModel
    data = [torch.randn(16, 64, device="cuda") for _ in range(3)]
    sim = QuantizationSimModel(InplaceNet(late=True).cuda().eval(), torch.randn(1, 64, device="cuda"))
    with pytest.raises(RuntimeError, match="written in place"):
        sim.compute_encodings(lambda m, d: [m(x) for x in d], data)


def test_quantsim_resnet_calibration_copies_first_forward_only():
    """ResNet-50 (no in-place write reaches a quantized conv / fc output): after the first forward
    nothing is copied (config 1's 8 forwards: 1/8 of the round-5 copies)."""
    from aimet_amd.quantsim import QuantizationSimModel
    from workloads.resnet import resnet50
    dev = torch.device("cuda", 0)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(4 * 8, 3, 64, 64, device=dev)
    sim = QuantizationSimModel(model, x[:1], quant_scheme="tf_enhanced")
    per_fwd = []

    def calibrate(m, _):
        for b in range(4):
            m(x[b * 8:(b + 1) * 8])
    sim.compute_encodings(calibrate, None)
    info = sim._last_calibration
    acts = []
    hooks = [mod.register_forward_hook(lambda mm, i, o: acts.append(o.numel()))
             for mod in model.modules() if isinstance(mod, (nn.Conv2d, nn.Linear))]
    with torch.no_grad():
        model(x[:8])
    for h in hooks:
        h.remove()
    per_fwd.append(sum(acts) + x[:8].numel())
    assert info["copied_quantizers"] == 0
    assert info["copied_elements"] == per_fwd[0]
