"""BASELINE.json's ResNet-50 configurations at their stated workloads, every encoding checked
against the CPU oracle (oracle/dlq_oracle.c, pinned to the reference C++ by tests/golden) fed the
exact tensors each quantizer saw.

* config 1: QuantizationSimModel.compute_encodings, ResNet-50 W8A8 per-tensor, 8 batches x 32
  images U(0,1) seed 1234, TF-Enhanced and TF;
* the bench's own calibration path (bench.py -> aimet_amd.calibration.compute_encodings_resident:
  batched activation statistics, per-channel weight statistics and device searches on a second
  stream) on the config-1 network: one 32-image batch, TF-Enhanced and TF, every activation
  encoding and every one of the 27,560 weight-channel encodings;
* config 4: ViT-L/16 TF-Enhanced calibration of every activation QuantSim quantizes (318
  quantizers, ~122.6 M elements per image), one 32-image batch sharded over 2 ranks (gloo, both on
  cuda:0) through aimet_amd.distributed.sharded_update_stats, the calibration plan, and the
  drop-in QuantizationSimModel.compute_encodings; both ranks' encodings == the oracle fed the whole
  batch (tests/vit_dist_worker.py).

The oracle work runs in a thread pool (ctypes releases the GIL); tensors stream to it one batch at
a time so host memory stays at one batch of activations."""
import concurrent.futures as cf
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import gpu_available
from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

DEV = torch.device("cuda", 0)
THREADS = min(16, os.cpu_count() or 4)


def _images(n, seed=1234):
    return torch.rand(n, 3, 224, 224, generator=torch.Generator().manual_seed(seed)).to(DEV)


def _resnet():
    from workloads.resnet import resnet50
    return resnet50(seed=0, device=DEV)


@pytest.mark.parametrize("scheme_name", ["post_training_tf_enhanced", "post_training_tf"])
def test_config1_quantsim_compute_encodings_equals_oracle(scheme_name, monkeypatch):
    from aimet_amd.quantizers import QuantScheme, StaticGridPerTensorQuantizer
    from aimet_amd.quantsim import QuantizationSimModel
    scheme = getattr(QuantScheme, scheme_name)
    mode = O.QUANTIZATION_TF_ENHANCED if scheme == QuantScheme.post_training_tf_enhanced else O.QUANTIZATION_TF
    model = _resnet()
    images = _images(8 * 32)
    batches = [images[b * 32:(b + 1) * 32] for b in range(8)]
    sim = QuantizationSimModel(model, batches[0][:1], quant_scheme=scheme, default_output_bw=8, default_param_bw=8)

    # every per-tensor quantizer feeds a CPU oracle analyzer with exactly what it was given
    # (the parameter quantizers' statistics are computed for every wrapper at once before the
    # forwards, quantsim._precompute_param_encodings, not through update_encoding_stats: their
    # analyzers are fed the parameter itself, what the first forward would have given them)
    analyzers, pending = {}, []
    pool = cf.ThreadPoolExecutor(THREADS)
    qmap, params = {}, {}
    for name, w in sim.quant_wrappers():
        pnames = list(w.param_quantizers.keys())
        for kind, qs in (("in", list(w.input_quantizers)), ("out", list(w.output_quantizers)),
                         ("param", list(w.param_quantizers.values()))):
            for i, q in enumerate(qs):
                if not isinstance(q, StaticGridPerTensorQuantizer):
                    continue
                key = (name, kind, i)
                qmap[key] = q
                if kind == "param":
                    params[key] = getattr(w._module_to_wrap, pnames[i])
                upd = q.update_encoding_stats

                def u(t, upd=upd, key=key, q=q):
                    if q.enabled and not q.is_encoding_frozen and q.bitwidth != 32:
                        pending.append((key, t.detach().float().reshape(-1).cpu().numpy()))
                    return upd(t)
                q.update_encoding_stats = u

    # the ANALYSIS forwards hand the activation quantizers' tensors to a StatsBatch (one batched
    # update per forward) instead of update_encoding_stats: record them there too
    from aimet_amd import qc_quantize_op as QO
    keys = {id(q): key for key, q in qmap.items()}
    orig_add = QO.StatsBatch.add

    def add(self, q, t, owned=False):
        if id(q) in keys:
            pending.append((keys[id(q)], t.detach().float().reshape(-1).cpu().numpy()))
        return orig_add(self, q, t, owned)
    monkeypatch.setattr(QO.StatsBatch, "add", add)

    def flush():
        # one batch: the analyzers of different quantizers update in parallel, each in batch order
        by_key = {}
        for key, x in pending:
            by_key.setdefault(key, []).append(x)
        pending.clear()

        def run(key, xs):
            a = analyzers.setdefault(key, O.Analyzer(mode))
            for x in xs:
                a.update(x)
        for f in [pool.submit(run, k, xs) for k, xs in by_key.items()]:
            f.result()

    def calibrate(m, _):
        for b in batches:
            m(b)
            flush()

    sim.compute_encodings(calibrate, None)
    torch.cuda.synchronize()
    pool.shutdown()
    for key, t in params.items():
        if key not in analyzers:
            analyzers[key] = O.Analyzer(mode)
            analyzers[key].update(t.detach().float().reshape(-1).cpu().numpy())
    checked, bad = 0, []
    for key, q in qmap.items():
        if not q.enabled or q.encoding is None or key not in analyzers:
            continue
        want = analyzers[key].compute(q.bitwidth, q.use_symmetric_encodings, q.use_strict_symmetric,
                                      q.use_unsigned_symmetric).as_tuple()
        checked += 1
        if q.encoding.to_tuple() != want:
            bad.append((key, q.encoding.to_tuple(), want))
    # 54 conv/fc weights + the model input + every conv/fc/relu/add output the default config quantizes
    assert checked >= 100, checked
    assert not bad, bad[:3]


@pytest.mark.parametrize("mode", [O.QUANTIZATION_TF_ENHANCED, O.QUANTIZATION_TF])
def test_bench_calibration_path_equals_oracle(mode):
    """bench.py's compute_encodings (compute_encodings_resident) on ResNet-50 with one 32-image
    batch: the input + 54 conv/fc outputs per-tensor asymmetric, 54 weights per-channel symmetric
    (27,560 channels); every encoding == the oracle analyzer fed the same tensor / channel."""
    import bench
    from aimet_amd.calibration import compute_encodings_resident
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    model = _resnet()
    acts, weights = bench.collect_tensors(model, _images(32))
    del model
    qm = QuantizationMode(int(mode))
    aq = [AimetTensorQuantizer(qm) for _ in acts]
    wq = [AimetTensorQuantizer(qm, num_channels=w.shape[0]) for _, w in weights]
    a_res, w_res = compute_encodings_resident(aq, [t for _, t in acts], wq, [w for _, w in weights],
                                              act_settings=(8, False, False, False),
                                              param_settings=(8, True, False, False))

    def act_oracle(t):
        a = O.Analyzer(mode)
        a.update(t.cpu().numpy().ravel())
        return a.compute(8).as_tuple()

    def weight_oracle(w2):
        out = []
        for row in w2:
            a = O.Analyzer(mode)
            a.update(row)
            out.append(a.compute(8, True).as_tuple())
        return out

    with cf.ThreadPoolExecutor(THREADS) as pool:
        fa = [pool.submit(act_oracle, t) for _, t in acts]
        fw = []
        for _, w in weights:
            w2 = w.cpu().numpy().reshape(w.shape[0], -1)
            # slices of channels so the 27,560 searches spread over the pool
            fw.append([pool.submit(weight_oracle, w2[s:s + 256]) for s in range(0, w2.shape[0], 256)])
        want_a = [f.result() for f in fa]
        want_w = [[e for f in fs for e in f.result()] for fs in fw]
    assert len(a_res) == 55 and len(w_res) == 54
    for i, ((e, v), want) in enumerate(zip(a_res, want_a)):
        assert v and e.to_tuple() == want, (acts[i][0], e.to_tuple(), want)
    n_ch = 0
    for i, ((es, v), want) in enumerate(zip(w_res, want_w)):
        got = [e.to_tuple() for e in es]
        assert v and len(got) == len(want)
        bad = [c for c in range(len(got)) if got[c] != want[c]]
        assert not bad, (weights[i][0], bad[:5], got[bad[0]], want[bad[0]])
        n_ch += len(got)
    assert n_ch == 27560


def test_config4_vit_sharded_calibration(tmp_path):
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vit_dist_worker.py")

    def run(world, out, mode="phased"):
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        procs = [subprocess.Popen([sys.executable, worker], env=dict(
            os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
            OUT=out, MODE=mode)) for r in range(world)]
        for p in procs:
            assert p.wait(timeout=300) == 0
        return [json.load(open(out + ".%d" % r)) for r in range(world)]

    oracles = {"hooks": run(1, str(tmp_path / "oracle"))[0], "sim": run(1, str(tmp_path / "oracle_sim"), "sim")[0]}
    for oracle in oracles.values():
        assert len(oracle["encodings"]) == 318
        assert oracle["elements"] > 32 * 120e6
    # sharded_update_stats / the calibration plan's staged launch (on the model's own activations)
    # / the drop-in QuantizationSimModel sharding by itself (its ANALYSIS forwards: weights QDQ'd)
    for mode in ("phased", "plan", "sim"):
        oracle = oracles["sim" if mode == "sim" else "hooks"]
        for r, res in enumerate(run(2, str(tmp_path / mode), mode)):
            assert res["elements"] == oracle["elements"]
            bad = [i for i, (a, b) in enumerate(zip(res["encodings"], oracle["encodings"])) if a != b]
            assert not bad, "%s, rank %d: %d of %d encodings differ from the oracle (first %s)" % (
                mode, r, len(bad), len(oracle["encodings"]), bad[:5])
