"""Config 5's data-parallel form (BASELINE.json: "data-parallel 8xMI355X"; the reference's multi-GPU
QAT mode, Docs/api_docs/torch_multi_gpu.rst:27-37): DistributedDataParallel over a range-learning
QuantizationSimModel (2 Llama decoder layers, 4-bit per-channel weights, 16-bit outputs,
LearnedGridQuantWrapper with the fused kernels), world size 2 over gloo with both ranks on one
GPU. DDP all-reduces every gradient -- the *_encoding_min / *_encoding_max range parameters and
the weights -- so each rank must hold the gradient one process computes on the union batch.

The single process runs the union batch as one micro-batch per rank with gradient accumulation:
the same GEMM shapes, so every forward value is the ranks' bit for bit and g0 / 2 + g1 / 2 is
exactly DDP's (g0 + g1) / 2 (halving is exact). Bar: bit-identical gradients for every parameter
-- the range parameters included, whose gradients (sums of rounding residuals x gradient) are
ill-conditioned: a batch-of-2 reference, whose GEMM outputs differ in their last bits, moves them
by up to 58x. A parameter whose gradient comes from a non-deterministic ROCm kernel would be
reported with its norm-wise relative error (bar 1e-6). Both ranks hold identical gradients."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "qat_ddp_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, out, autocast):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OUT=out, AUTOCAST="1" if autocast else "0")
        procs.append(subprocess.Popen([sys.executable, WORKER], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    return [json.load(open(out + ".%d" % r)) for r in range(world)]


def _rel(a, b):
    a, b = torch.tensor(a, dtype=torch.float64), torch.tensor(b, dtype=torch.float64)
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("autocast", [False, True])
def test_ddp_range_learning_equals_union_batch(tmp_path, autocast):
    ref, = _run(1, str(tmp_path / "one"), autocast)
    r0, r1 = _run(2, str(tmp_path / "ddp"), autocast)
    tol = 1e-6
    assert r0.keys() == ref.keys()
    errs, n_enc = {}, 0
    for name, want in ref.items():
        if name == "loss":
            continue
        assert want is not None, name
        a, b = r0[name], r1[name]
        assert a == b, "ranks disagree on %s" % name
        if "full" in want:
            n_enc += 1
            errs[name] = _rel(a["full"], want["full"])
        else:
            errs[name] = max(abs(a["norm"] - want["norm"]) / want["norm"], _rel(a["sample"], want["sample"]))
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:8]
    exact = sum(v == 0.0 for v in errs.values())
    print("bit-identical gradients: %d of %d; worst norm-wise relative errors: %s" % (exact, len(errs), worst))
    assert worst[0][1] <= tol, worst
    assert n_enc >= 4 * (2 * 7 + 1)   # min / max of the weight and output ranges of every Linear
    # the union loss is the mean of the ranks' losses (equal token counts)
    assert abs((r0["loss"] + r1["loss"]) / 2 - ref["loss"]) <= 1e-3 * abs(ref["loss"])
