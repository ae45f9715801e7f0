"""AdaRound data parallelism on the GPU kernels (world size 2, both ranks on cuda:0 over gloo):
identical alpha on both ranks, the HIP-graph form (graphs split around the all_reduce) equal to
the eager loop, and both equal to ONE process seeing the union of the ranks' batches through the
reference's torch ops (adaround_optimizer.py:139-160,214-216), within fp32 trajectory tolerance."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "adaround_dist_worker.py")
N, WORLD, SEEDS = 512, 2, (11, 23)


def problem():
    g = torch.Generator().manual_seed(3)
    conv = torch.nn.Conv2d(16, 24, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.1)
        conv.bias.zero_()
    inp = torch.randn(N, 16, 8, 8, generator=g)
    with torch.no_grad():
        out = conv(inp) + 0.01 * torch.randn(N, 24, 8, 8, generator=g)
    conv = conv.cuda()
    w = conv.weight.detach()
    d = (w.abs().amax(dim=(1, 2, 3)) / 7).contiguous()
    o = torch.full((24,), -8.0, device="cuda")
    return conv, inp.cuda(), out.cuda(), d, o


def params():
    from aimet_amd.adaround_optimizer import AdaroundHyperParameters
    return AdaroundHyperParameters(num_iterations=160, warm_start=0.25)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _union_reference():
    from aimet_amd.adaround import compute_beta, init_alpha
    from aimet_amd.adaround_optimizer import BATCH_SIZE, layer_forward, recon_loss
    from oracle import torch_ref as T
    conv, inp, out, d, o = problem()
    p = params()
    act = torch.nn.ReLU6()
    w = conv.weight.detach()
    alpha = init_alpha(w, d.view(-1, 1, 1, 1))
    opt = torch.optim.Adam([alpha], lr=1e-3 * WORLD)
    gens = [torch.Generator().manual_seed(s) for s in SEEDS]
    shards = [torch.arange(r, N, WORLD, device="cuda") for r in range(WORLD)]
    for it in range(p.num_iterations // WORLD):
        opt.zero_grad()
        wq = T.adaround_forward(w, alpha, d.view(-1, 1, 1, 1), o.view(-1, 1, 1, 1), 4)
        losses = []
        for r in range(WORLD):
            idx = shards[r][torch.randperm(len(shards[r]), generator=gens[r])[:BATCH_SIZE].cuda()]
            losses.append(recon_loss(act(layer_forward(conv, inp[idx], wq)), act(out[idx])))
        loss = sum(losses) / WORLD
        if it >= p.num_iterations * p.warm_start:
            loss = loss + T.adaround_round_loss(alpha, p.reg_param,
                                                compute_beta(p.num_iterations, it, p.beta_range, p.warm_start))
        loss.backward()
        opt.step()
    return alpha.detach().cpu()


def test_adaround_data_parallel_on_gpu(tmp_path):
    port = _free_port()
    out = str(tmp_path / "alpha")
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OUT=out)
        procs.append(subprocess.Popen([sys.executable, WORKER], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    res = [torch.load(out + ".%d" % r, weights_only=True) for r in range(WORLD)]
    for mode in ("eager", "graph"):
        assert torch.equal(res[0][mode], res[1][mode]), mode
        assert torch.equal(res[0][mode + "_loss"], res[1][mode + "_loss"]), mode
    torch.testing.assert_close(res[0]["graph"], res[0]["eager"], rtol=1e-5, atol=1e-6)
    want = _union_reference()
    torch.testing.assert_close(res[0]["eager"], want, rtol=1e-3, atol=2e-4)
