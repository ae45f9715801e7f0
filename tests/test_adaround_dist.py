"""AdaRound data parallelism (adaround_optimizer.py:139-160,214-216) at world size 2 over gloo on
the CPU: the cached samples sharded rank::world, the learning rate scaled by the world size,
num_iterations // world iterations, alpha.grad all-reduced and divided by the world size. Every
rank must end with the alpha of ONE process that sees the union of the ranks' batches (the mean
of their reconstruction losses + the rounding loss, the same scaled Adam), within fp32 tolerance.

The orchestration under test is the product code (aimet_amd.adaround_optimizer); the soft
quantization and the reconstruction gradient, gfx950 kernels in the product, are replaced by
their torch-op restatements (oracle/torch_ref.py) because this container has no GPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import torch_ref as T

N, WORLD, SEEDS = 96, 2, (11, 23)


def _problem():
    g = torch.Generator().manual_seed(3)
    conv = torch.nn.Conv2d(6, 8, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.zero_()
    inp = torch.randn(N, 6, 5, 5, generator=g)
    with torch.no_grad():
        out = conv(inp) + 0.01 * torch.randn(N, 8, 5, 5, generator=g)
    w = conv.weight.detach()
    d = (w.abs().amax(dim=(1, 2, 3)) / 7).contiguous()
    o = torch.full((8,), -8.0)
    return conv, inp, out, d, o


def _params():
    from aimet_amd.adaround_optimizer import AdaroundHyperParameters
    return AdaroundHyperParameters(num_iterations=40, warm_start=0.25)


class CpuSoftQuant:
    """Stand-in for adaround_optimizer._BoundSoftQuant (same interface) on torch ops."""

    def __init__(self, w, alpha, d, o, bitwidth, ch_axis, round_loss_out):
        shape = [1] * w.dim()
        shape[ch_axis] = -1
        self.w, self.alpha, self.bw = w, alpha, int(bitwidth)
        self.db, self.ob = d.view(shape), o.view(shape)
        self.reg = self.beta = 0.0
        self.reg_beta = None

    def forward(self):
        with torch.no_grad():
            return T.adaround_forward(self.w, self.alpha, self.db, self.ob, self.bw)

    def backward(self, grad):
        with torch.enable_grad():   # called from inside an autograd backward
            a = self.alpha.detach().clone().requires_grad_(True)
            loss = (T.adaround_forward(self.w, a, self.db, self.ob, self.bw) * grad).sum()
            if self.reg:
                loss = loss + T.adaround_round_loss(a, self.reg, self.beta)
            loss.backward()
        return a.grad


def _recon_backward(q, t, act):
    from aimet_amd.adaround_optimizer import recon_loss
    recon_loss(act(q), act(t)).backward()


def _patch():
    import aimet_amd.adaround_optimizer as AO
    AO._BoundSoftQuant = CpuSoftQuant
    AO.recon_loss_backward = _recon_backward


def _worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        _patch()
        from aimet_amd.adaround_optimizer import AdaroundOptimizer
        conv, inp, out, d, o = _problem()
        alpha = AdaroundOptimizer.optimize_rounding(conv, inp, out, d, o, 4, 0, _params(), torch.nn.ReLU(),
                                                    torch.Generator().manual_seed(SEEDS[rank]), use_graph=False)
        q.put((rank, alpha.detach().numpy().copy()))   # by value: no shared-memory handle to outlive the child
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def union_reference(world=WORLD, seeds=SEEDS):
    """One process, the union of the ranks' batches per iteration."""
    from aimet_amd.adaround import compute_beta, init_alpha
    from aimet_amd.adaround_optimizer import BATCH_SIZE, layer_forward, recon_loss
    conv, inp, out, d, o = _problem()
    p = _params()
    act = torch.nn.ReLU()
    w = conv.weight.detach()
    alpha = init_alpha(w, d.view(-1, 1, 1, 1))
    opt = torch.optim.Adam([alpha], lr=1e-3 * world)
    gens = [torch.Generator().manual_seed(s) for s in seeds]
    shards = [torch.arange(r, N, world) for r in range(world)]
    for it in range(p.num_iterations // world):
        opt.zero_grad()
        wq = T.adaround_forward(w, alpha, d.view(-1, 1, 1, 1), o.view(-1, 1, 1, 1), 4)
        losses = []
        for r in range(world):
            idx = shards[r][torch.randperm(len(shards[r]), generator=gens[r])[:BATCH_SIZE]]
            qo = layer_forward(conv, inp[idx], wq)
            losses.append(recon_loss(act(qo), act(out[idx])))
        loss = sum(losses) / world
        if it >= p.num_iterations * p.warm_start:
            loss = loss + T.adaround_round_loss(alpha, p.reg_param,
                                                compute_beta(p.num_iterations, it, p.beta_range, p.warm_start))
        loss.backward()
        opt.step()
    return alpha.detach()


def test_adaround_data_parallel_equals_union_of_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    import queue
    while len(res) < WORLD:
        try:
            r, a = q.get(timeout=2)
            res[r] = torch.from_numpy(a)
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.testing.assert_close(res[0], res[1], rtol=0, atol=0)   # identical on every rank
    want = union_reference()
    torch.testing.assert_close(res[0], want, rtol=1e-5, atol=1e-6)
    # the reference's quirk, mirrored: the rounding-loss horizon stays num_iterations, so with
    # world 2 the 20 iterations run span warm start (10) + the first half of the annealing


def test_adaround_world_one_unchanged():
    """No process group: every iteration on the whole cache, lr 1e-3 (the single-process loop)."""
    _patch()
    from aimet_amd.adaround_optimizer import AdaroundOptimizer
    torch.set_num_threads(1)
    conv, inp, out, d, o = _problem()
    a = AdaroundOptimizer.optimize_rounding(conv, inp, out, d, o, 4, 0, _params(), torch.nn.ReLU(),
                                            torch.Generator().manual_seed(SEEDS[0]), use_graph=False)
    # == the union reference with one "rank" holding everything
    want = union_reference(world=1, seeds=SEEDS[:1])
    torch.testing.assert_close(a.detach(), want, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("iters", [0, 1])
def test_adaround_fewer_iterations_than_ranks(iters, monkeypatch):
    """num_iterations // world == 0 (world 2, 0 or 1 iteration): the reference's loop runs zero
    times and returns the initial alpha; no batch is drawn and no graph captured (use_graph=True
    must not reach the capture path, which needs a GPU)."""
    _patch()
    import aimet_amd.adaround_optimizer as AO
    from aimet_amd.adaround import init_alpha
    monkeypatch.setattr(AO, "_group_world", lambda group: (0, 2))
    conv, inp, out, d, o = _problem()
    p = AO.AdaroundHyperParameters(num_iterations=iters)
    a = AO.AdaroundOptimizer.optimize_rounding(conv, inp, out, d, o, 4, 0, p, torch.nn.ReLU(),
                                               torch.Generator().manual_seed(1), use_graph=True)
    want = init_alpha(conv.weight.detach(), d.view(-1, 1, 1, 1))
    torch.testing.assert_close(a.detach(), want.detach(), rtol=0, atol=0)
