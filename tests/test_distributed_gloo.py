"""Sharded calibration (aimet_amd.distributed) at world_size 2 over gloo on the CPU.

The exchange logic (packing, collective ops, global counts, fold order) is the product code; the
per-rank statistics are produced by an oracle-backed stand-in implementing the same duck-typed
quantizer interface as the gfx950 AimetTensorQuantizer (this container has no GPU). The sharded
result must be identical to one analyzer seeing the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O


class OracleShardQuantizer:
    """Test stand-in: reference-exact statistics on the CPU, same phase interface."""

    def __init__(self, scheme, num_channels=1, percentile=None):
        self.scheme = scheme
        self.num_channels = num_channels
        self.uses_histogram = scheme != O.QUANTIZATION_TF
        self.an = [O.Analyzer(scheme) for _ in range(num_channels)]
        if percentile is not None:
            for a in self.an:
                a.set_percentile(percentile)
        self.active = [False] * num_channels

    def bind_exchange(self, minmax, counts=None):
        self.mm, self.cnt = minmax, counts

    def _channels(self, t, ax):
        x = t.numpy()
        if self.num_channels == 1:
            return [x.ravel()]
        return [np.ascontiguousarray(np.take(x, c, axis=ax)).ravel() for c in range(self.num_channels)]

    def batch_minmax(self, t, ax=0):
        for c, x in enumerate(self._channels(t, ax)):
            self.mm[2 * c] = -O.get_min(x)
            self.mm[2 * c + 1] = O.get_max(x)

    def fold_minmax(self):
        for c, a in enumerate(self.an):
            self.active[c] = a.fold_minmax(-float(self.mm[2 * c]), float(self.mm[2 * c + 1]))

    def batch_histogram(self, t, ax=0):
        for c, x in enumerate(self._channels(t, ax)):
            if not self.active[c]:
                continue
            xl, _ = self.an[c].histogram()
            bucket = np.float32(xl[1] - xl[0])
            off = np.float32(np.float32(xl[0]) / bucket)
            self.cnt[512 * c:512 * (c + 1)] = torch.from_numpy(O.histogram(x, bucket, off).astype(np.int64))

    def fold_histogram(self, n):
        for c, a in enumerate(self.an):
            if self.active[c]:
                a.update_from_counts(self.cnt[512 * c:512 * (c + 1)].numpy().astype(np.uint64), n)
            self.cnt[512 * c:512 * (c + 1)] = 0

    def encodings(self, bw, *flags):
        return [a.compute(bw, *flags).as_tuple() for a in self.an]


def make_batches(seed=0, n_batches=3, batch=8):
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_batches):
        act = (rng.standard_normal((batch, 6, 5, 5)) * (1 + b)).astype(np.float32)
        if b == 0:
            act[:, 2] = 0.0
        relu = np.maximum(act, 0)
        out.append((act, relu))
    return out


CONFIGS = [("tf", O.QUANTIZATION_TF, 1, None, 0), ("tfe", O.QUANTIZATION_TF_ENHANCED, 1, None, 1),
           ("pct", O.QUANTIZATION_PERCENTILE, 1, 99.0, 0), ("tfe_pc", O.QUANTIZATION_TF_ENHANCED, 6, None, 0),
           ("mse", O.QUANTIZATION_MSE, 1, None, 1)]


def _quantizers():
    return [OracleShardQuantizer(s, c, p) for _, s, c, p, _ in CONFIGS]


def _tensors(batch, rank, world):
    act, relu = batch
    n = act.shape[0]
    sl = slice(rank * n // world, (rank + 1) * n // world)
    src = [act, relu]
    return [torch.from_numpy(np.ascontiguousarray(src[which][sl])) for _, _, _, _, which in CONFIGS]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from aimet_amd.distributed import sharded_update_stats
        qs = _quantizers()
        ex = None
        for batch in make_batches():
            ex = sharded_update_stats(qs, _tensors(batch, rank, world), ch_axes=[0, 0, 0, 1, 0], exchange=ex)
        res = [qq.encodings(8, 0, 0, 0) + qq.encodings(8, 1, 0, 0) for qq in qs]
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_sharded_calibration_equals_whole_batch(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # whole-batch reference: one analyzer per quantizer/channel over the full batch
    whole = _quantizers()
    for batch in make_batches():
        for qq, t, ax in zip(whole, _tensors(batch, 0, 1), [0, 0, 0, 1, 0]):
            for c, x in enumerate(qq._channels(t, ax)):
                qq.an[c].update(x)
    want = [qq.encodings(8, 0, 0, 0) + qq.encodings(8, 1, 0, 0) for qq in whole]
    for r in range(world):
        assert results[r] == want, r


def test_single_process_path_matches_whole_batch():
    """world_size 1 (no process group): the same code path without collectives."""
    from aimet_amd.distributed import sharded_update_stats
    qs = _quantizers()
    ex = None
    for batch in make_batches(seed=4):
        ex = sharded_update_stats(qs, _tensors(batch, 0, 1), ch_axes=[0, 0, 0, 1, 0], exchange=ex)
    whole = _quantizers()
    for batch in make_batches(seed=4):
        for qq, t, ax in zip(whole, _tensors(batch, 0, 1), [0, 0, 0, 1, 0]):
            for c, x in enumerate(qq._channels(t, ax)):
                qq.an[c].update(x)
    assert [qq.encodings(8, 0, 0, 0) for qq in qs] == [qq.encodings(8, 0, 0, 0) for qq in whole]
