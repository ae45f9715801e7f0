"""Sharded calibration on the GPU kernels (world size 2, both ranks on cuda:0 over gloo): every
rank's encodings == one process seeing the whole batches, for TF / TF-E / percentile / MSE,
per-tensor and per-channel. Ranks are separate child processes."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_gpu_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, out, **extra):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OUT=out, **extra)
        procs.append(subprocess.Popen([sys.executable, WORKER], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    return [json.load(open(out + ".%d" % r)) for r in range(world)]


def test_sharded_calibration_equals_whole_batch_on_gpu(tmp_path):
    whole, = _run(1, str(tmp_path / "whole"))
    shards = _run(2, str(tmp_path / "shard"))
    for r, res in enumerate(shards):
        assert res == whole, "rank %d" % r


def test_rccl_world1_device_exchange_equals_unsharded(tmp_path):
    """A world-size-1 RCCL ("nccl") group formed in a fresh process before any other GPU call;
    every batch's two packed collectives run on the device buffers (distributed.py _all_reduce's
    RCCL branch, stream-ordered between the statistics kernels): the encodings equal the unsharded
    path bit for bit."""
    whole, = _run(1, str(tmp_path / "whole"))
    rccl, = _run(1, str(tmp_path / "rccl"), BACKEND="nccl", FORCE_EXCHANGE="1")
    assert open(str(tmp_path / "rccl") + ".backend").read() == "nccl"
    assert rccl == whole


def test_plan_sharded_calibration_equals_whole_batch_on_gpu(tmp_path):
    """The calibration plan's sharded form (bench.py's path at N > 1: stage 1, packed MAX, stage 2,
    packed SUM with the element counts formed on the device, stage 4), two ranks over gloo on one
    GPU, three batches refilled in place: every rank's encodings == each quantizer's own
    updateStats over the whole batches (per-tensor activations sharded, per-channel parameters)."""
    whole, = _run(1, str(tmp_path / "whole"), MODE="plan")
    shards = _run(2, str(tmp_path / "shard"), MODE="plan")
    for r, res in enumerate(shards):
        assert res == whole, "rank %d" % r


def test_rccl_world1_plan_exchange_equals_unsharded(tmp_path):
    """The calibration plan's sharded form over a world-size-1 RCCL group: both packed collectives
    of every batch run on the device buffers between the plan's stages; encodings == unsharded."""
    whole, = _run(1, str(tmp_path / "whole"), MODE="plan")
    rccl, = _run(1, str(tmp_path / "rccl"), MODE="plan", BACKEND="nccl", FORCE_EXCHANGE="1")
    assert open(str(tmp_path / "rccl") + ".backend").read() == "nccl"
    assert rccl == whole
