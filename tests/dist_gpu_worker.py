"""Worker of tests/test_distributed_gpu.py (not collected by pytest): one rank of a sharded
calibration on the GPU. Every rank uses cuda:0 (one-GPU box) and a gloo group (the exchange
buffers are staged through host memory); the statistics are computed by the gfx950 kernels.

BACKEND=nccl with WORLD_SIZE=1 and FORCE_EXCHANGE=1: a world-size-1 RCCL group formed before any
other GPU call, and both packed collectives of every batch run on the device buffers (the branch
of aimet_amd.distributed._all_reduce that the N-GPU bench takes).

MODE=plan: the native path of bench.py / compute_encodings_resident -- an
aimet_amd.calibration.CalibrationPlan over per-tensor activation quantizers (sharded, exchanged)
and per-channel parameter quantizers (replicated), its tensors refilled in place every batch; the
unsharded reference of it (WORLD_SIZE=1, no FORCE_EXCHANGE) is every quantizer's own updateStats."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from aimet_amd.distributed import sharded_update_stats  # noqa: E402
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402

SCHEMES = [QuantizationMode.QUANTIZATION_TF, QuantizationMode.QUANTIZATION_TF_ENHANCED,
           QuantizationMode.QUANTIZATION_PERCENTILE, QuantizationMode.QUANTIZATION_MSE]
FLAGS = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 1)]
# the plan's forms also carry the entropy analyzer (its per-batch range widening from the global
# min/max)
PLAN_SCHEMES = SCHEMES + [QuantizationMode.QUANTIZATION_ENTROPY]


def batches(n_batches=3, batch=8, seed=0):
    """(activation [batch, 6, 5, 5], relu of it) per batch; batch 0 has an all-zero channel."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_batches):
        act = (rng.standard_normal((batch, 6, 5, 5)) * (1 + b)).astype(np.float32)
        if b == 0:
            act[:, 2] = 0.0
        out.append((act, np.maximum(act, 0)))
    return out


def make_quantizers():
    qs = []
    for s in SCHEMES:
        qs.append(AimetTensorQuantizer(s))                     # per-tensor activation
        qs.append(AimetTensorQuantizer(s, num_channels=6))     # per-channel (axis 1)
    for q in qs:
        if q.quant_scheme == QuantizationMode.QUANTIZATION_PERCENTILE:
            q.setPercentileValue(99.0)
    return qs


def encodings(qs):
    out = []
    for q in qs:
        for fl in FLAGS:
            e, valid = q.getEncoding(8, *fl)
            out.append([x.to_tuple() for x in (e if isinstance(e, list) else [e])] + [bool(valid)])
    return out


def plan_main(rank, world, force, dev):
    """MODE=plan (see the module docstring)."""
    from aimet_amd.calibration import CalibrationPlan
    aq = [AimetTensorQuantizer(s) for s in PLAN_SCHEMES]
    pq = [AimetTensorQuantizer(s, num_channels=6) for s in PLAN_SCHEMES]
    for q in aq + pq:
        if q.quant_scheme == QuantizationMode.QUANTIZATION_PERCENTILE:
            q.setPercentileValue(99.0)
    sharded = world > 1 or force
    plan, bufs, wbufs = None, None, None
    last = None
    for b, (act, relu) in enumerate(batches()):
        shard = slice(rank, None, world)
        acts = [np.ascontiguousarray((act if i % 2 == 0 else relu)[shard]) for i in range(len(aq))]
        # the parameters (replicated): a [6, 5, 5] slice of the batch, channel axis 0
        ws = [np.ascontiguousarray((act if i % 2 == 0 else relu)[b % act.shape[0]]) for i in range(len(pq))]
        if not sharded:
            for q, a in zip(aq, acts):
                q.updateStats(torch.from_numpy(a).to(dev), True)
            for q, w in zip(pq, ws):
                q.updateStatsPerChannel(torch.from_numpy(w).to(dev), 0, True)
            last = None
            continue
        if plan is None:
            bufs = [torch.from_numpy(a).to(dev) for a in acts]
            wbufs = [torch.from_numpy(w).to(dev) for w in ws]
            plan = CalibrationPlan(aq, bufs, pq, wbufs, force_exchange=force)
        else:
            for t, a in zip(bufs, acts):
                t.copy_(torch.from_numpy(a))
            for t, w in zip(wbufs, ws):
                t.copy_(torch.from_numpy(w))
        last = plan.run(reset=False)
    res = encodings(aq + pq)
    if last is not None:
        # the plan's own (batched) encodings at its default settings == getEncoding's
        for q, (e, v) in zip(aq, last[0]):
            assert v and e.to_tuple() == q.getEncoding(8, False, False, False)[0].to_tuple()
        for q, (es, v) in zip(pq, last[1]):
            assert v and [x.to_tuple() for x in es] == [x.to_tuple() for x in q.getEncoding(8, True, False, False)[0]]
    if plan is not None:
        plan.close()
    return res


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    backend = os.environ.get("BACKEND", "gloo")
    force = os.environ.get("FORCE_EXCHANGE") == "1"
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        # the process group first, bound to the device, as bench.py forms it
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    torch.cuda.set_device(0)
    if world > 1 and backend == "gloo":
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if os.environ.get("MODE") == "plan":
        res = plan_main(rank, world, force, dev)
        with open(os.environ["OUT"] + ".%d" % rank, "w") as f:
            json.dump(res, f)
        if dist.is_initialized():
            with open(os.environ["OUT"] + ".backend", "w") as f:
                f.write(dist.get_backend())
            dist.barrier()
            dist.destroy_process_group()
        return
    qs = make_quantizers()
    sharded = world > 1 or force
    ex = None
    for act, relu in batches():
        shard = slice(rank, None, world)      # per-sample sharding
        tensors, axes = [], []
        for i, q in enumerate(qs):
            src = act if (i // 2) % 2 == 0 else relu
            tensors.append(torch.from_numpy(np.ascontiguousarray(src[shard])).to(dev))
            axes.append(1)
        if sharded:
            ex = sharded_update_stats(qs, tensors, axes, exchange=ex, force_exchange=force)
        else:
            for q, t, ax in zip(qs, tensors, axes):
                if q.num_channels == 1:
                    q.updateStats(t, True)
                else:
                    q.updateStatsPerChannel(t, ax, True)
    res = encodings(qs)
    with open(os.environ["OUT"] + ".%d" % rank, "w") as f:
        json.dump(res, f)
    if dist.is_initialized():
        with open(os.environ["OUT"] + ".backend", "w") as f:
            f.write(dist.get_backend())
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
