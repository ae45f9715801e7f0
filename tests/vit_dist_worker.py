"""Worker of tests/test_configs_gpu.py::test_config4_vit_sharded_calibration (not collected by
pytest). Config 4 at its stated workload and batch: every activation
QuantizationSimModel quantizes on ViT-L/16 (workloads/vit.py activation_modules + the model
input), TF-Enhanced, per-tensor, over one 32-image calibration batch (config 4's batch size).

  WORLD_SIZE=2: rank r forwards images [16r, 16r+16) on cuda:0 and the ranks calibrate over a gloo
                group (one MAX + one SUM): MODE=phased through
                aimet_amd.distributed.sharded_update_stats, MODE=plan through
                compute_encodings_resident -- the native calibration plan's staged launch (318
                quantizers: the min/max walk form) with the two collectives between its stages;
  WORLD_SIZE=1 (oracle): forwards the same two 16-image shards, feeds the CPU oracle analyzers
                each quantizer's two shards concatenated as ONE batch (min/max and bin counts do
                not depend on element order), in a host thread pool.
Writes every quantizer's 8-bit asymmetric encoding (and the element count) to OUT.<rank>."""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from aimet_amd.calibration import compute_encodings_resident  # noqa: E402
from aimet_amd.distributed import sharded_update_stats  # noqa: E402
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402
from workloads.vit import activation_modules, vit_l16  # noqa: E402

IMAGES, SHARDS = 32, 2


def shard_activations(model, images, s):
    acts = []
    hooks = [m.register_forward_hook(lambda mod, i, o: acts.append(o.contiguous()))
             for m in activation_modules(model)]
    x = images[s * IMAGES // SHARDS:(s + 1) * IMAGES // SHARDS].cuda()
    with torch.no_grad():
        model(x)
    for h in hooks:
        h.remove()
    return [x] + acts


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    model = vit_l16(seed=0, device="cuda")
    images = torch.randn(IMAGES, 3, 224, 224, generator=torch.Generator().manual_seed(3))
    if world == 1:
        from oracle import oracle as O
        shards = [[t.cpu().numpy().ravel() for t in shard_activations(model, images, s)] for s in range(SHARDS)]
        n = len(shards[0])
        analyzers = [O.Analyzer(O.QUANTIZATION_TF_ENHANCED) for _ in range(n)]

        def feed(i):
            analyzers[i].update(np.concatenate([sh[i] for sh in shards]))
            return analyzers[i].compute(8).as_tuple()
        with ThreadPoolExecutor(16) as pool:
            encs = list(pool.map(feed, range(n)))
        elems = sum(a.size for sh in shards for a in sh)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        tensors = shard_activations(model, images, rank)
        qs = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in tensors]
        if os.environ.get("MODE") == "plan":
            a_res, _ = compute_encodings_resident(qs, tensors, [], [])
            encs = [e.to_tuple() for e, _ in a_res]
        else:
            sharded_update_stats(qs, tensors)
            encs = [e.to_tuple() for e, _ in AimetTensorQuantizer.getEncodings(qs, 8, False, False, False)]
        t = torch.tensor([sum(x.numel() for x in tensors)], dtype=torch.int64)
        dist.all_reduce(t)
        elems = int(t)
    with open(os.environ["OUT"] + ".%d" % rank, "w") as f:
        json.dump({"encodings": [list(e) for e in encs], "elements": elems}, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
