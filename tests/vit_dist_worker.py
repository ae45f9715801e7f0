"""Worker of tests/test_configs_gpu.py::test_config4_vit_sharded_calibration (not collected by
pytest). Config 4 at its stated workload and batch: every activation
QuantizationSimModel quantizes on ViT-L/16 (workloads/vit.py activation_modules + the model
input), TF-Enhanced, per-tensor, over one 32-image calibration batch (config 4's batch size).

  WORLD_SIZE=2: rank r forwards images [16r, 16r+16) on cuda:0 and the ranks calibrate over a gloo
                group (one MAX + one SUM): MODE=phased through
                aimet_amd.distributed.sharded_update_stats, MODE=plan through
                compute_encodings_resident -- the native calibration plan's staged launch (318
                quantizers: the min/max walk form) with the two collectives between its stages;
                MODE=sim through the drop-in QuantizationSimModel(quantizable_types = the modules
                whose outputs QuantSim quantizes).compute_encodings, each rank calling it on its
                shard: the sim shards by itself (the ranks form a process group);
  WORLD_SIZE=1 (oracle): forwards the same two 16-image shards, feeds the CPU oracle analyzers
                each quantizer's two shards concatenated as ONE batch (min/max and bin counts do
                not depend on element order), in a host thread pool. MODE=sim: the shards are
                forwarded through the same sim (its weights quantize-dequantized as in the ranks'
                ANALYSIS forwards) and the oracle is fed what each of its activation quantizers is
                handed.
Writes every quantizer's 8-bit asymmetric encoding (and the element count) to OUT.<rank>, ordered
as the model input, then the quantized modules in forward order."""
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


def sim_of(model, images):
    from aimet_amd.quantsim import QuantizationSimModel
    from workloads.vit import QUANTIZED_OUTPUT_TYPES
    return QuantizationSimModel(model, images[:1].cuda(), quant_scheme="tf_enhanced", in_place=True,
                                quantizable_types=QUANTIZED_OUTPUT_TYPES)


def forward_order(sim):
    """(wrapper name, kind) of every enabled activation quantizer: the model input, then the
    quantized outputs in the order the forward runs them (as the hooks of the other modes)."""
    from aimet_amd.qc_quantize_op import QcQuantizeWrapper
    order = []
    hooks = [w.register_forward_hook(lambda m, i, o, n=n: order.append(n))
             for n, w in sim.model.named_modules() if isinstance(w, QcQuantizeWrapper)]
    with torch.no_grad():
        sim.model(torch.zeros(1, 3, 224, 224, device="cuda"))
    for h in hooks:
        h.remove()
    return [(order[0], "input")] + [(n, "output") for n in order]


def sim_main(rank, world, model, images):
    """MODE=sim: the drop-in QuantizationSimModel on ViT-L/16."""
    import aimet_amd.qc_quantize_op as QO
    sim = sim_of(model, images)
    order = forward_order(sim)
    if world == 1:
        from oracle import oracle as O
        names = {}
        for n, w in sim.quant_wrappers():
            names[id(w.input_quantizers[0])] = (n, "input")
            names[id(w.output_quantizers[0])] = (n, "output")
        seen = {}
        orig_add = QO.StatsBatch.add

        def add(self, q, t, owned=False):
            seen.setdefault(names[id(q)], []).append(t.detach().cpu().numpy().ravel())
        QO.StatsBatch.add = add
        sim.compute_encodings(lambda m, _: [m(images[s * IMAGES // SHARDS:(s + 1) * IMAGES // SHARDS].cuda())
                                            for s in range(SHARDS)], None)
        QO.StatsBatch.add = orig_add

        def feed(key):
            a = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
            a.update(np.concatenate(seen[key]))
            return a.compute(8).as_tuple()
        with ThreadPoolExecutor(16) as pool:
            encs = list(pool.map(feed, order))
        elems = sum(a.size for v in seen.values() for a in v)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        seen = []
        orig_add = QO.StatsBatch.add

        def add(self, q, t, owned=False):
            seen.append(t.numel())
            return orig_add(self, q, t, owned)
        QO.StatsBatch.add = add
        x = images[rank * IMAGES // SHARDS:(rank + 1) * IMAGES // SHARDS].cuda()
        sim.compute_encodings(lambda m, _: m(x), None)
        QO.StatsBatch.add = orig_add
        assert sim._last_calibration["sharded"], sim._last_calibration
        act = sim.get_encodings_dict()["activation_encodings"]
        encs = []
        for n, kind in order:
            e = act[n][kind]["0"]
            encs.append((e["min"], e["max"], e["scale"], float(e["offset"]), e["bitwidth"]))
        t = torch.tensor([sum(seen)], dtype=torch.int64)
        dist.all_reduce(t)
        elems = int(t)
    return encs, elems


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    model = vit_l16(seed=0, device="cuda")
    images = torch.randn(IMAGES, 3, 224, 224, generator=torch.Generator().manual_seed(3))
    if os.environ.get("MODE") == "sim":
        encs, elems = sim_main(rank, world, model, images)
    elif world == 1:
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
