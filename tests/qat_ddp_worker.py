"""Worker of tests/test_qat_ddp_gpu.py: range-learning QAT (config 5's form) on a 2-decoder-layer
Llama (workloads/llama.py, vocab 1024) through QuantizationSimModel, under DistributedDataParallel
when WORLD_SIZE > 1 (gloo; every rank on cuda:0), else one process on the union batch.

Every rank calibrates on ITS shard of the calibration batch (rank r: sequence r of UNION
sequences): QuantizationSimModel.compute_encodings shards by itself (the ranks form a process
group), exchanging each forward's activation statistics. The one process calibrates on the union
batch as ONE statistics batch whose tensors come from one forward per sequence (the ranks' GEMM
shapes, so every activation is the ranks' bit for bit): each quantizer's two tensors are
concatenated and updated once, as one device fed the whole batch. Then every rank runs ONE step on
its share (rank r: sequence r), loss = mean token cross-entropy, backward (DDP all-reduces and
averages the gradients). One process runs the union batch as UNION micro-batches with gradient
accumulation (the ranks' GEMM shapes). Saves, per parameter: the full gradient of
every *_encoding_min / *_encoding_max, and a fixed sample of 4096 elements + the norm of every
other gradient."""
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

UNION, SEQ, VOCAB = 2, 128, 1024


def main():
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    autocast = os.environ.get("AUTOCAST", "1") == "1"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.backends.cuda.matmul.allow_tf32 = False
    from aimet_amd.qc_quantize_op import LearnedGridQuantWrapper
    from aimet_amd.quantizers import QuantScheme
    from aimet_amd.quantsim import QuantizationSimModel
    from workloads.llama import Llama

    torch.manual_seed(0)
    with torch.device(dev):
        model = Llama(lambda i, o: nn.Linear(i, o, bias=False), layers=2, vocab=VOCAB)
    with torch.no_grad():
        g = torch.Generator(device=dev).manual_seed(0)
        for p in model.parameters():
            if p.dim() > 1:
                p.normal_(0, 0.02, generator=g)
    cfg = {"defaults": {"ops": {"is_output_quantized": "True"},
                        "params": {"is_quantized": "True", "is_symmetric": "True"},
                        "strict_symmetric": "False", "per_channel_quantization": "True"}}
    sim = QuantizationSimModel(model, quant_scheme=QuantScheme.training_range_learning_with_tf_init,
                               default_param_bw=4, default_output_bw=16, in_place=True, config_file=cfg)
    ids_all = torch.randint(VOCAB, (UNION, SEQ + 1), device=dev, generator=torch.Generator(device=dev).manual_seed(5))

    def fwd(m, ids):
        if autocast:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return m(ids)
        return m(ids)

    if world > 1:
        sim.compute_encodings(lambda m, ids: fwd(m, ids), ids_all[rank:rank + 1, :-1])
        assert sim._last_calibration["sharded"], sim._last_calibration
    else:
        import aimet_amd.qc_quantize_op as QO
        stash = {}
        orig_add, orig_flush, orig_accepts = QO.StatsBatch.add, QO.StatsBatch.flush, QO.StatsBatch.accepts
        orig_end = QO.StatsBatch.end_forward

        def add(self, q, t, owned=False):   # every forward's tensors held until the end
            stash.setdefault(id(q), (q, []))[1].append(t.detach().float().clone())

        def flush(self):                    # then one update per quantizer of the concatenation
            for q, ts in stash.values():
                orig_add(self, q, torch.cat([t.reshape(-1) for t in ts]), True)
            stash.clear()
            orig_flush(self)
        QO.StatsBatch.add, QO.StatsBatch.flush, QO.StatsBatch.end_forward = add, flush, lambda self: None
        # the 16-bit (autocast) activations too, as the sharded batch takes them
        QO.StatsBatch.accepts = lambda self, q, t: self.eligible_sharded(q, t)
        sim.compute_encodings(lambda m, ids: [fwd(m, ids[i:i + 1]) for i in range(UNION)], ids_all[:, :-1])
        QO.StatsBatch.add, QO.StatsBatch.flush, QO.StatsBatch.accepts = orig_add, orig_flush, orig_accepts
        QO.StatsBatch.end_forward = orig_end
    assert sum(isinstance(w, LearnedGridQuantWrapper) for w in sim.model.modules()) >= 2 * 7 + 1
    net = sim.model
    net.train()
    if world > 1:
        # rank r: sequence r; DDP averages the ranks' gradients
        mine = ids_all[rank:rank + 1]
        ddp = torch.nn.parallel.DistributedDataParallel(net)
        logits = fwd(ddp, mine[:, :-1])
        loss = F.cross_entropy(logits.float().reshape(-1, VOCAB), mine[:, 1:].reshape(-1))
        loss.backward()
    else:
        # one process, the union batch as UNION micro-batches of one sequence with gradient
        # accumulation (loss / UNION each): the very GEMM shapes of the ranks, so the forward values
        # are the ranks' bit for bit, and g0 / 2 + g1 / 2 is what DDP forms ((g0 + g1) / 2, the
        # halving exact)
        loss = 0.0
        for i in range(UNION):
            seq = ids_all[i:i + 1]
            logits = fwd(net, seq[:, :-1])
            li = F.cross_entropy(logits.float().reshape(-1, VOCAB), seq[:, 1:].reshape(-1)) / UNION
            li.backward()
            loss = loss + li.detach()
    torch.cuda.synchronize()
    out = {"loss": float(loss)}
    gen = torch.Generator().manual_seed(11)
    for name, p in net.named_parameters():
        if p.grad is None:
            out[name] = None
            continue
        gr = p.grad.detach().float().reshape(-1).cpu()
        if "_encoding_" in name:
            out[name] = {"full": gr.tolist()}
        else:
            idx = torch.randint(gr.numel(), (4096,), generator=gen)
            out[name] = {"sample": gr[idx].tolist(), "norm": float(gr.double().norm())}
    with open(os.environ["OUT"] + ".%d" % rank, "w") as f:
        json.dump(out, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
