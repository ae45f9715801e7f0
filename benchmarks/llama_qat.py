"""Config 5 (BASELINE.json / SURVEY §8(d)): Llama-3-8B W4A16 QAT with learned-grid (range
learning) per-channel 4-bit symmetric weight quantizers, seq 2048, micro-batch 1 per GPU.

  python benchmarks/llama_qat.py [--layers 32] [--path quantsim|module] [--impl fused|reference]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 benchmarks/llama_qat.py

--path quantsim (default): the reference's workflow. QuantizationSimModel(model,
  quant_scheme=training_range_learning_with_tf_init, default_param_bw=4, default_output_bw=16,
  per-channel symmetric params) wraps every linear layer (q/k/v/o, gate/up/down, lm_head);
  compute_encodings calibrates them on one batch (TF, static grid), then QuantSim swaps in
  LearnedGridQuantWrapper: each linear quantize-dequantizes its fp32 master weight (4-bit,
  learnable per-output-channel range) and its output (16-bit, learnable per-tensor range) with
  the fused learned-grid kernels; matmuls run in bf16 (torch.autocast); Adam (fused) updates
  weights and ranges.
  --impl reference: the same QuantSim with the reference's torch-op QuantizeDequantizeFunc for
  every learned-grid quantizer (RefQuantizeDequantize), for a like-for-like step time.
--path module: the weight-only hand-built QAT linear of round 1 (no activation quantizers):
  --impl fused      aimet_amd's learned-grid kernels (one forward pass, one backward pass per weight)
  --impl reference  the reference's torch-op QuantizeDequantizeFunc (v1/tensor_quantizer.py:896-986 over
                    quantsim_straight_through_grad.py:121-347, restated in oracle/torch_ref.py)
Unit of work = weight QDQ + STE elements per step (forward + backward over all linear weights);
the activation elements quantized per step are reported beside it.
Synthetic data: random token ids, random-init weights N(0, 0.02) (seed 0).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

BITWIDTH = 4


class RefLearnedGrid(torch.autograd.Function):
    """The reference's QuantizeDequantizeFunc with symmetric per-channel encodings: forward saves
    the mask and x_quant, backward = symmetric_gradients (quantsim_straight_through_grad.py)."""

    @staticmethod
    def forward(ctx, x, emin, emax):
        from oracle import torch_ref as T
        y, mask, x_quant, delta, offset, steps = T.lg_forward(x, emin, emax, BITWIDTH, True)
        ctx.save_for_backward(x, mask, x_quant, delta, offset)
        ctx.steps = steps
        return y

    @staticmethod
    def backward(ctx, grad):
        x, mask, x_quant, delta, offset = ctx.saved_tensors
        grad_x = mask * grad
        gmax = ((x_quant + offset) * grad).sum(dim=1) - (mask * (x / delta) * grad).sum(dim=1)
        gmax = gmax / torch.div(ctx.steps, 2, rounding_mode="floor")
        return grad_x, -gmax, gmax


class RefQuantizeDequantize(torch.autograd.Function):
    """--path quantsim --impl reference: the reference's QuantizeDequantizeFunc for every quantizer
    QuantSim wraps (4-bit per-channel weights AND 16-bit per-tensor outputs), torch ops in float32
    (v1/tensor_quantizer.py:896-986 over quantsim_straight_through_grad.py:191-328): the forward saves
    mask and x_quant, the backward forms grad_x and the range gradients from them. Swapped in for
    aimet_amd.learned_grid.LearnedGridQuantizeDequantize (same apply signature; `out_dtype`, the
    dtype autocast would cast the result to, is applied as that cast after the float32 result)."""

    @staticmethod
    def forward(ctx, x, emin, emax, bw, sym=False, strict=False, unsigned=False, ch_axis=0, out_dtype=None):
        from oracle import torch_ref as T
        x32 = x.float()
        y, mask, x_quant, delta, offset, steps = T.lg_forward(x32, emin.float(), emax.float(), bw, sym, strict,
                                                              unsigned, ch_axis)
        ctx.save_for_backward(x32, mask, x_quant, delta, offset, emin, emax)
        ctx.meta = (sym, steps, ch_axis, x.dtype)
        return y.to(x.dtype).to(out_dtype if out_dtype is not None else x.dtype)

    @staticmethod
    def backward(ctx, grad):
        x, mask, x_quant, delta, offset, emin, emax = ctx.saved_tensors
        sym, steps, ch_axis, dtype = ctx.meta
        g = grad.float()
        grad_x = (mask * g).to(dtype)
        dims = list(range(x.dim()))
        if emin.numel() > 1:
            dims.pop(ch_axis)
        if sym:
            gmax = ((x_quant + offset) * g).sum(dim=dims) - (mask * (x / delta) * g).sum(dim=dims)
            gmax = gmax / torch.div(steps, 2, rounding_mode="floor")
            return grad_x, (-gmax).view_as(emin), gmax.view_as(emax), None, None, None, None, None, None
        grad_scale = (x_quant + offset - x * mask / delta) * g
        grad_offset = (delta * g) * (~mask)
        t1 = grad_scale.sum(dim=dims) / steps
        t2 = steps / (emax - emin) ** 2 * grad_offset.sum(dim=dims)
        return grad_x, (-t1 + emax * t2).view_as(emin), (t1 - emin * t2).view_as(emax), None, None, None, None, None, None


class QatLinear(nn.Module):
    impl = "fused"

    def __init__(self, fin, fout):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(fout, fin))
        self.encoding_min = nn.Parameter(torch.empty(fout))
        self.encoding_max = nn.Parameter(torch.empty(fout))

    def forward(self, x):
        if QatLinear.impl == "fused":
            from aimet_amd.learned_grid import LearnedGridQuantizeDequantize
            wq = LearnedGridQuantizeDequantize.apply(self.weight, self.encoding_min, self.encoding_max, BITWIDTH, True,
                                                     False, False, 0)
        else:
            wq = RefLearnedGrid.apply(self.weight, self.encoding_min, self.encoding_max)
        return F.linear(x, wq)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--impl", choices=["fused", "reference"], default="fused")
    ap.add_argument("--path", choices=["quantsim", "module", "plain"], default="quantsim",
                    help="plain: the same model and step without any quantizer (the floor QAT adds to)")
    ap.add_argument("--act-bw", type=int, default=16)
    ap.add_argument("--profile-calib", action="store_true",
                    help="print a cProfile of QuantizationSimModel.compute_encodings (top functions by own time)")
    ap.add_argument("--dump-first", default=None,
                    help="save the first step's loss, per-parameter weight-gradient sums and the encoding "
                         "range gradients to this path (full-size parity of --impl fused vs reference: "
                         "tools/studies/llama_first_step_compare.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    from workloads.llama import Llama

    QatLinear.impl = args.impl
    torch.manual_seed(0)
    linear_type = QatLinear if args.path == "module" else nn.Linear
    linear_cls = QatLinear if args.path == "module" else (lambda i, o: nn.Linear(i, o, bias=False))
    with torch.device(dev):
        model = Llama(linear_cls, layers=args.layers)
    qlin = [m for m in model.modules() if isinstance(m, linear_type)]
    vocab = model.lm_head.weight.shape[0]
    with torch.no_grad():
        g = torch.Generator(device=dev).manual_seed(0)
        model.embed_tokens.weight.normal_(0, 0.02, generator=g)
        for m in qlin:
            m.weight.normal_(0, 0.02, generator=g)
            if args.path == "module":
                # TF per-channel symmetric init of the learnable range (QuantSim compute_encodings)
                q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF, num_channels=m.weight.shape[0])
                q.updateStatsPerChannel(m.weight, 0, True)
                encs, _ = q.getEncoding(BITWIDTH, True, False, False)
                m.encoding_min.copy_(torch.tensor([e.min for e in encs], dtype=torch.float32))
                m.encoding_max.copy_(torch.tensor([e.max for e in encs], dtype=torch.float32))
    n_weights = sum(m.weight.numel() for m in qlin)
    calib_s, n_act = None, 0
    if args.path == "quantsim":
        from aimet_amd.qc_quantize_op import LearnedGridQuantWrapper
        from aimet_amd.quantizers import QuantScheme
        from aimet_amd.quantsim import QuantizationSimModel
        if args.impl == "reference":
            import aimet_amd.learned_grid as LG
            LG.LearnedGridQuantizeDequantize = RefQuantizeDequantize
        cfg = {"defaults": {"ops": {"is_output_quantized": "True"},
                            "params": {"is_quantized": "True", "is_symmetric": "True"},
                            "strict_symmetric": "False", "per_channel_quantization": "True"}}
        sim = QuantizationSimModel(model, quant_scheme=QuantScheme.training_range_learning_with_tf_init,
                                   default_param_bw=BITWIDTH, default_output_bw=args.act_bw, in_place=True,
                                   config_file=cfg)
        cal = torch.Generator(device=dev).manual_seed(99)
        ids_cal = torch.randint(vocab, (1, args.seq), device=dev, generator=cal)
        torch.cuda.synchronize()
        t0 = time.perf_counter()

        def calibrate(m, ids):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                m(ids)
        if args.profile_calib:
            import cProfile
            import io
            import pstats
            pr = cProfile.Profile()
            pr.enable()
        sim.compute_encodings(calibrate, ids_cal)
        torch.cuda.synchronize()
        calib_s = time.perf_counter() - t0
        if args.profile_calib:
            pr.disable()
            buf = io.StringIO()
            pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
            print(buf.getvalue(), file=sys.stderr)
            buf = io.StringIO()
            pstats.Stats(pr, stream=buf).sort_stats("cumtime").print_stats(25)
            print(buf.getvalue(), file=sys.stderr)
        wrappers = [w for w in sim.model.modules() if isinstance(w, LearnedGridQuantWrapper)]
        assert len(wrappers) == len(qlin), (len(wrappers), len(qlin))
        n_act = sum(w._module_to_wrap.weight.shape[0] for w in wrappers) * args.seq
        model = sim.model
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local]) if world > 1 else model
    try:
        opt = torch.optim.Adam(model.parameters(), lr=1e-5, fused=True)
    except (RuntimeError, TypeError):
        opt = torch.optim.Adam(model.parameters(), lr=1e-5)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    first = [args.dump_first]

    def step():
        ids = torch.randint(vocab, (1, args.seq + 1), device=dev, generator=gen)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = ddp(ids[:, :-1])
        loss = F.cross_entropy(logits.float().view(-1, vocab), ids[:, 1:].reshape(-1))
        loss.backward()
        if first[0] and rank == 0:
            # the first step's results before any update: the loss, every weight gradient's float64
            # sum (in parameter order) and the encoding range gradients, for a run of each impl
            named = list(model.named_parameters())
            torch.save({"impl": args.impl, "loss": loss.detach().float().cpu(),
                        "weight_grad_sums": torch.stack([p.grad.double().sum() for n, p in named
                                                         if p.grad is not None and "encoding" not in n]).cpu(),
                        "range_grads": {n: p.grad.detach().float().cpu() for n, p in named
                                        if p.grad is not None and "encoding" in n}}, first[0])
            first[0] = None
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    if rank == 0:
        ms = dt / args.steps * 1e3
        print(json.dumps({
            "metric": "Llama-3-8B W4A16 learned-grid QAT step (weight QDQ + STE elements / s)",
            "scheme": {"quantsim": "training_range_learning_with_tf_init", "module": "hand-built QAT linear",
                       "plain": "no quantization (floor)"}[args.path],
            "value": round(2 * n_weights * world / (ms * 1e-3) / 1e9, 3), "unit": "Gelem/s", "n_gpus": world,
            "path": args.path, "impl": args.impl,
            "ms_per_step": round(ms, 2), "layers": args.layers, "seq_len": args.seq,
            "micro_batch": 1, "quantized_weight_elems": n_weights,
            "quantized_act_elems_per_step": n_act, "act_bw": args.act_bw if args.path == "quantsim" else None,
            "compute_encodings_s": None if calib_s is None else round(calib_s, 3),
            "final_loss": round(loss.item(), 4),
            "peak_mem_GB": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1),
            "data": "synthetic token ids, random-init weights N(0, 0.02) (seed 0)"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
