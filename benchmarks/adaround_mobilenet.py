"""Config 3 (BASELINE.json / SURVEY §8(d)): MobileNet-v2 W8 AdaRound on one GPU.

For every conv / linear layer in order (53 layers): cache the layer's input from the model whose
previous layers already carry their adarounded weights and the layer's output from the FP model
over 1024 images U(0,1) (seed 7); then optimise the rounding with
aimet_amd.adaround_optimizer (Adam on alpha, batch 32, 10k iterations, reg 0.01, beta 20->2,
warm start 0.2, ReLU6 applied to both outputs when the layer feeds one); then write the
hard-rounded weight. Weight encodings: 8-bit symmetric per-tensor TF-Enhanced (AIMET's AdaRound
default) from the device analyzers.

Reported (one JSON line): total AdaRound wall-clock, mean ms per iteration, and per layer its ms
per iteration and the loop form that ran it (dw: native depthwise kernels; pointwise / linear:
direct GEMMs; autograd: MIOpen through autograd -- layers with two forms time both at capture and
keep the faster); with --reference-iters the same loop using the reference's torch-op soft
quantization + rounding loss (oracle/torch_ref.py) for comparison. The per-kernel split of the
loop comes from rocprofv3 (tools/studies/ada_trace_summary.py), not from host-timed launches.
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=10000)
    ap.add_argument("--images", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=0, help="only the first N layers (0 = all)")
    ap.add_argument("--eager", action="store_true",
                    help="launch every iteration from Python instead of replaying one captured HIP graph")
    ap.add_argument("--reference-iters", type=int, default=0,
                    help="also time N iterations per layer of the torch-op reference loop")
    ap.add_argument("--exact-pow", action="store_true",
                    help="the rounding loss's bit-exact emulation of torch's pow (default: the f64 pow, within 1 ulp)")
    ap.add_argument("--miopen-find", action="store_true",
                    help="torch.backends.cudnn.benchmark: MIOpen benchmarks its convolution solvers per shape "
                         "(a fresh box has no find database; immediate mode may fall back to naive kernels)")
    args = ap.parse_args()
    if args.miopen_find:
        torch.backends.cudnn.benchmark = True

    from aimet_amd.adaround import AdaroundFunction, compute_beta, init_alpha, set_exact_pow
    from aimet_amd.adaround_optimizer import (AdaroundHyperParameters, AdaroundOptimizer, layer_forward,
                                              recon_loss)
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    from workloads.mobilenet_v2 import mobilenet_v2

    dev = torch.device("cuda", 0)
    set_exact_pow(args.exact_pow)
    fp = mobilenet_v2(seed=0, device=dev)
    qm = mobilenet_v2(seed=0, device=dev)     # receives the adarounded weights layer by layer
    images = torch.rand(args.images, 3, 224, 224, generator=torch.Generator().manual_seed(7)).to(dev)
    names = [n for n, m in fp.named_modules() if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear))]
    if args.layers:
        names = names[:args.layers]
    mods_fp, mods_q = dict(fp.named_modules()), dict(qm.named_modules())
    # the activation following each layer (AIMET applies it to both outputs)
    follow = {}
    for pname, parent in fp.named_modules():
        kids = list(parent.named_children())
        for (a, m), (_, nxt) in zip(kids, kids[1:]):
            if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear)) and isinstance(nxt, torch.nn.ReLU6):
                follow[(pname + "." + a) if pname else a] = nxt

    def cache(model, name, want_input):
        out = []
        mod = dict(model.named_modules())[name]
        h = mod.register_forward_hook(lambda m, i, o: out.append((i[0] if want_input else o).detach()))
        with torch.no_grad():
            for b in range(0, images.shape[0], 128):
                model(images[b:b + 128])
        h.remove()
        return torch.cat(out)

    params = AdaroundHyperParameters(num_iterations=args.iterations)
    gen = torch.Generator().manual_seed(0)
    loss_buf = torch.zeros(1, device=dev)
    t_opt = t_cache = t_ref = 0.0
    per_layer = []
    for name in names:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        inp = cache(qm, name, True)
        out = cache(fp, name, False)
        torch.cuda.synchronize()
        t_cache += time.perf_counter() - t0
        m = mods_q[name]
        w = m.weight.detach()
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
        q.updateStats(w.contiguous().view(-1), True)
        e, _ = q.getEncoding(8, True, False, False)
        d = torch.tensor([e.delta], dtype=torch.float32, device=dev)
        o = torch.tensor([e.offset], dtype=torch.float32, device=dev)
        act = follow.get(name)
        # untimed warm-up of this layer's shapes (MIOpen kernel selection, allocator) for both loops
        warm = AdaroundHyperParameters(num_iterations=5, warm_start=0.2)
        AdaroundOptimizer.optimize_rounding(m, inp, out, d, o, 8, 0, warm, act, torch.Generator().manual_seed(1),
                                            use_graph=not args.eager)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        alpha = AdaroundOptimizer.optimize_rounding(m, inp, out, d, o, 8, 0, params, act, gen, loss_buf,
                                                    use_graph=not args.eager)
        torch.cuda.synchronize()
        dt_ours = time.perf_counter() - t0
        t_opt += dt_ours
        per_layer.append([name, list(w.shape), round(dt_ours / args.iterations * 1e3, 4),
                          AdaroundOptimizer.last_loop_form])
        with torch.no_grad():
            m.weight.copy_(AdaroundOptimizer.hard_rounded_weight(m, alpha, d, o, 8))
        if args.reference_iters:
            from oracle import torch_ref as T
            a_ref = init_alpha(w, d)
            opt = torch.optim.Adam([a_ref])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for it in range(args.reference_iters):
                idx = torch.randperm(inp.shape[0], generator=gen)[:32].to(dev)
                x, target = inp.index_select(0, idx), out.index_select(0, idx)
                opt.zero_grad()
                wq_r = T.adaround_forward(w, a_ref, d, o, 8)
                qo = layer_forward(m, x, wq_r)
                if act is not None:
                    qo, target = act(qo), act(target)
                loss = recon_loss(qo, target)
                if it >= params.num_iterations * params.warm_start:
                    beta = compute_beta(params.num_iterations, it, params.beta_range, params.warm_start)
                    loss = loss + T.adaround_round_loss(a_ref, params.reg_param, beta)
                loss.backward()
                opt.step()
            torch.cuda.synchronize()
            t_ref += time.perf_counter() - t0
            per_layer[-1].append(round((time.perf_counter() - t0) / args.reference_iters * 1e3, 4))
        del inp, out

    iters = args.iterations * len(names)
    res = {
        "metric": "AdaRound wall-clock (MobileNet-v2, W8, all layers)",
        "value": round(t_opt, 3), "unit": "s", "higher_is_better": False, "n_gpus": 1,
        "layers": len(names), "iterations_per_layer": args.iterations, "images": args.images,
        "ms_per_iteration": round(t_opt / iters * 1e3, 4), "activation_caching_s": round(t_cache, 3),
        "loop": "eager" if args.eager else "hipgraph (one captured iteration replayed per iteration)",
        "miopen_find": bool(args.miopen_find),
        "rounding_loss_pow": "exact (torch's CPU pow, bit for bit)" if args.exact_pow else "table-driven f32 (within 1 ulp of torch's)",
        "weights_elems": sum(int(torch.Size(p[1]).numel()) for p in per_layer),
        "kernel_split": "per-kernel time of the loop: rocprofv3 --kernel-trace + tools/studies/ada_trace_summary.py "
                        "(profiles/r02/adaround_loop_kernels_*.csv)",
        "data": "synthetic U(0,1) images (seed 7), random-init MobileNet-v2 with folded BN (seed 0)",
    }
    if args.reference_iters:
        res["reference_torch_ops_ms_per_iteration"] = round(t_ref / (args.reference_iters * len(names)) * 1e3, 4)
        res["speedup_vs_reference_loop"] = round(res["reference_torch_ops_ms_per_iteration"] /
                                                 res["ms_per_iteration"], 2)
    res["per_layer_ms_per_iteration"] = per_layer   # [name, weight shape, ours, loop form(, reference)]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
