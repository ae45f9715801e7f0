"""Study: how far the fused AdaRound loop ends from the reference's torch-op
loop after 10k iterations, on three MobileNet-v2 layers (the stem conv, a depthwise conv, a
pointwise conv) -- the fraction of hard-rounding decisions (alpha >= 0) that differ.

Both loops get the same cached activations (256 images U(0,1), seed 7), the same per-tensor 8-bit
TF-Enhanced weight encoding, the same initial alpha and the same batch draws (torch.randperm from
generators with one seed). The reference loop is adaround_optimizer.py:115-221 restated with torch
ops on the GPU (AdaroundWrapper.apply_adaround, AdaroundLoss, torch.optim.Adam default), as the
reference runs AdaRound on a CUDA device. A second run of the fused loop checks determinism.
Prints one JSON line."""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=10000)
    ap.add_argument("--images", type=int, default=256)
    args = ap.parse_args()
    from aimet_amd.adaround import compute_beta, init_alpha
    from aimet_amd.adaround_optimizer import AdaroundHyperParameters, AdaroundOptimizer, layer_forward, recon_loss
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    from oracle import torch_ref as T
    from workloads.mobilenet_v2 import mobilenet_v2

    dev = torch.device("cuda", 0)
    fp = mobilenet_v2(seed=0, device=dev)
    images = torch.rand(args.images, 3, 224, 224, generator=torch.Generator().manual_seed(7)).to(dev)
    mods = dict(fp.named_modules())
    layers = ["features.0.0" if "features.0.0" in mods else "features.0", "features.2.conv.0", "features.3.conv.0"]
    layers = [n for n in layers if n in mods]
    params = AdaroundHyperParameters(num_iterations=args.iterations)
    rows = []
    for name in layers:
        m = mods[name]
        if not isinstance(m, (torch.nn.Conv2d, torch.nn.Linear)):
            m = next(c for c in m.modules() if isinstance(c, torch.nn.Conv2d))
        ins, outs = [], []
        h = m.register_forward_hook(lambda mod, i, o: (ins.append(i[0].detach()), outs.append(o.detach())) and None)
        with torch.no_grad():
            for b in range(0, args.images, 64):
                fp(images[b:b + 64])
        h.remove()
        inp, out = torch.cat(ins), torch.cat(outs)
        w = m.weight.detach()
        q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
        q.updateStats(w.contiguous().view(-1), True)
        e, _ = q.getEncoding(8, True, False, False)
        d = torch.tensor([e.delta], dtype=torch.float32, device=dev)
        o = torch.tensor([e.offset], dtype=torch.float32, device=dev)
        act = torch.nn.ReLU6()
        ours = AdaroundOptimizer.optimize_rounding(m, inp, out, d, o, 8, 0, params, act,
                                                   torch.Generator().manual_seed(11)).detach().clone()
        again = AdaroundOptimizer.optimize_rounding(m, inp, out, d, o, 8, 0, params, act,
                                                    torch.Generator().manual_seed(11)).detach().clone()
        # the reference's loop (torch ops, default Adam, the same draws)
        a_ref = init_alpha(w, d)
        opt = torch.optim.Adam([a_ref])
        gen = torch.Generator().manual_seed(11)
        for it in range(args.iterations):
            idx = torch.randperm(inp.shape[0], generator=gen)[:32].to(dev)
            x, target = inp.index_select(0, idx), out.index_select(0, idx)
            opt.zero_grad()
            qo = layer_forward(m, x, T.adaround_forward(w, a_ref, d, o, 8))
            loss = recon_loss(act(qo), act(target))
            if it >= params.num_iterations * params.warm_start:
                loss = loss + T.adaround_round_loss(a_ref, params.reg_param,
                                                    compute_beta(params.num_iterations, it, params.beta_range,
                                                                 params.warm_start))
            loss.backward()
            opt.step()
        ref = a_ref.detach()
        hard_o, hard_r = ours >= 0, ref >= 0
        rows.append({"layer": name, "weight_shape": list(w.shape), "elements": w.numel(),
                     "loop_form": AdaroundOptimizer.last_loop_form,
                     "hard_rounding_differs": int((hard_o != hard_r).sum()),
                     "hard_rounding_differs_frac": round(float((hard_o != hard_r).float().mean()), 6),
                     "alpha_max_abs_diff": float((ours - ref).abs().max()),
                     "alpha_median_abs": float(ref.abs().median()),
                     "rerun_bit_identical": bool(torch.equal(ours, again))})
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"study": "fused AdaRound loop vs the reference's torch-op loop (GPU), 10k iterations",
                      "iterations": args.iterations, "images": args.images, "layers": rows}), flush=True)


if __name__ == "__main__":
    main()
