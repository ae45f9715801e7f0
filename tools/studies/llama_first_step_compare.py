"""Full-size parity of config 5: the first QAT step of `benchmarks/llama_qat.py --dump-first` run
with our kernels (--impl fused) and with the reference's torch-op QuantizeDequantize (--impl
reference), same seeds: the loss and every weight gradient's sum compared bit for bit, the encoding
range gradients as the largest error relative to each tensor's largest magnitude (their sums run
in another order than torch's reductions; the bound the tests assert is in DESIGN §2).

usage: python tools/studies/llama_first_step_compare.py fused.pt reference.pt
"""
import json
import sys

import torch


def main():
    a = torch.load(sys.argv[1], weights_only=True)
    b = torch.load(sys.argv[2], weights_only=True)
    ws_a, ws_b = a["weight_grad_sums"], b["weight_grad_sums"]
    rel = []
    for n, ga in a["range_grads"].items():
        gb = b["range_grads"][n]
        scale = max(float(gb.abs().max()), 1e-30)
        rel.append(float((ga - gb).abs().max()) / scale)
    print(json.dumps({
        "loss_fused": float(a["loss"]), "loss_reference": float(b["loss"]),
        "loss_bit_equal": bool(torch.equal(a["loss"], b["loss"])),
        "weight_grad_tensors": int(ws_a.numel()),
        "weight_grad_sums_bit_equal": int((ws_a == ws_b).sum()),
        "range_grad_tensors": len(rel),
        "range_grad_max_rel_err": max(rel) if rel else None,
        "range_grad_median_rel_err": sorted(rel)[len(rel) // 2] if rel else None}))


if __name__ == "__main__":
    main()
