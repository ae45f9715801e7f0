"""Roofline of the learned-grid 16-bit activation kernels at Llama-3-8B QAT sizes (config 5,
VERDICT r02 item 4): aimet_lg_forward_16_range (4 B/elem: bf16 x in, bf16 y out) and
aimet_lg_backward_16 with the range gradients (6 B/elem: x, grad in, grad_x out), per-tensor
16-bit asymmetric encodings as QuantSim's output quantizers of every Linear.

Sizes: seq 2048 x {4096 (q / o / down outputs), 14336 (gate / up), 1024 (k / v)} and the
mean call of the QAT step (13.69 M elements: 3,081,240,576 activation elements over 225 calls,
profiles/r02/llama_qat_kernel_stats_q2.csv). HIP events on the launch stream over --reps calls.
"""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

HBM_PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--bitwidth", type=int, default=16)
    args = ap.parse_args()
    from aimet_amd import _native
    from aimet_amd.learned_grid import _RangeSpec, num_steps_of
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    out = []
    for name, n in (("seq2048x4096", 2048 * 4096), ("mean_call", 13_688_832), ("seq2048x14336", 2048 * 14336),
                    ("seq2048x1024", 2048 * 1024)):
        x = (torch.randn(n, device=dev, generator=g) * 1.3 + 0.1).to(torch.bfloat16)
        gr = torch.randn(n, device=dev, generator=g).to(torch.bfloat16)
        y, gx = torch.empty_like(x), torch.empty_like(x)
        emin = torch.tensor([-4.1], device=dev)
        emax = torch.tensor([4.7], device=dev)
        enc = torch.empty(4, 1, device=dev)
        sums = torch.empty(3, device=dev)
        gmin, gmax = torch.empty(1, device=dev), torch.empty(1, device=dev)
        steps = num_steps_of(args.bitwidth, False, False)
        spec = ctypes.byref(_RangeSpec(enc[2].data_ptr(), enc[3].data_ptr(), enc[0].data_ptr(), gmin.data_ptr(),
                                       gmax.data_ptr(), 0))

        def fwd():
            _native.call("aimet_lg_forward_16_range", x.data_ptr(), y.data_ptr(), n, 2, emin.data_ptr(),
                         emax.data_ptr(), args.bitwidth, 0, 0, 0, enc[0].data_ptr(), enc[1].data_ptr(),
                         enc[2].data_ptr(), sp)

        def bwd():
            _native.call("aimet_lg_backward_16", x.data_ptr(), gr.data_ptr(), gx.data_ptr(), sums.data_ptr(), n, 2,
                         enc[0].data_ptr(), enc[1].data_ptr(), ctypes.c_float(steps), spec, sp)

        cp = torch.empty_like(x)

        def copy():   # the same bytes as the forward: one 16-bit read + one write (torch's copy kernel)
            cp.copy_(x)

        def add():    # the same bytes as the backward: two 16-bit reads + one write
            torch.add(x, gr, out=cp)

        for label, fn, nbytes in (("lg_forward_16", fwd, 4), ("lg_backward_16", bwd, 6),
                                  ("control_copy", copy, 4), ("control_add", add, 6)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                fn()
            e1.record(stream)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            gbs = n * nbytes / (us * 1e-6) / 1e9
            r = {"kernel": label, "size": name, "elems": n, "bytes_per_elem": nbytes, "bitwidth": args.bitwidth,
                 "us_per_call": round(us, 2), "achieved_GBps": round(gbs, 1), "frac_of_peak": round(gbs / HBM_PEAK, 3)}
            out.append(r)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
