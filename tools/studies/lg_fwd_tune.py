"""The learned-grid forward of a float32 weight with its per-channel encodings formed in the kernel
and the result cast to bf16 (aimet_lg_forward_range, lg_fwd_kernel<IO_BF16>: the Llama-3-8B W4A16
QAT weight path) at Llama-3-8B's weight shapes: HBM rate per shape (6 B per element: 4 read, 2
written). Prints one JSON line per shape; `checksum` lets builds be compared bit for bit.

    python tools/studies/lg_fwd_tune.py [--reps R] [--tag NAME] [--lib PATH] [--out f32|bf16]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import aimet_amd  # noqa: E402

SHAPES = {"q_o_proj": (4096, 4096), "k_v_proj": (1024, 4096), "gate_up_proj": (14336, 4096),
          "down_proj": (4096, 14336), "lm_head": (128256, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default="")
    ap.add_argument("--lib", default=None)
    ap.add_argument("--out", default="bf16", choices=["f32", "bf16"])
    args = ap.parse_args()
    if args.lib:
        aimet_amd._native.LIB_PATH = os.path.abspath(args.lib)
    lib = aimet_amd.native_library()
    dev = torch.device("cuda", 0)
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    out_code, ysz = (2, 2) if args.out == "bf16" else (0, 4)
    for name, (C, K) in SHAPES.items():
        g = torch.Generator(device=dev).manual_seed(0)
        w = torch.randn(C, K, device=dev, generator=g) * 0.02
        emax = w.abs().amax(1)
        emin = -emax
        y = torch.empty(C, K, device=dev, dtype=torch.bfloat16 if args.out == "bf16" else torch.float32)
        d_out = torch.empty(C, device=dev)
        o_out = torch.empty(C, device=dev)

        def call():
            rc = lib.aimet_lg_forward_range(P(w), P(y), 1, C, K, out_code, P(emin), P(emax), 4, 1, 0, 0, P(d_out),
                                            P(o_out), None, s)
            assert rc == 0, rc
        call()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(args.reps):
            call()
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / args.reps
        nbytes = (4 + ysz) * C * K
        gbps = nbytes / ms / 1e6
        bits = y.view(torch.int16 if args.out == "bf16" else torch.int32).to(torch.int64)
        print(json.dumps({"kernel": "lg_fwd_kernel", "tag": args.tag, "out": args.out, "shape": name, "C": C, "K": K,
                          "avg_us": round(ms * 1e3, 2), "achieved_GBps": round(gbps, 1),
                          "frac_of_peak": round(gbps / 8000, 4), "checksum": int(bits.sum().item())}), flush=True)


if __name__ == "__main__":
    main()
