"""AdaRound backward kernel (aimet_adaround_backward, adaround_bwd_vec_kernel) at 2^28 elements:
HBM rate for alpha drawn N(0, s^2) -- s = 1: ~2 % of the rectified sigmoids saturate, s = 4: ~55 % --
with the round-loss value requested (want_loss) or not (the optimisation loop's form). Prints one
JSON line per case; `checksum` (sum of the gradient's bit patterns) lets runs of different kernel
forms be compared bit for bit (--tag names the form in the output).

    python tools/studies/ada_bwd_tune.py [--elems N] [--reps R] [--tag NAME] [--lib PATH] [--reg R] [--skew BYTES]
"""
import argparse
import ctypes
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import aimet_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=1 << 28)
    ap.add_argument("--channels", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--scales", default="1,4")
    ap.add_argument("--tag", default="")
    ap.add_argument("--reg", type=float, default=0.01, help="reg_param (0: no rounding loss, no pow)")
    ap.add_argument("--lib", default=None, help="another build of libaimet_amd.so")
    ap.add_argument("--skew", type=int, default=0, help="start buffer k (w, grad, out, alpha) k x SKEW bytes into its allocation")
    ap.add_argument("--exact-pow", action="store_true", help="the bit-exact Sleef pow instead of the fast (table-driven f32) pow")
    args = ap.parse_args()
    if args.lib:
        aimet_amd._native.LIB_PATH = os.path.abspath(args.lib)
    lib = aimet_amd.native_library()
    lib.aimet_adaround_set_exact_pow(1 if args.exact_pow else 0)
    dev = torch.device("cuda", 0)
    N, C = args.elems, args.channels
    K = N // C
    g = torch.Generator(device=dev).manual_seed(0)
    assert args.skew % 16 == 0

    def buf(k):   # N floats starting k x skew bytes into a fresh allocation
        off = k * args.skew // 4
        return torch.empty(N + off, device=dev)[off:]

    w = buf(0).copy_(torch.randn(N, device=dev, generator=g) * 0.05)
    grad = buf(1).copy_(torch.randn(N, device=dev, generator=g))
    out = buf(2)
    delta = (w.view(C, K).abs().amax(1) / 127).contiguous()
    offset = torch.full((C,), -128.0, device=dev)
    rloss = torch.zeros(1, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    for scale in [float(v) for v in args.scales.split(",")]:
        alpha = buf(3).copy_(torch.randn(N, device=dev, generator=torch.Generator(device=dev).manual_seed(1)) * scale)
        sat = float((alpha.abs() > math.log(11.0)).float().mean())
        for want_loss in (True, False):
            def call():
                if want_loss:
                    rloss.zero_()
                rc = lib.aimet_adaround_backward(P(w), P(alpha), P(grad), P(out), 1, C, K, P(delta), P(offset), 8,
                                                 ctypes.c_double(args.reg), ctypes.c_double(10.0),
                                                 P(rloss) if want_loss else None, s)
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
            gbps = 16 * N / ms / 1e6
            print(json.dumps({"kernel": "adaround_bwd_vec_kernel", "tag": args.tag, "reg": args.reg, "skew": args.skew,
                              "pow": "exact" if args.exact_pow else "fast", "elems": N, "alpha_scale": scale,
                              "saturated_frac": round(sat, 4), "want_loss": want_loss, "avg_ms": round(ms, 4),
                              "achieved_GBps": round(gbps, 1), "frac_of_peak": round(gbps / 8000, 4),
                              "checksum": int(out.view(torch.int32).to(torch.int64).sum().item()),
                              "round_loss": float(rloss.item()) if want_loss else None}), flush=True)


if __name__ == "__main__":
    main()
