"""AdaRound loop, 1x1 layers at 14x14 / 7x7 (MobileNet-v2): per-iteration time of the channel-major
step on the f32 matrix cores (aimet_adaround_pw_cm_forward + _wgrad + backward_adam_parts) against
the library-GEMM chain it replaces (gather_cm + mm + recon_grad_indexed_cm + mm + backward_adam),
both captured in a HIP graph and replayed. Prints one JSON line per layer shape.

    python tools/studies/pw_cm_bench.py [--reps 200]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aimet_amd import _native  # noqa: E402

SHAPES = [(64, 384, 196), (384, 64, 196), (96, 576, 196), (576, 96, 196), (160, 960, 49), (960, 160, 49),
          (960, 320, 49), (192, 64, 196)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--nb", type=int, default=32)
    ap.add_argument("--forms", default="mfma,library")
    ap.add_argument("--shapes", default="", help="indices into SHAPES, comma-separated (default: all)")
    ap.add_argument("--seq", action="store_true", help="batch rows 0 .. nb-1 every iteration (no random gather)")
    args = ap.parse_args()
    shapes = [SHAPES[int(i)] for i in args.shapes.split(",")] if args.shapes else SHAPES
    lib = _native.load()
    dev = torch.device("cuda", 0)
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
    nb, rows, iters = args.nb, 256, args.reps + 8
    for cin, cout, hw in shapes:
        g = torch.Generator(device=dev).manual_seed(cin + cout)
        x = torch.rand(rows, cin, hw, device=dev, generator=g)
        t = torch.randn(rows, cout, hw, device=dev, generator=g)
        w = torch.randn(cout, cin, device=dev, generator=g) * 0.05
        bias = torch.randn(cout, device=dev, generator=g) * 0.1
        if args.seq:
            idx = torch.arange(nb, device=dev).repeat(iters, 1).contiguous()
        else:
            idx = torch.stack([torch.randperm(rows, device=dev, generator=g)[:nb] for _ in range(iters)]).contiguous()
        d = (w.abs().amax(1) / 127).contiguous()
        o = torch.full((cout,), -128.0, device=dev)
        rb = torch.tensor([[0.01, 10.0, 9.0]] * iters, device=dev)
        adam = (ctypes.c_double(1e-3), ctypes.c_double(0.9), ctypes.c_double(0.999), ctypes.c_double(1e-8))
        res = {"cin": cin, "cout": cout, "hw": hw, "nb": nb, "seq": args.seq}
        for form in args.forms.split(","):
            alpha = torch.randn(cout, cin, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
            m, v = torch.zeros_like(alpha), torch.zeros_like(alpha)
            wq = w.clone()
            ctr = torch.zeros(2, dtype=torch.long, device=dev)
            it_cur, it_next = ctypes.c_void_p(ctr.data_ptr()), ctypes.c_void_p(ctr.data_ptr() + 8)
            if form == "mfma":
                sl = ctypes.c_int64()
                _native.check(lib.aimet_adaround_pw_cm_wgrad_slices(nb, cin, cout, hw, ctypes.byref(sl)))
                g_cm = torch.empty(cout, nb * hw, device=dev)
                parts = torch.empty(sl.value, cout, cin, device=dev)
                res["slices"] = sl.value

                def step(s):
                    _native.check(lib.aimet_adaround_pw_cm_forward(P(x), P(t), P(idx), it_cur, it_next, P(wq), P(bias),
                                                                   P(g_cm), nb, cin, cout, hw, 2, s))
                    _native.check(lib.aimet_adaround_pw_cm_wgrad(P(x), P(idx), it_cur, P(g_cm), P(parts), sl.value, nb,
                                                                 cin, cout, hw, s))
                    _native.check(lib.aimet_adaround_backward_adam_parts(P(w), P(alpha), P(parts), sl.value, 0, P(m), P(v),
                                                                         1, cout, cin, P(d), P(o), 8, P(rb), it_next,
                                                                         it_cur, *adam, None, P(wq), None, s))
            else:
                x_cm = torch.empty(cin, nb * hw, device=dev)
                q_cm = torch.empty(cout, nb * hw, device=dev)
                g_cm = torch.empty_like(q_cm)

                def step(s):
                    _native.check(lib.aimet_adaround_gather_cm(P(x), P(x_cm), P(idx), it_cur, it_next, nb, cin, hw, s))
                    torch.mm(wq, x_cm, out=q_cm)
                    _native.check(lib.aimet_adaround_recon_grad_indexed_cm(P(q_cm), P(t), P(idx), it_cur, P(g_cm), nb,
                                                                           cout, hw, P(bias), 2, s))
                    gw = torch.mm(g_cm, x_cm.t())
                    _native.check(lib.aimet_adaround_backward_adam(P(w), P(alpha), P(gw), P(m), P(v), 1, cout, cin,
                                                                   P(d), P(o), 8, P(rb), it_next, it_cur, *adam, None,
                                                                   P(wq), s))
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(3):
                    step(ctypes.c_void_p(side.cuda_stream))
            torch.cuda.current_stream(dev).wait_stream(side)
            ctr.zero_()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                step(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
            ctr.zero_()
            for _ in range(3):
                graph.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                graph.replay()
            e1.record()
            e1.synchronize()
            res[form + "_us"] = round(e0.elapsed_time(e1) / args.reps * 1e3, 2)
            res[form + "_alpha_checksum"] = float(alpha.double().sum())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
