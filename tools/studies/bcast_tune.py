"""Timing of the blockwise (broadcast) QDQ kernels at 2^28 fp32 elements, 64-element blocks:
[4096 x 65536] with blocks along the inner dim (contiguous: bcast_vec_kernel) and its transpose
[65536 x 4096] with blocks along the outer dim (strided: bcast_colblock_kernel); 8 B/elem
algorithmic. A checksum of the output bits compares study builds (--lib).
usage: bcast_tune.py [--lib PATH] [--tag T] [--reps R]"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tag", default="")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import aimet_amd._native as nat
    if args.lib:
        nat.LIB_PATH = os.path.abspath(args.lib)
    import aimet_amd
    from aimet_amd.onnx_op import BroadcastShapeInfo
    lib = aimet_amd.native_library()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    N, C = 1 << 28, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, device=dev, generator=g) * 2 + 0.3
    y = torch.empty_like(x)
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
    for shape, ch, ba in (((C, N // C), 0, 1), ((N // C, C), 1, 0)):
        info = BroadcastShapeInfo(shape, ch, ba, 64)
        E = info.numEncodings
        etab = torch.empty(4, E, device=dev)
        etab[2].uniform_(0.01, 0.02, generator=g)
        etab[3].fill_(-8.0)
        etab[0] = etab[2] * -8
        etab[1] = etab[2] * 7
        nd = info.numDims
        ts = (ctypes.c_int64 * nd)(*info.tensorStrides)
        es = (ctypes.c_int64 * nd)(*info.encodingStrides)

        def run():
            lib.aimet_qdq_broadcast(P(x), P(y), N, nd, ts, es, P(etab[0]), P(etab[1]), P(etab[2]), P(etab[3]), sp)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.reps):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        gbs = 8.0 * N / (ms * 1e-3) / 1e9
        print(json.dumps({"tag": args.tag, "shape": list(shape), "blocks": "contiguous" if info.hasContiguousBlocks()
                          else "strided", "encodings": E, "avg_ms": round(ms, 4), "GBps": round(gbs, 1),
                          "frac_of_8TBps": round(gbs / 8000.0, 4),
                          "checksum": int(y.view(torch.int32).to(torch.int64).sum().item())}), flush=True)


if __name__ == "__main__":
    main()
