"""Isolated timing of the device encoding searches (TF-Enhanced tfe_search_kernel, MSE
mse_search_kernel, entropy entropy_search_kernel) on ResNet-50's weights: 27,560 channels,
per-channel symmetric and asymmetric 8-bit, statistics computed once, then getEncodings repeated.
usage: tfe_search_time.py [--lib PATH] [TF_ENHANCED] [MSE] [ENTROPY] (--lib: another build of
libaimet_amd.so, e.g. tools/studies/ent_variants.sh's). Run under `rocprofv3 --kernel-trace --stats`
for the kernel durations; the wall-clock per batched getEncodings (search + copy + host encodings) is printed. Tuning tool."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402
from workloads.resnet import resnet50  # noqa: E402


def main():
    args = sys.argv[1:]
    if args[:1] == ["--lib"]:
        import aimet_amd._native
        aimet_amd._native.LIB_PATH = os.path.abspath(args[1])
        args = args[2:]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = resnet50(seed=0, device=dev)
    ws = [m.weight.detach().contiguous() for m in model.modules() if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear))]
    schemes = args or ["TF_ENHANCED"]
    for scheme in schemes:
        qs = [AimetTensorQuantizer(getattr(QuantizationMode, "QUANTIZATION_" + scheme), num_channels=w.shape[0])
              for w in ws]
        AimetTensorQuantizer.updateStatsPerChannelMany(qs, ws)
        torch.cuda.synchronize()
        run(scheme, qs, ws)


def run(scheme, qs, ws):
    phases(scheme, qs)
    for sym in (True, False):
        AimetTensorQuantizer.getEncodings(qs, 8, sym, False, False)   # warm
        t = []
        for _ in range(10):
            t0 = time.perf_counter()
            AimetTensorQuantizer.getEncodings(qs, 8, sym, False, False)
            t.append(time.perf_counter() - t0)
        t.sort()
        print("%s %s: %d channels, getEncodings median %.3f ms" % (scheme, "sym" if sym else "asym",
                                                                 sum(w.shape[0] for w in ws), t[len(t) // 2] * 1e3),
              flush=True)


def phases(scheme, qs):
    """launch (host enqueue), device (until the stream is done), finish (read-back, host fallbacks,
    the per-channel Python objects), medians of 10, symmetric"""
    from aimet_amd.tensor_quantizer import PendingEncodings
    AimetTensorQuantizer.getEncodings(qs, 8, True, False, False)
    t = {"launch": [], "device": [], "finish": []}
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pend = PendingEncodings(qs, 8, True, False, False)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        pend.result()
        t3 = time.perf_counter()
        t["launch"].append(t1 - t0)
        t["device"].append(t2 - t1)
        t["finish"].append(t3 - t2)
    print("%s sym phases (median ms): %s" % (scheme, {k: round(sorted(v)[5] * 1e3, 3) for k, v in t.items()}), flush=True)


if __name__ == "__main__":
    main()
