"""Time the phases of bench.py's compute_encodings (ResNet-50 bs256, TF-E act + per-channel TF-E
weights) twice: cold (first use) and warm. Tuning tool."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402
from workloads.resnet import resnet50  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
    acts, weights = bench.collect_tensors(model, x)
    del model
    TFE = QuantizationMode.QUANTIZATION_TF_ENHANCED
    for rep in range(3):
        t = {}

        def mark(k, t0):
            torch.cuda.synchronize()
            t[k] = time.perf_counter() - t0
            return time.perf_counter()
        t0 = time.perf_counter()
        aq = [AimetTensorQuantizer(TFE) for _ in acts]
        wq = [AimetTensorQuantizer(TFE, num_channels=w.shape[0]) for _, w in weights]
        t0 = mark("create", t0)
        if rep == 0:
            for q, (_, a) in zip(aq, acts):
                q.updateStats(a, True)
            t0 = mark("act_update_each", t0)
            for q in aq:
                q.resetEncodingStats()
            t0 = mark("reset", t0)
        AimetTensorQuantizer.updateStatsMany(aq, [a for _, a in acts])
        t0 = mark("act_update_many", t0)
        if rep == 0:
            for q, (_, w) in zip(wq, weights):
                q.updateStatsPerChannel(w, 0, True)
            t0 = mark("w_update_each", t0)
            for q in wq:
                q.resetEncodingStats()
            t0 = mark("w_reset", t0)
        AimetTensorQuantizer.updateStatsPerChannelMany(wq, [w for _, w in weights])
        t0 = mark("w_update_many", t0)
        if rep == 0:
            [q.getEncoding(8, False, False, False) for q in aq]
            t0 = mark("act_getenc_each", t0)
            [q.getEncoding(8, True, False, False) for q in wq]
            t0 = mark("w_getenc_each", t0)
        AimetTensorQuantizer.getEncodings(aq, 8, False, False, False)
        t0 = mark("act_getencs", t0)
        AimetTensorQuantizer.getEncodings(wq, 8, True, False, False)
        t0 = mark("w_getencs", t0)
        print("rep %d: " % rep + "  ".join("%s %.2f ms" % (k, v * 1e3) for k, v in t.items()),
              "total %.2f ms" % (sum(t.values()) * 1e3), flush=True)
        del aq, wq
    for rep in range(4):
        *_, secs, aq, wq = bench.compute_encodings(acts, weights)
        del aq, wq
        print("bench.compute_encodings rep %d: %.2f ms" % (rep, secs * 1e3), flush=True)


if __name__ == "__main__":
    main()
