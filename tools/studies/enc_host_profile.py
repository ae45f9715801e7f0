"""Host-side timeline of bench.py's compute_encodings (ResNet-50 bs256, TF-E activations + per-channel
TF-E weights): the wall-clock of every phase of aimet_amd.calibration.compute_encodings_resident
with NO extra synchronisation, so the numbers show where the host spends the time between the
launches (tuning tool; GPU kernel time comes from rocprofv3)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from aimet_amd import calibration as CAL  # noqa: E402
from aimet_amd import distributed as D  # noqa: E402
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402
from workloads.resnet import resnet50  # noqa: E402


def one(acts, weights, dev, qs=None):
    """qs None: new quantizers (constructed + created in the call); else (aq, wq) reset."""
    TFE = QuantizationMode.QUANTIZATION_TF_ENHANCED
    t = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()

    def mark(k):
        t.append((k, time.perf_counter()))
    if qs is None:
        aq = [AimetTensorQuantizer(TFE) for _ in acts]
        wq = [AimetTensorQuantizer(TFE, num_channels=w.shape[0]) for w in weights]
        mark("construct")
    else:
        aq, wq = qs
        AimetTensorQuantizer.resetEncodingStatsMany(aq + wq)
        mark("reset_many")
    torch.cuda.synchronize(dev)
    mark("sync_in")
    AimetTensorQuantizer._ensure_many(aq + wq, dev)
    mark("ensure_many")
    side = CAL._side_stream(dev)
    with torch.cuda.stream(side):
        keep = AimetTensorQuantizer.updateStatsPerChannelMany(wq, weights)
        mark("w_update_launch")
        pw = AimetTensorQuantizer.getEncodingsAsync(wq, 8, True, False, False)
        mark("w_getencs_launch")
    D.sharded_update_stats(aq, acts)
    mark("act_update_launch")
    pa = AimetTensorQuantizer.getEncodingsAsync(aq, 8, False, False, False)
    mark("act_getencs_launch")
    pw.result()
    mark("w_result(waits side)")
    del keep
    pa.result()
    mark("act_result(waits main)")
    torch.cuda.synchronize(dev)
    mark("sync_out")
    prev, parts = t0, []
    for k, v in t:
        parts.append("%s %.3f" % (k, (v - prev) * 1e3))
        prev = v
    return (prev - t0) * 1e3, parts, aq, wq


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
    acts, weights = bench.collect_tensors(model, x)
    del model
    acts = [a for _, a in acts]
    weights = [w for _, w in weights]
    keep = None
    for rep in range(4):
        del keep
        total, parts, aq, wq = one(acts, weights, dev)
        keep = (aq, wq)
        print("fresh rep %d total %.3f ms | %s" % (rep, total, " | ".join(parts)), flush=True)
    for rep in range(6):
        total, parts, aq, wq = one(acts, weights, dev, keep)
        print("reset rep %d total %.3f ms | %s" % (rep, total, " | ".join(parts)), flush=True)
    del keep
    for rep in range(4):
        *_, secs, aq, wq = bench.compute_encodings([("a", a) for a in acts], [("w", w) for w in weights])
        del aq, wq
        print("bench.compute_encodings rep %d: %.3f ms" % (rep, secs * 1e3), flush=True)


if __name__ == "__main__":
    main()
