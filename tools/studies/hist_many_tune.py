"""Tuning tool: time the batched histogram pass (aimet_tq_batch_histogram_many) over ResNet-50
bs256's 55 activation tensors with HIP events. Block size / elements per block come from
AIMET_TUNE_HIST_BLOCK / AIMET_TUNE_HIST_ELEMS (read once per process: run one process per setting)."""
import os
import sys

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
    acts, _ = bench.collect_tensors(model, x)
    del model
    ts = [t for _, t in acts]
    n = sum(t.numel() for t in ts)
    qs = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in ts]
    AimetTensorQuantizer.batch_minmax_many(qs, ts)
    AimetTensorQuantizer.fold_minmax_many(qs)
    ms = []
    for r in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        AimetTensorQuantizer.batch_histogram_many(qs, ts)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
        AimetTensorQuantizer.fold_histogram_many(qs, [t.numel() for t in ts])
    ms.sort()
    med = ms[len(ms) // 2]
    print("block %s elems %s: %.3f ms  %.1f GB/s" % (os.environ.get("AIMET_TUNE_HIST_BLOCK", "256"),
                                                    os.environ.get("AIMET_TUNE_HIST_ELEMS", "131072"), med,
                                                    4 * n / med / 1e6), flush=True)


if __name__ == "__main__":
    main()
