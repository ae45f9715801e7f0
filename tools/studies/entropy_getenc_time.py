"""Timing tool: batched getEncodings of 55 per-tensor entropy quantizers (ResNet-50-like count);
the host KL searches run in one thread pool across quantizers."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    ts = [torch.relu(torch.randn(1 << 20, device="cuda", generator=g) * (1 + i % 5)) for i in range(55)]
    qs = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY) for _ in ts]
    AimetTensorQuantizer.updateStatsMany(qs, ts)
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        AimetTensorQuantizer.getEncodings(qs, 8, False, False, False)
        t1 = time.perf_counter()
        [q.getEncoding(8, False, False, False) for q in qs]
        t2 = time.perf_counter()
        print("55 entropy quantizers: batched %.1f ms, one by one %.1f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3),
              flush=True)


if __name__ == "__main__":
    main()
