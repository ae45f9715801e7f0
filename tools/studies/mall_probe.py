"""Does the histogram pass gain when its tensor is still in the Infinity Cache (MALL, 256 MiB)?
For tensors of 32-1024 MB: time batch_histogram_many right after batch_minmax_many of the SAME
tensor (warm: the min/max pass just streamed it) and after a min/max pass over an unrelated 2 GB
tensor (cold). Also the reverse-order effect is not measurable here (the kernel's block order is
fixed); this only bounds what a cache-aware schedule can gain."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer as Q  # noqa: E402

dev = torch.device("cuda", 0)
big = torch.randn(512 << 20, device=dev)   # 2 GB flush tensor
flush_q = Q(QuantizationMode.QUANTIZATION_TF)


def ev():
    return torch.cuda.Event(enable_timing=True)


def run(mb, warm, reps=5):
    n = mb * (1 << 20) // 4
    x = torch.randn(n, device=dev)
    out_mm, out_h = [], []
    for _ in range(reps):
        q = Q(QuantizationMode.QUANTIZATION_TF_ENHANCED)
        if warm:
            a, b, c = ev(), ev(), ev()
            a.record()
            q.batch_minmax(x)
            q.fold_minmax()
            b.record()
            q.batch_histogram(x)
            c.record()
        else:
            q.batch_minmax(x)
            q.fold_minmax()
            flush_q.batch_minmax(big)   # evict
            a, b, c = ev(), ev(), ev()
            a.record()
            b.record()
            q.batch_histogram(x)
            c.record()
        torch.cuda.synchronize()
        out_mm.append(a.elapsed_time(b))
        out_h.append(b.elapsed_time(c))
    h = sorted(out_h)[len(out_h) // 2]
    m = sorted(out_mm)[len(out_mm) // 2]
    return h, mb * (1 << 20) / (h * 1e-3) / 1e12, m


for mb in (32, 64, 128, 192, 256, 512, 1024):
    hw, bw, m = run(mb, True)
    hc, bc, _ = run(mb, False)
    print("%5d MB  minmax %.3f ms (%.2f TB/s) | histogram after its own min/max: %.3f ms (%.2f TB/s)   cold: %.3f ms "
          "(%.2f TB/s)  gain %.1f%%" % (mb, m, mb * (1 << 20) / (m * 1e-3) / 1e12, hw, bw, hc, bc, 100 * (hc - hw) / hc),
          flush=True)
