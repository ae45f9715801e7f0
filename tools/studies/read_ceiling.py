"""Raw read ceiling of bench.py's 55 ResNet-50 bs256 activation tensors (tools/studies/read_ceiling.hip: one
launch, 16-KiB tiles, nontemporal 16-B loads, no reduction) against the min/max and histogram
passes of compute_encodings over the same tensors (aimet_tq_*_many), HIP-event timed."""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402
from workloads.resnet import resnet50  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "read_ceiling.so"))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
model = resnet50(seed=0, device=dev)
x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
acts, _ = bench.collect_tensors(model, x)
del model
torch.cuda.empty_cache()
ts = [t for _, t in acts]
nbytes = sum(t.numel() * 4 for t in ts)
bufs, tab, tile = [], [], 0
for k, t in enumerate(ts):
    nq = t.numel() // 4
    tiles = (nq + 1023) // 1024
    bufs.append((t.data_ptr(), nq, tile))
    tab += [k] * tiles
    tile += tiles
B = torch.tensor([v for b in bufs for v in b], dtype=torch.int64, device=dev)
T = torch.tensor(tab, dtype=torch.int32).to(torch.int16).to(dev)   # uint16 bit pattern (< 32768 buffers)
out = torch.zeros(1, device=dev)
s = torch.cuda.current_stream()


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1))
    return sorted(res)[len(res) // 2]


ms_raw = timed(lambda: lib.read_many(ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(T.data_ptr()), ctypes.c_int64(tile),
                                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s.cuda_stream)))
gate = torch.zeros(len(ts), dtype=torch.int32, device=dev)
part = torch.empty(tile * 4, 2, device=dev)
ms_v = {}
for v in (1, 2, 3):
    ms_v[v] = timed(lambda v=v: lib.mm_many_v(v, ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(T.data_ptr()),
                                              ctypes.c_int64(tile), ctypes.c_void_p(gate.data_ptr()),
                                              ctypes.c_void_p(part.data_ptr()), ctypes.c_void_p(s.cuda_stream)))
qs = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in ts]
AimetTensorQuantizer._ensure_many(qs, dev)


def minmax():
    AimetTensorQuantizer.resetEncodingStatsMany(qs)
    AimetTensorQuantizer.batch_minmax_many(qs, ts)


def both():
    AimetTensorQuantizer.resetEncodingStatsMany(qs)
    AimetTensorQuantizer.updateStatsMany(qs, ts)


ms_mm = timed(minmax)
ms_both = timed(both)
gb = nbytes / 1e9
print("activation bytes %.3f GB" % gb)
print("raw read (16-KiB tiles, nt loads, no reduction): %.3f ms  %.2f TB/s" % (ms_raw, gb / ms_raw))
for v, name in ((1, "+ block min/max, partial per tile"), (2, "+ a gate load (like pdf_init)"),
                (3, "min/max, partial per wave (no LDS)")):
    print("probe %d %-34s %.3f ms  %.2f TB/s" % (v, name, ms_v[v], gb / ms_v[v]))
print("reset + min/max pass:                            %.3f ms  %.2f TB/s" % (ms_mm, gb / ms_mm))
print("reset + min/max + histogram (updateStatsMany):   %.3f ms  %.2f TB/s (two passes)" % (ms_both, 2 * gb / ms_both))
