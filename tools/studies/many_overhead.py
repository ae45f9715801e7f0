"""Host-side cost of the batched statistics call (tuning tool): 99 tensors like ViT-L's."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aimet_amd import _native  # noqa: E402
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [4816896, 6422528] + [19365888, 6455296, 25821184, 6455296] * 24 + [32000]
ts = [torch.randn(n, device=dev) for n in sizes]
qs = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in ts]
AimetTensorQuantizer.updateStatsMany(qs, ts)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    AimetTensorQuantizer.updateStatsMany(qs, ts)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("updateStatsMany host %.3f ms, +sync %.3f ms" % ((t1 - t0) * 1e3, (t2 - t0) * 1e3))
# the native call alone
n = len(qs)
hs = (ctypes.c_void_p * n)(*[q._handle for q in qs])
xs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
ns = (ctypes.c_int64 * n)(*[t.numel() for t in ts])
s = torch.cuda.current_stream().cuda_stream
for rep in range(3):
    t0 = time.perf_counter()
    _native.call("aimet_tq_update_stats_many", hs, xs, ns, n, s)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("native call %.3f ms, +sync %.3f ms" % ((t1 - t0) * 1e3, (t2 - t0) * 1e3))
lib = _native.load()
p = ctypes.c_void_p(ts[0].data_ptr())
t0 = time.perf_counter()
for _ in range(100):
    lib.aimet_qdq_per_tensor(p, p, 0, None, 0, 0, ctypes.c_void_p(s))
print("100 trivial calls %.3f ms" % ((time.perf_counter() - t0) * 1e3))
