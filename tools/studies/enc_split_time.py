"""compute_encodings (bench.py's ResNet-50 bs256 workload, reset + recompute) split: both halves,
the activations alone, the per-channel weights alone (median of 9 calls each, wall-clock), to see
what the overlap of the two streams buys. Then 3 more full calls for a kernel trace."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from aimet_amd.calibration import compute_encodings_resident  # noqa: E402
from aimet_amd.libpymo import QuantizationMode  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402
from workloads.resnet import resnet50  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
model = resnet50(seed=0, device=dev)
x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
acts, weights = bench.collect_tensors(model, x)
del model, x
torch.cuda.empty_cache()
TFE = QuantizationMode.QUANTIZATION_TF_ENHANCED
aq = [AimetTensorQuantizer(TFE) for _ in acts]
wq = [AimetTensorQuantizer(TFE, num_channels=w.shape[0]) for _, w in weights]
A = [t for _, t in acts]
W = [w for _, w in weights]


def timed(a_q, a_t, w_q, w_t, reps=9):
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        compute_encodings_resident(a_q, a_t, w_q, w_t, param_settings=(8, True, False, False), reset=True)
        ts.append((time.perf_counter() - t0) * 1e3)
    ts = sorted(ts[1:])
    return round(ts[len(ts) // 2], 3)


res = {"both_ms": timed(aq, A, wq, W), "acts_only_ms": timed(aq, A, [], []), "weights_only_ms": timed([], [], wq, W)}
res["both_again_ms"] = timed(aq, A, wq, W)
print(json.dumps(res), flush=True)
for _ in range(3):
    compute_encodings_resident(aq, A, wq, W, param_settings=(8, True, False, False), reset=True)
torch.cuda.synchronize()
