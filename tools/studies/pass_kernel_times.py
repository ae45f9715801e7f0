"""The two halves of compute_encodings alone, 12 calls each (bench.py's ResNet-50 bs256 workload,
reset + recompute): `acts` = the 55 TF-Enhanced activation quantizers (min/max and histogram
passes), `weights` = the 54 per-channel symmetric weight quantizers (channel statistics + the
27,560-channel TF-E search). Run under rocprofv3 --kernel-trace --stats for per-kernel durations."""
import os
import sys

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
which = sys.argv[1] if len(sys.argv) > 1 else "acts"
aq = [AimetTensorQuantizer(TFE) for _ in acts] if which == "acts" else []
A = [t for _, t in acts] if which == "acts" else []
wq = [AimetTensorQuantizer(TFE, num_channels=w.shape[0]) for _, w in weights] if which == "weights" else []
W = [w for _, w in weights] if which == "weights" else []
for _ in range(12):
    compute_encodings_resident(aq, A, wq, W, param_settings=(8, True, False, False), reset=True)
torch.cuda.synchronize()
print("done", flush=True)
