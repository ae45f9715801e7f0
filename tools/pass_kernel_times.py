"""The activation passes of compute_encodings alone (bench.py's ResNet-50 bs256 activations, 55
TF-Enhanced quantizers, reset + recompute, no weights), 12 calls: run under
rocprofv3 --kernel-trace --stats for the per-kernel durations of the min/max and histogram passes."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
acts, _ = bench.collect_tensors(model, x)
del model, x
torch.cuda.empty_cache()
aq = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in acts]
A = [t for _, t in acts]
for _ in range(12):
    compute_encodings_resident(aq, A, [], [], reset=True)
torch.cuda.synchronize()
print("done", flush=True)
