"""What the weights cost a compute_encodings call: bench.py's workload (ResNet-50 bs256 activations
+ weights), the median wall-clock of reset-and-recompute calls with both, with the activations
only and with the weights only (compute_encodings_resident, as bench.py times it).

    python tools/studies/enc_split_cost.py [--reps 15]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    args = ap.parse_args()
    import bench
    from aimet_amd.calibration import compute_encodings_resident
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    from workloads.resnet import resnet50
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
    acts, weights = bench.collect_tensors(model, x)
    del model
    torch.cuda.empty_cache()
    A = [t for _, t in acts]
    W = [w for _, w in weights]
    aq = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in A]
    wq = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED, num_channels=w.shape[0]) for w in W]
    gb = {"both": 4 * (sum(t.numel() for t in A) + sum(w.numel() for w in W)) * 2 / 1e9,
          "acts": 4 * sum(t.numel() for t in A) * 2 / 1e9, "weights": 4 * sum(w.numel() for w in W) * 2 / 1e9}
    forms = {"both": (aq, A, wq, W), "acts": (aq, A, [], []), "weights": ([], [], wq, W)}
    for name, (q1, t1, q2, t2) in forms.items():
        compute_encodings_resident(q1, t1, q2, t2, act_settings=(8, False, False, False),
                                   param_settings=(8, True, False, False), reset=False)
    res = {}
    for _ in range(2):   # the forms interleaved, twice
        for name, (q1, t1, q2, t2) in forms.items():
            ts = []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                compute_encodings_resident(q1, t1, q2, t2, act_settings=(8, False, False, False),
                                           param_settings=(8, True, False, False), reset=True)
                ts.append(time.perf_counter() - t0)
            res.setdefault(name, []).append(sorted(ts)[len(ts) // 2])
    for name, v in res.items():
        ms = min(v) * 1e3
        print(json.dumps({"form": name, "median_ms_per_round": [round(t * 1e3, 3) for t in v],
                          "algorithmic_gb": round(gb[name], 3), "frac_of_8TBps": round(gb[name] / (ms * 1e-3) / 8000, 4)}))


if __name__ == "__main__":
    main()
