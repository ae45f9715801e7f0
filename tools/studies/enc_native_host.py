"""Host-side split of bench.py's compute_encodings on the native path (one aimet_calibrate_launch):
time in the Python preparation + native launch, in waiting for / building the parameters' and the
activations' encodings, with no extra synchronisation (tuning tool).
usage: python tools/studies/enc_native_host.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from aimet_amd import calibration as CAL  # noqa: E402
from aimet_amd.tensor_quantizer import AimetTensorQuantizer  # noqa: E402
from workloads.resnet import resnet50  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
    acts, weights = bench.collect_tensors(model, x)
    del model
    _, _, _, aq, wq = bench.compute_encodings(acts, weights)
    a_t, w_t = [t for _, t in acts], [w for _, w in weights]
    rows = []
    for rep in range(12):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        main_s = torch.cuda.current_stream(dev)
        a_p, p_p, keep = AimetTensorQuantizer.calibrateResidentAsync(
            aq, a_t, wq, w_t, None, (8, False, False, False), (8, True, False, False), reset=True,
            main_stream=main_s, side_stream=CAL._side_stream(dev))
        t1 = time.perf_counter()
        p_res = p_p.result()
        t2 = time.perf_counter()
        a_res = a_p.result()
        t3 = time.perf_counter()
        del keep, p_res, a_res
        rows.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0))
    rows = rows[2:]
    med = [sorted(r[i] for r in rows)[len(rows) // 2] * 1e3 for i in range(4)]
    print(json.dumps({"prep_and_launch_ms": round(med[0], 4), "param_results_ms": round(med[1], 4),
                      "act_results_ms": round(med[2], 4), "total_ms": round(med[3], 4)}))


if __name__ == "__main__":
    main()
