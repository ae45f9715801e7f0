"""Per-run wall clock and GPU span of the calibration plan on bench.py's workload (ResNet-50 batch
256, TF-E activations + per-channel TF-E weights), and the same for the plan's parts alone:
  both      -- the bench's headline (activations on the main stream, weights on the side stream)
  acts      -- the activations only
  weights   -- the weights only
  serial    -- both, the weights on the main stream ahead of the activations (no overlap)
Each run: synchronize, t0, plan.run(reset=True), t1; the GPU span is a HIP event recorded on the
main stream before the launch and one enqueued right after it (behind the activations' search,
the last kernel on that stream, and the join of the side stream). Prints one JSON line per form.

usage: python tools/studies/enc_plan_runs.py [--reps 30]
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--forms", default="both,both_after_resident")
    ap.add_argument("--lib", default=None, help="another build of libaimet_amd.so")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    if args.lib:
        import aimet_amd
        aimet_amd._native.LIB_PATH = os.path.abspath(args.lib)
    from aimet_amd.calibration import CalibrationPlan
    from workloads.resnet import resnet50
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
    acts, weights = bench.collect_tensors(model, x)
    del model, x
    A, W = [t for _, t in acts], [w for _, w in weights]
    n_elem = sum(t.numel() for t in A) + sum(w.numel() for w in W)
    main_s = torch.cuda.current_stream(dev)
    for form in args.forms.split(","):
        if form == "both_after_resident":
            # bench.py's order: the cold call, 9 calls on fresh quantizers, 9 on the same ones
            # (compute_encodings_resident), then the plan
            _, _, _, aq0, wq0 = bench.compute_encodings(acts, weights)
            for _ in range(9):
                del aq0, wq0
                _, _, _, aq0, wq0 = bench.compute_encodings(acts, weights)
            for _ in range(9):
                _, _, _, aq0, wq0 = bench.compute_encodings(acts, weights, (aq0, wq0))
        aq, wq = bench.make_quantizers(acts, weights)
        if form == "acts":
            plan = CalibrationPlan(aq, A)
        elif form == "weights":
            plan = CalibrationPlan([], [], wq, W)
        else:
            plan = CalibrationPlan(aq, A, wq, W)
        wall, span, host = [], [], []
        for i in range(args.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(main_s)
            if form == "serial":
                a, p = plan.launch(reset=True, side_stream=main_s)
            else:
                a, p = plan.launch(reset=True)
            e1.record(main_s)   # behind the activations' search (and the join of the side stream)
            tl = time.perf_counter()
            p.result()
            tp = time.perf_counter()
            a.result()
            t1 = time.perf_counter()
            if i >= 2:
                host.append((round((tl - t0) * 1e3, 3), round((tp - t0) * 1e3, 3)))
            torch.cuda.synchronize()
            if i >= 2:
                wall.append((t1 - t0) * 1e3)
                span.append(e0.elapsed_time(e1))
        med = lambda v: sorted(v)[len(v) // 2]
        print(json.dumps({"form": form, "tag": args.tag, "wall_ms_median": round(med(wall), 4), "wall_ms_min": round(min(wall), 4),
                          "gpu_span_ms_median": round(med(span), 4), "gpu_span_ms_min": round(min(span), 4),
                          "frac_of_8TBps_wall_median": round(8 * n_elem / (med(wall) / 1e3) / 8e12, 4),
                          "wall_ms": [round(v, 3) for v in wall], "host_launch_params_ms": host[:8]}), flush=True)
        plan.close()
        del aq, wq


if __name__ == "__main__":
    main()
