"""Where bench.py's compute_encodings wall clock goes on the host (round 5: bench.py's plan runs
measured ~0.25 ms above their GPU span, tools/studies/enc_plan_runs.py's ~0.02 ms). Replicates
bench.main() up to the headline plan, then times the plan runs with the host split into: launch
returned, parameters' encodings built, the activations' request event done (e_done.synchronize),
activations' encodings built -- in variants: as bench.py, without the wait on the event behind the launch (bench.py's own form),
after gc.freeze(), with gc disabled.
One JSON line per variant.

usage: python tools/studies/enc_bench_host.py [--reps 20]
"""
import argparse
import gc
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
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    rank, world, dev = bench.setup_dist(args)
    import aimet_amd
    from aimet_amd.calibration import CalibrationPlan
    from workloads.resnet import resnet50
    aimet_amd.native_library()
    torch.manual_seed(1234 + rank)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(args.batch, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234 + rank))
    acts, weights = bench.collect_tensors(model, x)
    del x
    torch.cuda.empty_cache()
    act_enc, w_enc, enc_cold, aq, wq = bench.compute_encodings(acts, weights)
    for _ in range(args.enc_reps):
        del aq, wq
        act_enc, w_enc, secs, aq, wq = bench.compute_encodings(acts, weights)
    for _ in range(args.enc_reps):
        act_enc, w_enc, secs, aq, wq = bench.compute_encodings(acts, weights, (aq, wq))
    plan = CalibrationPlan(aq, [t for _, t in acts], wq, [w for _, w in weights])
    stream = torch.cuda.current_stream()
    for variant in ("as_bench", "no_e1_sync", "gc_freeze", "gc_disabled", "as_bench_again"):
        if variant == "gc_freeze":
            gc.collect()
            gc.freeze()
        if variant == "gc_disabled":
            gc.disable()
        if variant == "as_bench_again":
            gc.enable()
            gc.unfreeze()
        rows = []
        for i in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(stream)
            ap_, pp = plan.launch(reset=True)
            e1.record(stream)
            t1 = time.perf_counter()
            pr = pp.result()
            t2 = time.perf_counter()
            if variant != "no_e1_sync":
                e1.synchronize()
            t3 = time.perf_counter()
            ar = ap_.result()
            t4 = time.perf_counter()
            torch.cuda.synchronize()
            if i >= 2:
                rows.append([round((t - t0) * 1e3, 3) for t in (t1, t2, t3, t4)] + [round(e0.elapsed_time(e1), 3)])
        med = lambda k: sorted(r[k] for r in rows)[len(rows) // 2]   # noqa: E731
        print(json.dumps({"variant": variant, "launch_ms": med(0), "params_built_ms": med(1),
                          "gpu_done_seen_ms": med(2), "wall_ms": med(3), "gpu_span_ms": med(4),
                          "gc_counts": gc.get_count(), "gc_objects": len(gc.get_objects()), "rows": rows[:6]}),
              flush=True)
    plan.close()
    del model


if __name__ == "__main__":
    main()
