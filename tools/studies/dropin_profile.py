"""Where QuantizationSimModel.compute_encodings spends its time beyond the plain forwards (bench.py's
drop-in surface, config 1: ResNet-50 W8A8 per-tensor TF-Enhanced, 8 x 32 U(0,1) images): the
phases of the call timed separately (reset + mode switch, the ANALYSIS forwards, the batched
encodings, the mode switch back), the plain forwards beside them, then a cProfile of one call
(top functions by own time).

    python tools/studies/dropin_profile.py [--reps 3]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import aimet_amd.quantsim as QS
    from aimet_amd.quantizers import QuantScheme
    from aimet_amd.quantsim import QuantizationSimModel
    from workloads.resnet import resnet50
    dev = torch.device("cuda", 0)
    model = resnet50(seed=0, device=dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    images = torch.rand(8 * 32, 3, 224, 224, device=dev, generator=g)
    batches = [images[b * 32:(b + 1) * 32] for b in range(8)]

    def calibrate(m, _):
        with torch.no_grad():
            for b in batches:
                m(b)

    sim = QuantizationSimModel(model, batches[0][:1], quant_scheme=QuantScheme.post_training_tf_enhanced,
                               default_output_bw=8, default_param_bw=8)
    # phase timing: wrap the pieces compute_encodings calls
    phases = {}
    orig_batched = QS.compute_encodings_batched

    def timed(name, fn):
        def w(*a, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn(*a, **k)
            torch.cuda.synchronize()
            phases.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
            return r
        return w
    QS.compute_encodings_batched = timed("encodings_batched", orig_batched)
    others = {n: getattr(QS, n) for n in ("_reset_many", "_precompute_param_encodings", "_forget_unused_param_encodings")}
    for n, fn in others.items():
        setattr(QS, n, timed(n.strip("_"), fn))
    cal_timed = timed("analysis_forwards", calibrate)
    for _ in range(args.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sim.compute_encodings(cal_timed, None)
        torch.cuda.synchronize()
        phases.setdefault("whole_call", []).append((time.perf_counter() - t0) * 1e3)
    plain = timed("plain_forwards", calibrate)
    for _ in range(args.reps + 1):
        plain(model, None)
    QS.compute_encodings_batched = orig_batched
    for n, fn in others.items():
        setattr(QS, n, fn)
    for k, v in phases.items():
        v = v[1:]
        print("%-20s median %.2f ms  runs %s" % (k, sorted(v)[len(v) // 2], [round(x, 2) for x in v]))
    pr = cProfile.Profile()
    pr.enable()
    sim.compute_encodings(calibrate, None)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
