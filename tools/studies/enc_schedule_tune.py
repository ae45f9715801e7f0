"""compute_encodings (bench.py's ResNet-50 bs256 workload) wall-clock under the calibration
schedule knobs: AIMET_CAL_SCHEDULE (params_first | acts_first) x AIMET_CAL_SIDE_PRIORITY (-1 high,
0 normal). Each configuration runs in its own process (the knobs are read at import)."""
import itertools
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r"""
import sys, time, json, torch
sys.path.insert(0, %r)
import bench
from workloads.resnet import resnet50
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
model = resnet50(seed=0, device=dev)
x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
acts, weights = bench.collect_tensors(model, x)
del model
torch.cuda.empty_cache()
ts, tr = [], []
for rep in range(9):
    *_, secs, aq, wq = bench.compute_encodings(acts, weights)
    ts.append(secs * 1e3)
for rep in range(9):
    *_, secs, aq, wq = bench.compute_encodings(acts, weights, (aq, wq))
    tr.append(secs * 1e3)
w, r = sorted(ts[1:]), sorted(tr)
print(json.dumps({"fresh_median_ms": round(w[len(w) // 2], 3), "reset_median_ms": round(r[len(r) // 2], 3),
                  "reset_min_ms": round(r[0], 3), "reset_all": [round(t, 3) for t in tr]}))
""" % REPO

if __name__ == "__main__":
    for sched, prio in itertools.product(("params_first", "acts_first"), ("-1", "0")):
        env = dict(os.environ, AIMET_CAL_SCHEDULE=sched, AIMET_CAL_SIDE_PRIORITY=prio)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(sched, prio, line[-1] if line else out.stderr[-2000:], flush=True)
