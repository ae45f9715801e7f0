"""compute_encodings (bench.py's ResNet-50 bs256 workload) wall-clock with the CUs partitioned
between the activation passes and the parameter searches (AIMET_CAL_SIDE_CUS_PER_XCD = k CUs per
XCD for the parameters' stream, 0 = no partition) under both launch orders. One process per
configuration (the knobs are read at import); median of 9 reset + recompute calls."""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from enc_schedule_tune import CHILD  # noqa: E402

configs = [c.split(":") for c in (sys.argv[1:] or ["params_first:0", "params_first:2", "params_first:4",
                                                   "acts_first:2", "acts_first:4", "params_first:6"])]
for cfg in configs:
    sched, k = cfg[0], cfg[1]
    env = dict(os.environ, AIMET_CAL_SCHEDULE=sched, AIMET_CAL_SIDE_CUS_PER_XCD=k,
               AIMET_CAL_PARAMS_SERIAL=cfg[2] if len(cfg) > 2 else "0",
               AIMET_TUNE_TFE_GRID=cfg[3] if len(cfg) > 3 else "65536")
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    print(json.dumps({"schedule": sched, "side_cus_per_xcd": int(k), "params_serial": cfg[2:3] == ["1"],
                      "tfe_grid": cfg[3] if len(cfg) > 3 else None}), line[-1] if line else out.stderr[-2000:],
          flush=True)
