"""compute_encodings (bench.py's form: reset + recompute of the sim's quantizers) with the native
work as two calls (activations first, the parameters' host preparation beside their min/max pass)
vs one call, interleaved A/B in one process so clock and thermal drift hit both alike.
usage: python tools/studies/enc_split_ab.py [reps]"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from aimet_amd import tensor_quantizer as TQ  # noqa: E402
from workloads.resnet import resnet50  # noqa: E402

GB = 23.276   # algorithmic bytes of one call (bench.py: two 4-B passes over 11.54 G activations + weights)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda", 0)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234))
    acts, weights = bench.collect_tensors(model, x)
    del model
    _, _, _, aq, wq = bench.compute_encodings(acts, weights)
    times = {True: [], False: []}
    encs = {}
    for rep in range(reps + 2):
        for split in (True, False):
            TQ._CAL_SPLIT = split
            a, w, s, aq, wq = bench.compute_encodings(acts, weights, (aq, wq))
            if rep >= 2:
                times[split].append(s)
            encs[split] = ([e.to_tuple() for e in a], [[c.to_tuple() for c in es] for es in w])
    assert encs[True] == encs[False], "the two forms disagree"
    out = {}
    for split, ts in times.items():
        med = statistics.median(ts)
        out["two_calls" if split else "one_call"] = {"median_ms": round(med * 1e3, 4),
                                                    "min_ms": round(min(ts) * 1e3, 4),
                                                    "frac_of_8TBs": round(GB / med / 8000.0, 4),
                                                    "reps": len(ts)}
    out["encodings_identical"] = True
    print(json.dumps(out))


if __name__ == "__main__":
    main()
