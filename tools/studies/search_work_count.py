"""The algorithmic work of the per-channel MSE and entropy searches on ResNet-50's 54 weights (27,560
channels, the workload of tools/studies/tfe_search_time.py), counted on the host from the same
random-init weights, for the counters' per-unit figures (profiles/r06/search_work_count.txt):

  MSE: candidates (nmins x nmaxs - 1, mse_core.hpp: setup) x non-empty bins (the bins the cost
       loop visits), i.e. the (candidate, bin) pairs an exhaustive search evaluates; the kernel's
       pruning stops most candidates early, so the counters' VALU per pair is below one loop step;
  entropy: windows (129) x window bins (the divergence terms), and the non-empty share.

The histogram is the analyzers' first-batch PDF: 512 equal bins over the channel's [min, max]
(an approximation of InitializePdf's exact bucket edges, good to a bin or two per channel).

    python tools/studies/search_work_count.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from workloads.resnet import resnet50  # noqa: E402


def main():
    model = resnet50(seed=0, device="cpu")
    ws = [m.weight.detach().reshape(m.weight.shape[0], -1).numpy() for m in model.modules()
          if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear))]
    channels = sum(w.shape[0] for w in ws)
    pairs = cands = nonempty = 0
    ent_terms = ent_nonempty = 0
    for w in ws:
        for row in w:
            lo, hi = float(row.min()), float(row.max())
            h, edges = np.histogram(row, bins=512, range=(lo, hi))
            ne = int((h > 0).sum())
            nmins = int((edges < 0).sum()) + 1
            nmaxs = int((edges > 0).sum()) + 1
            c = nmins * nmaxs - 1
            cands += c
            nonempty += ne
            pairs += c * ne
            # symmetric windows [n, 511 - n], n = 0 .. 128
            nz = (h > 0).astype(np.int64)
            pre = np.concatenate([[0], np.cumsum(nz)])
            for n in range(129):
                ent_terms += 512 - 2 * n
                ent_nonempty += int(pre[512 - n] - pre[n])
    print("channels %d" % channels)
    print("MSE: candidates %.4g (%.1f per channel), non-empty bins %.4g (%.1f per channel), "
          "(candidate, non-empty bin) pairs %.4g" % (cands, cands / channels, nonempty, nonempty / channels, pairs))
    print("entropy (symmetric windows): window x bin terms %.4g (%.0f per channel), non-empty %.4g (%.1f %%)"
          % (ent_terms, ent_terms / channels, ent_nonempty, 100.0 * ent_nonempty / ent_terms))


if __name__ == "__main__":
    main()
