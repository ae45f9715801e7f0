"""Per-iteration cost of the AdaRound loop variants on one layer (tuning tool)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aimet_amd import adaround_optimizer as AO  # noqa: E402
from aimet_amd.adaround import compute_beta, init_alpha  # noqa: E402
from oracle import torch_ref as T  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
for cin, cout, hw, groups in ((96, 576, 14, 1), (576, 576, 14, 576), (3, 32, 112, 1)):
    conv = torch.nn.Conv2d(cin, cout, 3 if groups > 1 or cin == 3 else 1, padding=1 if (groups > 1 or cin == 3) else 0,
                           groups=groups).to(dev)
    inp = torch.randn(1024, cin, hw, hw, device=dev)
    with torch.no_grad():
        out = conv(inp)
    w = conv.weight.detach()
    d = torch.tensor([float(w.abs().max()) / 127], device=dev)
    o = torch.tensor([-128.0], device=dev)
    P = AO.AdaroundHyperParameters(num_iterations=200, warm_start=0.2)
    for name in ("ours", "ours_foreach_adam", "reference"):
        def run():
            if name == "reference":
                a = init_alpha(w, d)
                opt = torch.optim.Adam([a])
                g = torch.Generator().manual_seed(0)
                for it in range(P.num_iterations):
                    idx = torch.randperm(1024, generator=g)[:32].to(dev)
                    x, t = inp.index_select(0, idx), out.index_select(0, idx)
                    opt.zero_grad()
                    loss = AO.recon_loss(AO.layer_forward(conv, x, T.adaround_forward(w, a, d, o, 8)), t)
                    if it >= 40:
                        loss = loss + T.adaround_round_loss(a, 0.01, compute_beta(200, it, (20, 2), 0.2))
                    loss.backward()
                    opt.step()
            else:
                orig = torch.optim.Adam
                if name == "ours_foreach_adam":
                    torch.optim.Adam = lambda params, fused=None: orig(params)
                try:
                    AO.AdaroundOptimizer.optimize_rounding(conv, inp, out, d, o, 8, 0, P, None,
                                                           torch.Generator().manual_seed(0))
                finally:
                    torch.optim.Adam = orig
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        print("layer %s %-20s %.3f ms/iter" % ((cin, cout, hw, groups), name, (time.perf_counter() - t0) / 200 * 1e3),
              flush=True)
