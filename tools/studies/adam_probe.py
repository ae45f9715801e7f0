"""Does aimet_adaround_backward_adam's Adam arithmetic match torch.optim.Adam(fused=True) bit for
bit? Runs both on the same params / grads for several steps (contracted and uncontracted forms)."""
import ctypes
import os
import sys

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "adam_probe.so"))
lib.adam_probe.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_int] + [ctypes.c_double] * 4 + [ctypes.c_int]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
n = 1 << 16
p0 = torch.randn(n, device=dev, generator=g)
grads = [torch.randn(n, device=dev, generator=g) * (10 ** (k % 5 - 3)) for k in range(20)]
for capturable in (False,):
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=1e-3, fused=True, capturable=capturable)
    res = {}
    for contract in (1, 11, 12, 13, 14, 15, 16):
        p, m, v = p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        res[contract] = (p, m, v)
    for step, gr in enumerate(grads, 1):
        ref.grad = gr.clone()
        opt.step()
        for contract, (p, m, v) in res.items():
            lib.adam_probe(p.data_ptr(), gr.data_ptr(), m.data_ptr(), v.data_ptr(), n, step, 1e-3, 0.9, 0.999, 1e-8,
                           contract)
        st = opt.state[ref]
        for contract, (p, m, v) in res.items():
            dp = int((p != ref.detach()).sum())
            dm = int((m != st["exp_avg"]).sum())
            dv = int((v != st["exp_avg_sq"]).sum())
            if step in (2, 5, 20):
                print("capturable=%d contract=%d step %2d: param diff %d, exp_avg diff %d, exp_avg_sq diff %d"
                      % (capturable, contract, step, dp, dm, dv), flush=True)
sys.exit(0)
