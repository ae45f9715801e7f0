"""Time aimet_adaround_dw_step on MobileNet-v2's depthwise shapes (batch 32 drawn from 1024 cached
rows) by HIP events; AIMET_TUNE_DW_U / AIMET_TUNE_DW_PER select the variant (tuning only).
usage: python tools/studies/dw_step_tune.py [label]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from aimet_amd import _native  # noqa: E402

dev = torch.device("cuda", 0)
label = sys.argv[1] if len(sys.argv) > 1 else ""
for (C, H, stride) in ((32, 112, 1), (96, 112, 2), (144, 56, 1), (384, 14, 1), (960, 7, 1)):
    rows, N, K, pad = 1024, 32, 3, 1
    OH = (H + 2 - 3) // stride + 1
    x = torch.rand(rows, C, H, H, device=dev)
    t = torch.rand(rows, C, OH, OH, device=dev)
    w = torch.randn(C, 1, 3, 3, device=dev) * 0.3
    idx = torch.randint(0, rows, (4, N), device=dev)
    ctr = torch.zeros(2, dtype=torch.long, device=dev)
    gw = torch.empty_like(w)
    n_ws = ctypes.c_int64()
    _native.call("aimet_dwconv2d_grad_weight_workspace", N, C, OH, OH, K, ctypes.byref(n_ws))
    ws = torch.empty(n_ws.value, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def call():
        _native.call("aimet_adaround_dw_step", x.data_ptr(), t.data_ptr(), idx.data_ptr(), ctr.data_ptr(),
                     ctr.data_ptr() + 8, w.data_ptr(), None, gw.data_ptr(), ws.data_ptr(), N, C, H, H, OH, OH, K,
                     stride, pad, 1, 2, s)
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        call()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    nb = (N * C * H * H + N * C * OH * OH) * 4
    print(json.dumps({"label": label, "C": C, "H": H, "stride": stride, "us": round(us, 2),
                      "GBps": round(nb / us / 1e3, 1)}), flush=True)
