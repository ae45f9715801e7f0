"""Timing tool: depthwise 3x3 conv forward + weight gradient (AdaRound's per-iteration layer
forward / backward on MobileNet-v2 shapes) through MIOpen vs PyTorch's native depthwise kernels."""
import torch
import torch.nn.functional as F


def bench(c, hw, stride, native, memfmt=torch.contiguous_format):
    x = torch.randn(32, c, hw, hw, device="cuda").to(memory_format=memfmt)
    w = torch.randn(c, 1, 3, 3, device="cuda", requires_grad=True)
    with torch.backends.cudnn.flags(enabled=not native):
        for _ in range(3):
            y = F.conv2d(x, w, None, stride, 1, 1, c)
            y.sum().backward()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            y = F.conv2d(x, w, None, stride, 1, 1, c)
            y.backward(torch.ones_like(y))
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 20


for c, hw, s in ((32, 112, 1), (96, 112, 2), (144, 56, 1), (144, 56, 2), (192, 28, 1), (384, 14, 1), (576, 14, 1),
                 (960, 7, 1)):
    print("C=%4d HW=%3d s=%d  miopen %.3f ms  native %.3f ms  miopen-NHWC %.3f ms" % (
        c, hw, s, bench(c, hw, s, False), bench(c, hw, s, True), bench(c, hw, s, False, torch.channels_last)),
          flush=True)
