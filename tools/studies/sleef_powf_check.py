"""Study: torch's CPU pow(tensor, float exponent) (the reference AdaRound rounding loss and its
pow_backward) == Sleef_powf_u10 (AVX512F build) in the vectorized part + the correctly rounded
value in the scalar tail (the last n mod 32 elements, one thread) + x*x / x*x*x for exponents 2 / 3.
The C form of the device restatement (tools/studies/sleef_powf.c) is compared bit for bit.
  gcc -O2 -ffp-contract=off -shared -fPIC -o /tmp/libsleef_powf.so tools/studies/sleef_powf.c -lm
  python tools/studies/sleef_powf_check.py"""
import ctypes
import math

import numpy as np
import torch

torch.set_num_threads(1)
lib = ctypes.CDLL("/tmp/libsleef_powf.so")
lib.sleef_powf_arr.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_long]


def model(x, e):
    n = x.size
    if e == 2.0:
        return x * x
    if e == 3.0:
        return x * x * x
    out = np.empty_like(x)
    lib.sleef_powf_arr(x.ctypes.data, e, out.ctypes.data, n)
    for i in range(n - n % 32, n):
        out[i] = np.float32(math.exp(float(e) * math.log(float(x[i])))) if x[i] != 0 else 0.0
    return out


rng = np.random.default_rng(2)
total = checked = 0
for n in [216, 315, 1000, 33, 31, 70000, (1 << 20) + 37]:
    for e in list(rng.uniform(1.0, 19.0, 30).astype(np.float32).tolist()) + [2.0, 3.0, 1.0]:
        x = rng.random(n, dtype=np.float32)
        want = torch.from_numpy(x).pow(e).numpy()
        total += int((model(x, e).view(np.uint32) != want.view(np.uint32)).sum())
        checked += n
print("checked %d elements: %d differ from torch.pow" % (checked, total))
