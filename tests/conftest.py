import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
sys.dont_write_bytecode = True


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "ref: needs /root/reference (build container only)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(params=[True, False], ids=["exact_pow", "fast_pow"])
def exact_pow(request):
    """Both forms of the AdaRound rounding loss's pow (aimet_amd.adaround.set_exact_pow): the
    bit-exact emulation of torch's CPU pow and the default table-driven f32 pow (within 1 ulp)."""
    from aimet_amd.adaround import set_exact_pow
    prev = set_exact_pow(request.param)
    yield request.param
    set_exact_pow(prev)


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")


@pytest.fixture(scope="session")
def golden_core(golden_dir):
    import numpy as np
    return dict(np.load(os.path.join(golden_dir, "golden_core.npz")))


@pytest.fixture(scope="session")
def golden_analyzers(golden_dir):
    import numpy as np
    return dict(np.load(os.path.join(golden_dir, "golden_analyzers.npz")))


@pytest.fixture(scope="session")
def golden_entropy(golden_dir):
    import numpy as np
    return dict(np.load(os.path.join(golden_dir, "golden_entropy.npz")))


def entropy_case(en, i):
    """Unpack entropy case i of golden_entropy.npz: batches, reference TensorProfilingParams and
    encodings {(bw, sym, strict, unsigned): (min, max, delta, offset, bw)}."""
    nb = int(en["e%d_nb" % i])
    encs = {}
    for k, v in zip(en["e%d_enc_keys" % i], en["e%d_enc_vals" % i]):
        bw, flags = str(k).split("_")
        encs[(int(bw), int(flags[0]), int(flags[1]), int(flags[2]))] = tuple(v[:4]) + (int(v[4]),)
    t = en["e%d_tpp" % i]
    return dict(batches=[en["e%d_b%d" % (i, k)] for k in range(nb)], encs=encs,
                tpp=dict(has_hist=int(t[0]), min=float(t[1]), max=float(t[2]), iterations=int(t[3]),
                         hist=en["e%d_hist" % i]))


@pytest.fixture(scope="session")
def golden_torch(golden_dir):
    import numpy as np
    return dict(np.load(os.path.join(golden_dir, "golden_torch.npz")))


@pytest.fixture(scope="session")
def kat(golden_dir):
    import json
    with open(os.path.join(golden_dir, "kat.json")) as f:
        return json.load(f)


def analyzer_case(an, i):
    """Unpack analyzer case i from golden_analyzers.npz."""
    nb = int(an["a%d_nb" % i])
    keys = [str(k) for k in an["a%d_enc_keys" % i]]
    vals = an["a%d_enc_vals" % i]
    encs = {}
    for k, v in zip(keys, vals):
        bw, flags = k.split("_")
        encs[(int(bw), int(flags[0]), int(flags[1]), int(flags[2]))] = tuple(v)
    return dict(scheme=int(an["a%d_scheme" % i]), percentile=float(an["a%d_percentile" % i]),
                batches=[an["a%d_b%d" % (i, k)] for k in range(nb)], encs=encs,
                xleft=an["a%d_xleft" % i], pdf=an["a%d_pdf" % i])


def per_channel_case(core, i):
    p = "pc%d_" % i
    return dict(x=core[p + "x"], outer=int(core[p + "outer"]), C=int(core[p + "C"]), K=int(core[p + "K"]),
                encs=core[p + "encs"], table=core[p + "table"], y=core[p + "y"])


def bits(a):
    """Bit pattern view for bit-exact comparisons (NaN payloads compared as NaN-ness)."""
    import numpy as np
    a = np.asarray(a, dtype=np.float32)
    b = a.view(np.uint32).copy()
    b[np.isnan(a)] = 0x7FC00000
    return b
