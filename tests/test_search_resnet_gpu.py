"""The per-channel device encoding searches on BASELINE config 2's weights (ResNet-50, 54 weights,
27,560 channels, per-channel 8-bit, symmetric and asymmetric) == the CPU oracle's host searches
(oracle/dlq_oracle.c, pinned to the reference C++ by tests/golden): MSE (mse_search.hip: zero-mass
bins skipped, guarded reciprocal) and entropy (entropy_search.hip). Every 4th channel of every
weight is checked (the oracle's MSE search costs ~10 ms per channel on one host core), in a
thread pool."""
import concurrent.futures as cf
import os

import pytest
import torch

from conftest import gpu_available
from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]
DEV = torch.device("cuda", 0)
THREADS = min(16, os.cpu_count() or 4)
STRIDE = 4


@pytest.mark.parametrize("scheme_name", ["QUANTIZATION_MSE", "QUANTIZATION_ENTROPY"])
def test_resnet50_weight_searches_equal_oracle(scheme_name):
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    from workloads.resnet import resnet50
    scheme = getattr(QuantizationMode, scheme_name)
    model = resnet50(seed=0, device=DEV)
    ws = [m.weight.detach().contiguous() for m in model.modules() if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear))]
    qs = [AimetTensorQuantizer(scheme, num_channels=w.shape[0]) for w in ws]
    AimetTensorQuantizer.updateStatsPerChannelMany(qs, ws)
    rows = [w.reshape(w.shape[0], -1).cpu().numpy() for w in ws]
    assert sum(w.shape[0] for w in ws) == 27560

    def oracle(i, c, sym):
        a = O.Analyzer(int(scheme))
        a.update(rows[i][c])
        return a.compute(8, sym).as_tuple()

    with cf.ThreadPoolExecutor(THREADS) as pool:
        for sym in (True, False):
            got = AimetTensorQuantizer.getEncodings(qs, 8, sym, False, False)
            jobs = {(i, c): pool.submit(oracle, i, c, sym) for i, r in enumerate(rows)
                    for c in range(0, r.shape[0], STRIDE)}
            bad = []
            for (i, c), f in jobs.items():
                encs, valid = got[i]
                assert valid
                if encs[c].to_tuple() != f.result():
                    bad.append((i, c, encs[c].to_tuple(), f.result()))
            assert not bad, (sym, len(bad), len(jobs), bad[:3])
