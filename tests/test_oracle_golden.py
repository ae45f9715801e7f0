"""Pins the CPU oracle (oracle/dlq_oracle.c) to the reference: golden vectors produced by the
reference C++ (tests/golden/*.npz, see make_golden.py) and the reference test-suites' KATs.
CPU only."""
import numpy as np
import pytest

from conftest import analyzer_case, bits, per_channel_case
from oracle import oracle as O


def test_kat_qdq_and_quantize(kat):
    for name in ("qdq_sanity", "qdq_gated_min", "qdq_gated_equal", "qdq_gated_max"):
        k = kat[name]
        y = O.qdq_per_tensor(np.array(k["x"], np.float32), k["min"], k["max"], k["bw"])
        # EXPECT_FLOAT_EQ == within 4 ulp
        np.testing.assert_array_max_ulp(y, np.array(k["expected"], np.float32), maxulp=4)
    for name in ("quantize_unsigned", "quantize_signed"):
        k = kat[name]
        y = O.quantize_per_tensor(np.array(k["x"], np.float32), k["min"], k["max"], k["bw"], k["shift"])
        np.testing.assert_array_equal(y, np.array(k["expected"], np.float32))


def test_kat_tfe(kat, golden_torch):
    k = kat["tfe_normal"]
    a = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
    a.update(golden_torch["tfe_kat_x"])
    e = a.compute(8, False, False, False)
    assert abs(e.min - k["expected_min"]) < k["tol"]
    assert abs(e.max - k["expected_max"]) < k["tol"]
    assert e.as_tuple() == tuple(k["ref_encoding"])  # bit-exact vs the reference re-run
    y = O.qdq_per_tensor(np.full(3, 5.0, np.float32), e.min, e.max, 8)
    assert abs(y[0] - k["expected_qdq5"]) < k["tol"]
    assert float(y[0]) == k["ref_qdq5"]


def test_kat_tfe_all_zero(kat):
    k = kat["tfe_all_zero"]
    a = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
    a.update(np.zeros(k["n"], np.float32))
    e = a.compute(8, False, False, False)
    assert abs(e.min - k["expected_min"]) < k["tol"] and abs(e.max - k["expected_max"]) < k["tol"]
    assert e.offset == k["expected_offset"] and e.bw == 8


@pytest.mark.parametrize("name", ["per_channel_symmetric", "per_channel_asymmetric"])
def test_kat_per_channel(kat, name):
    k = kat[name]
    x = np.array(k["x"], np.float32)
    table = O.per_channel_table([tuple(e) for e in k["encodings"]])
    y = O.qdq_per_channel(x, x.shape[0], x.shape[1], table)
    np.testing.assert_allclose(y, np.array(k["expected"], np.float32), atol=k["atol"])


def test_golden_per_tensor(golden_core):
    xs, encs = golden_core["pt_x"], golden_core["pt_enc"]
    for i, (x, e) in enumerate(zip(xs, encs)):
        mn, mx, bw = e[0], e[1], int(e[2])
        np.testing.assert_array_equal(bits(O.qdq_per_tensor(x, mn, mx, bw)), bits(golden_core["pt_qdq"][i]))
        np.testing.assert_array_equal(bits(O.quantize_per_tensor(x, mn, mx, bw, False)),
                                      bits(golden_core["pt_q_unsigned"][i]))
        np.testing.assert_array_equal(bits(O.quantize_per_tensor(x, mn, mx, bw, True)),
                                      bits(golden_core["pt_q_signed"][i]))
        assert O.fill_encoding_info(bw, mn, mx).as_tuple() == tuple(golden_core["pt_fill"][i][:4]) + (bw,)


def test_golden_computed_encodings(golden_core):
    for inp, out in zip(golden_core["gce_in"], golden_core["gce_out"]):
        bw, mn, mx, sym, strict, un = inp
        got = O.get_computed_encodings(int(bw), mn, mx, int(sym), int(strict), int(un)).as_tuple()
        np.testing.assert_array_equal(np.array(got[:4]), out[:4])


def test_golden_per_channel(golden_core):
    for i in range(int(golden_core["pc_count"])):
        c = per_channel_case(golden_core, i)
        table = O.per_channel_table([tuple(e) for e in c["encs"]])
        np.testing.assert_array_equal(bits(table), bits(c["table"]))
        y = O.qdq_per_channel(c["x"], c["C"], c["K"], table)
        np.testing.assert_array_equal(bits(y), bits(c["y"]))


def test_golden_analyzers(golden_analyzers):
    n = int(golden_analyzers["count"])
    assert n > 0
    for i in range(n):
        c = analyzer_case(golden_analyzers, i)
        a = O.Analyzer(c["scheme"])
        if c["scheme"] == O.QUANTIZATION_PERCENTILE:
            a.set_percentile(c["percentile"])
        for b in c["batches"]:
            a.update(b)
        for (bw, sym, strict, un), want in c["encs"].items():
            got = a.compute(bw, sym, strict, un).as_tuple()
            assert got == tuple(want[:4]) + (int(want[4]),), (i, c["scheme"], bw, sym, strict, un, got, want)
        if c["scheme"] != O.QUANTIZATION_TF:
            xl, pdf = a.histogram()
            np.testing.assert_array_equal(xl, c["xleft"])
            np.testing.assert_array_equal(pdf, c["pdf"])


def test_sharded_pdf_equals_whole_batch():
    """Counts summed over shards + PDF update with the global count == one-device UpdatePdf
    (the contract of the sharded calibration)."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal(4000).astype(np.float32)
    whole = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
    whole.update(x)
    xl, _ = whole.histogram()
    shard = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
    shard.update(x)  # initializes the PDF range on the same data
    shard2 = O.Analyzer(O.QUANTIZATION_TF_ENHANCED)
    shard2.update(x)
    # second batch: whole vs sharded counts
    y = rng.standard_normal(4000).astype(np.float32) * 1.5
    whole.update(y)
    bucket = np.float32(xl[1] - xl[0])
    off = np.float32(np.float32(xl[0]) / bucket)
    counts = sum(O.histogram(part, bucket, off).astype(np.uint64) for part in np.array_split(y, 4))
    shard.update_from_counts(counts, y.size)
    assert whole.compute(8).as_tuple() == shard.compute(8).as_tuple()
    np.testing.assert_array_equal(whole.histogram()[1], shard.histogram()[1])


@pytest.mark.ref
def test_oracle_vs_compiled_reference_random():
    """Randomized cross-check against the reference C++ compiled in place (build container only)."""
    from oracle import ref as R
    if not R.available():
        pytest.skip("reference not present")
    rng = np.random.default_rng(11)
    for t in range(60):
        x = (rng.standard_normal(1024) * rng.uniform(0.01, 20)).astype(np.float32)
        mn, mx = sorted(rng.uniform(-6, 6, 2))
        bw = int(rng.choice([4, 8, 16]))
        np.testing.assert_array_equal(bits(O.qdq_per_tensor(x, mn, mx, bw)), bits(R.qdq_per_tensor(x, mn, mx, bw)))
    for scheme in (0, 1, 3, 4):
        a, b = O.Analyzer(scheme), R.Analyzer(scheme)
        for _ in range(2):
            x = (rng.standard_normal(700) * 2 + 0.3).astype(np.float32)
            a.update(x)
            b.update(x)
        for fl in [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 0, 1)]:
            assert a.compute(8, *fl).as_tuple() == b.compute(8, *fl).as_tuple()


def test_torch_ref_learned_grid_vs_reference_python(golden_dir):
    """oracle/torch_ref.py (learned-grid restatement) == the reference module's own outputs."""
    import os
    import torch
    from oracle import torch_ref as T
    g = dict(np.load(os.path.join(golden_dir, "golden_lg.npz")))
    for i in range(int(g["count"])):
        x, grad = torch.from_numpy(g["c%d_x" % i]), torch.from_numpy(g["c%d_grad" % i])
        emin, emax = torch.from_numpy(g["c%d_emin" % i]), torch.from_numpy(g["c%d_emax" % i])
        bw, sym = (int(v) for v in g["c%d_cfg" % i])
        y = T.lg_forward(x, emin, emax, bw, bool(sym))[0]
        np.testing.assert_array_equal(bits(y.numpy()), bits(g["c%d_y" % i]))
        gx, gmin, gmax = T.lg_gradients(x, grad, emin, emax, bw, bool(sym))
        np.testing.assert_array_equal(bits(gx.numpy()), bits(g["c%d_gx" % i]))
        np.testing.assert_allclose(gmin.numpy(), g["c%d_gmin" % i], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(gmax.numpy(), g["c%d_gmax" % i], rtol=1e-6, atol=1e-6)


def test_torch_ref_adaround_round_loss_kat(kat):
    import torch
    from oracle import torch_ref as T
    k = kat["adaround_round_loss"]
    np.random.seed(k["seed"])
    alpha = torch.from_numpy(np.random.rand(*k["shape"]))
    loss = T.adaround_round_loss(alpha, k["reg_param"], kat["adaround_beta"]["expected"])
    assert abs(float(loss) - k["expected"]) < 10 ** -k["places"]


def test_torch_ref_adaround_pinned_to_reference(golden_dir):
    """oracle/torch_ref.adaround_forward / adaround_round_loss (the restatement the GPU tests and the
    optimizer-loop test use) reproduce the reference's apply_adaround / compute_round_loss
    (golden_adaround.npz) bit for bit on the CPU (one thread)."""
    import os
    import torch
    from oracle import torch_ref as T
    z = np.load(os.path.join(golden_dir, "golden_adaround.npz"))
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        for i in range(int(z["count"])):
            k = "c%d_" % i
            w = torch.from_numpy(z[k + "w"])
            shape = (-1,) + (1,) * (w.dim() - 1)
            d = torch.from_numpy(z[k + "delta"]).view(shape)
            o = torch.from_numpy(z[k + "offset"]).view(shape)
            a = torch.from_numpy(z[k + "alpha"]).requires_grad_(True)
            wq = T.adaround_forward(w, a, d, o, int(z[k + "bw"]))
            assert np.array_equal(wq.detach().numpy().view(np.int32), z[k + "wq"].view(np.int32)), i
            (wq * torch.from_numpy(z[k + "grad"])).sum().backward()
            assert np.array_equal(a.grad.numpy().view(np.int32), z[k + "ga_recon"].view(np.int32)), i
            rl = T.adaround_round_loss(a.detach(), float(z["reg_param"]), float(z[k + "beta"]))
            assert float(rl) == float(z[k + "round_loss"]), i
    finally:
        torch.set_num_threads(nt)


def test_lg_encoding_gradient_bound_holds_for_the_reference(golden_dir):
    """The stated bound of the learned-grid encoding gradients (oracle/torch_ref.py:
    lg_encoding_grads_bound): the reference module's own fp32 results (golden_lg.npz) lie within
    16 eps x (sum of |terms|) of the float64 sums -- the bound the GPU kernels are held to."""
    import os
    import numpy as np
    import torch
    from oracle import torch_ref as T
    g = dict(np.load(os.path.join(golden_dir, "golden_lg.npz")))
    for i in range(5):
        x, gr = torch.from_numpy(g["c%d_x" % i]), torch.from_numpy(g["c%d_grad" % i])
        emin, emax = torch.from_numpy(g["c%d_emin" % i]), torch.from_numpy(g["c%d_emax" % i])
        bw, sym = (int(v) for v in g["c%d_cfg" % i])
        ex_min, ex_max, b_min, b_max = T.lg_encoding_grads_bound(x, gr, emin, emax, bw, bool(sym))
        T.assert_within_sum_bound(torch.from_numpy(g["c%d_gmin" % i]), ex_min, b_min, 16, "grad_min %d" % i)
        T.assert_within_sum_bound(torch.from_numpy(g["c%d_gmax" % i]), ex_max, b_max, 16, "grad_max %d" % i)
