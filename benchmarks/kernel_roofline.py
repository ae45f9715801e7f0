"""Per-kernel roofline of every hot-path kernel on one MI355X.

For each kernel: average launch time over R launches (HIP events on the launch stream), achieved
GB/s from the ALGORITHMIC bytes per element of SURVEY §8(d), fraction of the 8 TB/s HBM peak,
and beside it
  * the CPU restatement of the reference (oracle/, 1 thread) on a bounded sample, and
  * for the rows the reference implements as torch ops (a13 STE, a14 learned grid, a15 AdaRound),
    that torch-op sequence (oracle/torch_ref.py) run on the same GPU: the reference's own GPU path.

usage: python benchmarks/kernel_roofline.py [--elems N] [--reps R] [--cpu-elems M] [--out FILE]
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

HBM_PEAK = 8000.0   # GB/s, MI355X_MICROARCH.md


def timed(fn, reps, stream):
    fn()   # warm
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def cpu_timed(fn, min_s=1.0):
    fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= min_s:
            return dt / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=1 << 28)
    ap.add_argument("--channels", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-elems", type=int, default=1 << 22)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import aimet_amd
    from aimet_amd import _native
    from aimet_amd.libpymo import QuantizationMode, TfEncoding, encodings_to_c
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    from oracle import oracle as O
    from oracle import torch_ref as T

    torch.set_num_threads(1)
    lib = aimet_amd.native_library()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    N, C = args.elems, args.channels
    K = N // C
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, device=dev, generator=g) * 2 + 0.3
    y = torch.empty_like(x)
    grad = torch.randn(N, device=dev, generator=g)
    gx = torch.empty_like(x)
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731

    enc = TfEncoding()
    enc.min, enc.max, enc.bw = -3.0, 5.0, 8
    encs = []
    for c in range(C):
        e = TfEncoding()
        e.min, e.max, e.bw = -2.5 - (c % 7) * 0.1, 3.0 + (c % 5) * 0.2, 8
        encs.append(e)
    table = torch.empty(4 * C, dtype=torch.float32, device=dev)
    _native.call("aimet_per_channel_table", encodings_to_c(encs), C, table.data_ptr(), sp)
    mins, maxs = table[:C].contiguous(), table[C:2 * C].contiguous()
    delta, offset = table[2 * C:3 * C].contiguous(), table[3 * C:].contiguous()
    alpha = torch.randn(N, device=dev, generator=g)
    w = (torch.randn(N, device=dev, generator=g) * 0.05)
    sums = torch.zeros(3 * C, dtype=torch.float32, device=dev)
    rloss = torch.zeros(1, dtype=torch.float32, device=dev)

    rows = []

    def row(name, ref, nbytes, ms, cpu=None, torch_gpu_ms=None, note=""):
        gbs = N * nbytes / (ms * 1e-3) / 1e9
        r = {"kernel": name, "row": ref, "elems": N, "bytes_per_elem": nbytes, "avg_ms": round(ms, 4),
             "achieved_GBps": round(gbs, 1), "frac_of_peak": round(gbs / HBM_PEAK, 4), "note": note}
        if cpu is not None:
            r["cpu_1core_Gelem_s"] = round(cpu, 4)
            r["gpu_vs_cpu"] = round(N / (ms * 1e-3) / 1e9 / cpu, 1)
        if torch_gpu_ms is not None:
            r["reference_torch_ops_on_gpu_ms"] = round(torch_gpu_ms, 4)
            r["speedup_vs_reference_torch_ops"] = round(torch_gpu_ms / ms, 2)
        rows.append(r)
        print(json.dumps(r), flush=True)

    # CPU samples
    M = args.cpu_elems
    xs = x[:M].cpu().numpy()
    gs = grad[:M].cpu().numpy()
    cpu = not args.no_cpu

    def cpu_rate(fn):
        return M / cpu_timed(fn) / 1e9 if cpu else None

    # a3: per-tensor QDQ / a4: quantize-only
    ms = timed(lambda: lib.aimet_qdq_per_tensor(P(x), P(y), N, ctypes.byref(enc), 0, 0, sp), args.reps, stream)
    row("qdq_per_tensor", "a3", 8, ms, cpu_rate(lambda: O.qdq_per_tensor(xs, enc.min, enc.max, 8)))
    ms = timed(lambda: lib.aimet_quantize_per_tensor(P(x), P(y), N, ctypes.byref(enc), 0, 1, 0, sp), args.reps,
               stream)
    row("quantize_per_tensor", "a4", 8, ms, cpu_rate(lambda: O.quantize_per_tensor(xs, enc.min, enc.max, 8, True)))
    # a3 / a5 with fp16 and bf16 I/O (casts fused: 4 B/elem) vs the reference's upcast-QDQ-downcast
    for dt, code in ((torch.float16, 1), (torch.bfloat16, 2)):
        x16, y16 = x.to(dt), torch.empty(N, dtype=dt, device=dev)
        ms = timed(lambda: lib.aimet_qdq_per_tensor_16(P(x16), P(y16), N, code, ctypes.byref(enc), 0, 0, sp),
                   args.reps, stream)

        def three_pass():
            xf = x16.to(torch.float32)
            lib.aimet_qdq_per_tensor(P(xf), P(y), N, ctypes.byref(enc), 0, 0, sp)
            return y.to(dt)
        t_ms = timed(three_pass, 2, stream)
        row("qdq_per_tensor %s I/O" % str(dt).split(".")[1], "a3", 4, ms, None, t_ms,
            note="reference: .to(float32) -> fp32 QDQ -> .to(dtype)")
        ms = timed(lambda: lib.aimet_qdq_per_channel_16(P(x16), P(y16), 1, C, K, code, P(table), 0, 0, sp),
                   args.reps, stream)
        row("qdq_per_channel %s I/O" % str(dt).split(".")[1], "a5", 4, ms)
        del x16, y16
    # a5: per-channel QDQ
    ms = timed(lambda: lib.aimet_qdq_per_channel(P(x), P(y), 1, C, K, P(table), 0, 0, sp), args.reps, stream)
    Cs = max(1, M // K)
    tab_h = table.view(4, C)[:, :Cs].contiguous().cpu().numpy().ravel()
    row("qdq_per_channel", "a5", 8, ms,
        cpu_rate(lambda: O.qdq_per_channel(xs[:Cs * K], Cs, K, tab_h)) if M >= K else None,
        note="C=%d K=%d" % (C, K))
    # a13: STE backward (per-channel bounds) vs the reference's torch ops
    ms = timed(lambda: lib.aimet_ste_backward(P(x), P(grad), P(gx), 1, C, K, P(mins), P(maxs), sp), args.reps, stream)
    xv, gv = x.view(C, K), grad.view(C, K)
    mn_b, mx_b = mins.view(C, 1), maxs.view(C, 1)
    t_ms = timed(lambda: gv * ((xv >= mn_b) & (xv <= mx_b)).float(), max(2, args.reps // 2), stream)
    row("ste_backward", "a13", 12, ms, cpu_rate(lambda: O.ste_backward(xs, gs, [-2.5], [3.0])), t_ms)
    # a7 / a8: statistics passes
    # (a TF quantizer: a histogram quantizer only takes min/max on its first batch)
    qt = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF)
    ms = timed(lambda: qt.batch_minmax(x), args.reps, stream)
    q = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED)
    q.batch_minmax(x)
    q.fold_minmax()
    row("minmax (stats pass 1)", "a7", 4, ms, cpu_rate(lambda: (O.get_min(xs), O.get_max(xs))))
    ms = timed(lambda: q.batch_histogram(x), args.reps, stream)
    row("histogram 512 bins (stats pass 2)", "a8", 4, ms,
        cpu_rate(lambda: O.histogram(xs, np.float32(0.0469), np.float32(-150.0))))
    # §8(f) row 3: entropy analyzer -- the histogram pass alone (binning with the range widened
    # every batch) and a whole updateStats (min/max + widen + histogram + fold: two reads of x)
    qe = AimetTensorQuantizer(QuantizationMode.QUANTIZATION_ENTROPY)
    qe.updateStats(x, True)
    ms = timed(lambda: qe.batch_histogram(x), args.reps, stream)
    row("entropy histogram 512 bins", "f3", 4, ms)
    oe = O.Analyzer(O.QUANTIZATION_ENTROPY)
    ms = timed(lambda: qe.updateStats(x, True), args.reps, stream)
    row("entropy updateStats (4 launches)", "f3", 8, ms, cpu_rate(lambda: oe.update(xs)),
        note="cpu = updateTensorHistogram_cpu restated (the reference GPU build copies to the host and runs it)")
    # §8(f) row 4: blockwise (LPBQ-style) QDQ over a [C, K] weight with 64-element blocks along K
    # (contiguous blocks: 2 merged dims) and over its transpose [K, C] (blocks strided: 3 dims),
    # plus the fp16 round trip of float quantizers
    from aimet_amd.onnx_op import BroadcastShapeInfo
    Kb = N // C
    for shape, ch, ba in (((C, Kb), 0, 1), ((Kb, C), 1, 0)):
        info = BroadcastShapeInfo(shape, ch, ba, 64)
        E = info.numEncodings
        etab = torch.empty(4, E, device=dev)
        etab[2].uniform_(0.01, 0.02)
        etab[3].fill_(-8.0)
        etab[0] = etab[2] * -8
        etab[1] = etab[2] * 7
        nd = info.numDims
        ts = (ctypes.c_int64 * nd)(*info.tensorStrides)
        es = (ctypes.c_int64 * nd)(*info.encodingStrides)
        ms = timed(lambda: lib.aimet_qdq_broadcast(P(x), P(y), N, nd, ts, es, P(etab[0]), P(etab[1]), P(etab[2]),
                                                   P(etab[3]), sp), args.reps, stream)
        row("qdq_blockwise %s block 64" % ("x".join(map(str, shape))), "f4", 8, ms,
            note="%d encodings, %s blocks" % (E, "contiguous" if info.hasContiguousBlocks() else "strided"))
    ms = timed(lambda: lib.aimet_qdq_fp16(P(x), P(y), N, sp), args.reps, stream)
    row("qdq_fp16 (float quantizer)", "f4", 8, ms)
    # a14: learned grid forward / backward vs the reference's torch ops
    steps = 255.0
    ms = timed(lambda: lib.aimet_lg_forward(P(x), P(y), 1, C, K, P(delta), P(offset), ctypes.c_float(steps), sp),
               args.reps, stream)
    emin, emax = mins.clone(), maxs.clone()
    t_ms = timed(lambda: T.lg_forward(xv, emin, emax, 8), 2, stream)
    row("learned_grid_forward", "a14", 8, ms, None, t_ms)
    ms = timed(lambda: (sums.zero_(), lib.aimet_lg_backward(P(x), P(grad), P(gx), P(sums), 1, C, K, P(delta),
                                                              P(offset), ctypes.c_float(steps), None, sp)),
               args.reps, stream)
    t_ms = timed(lambda: T.lg_gradients(xv, gv, emin, emax, 8), 2, stream)
    row("learned_grid_backward (+ per-channel sums)", "a14", 12, ms, None, t_ms)
    # a15: AdaRound soft-quant forward / backward (+ round loss)
    ms = timed(lambda: lib.aimet_adaround_forward(P(w), P(alpha), P(y), 1, C, K, P(delta), P(offset), 8, 1, sp),
               args.reps, stream)
    wv, av = w.view(C, K), alpha.view(C, K)
    d_b, o_b = delta.view(C, 1), offset.view(C, 1)
    t_ms = timed(lambda: T.adaround_forward(wv, av, d_b, o_b, 8), 2, stream)
    row("adaround_forward", "a15", 12, ms, None, t_ms)
    ms = timed(lambda: (rloss.zero_(), lib.aimet_adaround_backward(P(w), P(alpha), P(grad), P(gx), 1, C, K, P(delta),
                                                                     P(offset), 8, ctypes.c_double(0.01),
                                                                     ctypes.c_double(10.0), P(rloss), sp)),
               args.reps, stream)

    def torch_ada_bwd():
        a = av.detach().requires_grad_(True)
        out = T.adaround_forward(wv, a, d_b, o_b, 8)
        loss = (out * gv).sum() + T.adaround_round_loss(a, 0.01, 10.0)
        loss.backward()
    t_ms = timed(torch_ada_bwd, 2, stream)
    row("adaround_backward (+ round loss)", "a15", 16, ms, None, t_ms,
        note="reference: torch forward + autograd backward + round loss; alpha ~ N(0, 1): %.1f %% of the "
             "rectified sigmoids saturate" % (100 * float((alpha.abs() > math.log(11.0)).float().mean())))
    # a converging loop's alphas: N(0, 16) saturates ~55 % of them (the wave-compacted rounding-loss
    # pows then run for the rest only); with and without the loss value (the optimisation loop's form)
    alpha_sat = alpha * 4.0
    sat = 100 * float((alpha_sat.abs() > math.log(11.0)).float().mean())
    for want_loss in (True, False):
        ms = timed(lambda: (rloss.zero_(), lib.aimet_adaround_backward(
            P(w), P(alpha_sat), P(grad), P(gx), 1, C, K, P(delta), P(offset), 8, ctypes.c_double(0.01),
            ctypes.c_double(10.0), P(rloss) if want_loss else None, sp)), args.reps, stream)
        row("adaround_backward (%s), %.0f %% saturated" % ("+ round loss" if want_loss else "gradient only", sat),
            "a15", 16, ms, note="alpha ~ N(0, 16)")

    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
