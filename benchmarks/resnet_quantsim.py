"""Config 1 (BASELINE.json / SURVEY §8(d)): ResNet-50 W8A8 per-tensor QuantizationSimModel
compute_encodings, quant schemes TF-Enhanced and TF, 8 calibration batches x 32 images U(0,1)
(seed 1234), 224x224, random-init ResNet-50 (seed 0). Reported per scheme:
  * compute_encodings wall-clock on one MI355X (ANALYSIS forwards + statistics + encodings),
  * whether EVERY encoding (54 input/output activation quantizers + 54 weights) equals the CPU
    oracle's (oracle/dlq_oracle.c) fed exactly the tensors each quantizer saw, and
  * that CPU restatement's own time for the same statistics + encodings (1 thread): the
    reference's CPU path.
Plus config 2's end-to-end step: the W8A8 per-channel QuantSim forward of a batch of 256 (convs on
MIOpen, every activation / weight QDQ through the gfx950 kernels) against the fp32 forward.

  python benchmarks/resnet_quantsim.py [--batches 8] [--batch 32] [--e2e-batch 256] [--no-oracle]
  python benchmarks/resnet_quantsim.py --cpu-model --repeats 3   # config 1 as stated: the aimet_torch CPU path

--cpu-model: the model and the calibration images stay on the host (the reference's aimet_torch CPU
path: forwards on the host cores); every quantizer's statistics and QDQ run on the MI355X, the
tensors staged through HBM (aimet_amd.tensor_quantizer._stage). No config-2 step in this mode. The
host cores are shared on the GPU box, so host-forward times vary run to run: each figure is the
minimum of --repeats runs (all runs listed).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def record_stats(sim):
    """Patch every quantizer's update/reset to also keep a host copy of what it was fed."""
    from aimet_amd.quantizers import StaticGridPerTensorQuantizer
    seen = {}
    for name, w in sim.quant_wrappers():
        for kind, qs in (("in", list(w.input_quantizers)), ("out", list(w.output_quantizers)),
                         ("param", list(w.param_quantizers.values()))):
            for i, q in enumerate(qs):
                if not isinstance(q, StaticGridPerTensorQuantizer):
                    continue
                key = (name, kind, i)
                seen[key] = []
                upd, rst = q.update_encoding_stats, q.reset_encoding_stats

                def u(t, upd=upd, key=key, q=q):
                    if q.enabled and not q.is_encoding_frozen and q.bitwidth != 32:
                        seen[key].append(t.detach().float().reshape(-1).cpu().numpy())
                    return upd(t)

                def r(rst=rst, key=key, q=q):
                    if not q.is_encoding_frozen:
                        seen[key] = []
                    return rst()
                q.update_encoding_stats, q.reset_encoding_stats = u, r
    return seen


def quantizer_map(sim):
    out = {}
    for name, w in sim.quant_wrappers():
        for kind, qs in (("in", list(w.input_quantizers)), ("out", list(w.output_quantizers)),
                         ("param", list(w.param_quantizers.values()))):
            for i, q in enumerate(qs):
                out[(name, kind, i)] = q
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--e2e-batch", type=int, default=256)
    ap.add_argument("--e2e-steps", type=int, default=5)
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--cpu-model", action="store_true")
    ap.add_argument("--repeats", type=int, default=1,
                    help="timed compute_encodings (and, with --cpu-model, host forward) runs; the minimum is reported")
    args = ap.parse_args()

    from aimet_amd.quantizers import QuantScheme
    from aimet_amd.quantsim import QuantizationSimModel
    from workloads.resnet import resnet50

    torch.cuda.set_device(0)
    dev = torch.device("cpu") if args.cpu_model else torch.device("cuda", 0)
    model = resnet50(seed=0, device=dev).eval()
    g = torch.Generator().manual_seed(1234)
    images = torch.rand(args.batches * args.batch, 3, 224, 224, generator=g).to(dev)
    batches = [images[b * args.batch:(b + 1) * args.batch] for b in range(args.batches)]
    dummy = batches[0][:1]

    def calibrate(m, _):
        for b in batches:
            m(b)

    res = {"metric": "ResNet-50 W8A8 per-tensor compute_encodings wall-clock", "unit": "s",
           "higher_is_better": False, "n_gpus": 1, "calibration": "%d batches x %d images U(0,1) seed 1234"
           % (args.batches, args.batch), "model_device": str(dev),
           "host_threads": torch.get_num_threads() if args.cpu_model else None, "schemes": {}}
    for scheme in (QuantScheme.post_training_tf_enhanced, QuantScheme.post_training_tf):
        sim = QuantizationSimModel(model, dummy, quant_scheme=scheme, default_output_bw=8, default_param_bw=8)
        # warm (kernels, MIOpen algorithm selection); timed run on a fresh calibration
        sim.compute_encodings(calibrate, None)
        runs = []
        for _ in range(args.repeats):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sim.compute_encodings(calibrate, None)
            torch.cuda.synchronize()
            runs.append(time.perf_counter() - t0)
        secs = min(runs)
        qmap = quantizer_map(sim)
        n_enc = sum(1 for q in qmap.values() if q.enabled and q.encoding is not None)
        in_q = None
        if args.cpu_model:
            # one more calibration with every quantizer's statistics call timed (staging the host
            # tensor into HBM + the device statistics, synchronised): QuantSim's own share of the call
            spent = [0.0]
            saved = {}
            for key, q in qmap.items():
                upd = q.update_encoding_stats
                saved[key] = upd

                def u(t, upd=upd):
                    t0 = time.perf_counter()
                    r = upd(t)
                    torch.cuda.synchronize()
                    spent[0] += time.perf_counter() - t0
                    return r
                q.update_encoding_stats = u
            sim.compute_encodings(calibrate, None)
            torch.cuda.synchronize()
            for key, q in qmap.items():
                q.update_encoding_stats = saved[key]
            in_q = round(spent[0], 4)
        r = {"compute_encodings_s": round(secs, 4), "compute_encodings_runs_s": [round(v, 4) for v in runs],
             "quantizers": n_enc}
        if in_q is not None:
            r["quantizer_statistics_calls_s"] = in_q
        if not args.no_oracle:
            from oracle import oracle as O
            seen = record_stats(sim)
            sim.compute_encodings(calibrate, None)
            torch.cuda.synchronize()
            mode = O.QUANTIZATION_TF_ENHANCED if scheme == QuantScheme.post_training_tf_enhanced \
                else O.QUANTIZATION_TF
            ok, checked, elems, t_cpu = True, 0, 0, 0.0
            mismatch = []
            for key, chunks in seen.items():
                q = qmap[key]
                if not q.enabled or q.encoding is None or not chunks:
                    continue
                t0 = time.perf_counter()
                a = O.Analyzer(mode)
                for c in chunks:
                    a.update(c)
                    elems += c.size
                want = a.compute(q.bitwidth, q.use_symmetric_encodings, q.use_strict_symmetric,
                                 q.use_unsigned_symmetric).as_tuple()
                t_cpu += time.perf_counter() - t0
                checked += 1
                if q.encoding.to_tuple() != want:
                    ok = False
                    mismatch.append([list(key), q.encoding.to_tuple(), want])
            r.update({"encodings_equal_cpu_oracle": ok, "oracle_checked_quantizers": checked,
                      "statistics_elems": elems, "cpu_oracle_1thread_s": round(t_cpu, 3),
                      "speedup_vs_cpu_oracle": round(t_cpu / secs, 1)})
            if mismatch:
                r["mismatches"] = mismatch[:5]
            del seen
        res["schemes"][scheme.name] = r
        del sim
        torch.cuda.empty_cache()

    if args.cpu_model:
        # the same 8 forwards of the plain model: what the calibration costs without QuantSim
        fw = []
        with torch.no_grad():
            for _ in range(args.repeats):
                t0 = time.perf_counter()
                calibrate(model, None)
                fw.append(time.perf_counter() - t0)
        res["host_fp32_forwards_s"] = round(min(fw), 4)
        res["host_fp32_forwards_runs_s"] = [round(v, 4) for v in fw]
        for r in res["schemes"].values():
            r.pop("speedup_vs_cpu_oracle", None)   # the timed call includes the host forwards here
        res["note"] = ("host forwards dominate and the host cores are shared: compute_encodings_s vs "
                       "host_fp32_forwards_s is within run-to-run noise; quantizer_statistics_calls_s is "
                       "the time inside every quantizer's statistics call (HBM staging + device statistics)")
        res["data"] = "synthetic U(0,1) images (seed 1234), random-init ResNet-50 (seed 0) on the host"
        print(json.dumps(res), flush=True)
        return

    # config 2 end-to-end step: W8A8 per-channel QuantSim forward, batch 256
    cfg = {"defaults": {"params": {"is_symmetric": "True"}, "ops": {"is_symmetric": "False"},
                        "per_channel_quantization": "True"}}
    sim = QuantizationSimModel(model, dummy, quant_scheme=QuantScheme.post_training_tf_enhanced,
                               default_output_bw=8, default_param_bw=8, config_file=cfg)
    sim.compute_encodings(calibrate, None)
    x = torch.rand(args.e2e_batch, 3, 224, 224, generator=torch.Generator().manual_seed(99)).to(dev)

    def timed(fn):
        with torch.no_grad():
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.e2e_steps):
                fn()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.e2e_steps * 1e3

    q_ms = timed(lambda: sim.model(x))
    f_ms = timed(lambda: model(x))
    res["e2e_step"] = {"batch": args.e2e_batch, "quantsim_forward_ms": round(q_ms, 2),
                       "fp32_forward_ms": round(f_ms, 2), "quantization_overhead_ms": round(q_ms - f_ms, 2),
                       "note": "W8A8 per-channel TF-E QuantSim forward (MIOpen convs + gfx950 QDQ, eager) vs the "
                               "same model unquantized"}
    res["data"] = "synthetic U(0,1) images (seed 1234 / 99), random-init ResNet-50 (seed 0)"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
