"""bench.py -- fake-quant throughput of the MI355X quantization-simulation core.

Workload (BASELINE.json configs[1]): ResNet-50 W8A8 fake-quant forward, synthetic 224x224 batch of
256 per GPU, i.e. every tensor QuantizationSimModel quantize-dequantizes in one forward:
  * the model input + the 54 conv/fc outputs, per-tensor 8-bit (2.884 G elements), and
  * the 54 conv/fc weights, per-channel (axis 0) symmetric 8-bit (25.5 M elements, 27,560 channels).
Activations come from one real fp32 forward of a random-init ResNet-50 (seed 0) on U(0,1) images
(seed 1234 + rank) and stay resident in HBM; a "step" quantize-dequantizes all of them once.
Encodings are computed first (TF-Enhanced activations, TF-Enhanced per-channel weights =
QuantizationSimModel's default scheme) and that compute_encodings wall-clock is reported too.

Multi-GPU: one process per GPU (torch.distributed, RCCL). Each rank runs its own batch (weak
scaling, no data-path collective); calibration is sharded per sample across ranks with one RCCL
exchange of the packed statistics per batch (aimet_amd.distributed).

At N=1 the line also carries BASELINE configs 3 and 5 (`secondary`), each run by its own benchmark
in a child process after the headline (benchmarks/adaround_mobilenet.py: MobileNet-v2 AdaRound, all
53 layers x 10k iterations; benchmarks/llama_qat.py: Llama-3-8B W4A16 QAT at seq 2048, mb 1, full
model, beside the same step without quantizers), within a time budget that keeps the whole run
inside the driver's limit; a config that fails or does not fit is recorded as such in the line.
The process that launches them never touches the GPU (the headline runs in a child too).

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BYTES_QDQ = 8            # fp32 read + fp32 write per element
# HBM bytes per step of the activation QDQ launches from the rocprofv3 PMC passes of this bench
# (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM; separate --pmc FETCH_SIZE / WRITE_SIZE runs,
# tools/runs/r05/gpu_r05_g.sh): profiles/r05/bench_pmc_summary.txt, 11.5375 + 11.5359 = 23.0734 GB
# (measured at the default workload: 2,883,971,072 activation elements per step; other batch sizes
# report null). The same figure as rounds 1-4 (the QDQ kernels are unchanged).
TRAFFIC_GB = 23.0734
TRAFFIC_ELEMS = 2883971072


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)   # ~0.37 s timed region at N=1
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--cpu-sample-images", type=int, default=32,
                   help="images of each activation tensor (plus all weights) timed on the CPU oracle")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--enc-reps", type=int, default=9, help="timed compute_encodings_resident calls after the cold one")
    p.add_argument("--plan-reps", type=int, default=25,
                   help="timed CalibrationPlan runs (the compute_encodings headline), after 2 untimed ones")
    p.add_argument("--eager", action="store_true", help="launch every QDQ from Python instead of HIP graphs")
    p.add_argument("--per-weight-launches", action="store_true",
                   help="one per-channel QDQ launch per weight instead of the batched plan")
    p.add_argument("--no-dropin", action="store_true",
                   help="skip the drop-in surface timings (QuantizationSimModel.compute_encodings of config 1, "
                        "the StaticGridQuantWrapper forward of config 2)")
    p.add_argument("--no-secondary", action="store_true",
                   help="skip BASELINE configs 3 and 5 (run at N=1 after the headline, in child processes)")
    p.add_argument("--secondary-budget", type=float, default=480.0,
                   help="seconds from the start of bench.py by which the secondary configs must end")
    p.add_argument("--force-exchange", action="store_true",
                   help="at N=1 form a world-size-1 RCCL group before any GPU call and time the sharded "
                        "calibration's staged form (both packed collectives through RCCL) beside the headline")
    return p.parse_args()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N copies of this script, one per GPU, with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, and wait for them. This parent never touches the
    GPU (torch.cuda.device_count() does not initialise HIP on this image); it only counts devices.
    Rank 0 writes the JSON line to the inherited stdout. If any rank fails, the others are stopped
    and the parent exits with that rank's status."""
    backend = os.environ.get("AIMET_BENCH_BACKEND", "nccl")
    if backend == "nccl" and not os.environ.get("AIMET_BENCH_LAUNCH_CHECK"):
        ndev = torch.cuda.device_count()
        if ndev < n:
            print("bench.py --gpus %d: only %d GPU(s) visible; RCCL needs one GPU per rank "
                  "(AIMET_BENCH_BACKEND=gloo rehearses several ranks on fewer GPUs)" % (n, ndev), file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print("bench.py: rank %d exited with %d; stopping the other ranks" % (procs.index(p), code),
                      file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


def launch_check(world, rank):
    """AIMET_BENCH_LAUNCH_CHECK=1: form the process group exactly as the bench does (no GPU work)
    and report what formed: the CPU test of the launcher (tests/test_bench_launch.py)."""
    backend = os.environ.get("AIMET_BENCH_BACKEND", "nccl")
    if os.environ["AIMET_BENCH_LAUNCH_CHECK"] == "fail%d" % rank:
        sys.exit(3)   # the launcher's failure path (a rank dying before the group forms)
    dist.init_process_group(backend, rank=rank, world_size=world)
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": dist.get_world_size(), "dist_backend": dist.get_backend(),
                          "rank_sum": int(t.item())}), flush=True)
    dist.destroy_process_group()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher formed WORLD_SIZE=%d" % (args.gpus, world))
    # AIMET_BENCH_BACKEND=gloo rehearses the N-rank path with several ranks sharing fewer GPUs
    # (RCCL needs one GPU per rank); the statistics exchange then stages through host memory
    backend = os.environ.get("AIMET_BENCH_BACKEND", "nccl")
    if backend == "nccl" and world > 1 and torch.cuda.device_count() < world:
        raise SystemExit("bench.py: %d ranks over RCCL but only %d GPU(s) visible" % (world, torch.cuda.device_count()))
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1 or args.force_exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    else:
        torch.cuda.set_device(local)
    return rank, world, torch.device("cuda", local)


def collect_tensors(model, x):
    """Run the fp32 forward once; keep the model input and every conv/fc output resident."""
    acts = [("input", x)]
    hooks = []
    for name, mod in model.named_modules():
        if isinstance(mod, (torch.nn.Conv2d, torch.nn.Linear)):
            hooks.append(mod.register_forward_hook(
                lambda m, i, o, name=name: acts.append((name, o.detach().contiguous()))))
    with torch.no_grad():
        model(x)
    for h in hooks:
        h.remove()
    weights = [(name, mod.weight.detach().contiguous()) for name, mod in model.named_modules()
               if isinstance(mod, (torch.nn.Conv2d, torch.nn.Linear))]
    return acts, weights


def make_quantizers(acts, weights):
    """The sim's quantizers for this workload: TF-Enhanced per-tensor activations, TF-Enhanced
    per-channel weights (QuantizationSimModel's default scheme)."""
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    aq = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in acts]
    wq = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED, num_channels=w.shape[0]) for _, w in weights]
    return aq, wq


def time_plan(plan, reps, warm=2, spans=None, phases=None):
    """`warm` untimed, then `reps` timed plan runs that reset and recompute the plan's quantizers
    (one compute_encodings of an existing sim each); returns (median seconds, encodings of the last
    run, every timed run in ms). spans (a list): each run's GPU span in ms, a HIP event on the main
    stream before the launch to one enqueued right behind it (after the activations' search)."""
    secs, res = [], None
    stream = torch.cuda.current_stream()
    for i in range(warm + reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # the previous run's results are released before the clock starts: freeing its 27,560
        # encoding objects is not this run's work (it had sat behind the activations' result,
        # ~0.25 ms of every timed run, profiles/r05/README.md)
        res = p_res = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        a, p = plan.launch(reset=True)
        e1.record(stream)
        t1 = time.perf_counter()
        p_res = p.result()
        t2 = time.perf_counter()
        res = (a.result(), p_res)
        if i >= warm:
            secs.append(time.perf_counter() - t0)
            if phases is not None:   # host: launch returned, parameters' encodings built (ms)
                phases.append((round((t1 - t0) * 1e3, 3), round((t2 - t0) * 1e3, 3)))
            if spans is not None:
                torch.cuda.synchronize()
                spans.append(round(e0.elapsed_time(e1), 3))
    return sorted(secs)[len(secs) // 2], res, [round(v * 1e3, 3) for v in secs]


def compute_encodings(acts, weights, quantizers=None):
    """compute_encodings as QuantizationSimModel does it for this workload (v1/quantsim.py:381-449):
    TF-Enhanced stats for every activation, TF-Enhanced per-channel symmetric for every weight.
    quantizers=None: new quantizers are created inside the timed region (a first calibration);
    else the (aq, wq) of an earlier call -- the sim's quantizers, created with the sim -- are reset
    (resetEncodingStats of every quantizer, v1/quantsim.py:387-399) and recomputed."""
    from aimet_amd.calibration import compute_encodings_resident
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if quantizers is None:
        aq, wq = make_quantizers(acts, weights)
    else:
        aq, wq = quantizers
    # activations (sharded across ranks, one packed collective per phase) and per-channel weights
    # on a second stream, after the reset of the sim's quantizers: aimet_amd.calibration
    a_res, w_res = compute_encodings_resident(aq, [t for _, t in acts], wq, [w for _, w in weights],
                                              act_settings=(8, False, False, False),
                                              param_settings=(8, True, False, False),
                                              reset=quantizers is not None)
    act_enc = [e for e, _ in a_res]
    w_enc = [e for e, _ in w_res]
    return act_enc, w_enc, time.perf_counter() - t0, aq, wq


def dropin_surface(model, dev, qdq_kernel_ms, reps=3):
    """The caller surface a user of the reference drives (aimet_amd.quantsim, v1/quantsim.py:425-449,
    v1/qc_quantize_op.py:705-745), timed on the same random-init ResNet-50:
      * config 1: QuantizationSimModel(quant_scheme=post_training_tf_enhanced, W8A8 per-tensor)
        .compute_encodings over 8 x 32 U(0,1) images (seed 1234) -- ANALYSIS forwards through every
        StaticGridQuantWrapper + statistics + encodings -- beside the same 8 forwards of the plain
        model (median of `reps` runs each, after a warm run);
      * config 2: the W8A8 per-channel QuantSim forward of the bench's batch-256 shape (eager,
        MIOpen convolutions, every QDQ through the wrappers) minus the unquantized forward, beside
        the QDQ kernel time of the headline step (the wrappers' Python cost is the rest)."""
    from aimet_amd.quantizers import QuantScheme
    from aimet_amd.quantsim import QuantizationSimModel
    g = torch.Generator(device=dev).manual_seed(1234)
    images = torch.rand(8 * 32, 3, 224, 224, device=dev, generator=g)
    batches = [images[b * 32:(b + 1) * 32] for b in range(8)]

    def calibrate(m, _):
        with torch.no_grad():
            for b in batches:
                m(b)

    def median_s(fn):
        fn()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]

    sim = QuantizationSimModel(model, batches[0][:1], quant_scheme=QuantScheme.post_training_tf_enhanced,
                               default_output_bw=8, default_param_bw=8)
    ce = median_s(lambda: sim.compute_encodings(calibrate, None))
    fw = median_s(lambda: calibrate(model, None))
    n_q = sum(1 for _, w in sim.quant_wrappers() for q in list(w.output_quantizers) + list(w.input_quantizers) +
              list(w.param_quantizers.values()) if q.enabled and q.encoding is not None)
    del sim
    cfg = {"defaults": {"params": {"is_symmetric": "True"}, "ops": {"is_symmetric": "False"},
                        "per_channel_quantization": "True"}}
    sim = QuantizationSimModel(model, batches[0][:1], quant_scheme=QuantScheme.post_training_tf_enhanced,
                               default_output_bw=8, default_param_bw=8, config_file=cfg)
    sim.compute_encodings(calibrate, None)
    x = torch.rand(256, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(99))
    with torch.no_grad():
        q_ms = median_s(lambda: sim.model(x)) * 1e3
        f_ms = median_s(lambda: model(x)) * 1e3
    del sim, x, images, batches
    torch.cuda.empty_cache()
    return {"quantsim_compute_encodings_s": round(ce, 4), "quantsim_calibration_forwards_s": round(fw, 4),
            "quantsim_compute_encodings_minus_forwards_s": round(ce - fw, 4), "quantsim_quantizers": n_q,
            "quantsim_fwd_ms": round(q_ms, 2), "fp32_fwd_ms": round(f_ms, 2),
            "quantsim_fwd_qdq_overhead_ms": round(q_ms - f_ms, 2), "qdq_kernel_ms_per_step": round(qdq_kernel_ms, 3),
            "quantsim_fwd_python_overhead_ms": round(q_ms - f_ms - qdq_kernel_ms, 2),
            "what": "config 1: QuantizationSimModel(post_training_tf_enhanced, W8A8 per-tensor).compute_encodings "
                    "over 8 x 32 U(0,1) images vs the same 8 plain forwards; config 2: the W8A8 per-channel QuantSim "
                    "forward at batch 256 (eager, MIOpen convs) minus the fp32 forward, vs the headline step's QDQ "
                    "kernel time (weights + activations); medians of %d runs after a warm one" % reps}


def cpu_baseline(acts, weights, act_enc, w_enc, images, act_outs, w_outs):
    """The reference's CPU path on a bounded sample: oracle/_ref (the reference DlQuantization C++
    compiled from its own sources, TensorQuantizationSim::quantizeDequantizeTensor and
    quantizeDequantizePerChannel with COMP_MODE_CPU) when that library travelled with the tree,
    and the in-repo C restatement (oracle/dlq_oracle.c, single thread + OpenMP) beside it.

    The outputs of the timed reference run are then compared bit for bit with the GPU outputs of
    the same elements (act_outs / w_outs: the QDQ results of the last timed step), and the TF-E
    encodings the reference analyzers compute for the sampled weight channels with the GPU's."""
    from oracle import oracle as O
    xs, ws = [], []
    for (name, t), e in zip(acts, act_enc):
        xs.append((t[:images].cpu().numpy().ravel(), e))
    for (name, w), encs in zip(weights, w_enc):
        ws.append((w.cpu().numpy().ravel(), w.shape[0], w[0].numel(),
                   O.per_channel_table([e.to_tuple() for e in encs])))
    n = sum(x.size for x, _ in xs) + sum(w.size for w, _, _, _ in ws)

    def timed(qdq_t, qdq_c, keep=None):
        t0 = time.perf_counter()
        for x, e in xs:
            y = qdq_t(x, e)
            if keep is not None:
                keep.append(y)
        for w, C, K, tab in ws:
            y = qdq_c(w, C, K, tab)
            if keep is not None:
                keep.append(y)
        return time.perf_counter() - t0

    res = {"n": n}
    ref_lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle", "_ref", "libdlq_ref.so")
    have_ref = os.path.exists(ref_lib)
    outs = []
    res["port_s"] = timed(lambda x, e: O.qdq_per_tensor(x, e.min, e.max, 8), O.qdq_per_channel,
                          None if have_ref else outs)
    # the OpenMP variant of the same loops on the box's CPU share
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    res["omp_s"] = timed(lambda x, e: O.qdq_per_tensor_omp(x, e.min, e.max, 8, threads),
                         lambda w, C, K, tab: O.qdq_per_channel_omp(w, C, K, tab, threads))
    res["omp_threads"] = threads
    res["openmp"] = O.openmp_enabled()
    Analyzer = O.Analyzer
    if have_ref:
        from oracle import ref as R
        res["ref_s"] = timed(lambda x, e: R.qdq_per_tensor(x, e.min, e.max, 8), R.qdq_per_channel, outs)
        Analyzer = R.Analyzer
    # parity of the timed CPU outputs with the GPU's (bit patterns; NaN payloads canonicalised)
    gpu = [o[:images] for o in act_outs] + list(w_outs)
    mism = 0
    for want, got in zip(outs, gpu):
        a = np.asarray(want, np.float32).ravel()
        b = got.detach().cpu().numpy().ravel()
        ba, bb = a.view(np.uint32).copy(), b.view(np.uint32).copy()
        ba[np.isnan(a)] = 0x7FC00000
        bb[np.isnan(b)] = 0x7FC00000
        mism += int(np.count_nonzero(ba != bb)) if a.size == b.size else max(a.size, b.size)
    res["parity"] = {"parity_checked": len(outs) == len(gpu), "elements": n, "mismatches": mism,
                     "against": "oracle/_ref (reference C++)" if have_ref else "oracle/dlq_oracle.c"}
    # compute_encodings on the CPU, MEASURED on the whole batch (no projection): the reference
    # analyzers (TF-Enhanced) over every activation tensor (per-tensor, asymmetric) and every channel
    # of every weight (per-channel, symmetric), single-threaded, each tensor copied to the host
    # outside the timed spans; every encoding is compared with the GPU's. (The per-channel loop
    # calls the analyzers from Python, ~20 us per channel of call overhead the reference's C++ loop
    # would not have: the figure is an upper bound by that much.)
    TFE = 1
    act_s, act_mism = 0.0, 0
    for (name, t), e in zip(acts, act_enc):
        x = t.detach().cpu().numpy().ravel()
        t0 = time.perf_counter()
        a = Analyzer(TFE)
        a.update(x)
        got = a.compute(8).as_tuple()
        act_s += time.perf_counter() - t0
        act_mism += int(got != e.to_tuple())
        del x, a
    w_s, nch, enc_mism = 0.0, 0, 0
    for (w, C, K, _), encs in zip(ws, w_enc):
        w2 = w.reshape(C, K)
        t0 = time.perf_counter()
        row = []
        for c in range(C):
            a = Analyzer(TFE)
            a.update(w2[c])
            row.append(a.compute(8, True).as_tuple())
        w_s += time.perf_counter() - t0
        nch += C
        enc_mism += sum(1 for c, want in enumerate(row) if encs[c].to_tuple() != want)
    res["enc"] = {"value_s": round(act_s + w_s, 3), "activations_s": round(act_s, 3), "weights_s": round(w_s, 3),
                  "projected": False,
                  "sample": "the whole batch: TF-E statistics + encoding of all %d activation tensors (%d elements, "
                            "per-tensor) and all %d weight channels (per-channel symmetric), one thread"
                            % (len(acts), sum(t.numel() for _, t in acts), nch),
                  "act_encodings_checked": len(acts), "act_encoding_mismatches": act_mism,
                  "weight_channel_encodings_checked": nch, "weight_channel_encoding_mismatches": enc_mism,
                  "what": "reference analyzers (oracle/_ref)" if Analyzer is not O.Analyzer
                          else "C restatement analyzers (oracle/dlq_oracle.c)"}
    return res


def time_exchange(dev, act_quantizers, reps=20):
    """The two collectives of one sharded calibration batch (aimet_amd.distributed) at the packed
    sizes this workload exchanges: {-min, max} of every activation quantizer (all_reduce MAX) and
    512 int64 bin counts + 1 element count per histogram quantizer (all_reduce SUM). Median host
    wall time of `reps` synchronised calls, max over ranks, in ms."""
    from aimet_amd.distributed import _all_reduce
    n_hist = sum(1 for q in act_quantizers if q.uses_histogram)
    bufs = (("minmax_max", torch.zeros(2 * len(act_quantizers), dtype=torch.float32, device=dev), dist.ReduceOp.MAX),
            ("counts_sum", torch.zeros(513 * n_hist, dtype=torch.int64, device=dev), dist.ReduceOp.SUM))
    out = {}
    for key, t, op in bufs:
        ts = []
        for i in range(reps + 3):
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            _all_reduce(t, op, None)
            torch.cuda.synchronize()
            if i >= 3:
                ts.append(time.perf_counter() - t0)
        out[key] = round(_max_over_ranks(sorted(ts)[len(ts) // 2], dev) * 1e3, 4)
        out[key + "_bytes"] = t.numel() * t.element_size()
    return out


def _max_over_ranks(v, dev):
    t = torch.tensor([v], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _run_child(cmd, timeout, env=None):
    """One child benchmark: (its last JSON line or None, a note on failure)."""
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, timeout=timeout, env=env, cwd=REPO)
    except subprocess.TimeoutExpired:
        return None, "timed out after %.0f s" % timeout
    lines = [ln for ln in r.stdout.decode(errors="replace").splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return None, "exit status %d" % r.returncode
    try:
        return json.loads(lines[-1]), None
    except ValueError as e:
        return None, "unparsable line: %s" % e


def secondary_configs(t_start, budget):
    """BASELINE configs 3 and 5, each in a child process (its own GPU memory), in the time left of
    `budget` seconds since t_start; what ran, what failed and what did not fit."""
    out = {"budget_s": budget}
    runs = [
        # the AdaRound backward kernel alone at 2^28 elements, N(0, 1) alpha (its roofline line)
        ("adaround_backward_kernel_2p28", [sys.executable, "tools/studies/ada_bwd_tune.py", "--scales", "1",
                                           "--tag", "bench"], 20.0),
        ("config3_adaround_mobilenet_v2", [sys.executable, "benchmarks/adaround_mobilenet.py"], 150.0),
        ("config5_llama3_8b_w4a16_qat", [sys.executable, "benchmarks/llama_qat.py"], 150.0),
        ("config5_llama3_8b_no_quantizer", [sys.executable, "benchmarks/llama_qat.py", "--path", "plain"], 120.0),
    ]
    for key, cmd, need in runs:
        left = budget - (time.perf_counter() - t_start)
        if left < need:
            out[key] = {"skipped": "%.0f s of the budget left, %.0f s needed" % (left, need)}
            continue
        t0 = time.perf_counter()
        res, err = _run_child(cmd, timeout=left)
        wall = round(time.perf_counter() - t0, 1)
        out[key] = dict(res, child_wall_s=wall) if res is not None else {"error": err, "child_wall_s": wall}
    c3, c5, c5p = (out.get(k, {}) for k in ("config3_adaround_mobilenet_v2", "config5_llama3_8b_w4a16_qat",
                                             "config5_llama3_8b_no_quantizer"))
    if "value" in c3:
        out["config3_adaround_s"] = c3["value"]
    kb = out.get("adaround_backward_kernel_2p28", {})
    if "achieved_GBps" in kb:   # the last line: the loop's form, without the loss value
        out["adaround_bwd_GBps"] = kb["achieved_GBps"]
        out["adaround_bwd_frac_of_8TBps"] = kb["frac_of_peak"]
    if "ms_per_step" in c5:
        out["config5_qat_ms_per_step"] = c5["ms_per_step"]
        if "ms_per_step" in c5p:
            out["config5_no_quantizer_ms_per_step"] = c5p["ms_per_step"]
            out["config5_quantizer_ms_per_step"] = round(c5["ms_per_step"] - c5p["ms_per_step"], 2)
    return out


def orchestrate(args):
    """N=1 with the secondary configs: the headline bench in a child (this process never touches
    the GPU), then configs 3 and 5; one merged JSON line."""
    t_start = time.perf_counter()
    env = dict(os.environ, AIMET_BENCH_CHILD="1")
    res, err = _run_child([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], timeout=None, env=env)
    if res is None:
        print("bench.py: the headline run failed (%s)" % err, file=sys.stderr)
        return 1
    res["secondary"] = secondary_configs(t_start, args.secondary_budget)
    print(json.dumps(res), flush=True)
    return 0


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if (world_env is None and args.gpus == 1 and not args.no_secondary and not os.environ.get("AIMET_BENCH_CHILD")
            and not os.environ.get("AIMET_BENCH_LAUNCH_CHECK")):
        sys.exit(orchestrate(args))
    if os.environ.get("AIMET_BENCH_LAUNCH_CHECK"):
        return launch_check(int(world_env or 1), int(os.environ.get("RANK", "0")))
    rank, world, dev = setup_dist(args)
    import aimet_amd
    from aimet_amd import _native
    from aimet_amd._native import TfEncodingC
    from workloads.resnet import resnet50

    lib = aimet_amd.native_library()
    torch.manual_seed(1234 + rank)
    model = resnet50(seed=0, device=dev)
    x = torch.rand(args.batch, 3, 224, 224, device=dev, generator=torch.Generator(device=dev).manual_seed(1234 + rank))
    acts, weights = collect_tensors(model, x)
    del x
    torch.cuda.empty_cache()

    # compute_encodings wall-clock: the first call (cold: code objects load, pools grow, quantizers
    # created), the median of --enc-reps calls on fresh quantizers, and the median of --enc-reps
    # calls that reset and recompute the same quantizers (QuantizationSimModel.compute_encodings on
    # an existing sim: the headline); the encodings of the last call are used
    act_enc, w_enc, enc_cold, aq, wq = compute_encodings(acts, weights)
    fresh, warm = [], []
    for _ in range(args.enc_reps):
        del aq, wq
        act_enc, w_enc, secs, aq, wq = compute_encodings(acts, weights)
        fresh.append(secs)
    for _ in range(args.enc_reps):
        act_enc, w_enc, secs, aq, wq = compute_encodings(acts, weights, (aq, wq))
        warm.append(secs)
    enc_resident = sorted(warm)[len(warm) // 2] if warm else enc_cold
    enc_fresh = sorted(fresh)[len(fresh) // 2] if fresh else enc_cold
    # the headline: a calibration plan over the sim's quantizers and the resident activations,
    # prepared once (as the quantizers are created once with the sim), each timed run a reset +
    # recompute of every quantizer (aimet_amd.calibration.CalibrationPlan). Sharded at N > 1.
    from aimet_amd.calibration import CalibrationPlan
    cplan = CalibrationPlan(aq, [t for _, t in acts], wq, [w for _, w in weights])
    enc_spans, enc_phases = [], []
    enc_seconds, (a_res, w_res), enc_runs_ms = time_plan(cplan, max(1, args.plan_reps), spans=enc_spans,
                                                         phases=enc_phases)
    # the same on quantizers made for the plan alone (a new sim), for comparison
    nq, nw = make_quantizers(acts, weights)
    nplan = CalibrationPlan(nq, [t for _, t in acts], nw, [w for _, w in weights])
    new_spans = []
    enc_new_s, _, _ = time_plan(nplan, max(1, args.plan_reps), spans=new_spans)
    nplan.close()
    del nq, nw
    plan_act, plan_w = [e for e, _ in a_res], [e for e, _ in w_res]
    enc_plan_equal = ([e.to_tuple() for e in plan_act] == [e.to_tuple() for e in act_enc] and
                      [[x.to_tuple() for x in es] for es in plan_w] == [[x.to_tuple() for x in es] for es in w_enc])
    act_enc, w_enc = plan_act, plan_w
    enc_exchange = None
    if args.force_exchange and world == 1:
        # the sharded calibration's staged form on this rank (stage 1, RCCL MAX, stage 2, RCCL SUM,
        # stage 4) over a world-size-1 group: the per-rank cost the 1 -> N curve starts from.
        # Quantizers of their own (the plan binds them to the packed exchange buffers).
        xq, xw = make_quantizers(acts, weights)
        xplan = CalibrationPlan(xq, [t for _, t in acts], xw, [w for _, w in weights], force_exchange=True)
        x_s, (xa, xwr), x_runs = time_plan(xplan, max(1, args.plan_reps))
        enc_exchange = {"seconds": round(x_s, 4), "dist_backend": dist.get_backend(),
                        "world_formed": dist.get_world_size(),
                        "equal_to_headline": [e.to_tuple() for e, _ in xa] == [e.to_tuple() for e in act_enc] and
                        [[x.to_tuple() for x in es] for es, _ in xwr] == [[x.to_tuple() for x in es] for es in w_enc]}
        xplan.close()
        del xq, xw

    # ---- the step: every QDQ of one QuantSim forward, pre-bound C-ABI calls --------------------
    stream = torch.cuda.current_stream(dev)
    sptr = ctypes.c_void_p(stream.cuda_stream)
    act_calls, w_calls = [], []
    outs, act_outs = [], []
    for (name, t), e in zip(acts, act_enc):
        o = torch.empty_like(t)
        act_outs.append(o)
        act_calls.append((ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(o.data_ptr()), t.numel(), e.to_c()))
    for ((name, w), encs), q in zip(zip(weights, w_enc), wq):
        o = torch.empty_like(w)
        outs.append(o)
        table = q.channelTable(encs, dev)
        outs.append(table)
        w_calls.append((ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(o.data_ptr()), 1, w.shape[0], w[0].numel(),
                        ctypes.c_void_p(table.data_ptr())))
    n_act = sum(c[2] for c in act_calls)
    n_w = sum(c[2] * c[3] * c[4] for c in w_calls)
    n_step = n_act + n_w
    qdq_t = lib.aimet_qdq_per_tensor
    qdq_c = lib.aimet_qdq_per_channel

    def launch_acts(sp):
        for (a, o, n, e) in act_calls:
            rc = qdq_t(a, o, n, ctypes.byref(e), 0, 0, sp)
            if rc:
                _native.check(rc)

    # all 54 parameter QDQs of the forward in ONE launch (aimet_qdq_channel_plan_*)
    from aimet_amd.tensor_quantizer import ChannelQdqPlan
    plan = ChannelQdqPlan([(w, outs[2 * i], 0, outs[2 * i + 1]) for i, (_, w) in enumerate(weights)]) \
        if not args.per_weight_launches else None
    plan_run = lib.aimet_qdq_channel_plan_run

    def launch_weights(sp):
        if plan is not None:
            rc = plan_run(plan._handle, 0, 0, sp)
            if rc:
                _native.check(rc)
            return
        for (a, o, outer, C, K, tab) in w_calls:
            rc = qdq_c(a, o, outer, C, K, tab, 0, 0, sp)
            if rc:
                _native.check(rc)

    # The step is captured once into two HIP graphs (activation QDQs, weight QDQs) and replayed:
    # 109 launches per step would otherwise cost ~8 us of host launch each.
    use_graph = not args.eager
    if use_graph:
        cap = torch.cuda.Stream(dev)
        g_act, g_w = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        cap.wait_stream(stream)
        with torch.cuda.stream(cap):
            launch_acts(ctypes.c_void_p(cap.cuda_stream))   # warm (outside capture)
            launch_weights(ctypes.c_void_p(cap.cuda_stream))
        stream.wait_stream(cap)
        torch.cuda.synchronize()
        with torch.cuda.graph(g_act, stream=cap):
            launch_acts(ctypes.c_void_p(cap.cuda_stream))
        with torch.cuda.graph(g_w, stream=cap):
            launch_weights(ctypes.c_void_p(cap.cuda_stream))
        torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        if use_graph:
            g_act.replay()
        else:
            launch_acts(sptr)
        if i is not None:
            ev[i][1].record(stream)
        if use_graph:
            g_w.replay()
        else:
            launch_weights(sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # HIP events on the launch stream bracket the activation QDQ launches of every timed step
    act_ms = [s.elapsed_time(e) for s, e in ev]
    kernel_ms = sum(act_ms) / len(act_ms)
    if world > 1:
        tt = torch.tensor([dt, enc_seconds, enc_cold, enc_fresh, enc_resident], dtype=torch.float64,
                          device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt, enc_seconds, enc_cold, enc_fresh, enc_resident = (float(v) for v in tt)

    ms_per_step = dt / args.steps * 1e3
    value = n_step * world * args.steps / dt / 1e9
    achieved = n_act * BYTES_QDQ / (kernel_ms / 1e3) / 1e9
    result = {
        "metric": "fake-quant Gelem/s (ResNet-50 W8A8 QuantSim forward QDQ; + compute_encodings wall-clock)",
        "value": round(value, 3),
        "unit": "Gelem/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: U(0,1) 224x224 images (seed 1234+rank), activations of a random-init ResNet-50 (seed 0)",
        "config": {"workload": "resnet50_w8a8_per_channel_fake_quant_fwd", "launch": "hipgraph" if use_graph else "eager",
                   "weight_qdq": "per-weight launches" if plan is None else "one batched launch", "global_batch": args.batch * world,
                   "per_gpu_batch": args.batch, "act_elems_per_step": n_act, "weight_elems_per_step": n_w,
                   "act_quantizers": len(act_calls), "weight_quantizers": len(w_calls),
                   "weight_channels": int(sum(c[3] for c in w_calls)), "parallelism": "dp%d" % world,
                   "compute_encodings_s": round(enc_seconds, 4),
                   "compute_encodings_cold_s": round(enc_cold, 4),
                   "compute_encodings_fresh_quantizers_s": round(enc_fresh, 4),
                   "compute_encodings_resident_s": round(enc_resident, 4),
                   "compute_encodings_runs_ms": enc_runs_ms,
                   "compute_encodings_gpu_span_ms": enc_spans,
                   "compute_encodings_host_phases_ms": enc_phases,
                   "compute_encodings_new_sim_s": round(enc_new_s, 4),
                   "compute_encodings_new_sim_gpu_span_ms": sorted(new_spans)[len(new_spans) // 2] if new_spans else None,
                   "compute_encodings_plan_equals_resident": enc_plan_equal,
                   # two passes (min/max, histogram) of 4 B over every activation and weight element
                   "compute_encodings_roofline": {
                       "algorithmic_gb": round(8 * n_step / 1e9, 3),
                       "achieved_gbps": round(8 * n_step / enc_seconds / 1e9, 1),
                       "frac": round(8 * n_step / enc_seconds / 1e9 / HBM_PEAK_GBPS, 4)},
                   "compute_encodings_timing": "median of %d CalibrationPlan.run(reset=True) calls (after 2 "
                                               "untimed ones): reset and "
                                               "recompute the sim's quantizers (created once, as QuantizationSimModel "
                                               "does) with the plan prepared once over the resident activations; "
                                               "beside it the first call of the process (cold), %d "
                                               "compute_encodings_resident calls on fresh quantizers (plan made "
                                               "inside) and %d on the sim's quantizers (cached plan, its tensors "
                                               "checked by identity every call); max over ranks"
                                               % (max(1, args.plan_reps), args.enc_reps, args.enc_reps),
                   "compute_encodings_scheme": "tf_enhanced act per-tensor + tf_enhanced weight per-channel sym"},
        "roofline": {"bound": "hbm", "kernel": "qdq_per_tensor (tensor_vec_kernel)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": TRAFFIC_GB if n_act == TRAFFIC_ELEMS else None,
                     "bytes_per_elem": BYTES_QDQ, "launches_per_step": len(act_calls),
                     "avg_launch_us": round(kernel_ms * 1e3 / len(act_calls), 2),
                     "act_qdq_ms_per_step": round(kernel_ms, 4),
                     "timing": "HIP events on the launch stream around the %d activation QDQ launches of each "
                               "timed step (%s)" % (len(act_calls), "graph replay" if use_graph else "eager")},
    }
    if world == 1 and not args.no_dropin:
        # the whole step's QDQ kernel time: the activation launches (events) + the weights' launch
        w_ms = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if use_graph:
                g_w.replay()
            else:
                launch_weights(sptr)
            e1.record(stream)
            torch.cuda.synchronize()
            w_ms.append(e0.elapsed_time(e1))
        try:   # a secondary measurement: a failure here is recorded in the line, not fatal to it
            result["config"]["dropin"] = dropin_surface(model, dev, kernel_ms + sorted(w_ms)[2])
        except Exception as e:   # noqa: BLE001
            result["config"]["dropin"] = {"error": "%s: %s" % (type(e).__name__, e)}
    del model
    cb = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:   # a failure of the host-side baseline is recorded in the line, not fatal to it
            cb = cpu_baseline(acts, weights, act_enc, w_enc, args.cpu_sample_images, act_outs, outs[0::2])
        except Exception as e:   # noqa: BLE001
            result["cpu_baseline"] = {"value": None, "unit": "Gelem/s", "cores": 1, "kind": "reference",
                                      "sample": "not measured", "error": "%s: %s" % (type(e).__name__, e)}
    if cb is not None:
        n = cb["n"]
        sample = ("first %d images of each activation tensor + all weights (%d elems), per-tensor + per-channel "
                  "QDQ with the bench's encodings, single-threaded on the host" % (args.cpu_sample_images, n))
        port = {"value": round(n / cb["port_s"] / 1e9, 4), "cores": 1, "seconds": round(cb["port_s"], 3),
                "what": "oracle/dlq_oracle.c (C restatement)"}
        omp = {"value": round(n / cb["omp_s"] / 1e9, 4), "cores": cb["omp_threads"], "nproc": os.cpu_count(),
               "openmp": cb["openmp"], "what": "oracle/dlq_oracle.c with OpenMP"}
        if "ref_s" in cb:
            result["cpu_baseline"] = {"value": round(n / cb["ref_s"] / 1e9, 4), "unit": "Gelem/s", "cores": 1,
                                      "kind": "reference",
                                      "sample": sample + "; oracle/_ref/libdlq_ref.so = the reference "
                                                "DlQuantization CPU code compiled from its sources",
                                      "seconds": round(cb["ref_s"], 3), "port": port, "omp": omp,
                                      "parity": cb["parity"], "compute_encodings": cb["enc"]}
        else:
            result["cpu_baseline"] = {"value": port["value"], "unit": "Gelem/s", "cores": 1, "kind": "port",
                                      "sample": sample + "; " + port["what"], "seconds": port["seconds"],
                                      "omp": omp, "parity": cb["parity"], "compute_encodings": cb["enc"]}
    if enc_exchange is not None:
        result["config"]["compute_encodings_exchange_s"] = enc_exchange["seconds"]
        result["config"]["compute_encodings_exchange"] = dict(
            enc_exchange, ratio_to_headline=round(enc_exchange["seconds"] / enc_seconds, 4),
            what="the sharded calibration's staged plan (stage 1, all_reduce MAX, stage 2, all_reduce SUM, stage 4) "
                 "over a world-size-1 group formed before any GPU call; median of the same reset+recompute runs")
    if world > 1:
        # the calibration exchange of this workload: what formed, and the two collectives' cost
        result["config"]["dist_backend"] = dist.get_backend()
        result["config"]["world_formed"] = dist.get_world_size()
        result["config"]["allreduce_ms"] = time_exchange(dev, aq)
        result["config"]["allreduce_timing"] = ("median of 20 synchronised calls per collective, max over ranks; "
                                                "one MAX + one SUM per calibration batch")
        # the encodings every rank computed must agree (they are reduced from the same global stats)
        sig = torch.tensor([hash(tuple(e.to_tuple() for e in act_enc)) & 0x7FFFFFFFFFFF], dtype=torch.int64,
                           device=dev if dist.get_backend() == "nccl" else "cpu")
        lo, hi = sig.clone(), sig.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        result["config"]["encodings_identical_across_ranks"] = bool(lo.item() == hi.item())
    if rank == 0:
        print(json.dumps(result), flush=True)
    cplan.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
