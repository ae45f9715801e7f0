"""Config 4 (BASELINE.json / SURVEY §8(d)): ViT-L/16 INT8 TF-Enhanced histogram calibration with
the calibration batch sharded per sample across GPUs.

  python benchmarks/vit_calibration.py                       # 1 GPU
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
         benchmarks/vit_calibration.py                       # N GPUs (RCCL)

256 images N(0,1) (seed 3), global batch 32 (8 calibration batches), each rank runs the forward
on its 32/N images. Quantizers: one TF-Enhanced per-tensor activation quantizer on the model input
and on the output of every op QuantizationSimModel quantizes under the default config
(workloads/vit.py activation_modules: patch conv, concat, pos add, and per block LayerNorm x2,
qkv, q*scale, q@k^T, softmax, @v, proj, fc1, GELU, fc2, residual adds x2, final LN, head:
317 ops + input, about 122.6 M elements per image). Per batch
the ranks run the device statistics (min/max on the first batch, 512-bin histogram, PDF fold) and
exchange them with ONE all_reduce(MAX) + ONE all_reduce(SUM) of the packed buffers
(aimet_amd.distributed). Reported (rank 0, one JSON line):
  * stats Gelem/s per GPU and aggregate (elements histogrammed / wall time of the statistics
    path between two device synchronisations, forward excluded, max over ranks), in a process
    warmed by one untimed statistics pass on throwaway quantizers (--cold: without it),
  * time inside the two collectives, forward time,
  * encodings identical on every rank (all_gather of a digest) and, at N=1, bit-identical to the
    CPU oracle fed the same tensors, for every quantizer (--oracle-check N: the first N only; the
    oracle analyzers run in a thread pool on the host, outside the timed region).
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=256)
    ap.add_argument("--batch", type=int, default=32, help="global calibration batch")
    ap.add_argument("--oracle-check", type=int, default=-1, help="-1: every quantizer (N=1 only)")
    ap.add_argument("--oracle-threads", type=int, default=16)
    ap.add_argument("--phased", action="store_true", help="single rank: run the sharded phases anyway")
    ap.add_argument("--cold", action="store_true", help="time the first batch in a cold process (no warm-up pass)")
    ap.add_argument("--profile-host", action="store_true", help="cProfile the host side of the later batches")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from aimet_amd import distributed as D
    from aimet_amd.libpymo import QuantizationMode
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    from workloads.vit import activation_modules, vit_l16

    model = vit_l16(seed=0, device=dev)
    layers = activation_modules(model)
    quantizers = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in range(len(layers) + 1)]
    acts = []
    hooks = [m.register_forward_hook(lambda mod, i, o: acts.append(o)) for m in layers]
    per_rank = args.batch // world
    g = torch.Generator().manual_seed(3)
    images = torch.randn(args.images, 3, 224, 224, generator=g)       # the same 256 images on every rank
    n_check = 0 if world > 1 or args.oracle_check == 0 else \
        len(quantizers) if args.oracle_check < 0 else min(args.oracle_check, len(quantizers))
    oracle_pool = analyzers = None
    if n_check:
        from concurrent.futures import ThreadPoolExecutor

        from oracle import oracle as O
        analyzers = [O.Analyzer(O.QUANTIZATION_TF_ENHANCED) for _ in range(n_check)]
        oracle_pool = ThreadPoolExecutor(args.oracle_threads)

    stream = torch.cuda.current_stream(dev)
    t_fwd = t_stats = t_coll = 0.0
    per_batch, host_batch, gpu_batch = [], [], []
    shadow = None
    elems = 0
    ex = None
    for b0 in range(0, args.images, args.batch):
        x = images[b0 + rank * per_rank: b0 + (rank + 1) * per_rank].to(dev)
        acts.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            model(x)
        torch.cuda.synchronize()
        t_fwd += time.perf_counter() - t0
        tensors = [x] + [a.contiguous() for a in acts]
        assert len(tensors) == len(quantizers), (len(tensors), len(quantizers))
        elems += sum(t.numel() for t in tensors)
        if b0 == 0 and not args.cold:
            # warm the process once (code objects of the statistics kernels, allocator pools) on
            # throwaway quantizers: the timed calibration is what it costs in a warm process
            warm = [AimetTensorQuantizer(QuantizationMode.QUANTIZATION_TF_ENHANCED) for _ in quantizers]
            D.sharded_update_stats(warm, tensors, fused=not args.phased)
            AimetTensorQuantizer.getEncodings(warm, 8, False, False, False)
            shadow = warm if world == 1 else None
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        if args.profile_host:
            from aimet_amd import _native
            native_s = []
            orig_call = _native.call

            def timed_call(name, *a):
                t = time.perf_counter()
                r = orig_call(name, *a)
                native_s.append((name, (time.perf_counter() - t) * 1e3))
                return r
            _native.call = timed_call
        t0 = time.perf_counter()
        ex = D.sharded_update_stats(quantizers, tensors, exchange=ex, fused=not args.phased)
        host_batch.append(time.perf_counter() - t0)   # until every launch is enqueued
        if args.profile_host:
            _native.call = orig_call
            print("host: batch %d enqueue %.3f ms, native calls %s" % (b0 // args.batch, host_batch[-1] * 1e3,
                                                                      native_s), file=sys.stderr)
        torch.cuda.synchronize()
        per_batch.append(time.perf_counter() - t0)
        if shadow is not None:
            # the GPU time of the statistics alone, on the warm-up quantizers (the same state: they
            # saw every earlier batch too): the stream is held by a sleep kernel while the host
            # enqueues, so e_a .. e_b spans only the statistics kernels -- what a pipelined
            # calibration loop, which enqueues the statistics while the forward still runs, pays
            e_a, e_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(20_000_000)
            e_a.record(stream)
            D.sharded_update_stats(shadow, tensors, fused=not args.phased)
            e_b.record(stream)
            torch.cuda.synchronize()
            gpu_batch.append(e_a.elapsed_time(e_b) / 1e3)
        t_stats += per_batch[-1]
        if analyzers:
            # the oracle sees the same tensors, one update per quantizer per batch (untimed)
            host = [t.cpu().numpy().ravel() for t in tensors[:n_check]]
            list(oracle_pool.map(lambda ia: analyzers[ia[0]].update(ia[1]), enumerate(host)))
            del host
        # the collectives alone (same packed buffers, values already reduced: MAX / SUM of zeros
        # would change them, so time a copy of each buffer)
        if world > 1:
            mm, cnt = ex.minmax.clone(), ex.counts.clone()
            c0 = torch.cuda.Event(enable_timing=True)
            c1 = torch.cuda.Event(enable_timing=True)
            c0.record(stream)
            dist.all_reduce(mm, op=dist.ReduceOp.MAX)
            dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
            c1.record(stream)
            torch.cuda.synchronize()
            t_coll += c0.elapsed_time(c1) / 1e3
    for h in hooks:
        h.remove()
    encs = AimetTensorQuantizer.getEncodings(quantizers, 8, False, False, False)
    digest = hashlib.sha256(json.dumps([e.to_tuple() for e, _ in encs]).encode()).hexdigest()

    same = True
    if world > 1:
        tt = torch.tensor([t_stats, t_fwd, t_coll], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_stats, t_fwd, t_coll = (float(v) for v in tt)
        digests = [None] * world
        dist.all_gather_object(digests, digest)
        same = all(d == digest for d in digests)
    oracle_ok, mismatches = None, None
    if analyzers:
        mismatches = [i for i, a in enumerate(analyzers) if encs[i][0].to_tuple() != a.compute(8).as_tuple()]
        oracle_ok = not mismatches
        oracle_pool.shutdown()

    if rank == 0:
        per_gpu = elems / t_stats / 1e9
        print(json.dumps({
            "metric": "TF-Enhanced calibration statistics Gelem/s (ViT-L/16, batch sharded)",
            "value": round(per_gpu * world, 3), "unit": "Gelem/s", "n_gpus": world,
            "per_gpu_gelem_s": round(per_gpu, 3), "elements_per_rank": elems,
            "stats_s": round(t_stats, 4), "stats_ms_per_batch": [round(v * 1e3, 3) for v in per_batch],
            "stats_enqueue_ms_per_batch": [round(v * 1e3, 3) for v in host_batch],
            "stats_gpu_ms_per_batch": [round(v * 1e3, 3) for v in gpu_batch],
            "collectives_s": round(t_coll, 4), "forward_s": round(t_fwd, 3),
            "quantizers": len(quantizers), "images": args.images, "global_batch": args.batch,
            "act_elems_per_image": round(elems * world / args.images),
            "encodings_identical_across_ranks": same, "encodings_equal_cpu_oracle": oracle_ok,
            "oracle_checked_quantizers": n_check, "oracle_mismatches": mismatches,
            "data": "synthetic N(0,1) images (seed 3), random-init ViT-L/16 (seed 0)"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
