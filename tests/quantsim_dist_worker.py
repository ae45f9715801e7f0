"""Worker of tests/test_quantsim_sharded_gpu.py (not collected by pytest): BASELINE config 1 through
the drop-in QuantizationSimModel.compute_encodings -- ResNet-50 W8A8 per-tensor, 8 batches x 32
U(0,1) images (seed 1234), SCHEME = post_training_tf_enhanced | post_training_tf.

  WORLD_SIZE=2: rank r forwards images [32b + 16r, 32b + 16r + 16) of every batch b on cuda:0; the
                ranks form a gloo group, so compute_encodings shards (one MAX + one SUM per forward);
  WORLD_SIZE=1: one process fed the 8 whole batches: each batch's two 16-image halves are forwarded
                separately (the ranks' convolution shapes) and each
                quantizer's two tensors are concatenated and updated ONCE, one statistics batch of
                32 images, through the sim's own (unsharded) StatsBatch. The CPU oracle analyzers
                are fed the same concatenations (and the parameters), in a host thread pool.
Writes the sim's encodings, what the calibration copied / exchanged, the oracle's mismatches
(WORLD_SIZE=1), and a digest of every tensor the quantizers were handed, to OUT.<rank>."""
import concurrent.futures as cf
import hashlib
import json
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

N_BATCHES, BATCH = 8, 32


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # convolutions without MIOpen (im2col + GEMM): MIOpen's algorithm choice depends on the state
    # of its find-db, which the processes of the test share and update, so the same convolution can
    # differ in its last bits between processes
    torch.backends.cudnn.enabled = False
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import aimet_amd.qc_quantize_op as QO
    from aimet_amd.quantizers import QuantScheme
    from aimet_amd.quantsim import QuantizationSimModel
    from workloads.resnet import resnet50
    scheme = getattr(QuantScheme, os.environ["SCHEME"])
    model = resnet50(seed=0, device=dev)
    images = torch.rand(N_BATCHES * BATCH, 3, 224, 224, device=dev,
                        generator=torch.Generator(device=dev).manual_seed(1234))
    sim = QuantizationSimModel(model, images[:1], quant_scheme=scheme, default_output_bw=8, default_param_bw=8)
    half = BATCH // 2
    digests = []
    orig_add, orig_flush, orig_end = QO.StatsBatch.add, QO.StatsBatch.flush, QO.StatsBatch.end_forward
    out = {}
    if world > 1:
        def add(self, q, t, owned=False):
            digests.append([hashlib.sha1(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()])
            return orig_add(self, q, t, owned)
        QO.StatsBatch.add = add

        def calibrate(m, _):
            for b in range(N_BATCHES):
                lo = b * BATCH + rank * half
                m(images[lo:lo + half])
        sim.compute_encodings(calibrate, None)
    else:
        from oracle import oracle as O
        mode = O.QUANTIZATION_TF_ENHANCED if scheme == QuantScheme.post_training_tf_enhanced else O.QUANTIZATION_TF
        pool = cf.ThreadPoolExecutor(16)
        analyzers, futures = {}, []
        stash, order = {}, []
        fwd = [0]

        def add(self, q, t, owned=False):
            if id(q) not in stash:
                order.append(id(q))
            stash.setdefault(id(q), (q, []))[1].append(t.detach().clone())

        def end_forward(self):
            fwd[0] += 1
            if fwd[0] % 2:
                return   # the batch's first half
            for key in order:
                q, ts = stash[key]
                digests.append([hashlib.sha1(t.contiguous().cpu().numpy().tobytes()).hexdigest() for t in ts])
                x = torch.cat([t.reshape(-1) for t in ts])
                a = analyzers.setdefault(key, O.Analyzer(mode))
                futures.append(pool.submit(a.update, x.cpu().numpy()))
                orig_add(self, q, x, True)
            stash.clear()
            order.clear()
            orig_end(self)
            for f in futures:   # one batch at a time in host memory; each analyzer in batch order
                f.result()
            futures.clear()
        QO.StatsBatch.add, QO.StatsBatch.end_forward = add, end_forward

        def calibrate(m, _):
            for b in range(N_BATCHES):
                m(images[b * BATCH:b * BATCH + half])
                m(images[b * BATCH + half:(b + 1) * BATCH])
        sim.compute_encodings(calibrate, None)
        pool.shutdown()
        checked, bad = 0, []
        for name, w in sim.quant_wrappers():
            for q in list(w.input_quantizers) + list(w.output_quantizers):
                if q.enabled and q.encoding is not None:
                    checked += 1
                    want = analyzers[id(q)].compute(8, q.use_symmetric_encodings).as_tuple()
                    if q.encoding.to_tuple() != want:
                        bad.append(name)
            q = w.param_quantizers["weight"]
            a = O.Analyzer(mode)
            a.update(w._module_to_wrap.weight.detach().float().cpu().numpy().ravel())
            checked += 1
            if q.encoding.to_tuple() != a.compute(8, q.use_symmetric_encodings).as_tuple():
                bad.append(name + ".weight")
        out["oracle"] = {"checked": checked, "mismatches": bad}
    QO.StatsBatch.add, QO.StatsBatch.flush, QO.StatsBatch.end_forward = orig_add, orig_flush, orig_end
    enc = sim.get_encodings_dict()
    out.update({"encodings": {"activation": enc["activation_encodings"], "param": enc["param_encodings"]},
                "calibration": sim._last_calibration, "digests": digests})
    with open(os.environ["OUT"] + ".%d" % rank, "w") as f:
        json.dump(out, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
