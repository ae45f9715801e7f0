"""Sharded calibration through the drop-in QuantizationSimModel.compute_encodings (SURVEY §8(e),
v1/quantsim.py:381-449): BASELINE config 1 -- ResNet-50 W8A8 per-tensor, 8 batches x 32 U(0,1)
images (seed 1234) -- with every batch split 16 + 16 over two ranks. Every encoding of both ranks
must equal the encodings of one process fed the 8 whole batches.

CPU (this test file): world size 2 over gloo, the quantizers' operators replaced by the oracle
(tests/oracle_ops.py: the CPU restatement of the reference analyzers; this container has no GPU),
so the single process IS the oracle fed the whole batches; the sim, its wrappers, StatsBatch and the
packed exchange are the product code. The GPU form (gfx950 operators, two gloo ranks on cuda:0) is
tests/test_quantsim_sharded_gpu.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_BATCHES, BATCH = 8, 32


def _images():
    return torch.rand(N_BATCHES * BATCH, 3, 224, 224, generator=torch.Generator().manual_seed(1234))


def _run(rank, world, port, scheme, out_q, threads):
    torch.set_num_threads(threads)
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_ops
        from aimet_amd.quantsim import QuantizationSimModel
        from workloads.resnet import resnet50
        patch = pytest.MonkeyPatch()
        oracle_ops.install(patch)
        model = resnet50(seed=0, device=torch.device("cpu"))
        images = _images()
        sim = QuantizationSimModel(model, images[:1], quant_scheme=scheme, default_output_bw=8, default_param_bw=8)
        share = BATCH // world

        def calibrate(m, _):
            for b in range(N_BATCHES):
                lo = b * BATCH + rank * share
                m(images[lo:lo + share])
        sim.compute_encodings(calibrate, None)
        out_q.put((world, rank, sim.get_encodings_dict(), sim._last_calibration))
    except BaseException as e:   # noqa: BLE001 -- reported to the parent
        out_q.put((world, rank, "%s: %s" % (type(e).__name__, e), None))
        raise
    finally:
        if world > 1:
            dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("scheme", ["tf_enhanced"])
def test_config1_sharded_quantsim_equals_single_process_oracle(scheme):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    threads = max(1, (os.cpu_count() or 4) // 3)
    procs = [ctx.Process(target=_run, args=(r, 2, port, scheme, q, threads)) for r in range(2)]
    procs.append(ctx.Process(target=_run, args=(0, 1, 0, scheme, q, threads)))   # the single process
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        world, rank, enc, info = q.get(timeout=900)
        res[(world, rank)] = (enc, info)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single, info1 = res[(1, 0)]
    assert not isinstance(single, str), single
    assert info1["sharded"] is False
    act = single["activation_encodings"]
    n_act = sum(len(v) for e in act.values() for v in e.values())
    assert n_act == 55 and len(single["param_encodings"]) == 54
    for r in range(2):
        enc, info = res[(2, r)]
        assert not isinstance(enc, str), enc
        assert info["sharded"] is True and info["world"] == 2
        assert enc["activation_encodings"] == single["activation_encodings"], r
        assert enc["param_encodings"] == single["param_encodings"], r
