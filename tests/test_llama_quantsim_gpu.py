"""Config 5's QuantSim form at the model level (SURVEY §8 a14 through the caller, VERDICT r02 weak
item 7): a 2-decoder-layer Llama-3-8B (workloads/llama.py: dim 4096, GQA 32/8 heads, SwiGLU 14336;
vocab cut to 1024) in a range-learning QuantizationSimModel, W4 per-channel symmetric / A16, run
under bf16 autocast -- the Linear weights go through the cast-fused learned-grid kernels, the
activations through the 16-bit I/O kernels, the ranges through aimet_lg_gate_ranges.

Every quantized tensor of the forward is checked against the reference's calculate_forward_pass
(quantsim_straight_through_grad.py:191-249) restated in torch ops (oracle/torch_ref.lg_forward,
pinned by golden_lg.npz): the reference's op on a bf16 tensor computes in float32 (torch promotes
against the float32 range parameters), and the drop-in's 16-bit kernels return that float32
result rounded to the input's dtype, which is what autocast's next matmul consumes -- so the
comparison is the float32 restatement rounded to bfloat16, bit for bit.

Two shapes: the small one (2 decoder layers, vocab 1024, seq 64) and config 5's stated shapes with
one decoder layer -- the full 128,256-token vocabulary (the lm_head's W4 per-channel quantizer:
128256 x 4096 = 525 M elements, 128,256 channels, the largest per-channel table on the path) and
seq 2048 (the 16-bit activation quantizers at their real sizes), micro-batch 1."""
import pytest
import torch
from torch import nn

from conftest import gpu_available
from oracle import torch_ref as T

gpu = pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")

# (decoder layers, vocab, seq): the small model, and config 5's vocabulary and sequence length
SHAPES = [pytest.param((2, 1024, 64), id="small"), pytest.param((1, 128256, 2048), id="full_vocab_seq2048")]
CFG = {"defaults": {"ops": {"is_output_quantized": "True"},
                    "params": {"is_quantized": "True", "is_symmetric": "True"},
                    "strict_symmetric": "False", "per_channel_quantization": "True"}}


def _sim(shape):
    """The range-learning QuantizationSimModel of a `layers`-layer Llama-3-8B with `vocab` tokens,
    calibrated on one sequence of `seq` tokens; returns (sim, the other sequence, fwd)."""
    from aimet_amd.quantizers import QuantScheme
    from aimet_amd.quantsim import QuantizationSimModel
    from workloads.llama import Llama

    layers, vocab, seq = shape
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    with torch.device(dev):
        model = Llama(lambda i, o: nn.Linear(i, o, bias=False), layers=layers, vocab=vocab)
    with torch.no_grad():
        g = torch.Generator(device=dev).manual_seed(0)
        for p in model.parameters():
            if p.dim() > 1:
                p.normal_(0, 0.02, generator=g)
    sim = QuantizationSimModel(model, quant_scheme=QuantScheme.training_range_learning_with_tf_init,
                               default_param_bw=4, default_output_bw=16, in_place=True, config_file=CFG)
    ids = torch.randint(vocab, (2, seq), device=dev, generator=torch.Generator(device=dev).manual_seed(3))

    def fwd(m, x):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return m(x)

    sim.compute_encodings(fwd, ids[:1])
    return sim, ids[1:], fwd


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_llama_quantsim_forward_equals_reference_ops(shape):
    from aimet_amd.qc_quantize_op import LearnedGridQuantWrapper

    sim, ids, fwd = _sim(shape)
    wrappers = [(n, w) for n, w in sim.model.named_modules() if isinstance(w, LearnedGridQuantWrapper)]
    linears = [(n, w) for n, w in wrappers if isinstance(w._module_to_wrap, nn.Linear)]
    assert len(linears) == shape[0] * 7 + 1, [n for n, _ in wrappers]
    head = linears[-1][1]._module_to_wrap
    assert head.weight.shape == (shape[1], 4096)

    rec, outs = {}, {}

    def raw_hook(mod, i, o, n):   # inside the wrapper: the patched (quantized) weight, the raw output
        rec[n] = (o.detach().clone(), mod.weight.detach().clone() if isinstance(mod, nn.Linear) else None)

    def out_hook(mod, i, o, n):
        outs[n] = o.detach().clone()
    hooks = [w._module_to_wrap.register_forward_hook(lambda mod, i, o, n=n: raw_hook(mod, i, o, n))
             for n, w in wrappers]
    hooks += [w.register_forward_hook(lambda mod, i, o, n=n: out_hook(mod, i, o, n)) for n, w in wrappers]
    with torch.no_grad():
        logits = fwd(sim.model, ids)
    for h in hooks:
        h.remove()
    assert torch.isfinite(logits.float()).all()
    del logits

    checked_w = checked_o = 0
    for n, w in wrappers:
        raw_out, wq = rec[n]
        if wq is not None and w.param_quantizers["weight"].enabled:
            pq = w.param_quantizers["weight"]
            assert wq.dtype == torch.bfloat16, n   # the cast autocast applies, fused into the kernel
            want = T.lg_forward(w._module_to_wrap.weight.detach(), w.weight_encoding_min.detach(),
                                w.weight_encoding_max.detach(), 4, True, False, False, pq.channel_axis)[0]
            torch.testing.assert_close(wq, want.to(wq.dtype), rtol=0, atol=0, msg=n)
            checked_w += 1
        if w.output_quantizers[0].enabled and w.output0_encoding_min is not None:
            got = outs[n]
            assert got.dtype == raw_out.dtype, n
            want = T.lg_forward(raw_out.float(), w.output0_encoding_min.detach(), w.output0_encoding_max.detach(),
                                16)[0]
            torch.testing.assert_close(got, want.to(got.dtype), rtol=0, atol=0, msg=n)
            checked_o += 1
    assert checked_w == len(linears) and checked_o >= len(linears)


# range gradients: error bound in units of 2^-24 x (sum of |terms|) of the float64 sum (fixed: the
# bar is part of the test)
LG_BOUND_C = 2.0


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_llama_quantsim_backward_equals_reference_ops(shape):
    """The same model, one QAT backward (loss = mean square of the float32 logits): every weight's
    and every quantized output's gradient == the reference's straight-through gradient (mask x
    upstream gradient) bit for bit, and every range gradient (weight_encoding_min/max per channel,
    output0_encoding_min/max) within LG_BOUND_C = 2 float32 eps x the sum of |terms| of the float64
    value of the reference's sums (oracle/torch_ref.lg_encoding_grads_bound on the upstream
    gradients the hooks saw; float32 sums in another order than torch's)."""
    from aimet_amd.qc_quantize_op import LearnedGridQuantWrapper

    sim, ids, fwd = _sim(shape)
    wrappers = [(n, w) for n, w in sim.model.named_modules()
                if isinstance(w, LearnedGridQuantWrapper) and isinstance(w._module_to_wrap, nn.Linear)]
    raw, gw, gout = {}, {}, {}

    def raw_hook(mod, i, o, n):
        raw[n] = o.detach().clone()
        mod.weight.register_hook(lambda gr, n=n: gw.__setitem__(n, gr.detach().clone()))

    def out_hook(mod, i, o, n):
        o.register_hook(lambda gr, n=n: gout.__setitem__(n, gr.detach().clone()))
    hooks = [w._module_to_wrap.register_forward_hook(lambda mod, i, o, n=n: raw_hook(mod, i, o, n))
             for n, w in wrappers]
    hooks += [w.register_forward_hook(lambda mod, i, o, n=n: out_hook(mod, i, o, n)) for n, w in wrappers]
    sim.model.train()
    sim.model.zero_grad(set_to_none=True)
    raw_in_grads = {}
    for n, w in wrappers:   # the gradient that reaches each wrapped Linear's output (grad_x of the output quantizer)
        w._module_to_wrap.register_full_backward_hook(
            lambda mod, gi, go, n=n: raw_in_grads.__setitem__(n, go[0].detach().clone()))
    fwd(sim.model, ids).float().square().mean().backward()
    for h in hooks:
        h.remove()
    assert len(gw) == len(gout) == len(wrappers)

    for n, w in wrappers:
        pq = w.param_quantizers["weight"]
        W = w._module_to_wrap.weight
        emin, emax = w.weight_encoding_min.detach(), w.weight_encoding_max.detach()
        gx, gmin, gmax = T.lg_gradients(W.detach(), gw[n].float(), emin, emax, 4, True, False, False, pq.channel_axis)
        torch.testing.assert_close(W.grad, gx, rtol=0, atol=0, msg=n)
        ex_min, ex_max, bmin, bmax = T.lg_encoding_grads_bound(W.detach(), gw[n].float(), emin, emax, 4, True,
                                                               ch_axis=pq.channel_axis)
        T.report_sum_bound_units(gmin, ex_min, bmin, "llama %s weight grad_min, reference torch ops" % n)
        T.assert_within_sum_bound(w.weight_encoding_min.grad, ex_min, bmin, LG_BOUND_C, "llama %s weight grad_min" % n)
        T.assert_within_sum_bound(w.weight_encoding_max.grad, ex_max, bmax, LG_BOUND_C, "llama %s weight grad_max" % n)

        omin, omax = w.output0_encoding_min.detach(), w.output0_encoding_max.detach()
        x, up = raw[n].float(), gout[n].float()
        gx, gmin, gmax = T.lg_gradients(x, up, omin, omax, 16)
        torch.testing.assert_close(raw_in_grads[n], gx.to(raw_in_grads[n].dtype), rtol=0, atol=0, msg=n)
        ex_min, ex_max, bmin, bmax = T.lg_encoding_grads_bound(x, up, omin, omax, 16)
        T.report_sum_bound_units(gmin, ex_min, bmin, "llama %s output grad_min, reference torch ops" % n)
        T.report_sum_bound_units(gmax, ex_max, bmax, "llama %s output grad_max, reference torch ops" % n)
        r_min, r_max = T.lg_range_grads_rounded_sums(x, up, omin, omax, 16)
        T.report_sum_bound_units(r_min, ex_min, bmin, "llama %s output grad_min, formula on rounded exact sums" % n)
        T.report_sum_bound_units(r_max, ex_max, bmax, "llama %s output grad_max, formula on rounded exact sums" % n)
        T.assert_within_sum_bound(w.output0_encoding_min.grad, ex_min, bmin, LG_BOUND_C, "llama %s output grad_min" % n)
        T.assert_within_sum_bound(w.output0_encoding_max.grad, ex_max, bmax, LG_BOUND_C, "llama %s output grad_max" % n)
