"""Why StatsBatch copies what it queues: on a network that overwrites a quantized output in place
(tests/test_quantsim.py BranchNet: `a.relu_()`, `b += a` after fc1's output quantizer), batched
statistics over the queued tensors themselves see the overwritten values. Prints, per form, how
many quantizer encodings differ from the per-call updates' (the reference's behaviour).

    python tools/studies/statsbatch_inplace_check.py
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import aimet_amd.qc_quantize_op as QO
    from aimet_amd.quantsim import QuantizationSimModel
    from test_quantsim import BranchNet, _quantizer_state
    data = [torch.randn(16, 64, device="cuda", generator=torch.Generator(device="cuda").manual_seed(i))
            for i in range(2)]
    orig_add, orig_eligible = QO.StatsBatch.add, QO.StatsBatch.eligible

    def run(form):
        if form == "per_call":
            QO.StatsBatch.eligible = staticmethod(lambda q, t: False)
        elif form == "batched_no_copy":
            QO.StatsBatch.add = lambda self, q, t, owned=False: orig_add(self, q, t, True)
        torch.manual_seed(3)
        sim = QuantizationSimModel(BranchNet().cuda().eval(), torch.randn(1, 64, device="cuda"),
                                   quant_scheme="tf_enhanced")
        sim.compute_encodings(lambda m, d: [m(x) for x in d], data)
        QO.StatsBatch.add, QO.StatsBatch.eligible = orig_add, orig_eligible
        return _quantizer_state(sim)

    ref = run("per_call")
    for form in ("batched_no_copy", "batched"):
        st = run(form)
        differ = [k for k in ref if st[k] != ref[k]]
        print("%-16s encodings differing from the per-call updates: %d of %d %s" % (form, len(differ), len(ref),
                                                                                 differ[:3]))


if __name__ == "__main__":
    main()
