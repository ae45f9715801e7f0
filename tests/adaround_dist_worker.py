"""Worker of tests/test_adaround_dist_gpu.py (not collected by pytest): one rank of a data-parallel
AdaRound optimisation on the GPU kernels. Both ranks use cuda:0 (one-GPU box) over a gloo group
(alpha.grad is staged through host memory), in the eager loop and in the HIP-graph form (two
graphs with the collective between them)."""
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from test_adaround_dist_gpu import SEEDS, params, problem  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from aimet_amd.adaround_optimizer import AdaroundOptimizer
        conv, inp, out, d, o = problem()
        res = {}
        for mode in ("eager", "graph"):
            loss = torch.zeros(1, device="cuda")
            a = AdaroundOptimizer.optimize_rounding(conv, inp, out, d, o, 4, 0, params(), torch.nn.ReLU6(),
                                                    torch.Generator().manual_seed(SEEDS[rank]), loss,
                                                    use_graph=(mode == "graph"))
            res[mode] = a.detach().cpu()
            res[mode + "_loss"] = loss.cpu()
        torch.save(res, os.environ["OUT"] + ".%d" % rank)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
