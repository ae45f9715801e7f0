#!/usr/bin/env bash
# Round 4, session t (merged with the closing check A after the GPU pool outage): the whole GPU
# suite, smoke, the bench line; the AdaRound backward tuning and 2k-iteration loop at this commit.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python -u bench.py
run ada_tune 300 python -u tools/studies/ada_bwd_tune.py
run ada2k 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
AIMET_ADA_GRAPH_ITERS=50 run ada2k_k50 600 python -u benchmarks/adaround_mobilenet.py --iterations 2000
