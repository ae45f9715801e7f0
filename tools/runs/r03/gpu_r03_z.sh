#!/usr/bin/env bash
# Round 3: AdaRound tests + 10k-iteration MobileNet-v2 (config 3) + smoke.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adaround"
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
