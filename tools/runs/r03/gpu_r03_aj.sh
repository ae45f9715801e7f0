#!/usr/bin/env bash
# Round 3 checkpoint: the whole GPU suite, smoke, the default bench line, the Llama step twice.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python -u bench.py
run llama1 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run llama2 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
