#!/usr/bin/env bash
# Round 3 final check: the whole GPU suite, smoke, the default bench line and its kernel trace,
# config 3 (AdaRound 10k) and config 5 (Llama QAT step).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python -u bench.py
run bench_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o run -- python3 bench.py --steps 20 --no-cpu-baseline
rm -f $OUT/bench_trace/run_kernel_trace.csv
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
run llama 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
