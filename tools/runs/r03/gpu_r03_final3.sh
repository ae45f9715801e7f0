#!/usr/bin/env bash
# Round 3 closing check after the two-call compute_encodings and the Llama QuantSim tests: the whole
# GPU suite, smoke, the bench line and its kernel trace, config 3 (AdaRound 10k) and config 5 (Llama QAT).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " passed" $OUT/gpu_tests.log && ! grep -q " failed\| error" $OUT/gpu_tests.log || { echo "tests failed"; exit 1; }
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 300 python -u bench.py
run bench_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o run -- python3 bench.py --steps 20 --no-cpu-baseline
python tools/studies/prof_summary.py $OUT/bench_trace --steps 20 > $OUT/bench_trace_summary.txt 2>&1
rm -f $OUT/bench_trace/run_kernel_trace.csv
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
run llama 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
