#!/usr/bin/env bash
# Round 4 closing check A: the whole GPU suite, smoke, the default bench line and its kernel trace.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python -u bench.py
run bench_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o run -- python3 bench.py --steps 20 --no-cpu-baseline
python tools/studies/prof_summary.py $OUT/bench_trace --steps 20 > $OUT/bench_trace_summary.txt 2>&1
rm -f $OUT/bench_trace/run_kernel_trace.csv
