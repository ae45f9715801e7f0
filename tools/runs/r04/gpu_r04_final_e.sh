#!/usr/bin/env bash
# Round 4 closing check E (after the AdaRound backward / Adam tail flag, the 1x1 slices folded by
# Adam, the search-job upload on the side stream): the whole GPU suite, smoke, the default bench line
# and its kernel stats, config 3 at 10k iterations.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python -u bench.py
run bench_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_stats -o run -- python3 bench.py --steps 20 --no-cpu-baseline
python tools/studies/prof_summary.py $OUT/bench_stats --steps 20 > $OUT/bench_stats_summary.txt 2>&1
rm -f $OUT/bench_stats/run_kernel_trace.csv
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
