#!/usr/bin/env bash
# Round 3 profile set: full GPU tests, bench line, rocprof trace + PMC of the bench, ViT, AdaRound 10k.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gpu_tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 600 python -u bench.py
run prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
run prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
run prof_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
run summary 120 python3 tools/studies/prof_summary.py $OUT/prof_trace $OUT/prof_fetch $OUT/prof_write --steps 5
run vit 300 python -u benchmarks/vit_calibration.py --images 160 --oracle-check 0
run vit_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vit_trace -o run -- python3 benchmarks/vit_calibration.py --images 160 --oracle-check 0
run vit_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/vit_fetch -o run -- python3 benchmarks/vit_calibration.py --images 160 --oracle-check 0
run ada10k 900 python -u benchmarks/adaround_mobilenet.py --iterations 10000
