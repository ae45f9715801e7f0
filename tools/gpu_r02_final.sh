#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
run bench 600 python bench.py
run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
run prof_sum 120 python tools/prof_summary.py "$OUT/prof" "$OUT/pmc_fetch" "$OUT/pmc_write" --steps 5
rm -f "$OUT"/prof/*kernel_trace.csv "$OUT"/pmc_*/*kernel_trace.csv
run vit 300 python -u benchmarks/vit_calibration.py
run rq_gpu 600 python -u benchmarks/resnet_quantsim.py --repeats 3
echo ALLDONE
