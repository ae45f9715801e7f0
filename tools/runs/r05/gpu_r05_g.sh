#!/usr/bin/env bash
# Round 5, session g: host split of bench.py's plan runs; the bench's kernel trace and its two PMC
# passes (FETCH_SIZE, WRITE_SIZE: the roofline record's HBM traffic).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run enc_host 300 python -u tools/studies/enc_bench_host.py --reps 20
B="python3 bench.py --no-cpu-baseline --no-dropin --enc-reps 1 --plan-reps 1"
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 20
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- $B --steps 2 --warmup 1
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- $B --steps 2 --warmup 1
python3 tools/studies/prof_summary.py $OUT/trace $OUT/pmc_fetch $OUT/pmc_write --steps 20 > $OUT/bench_pmc_summary.txt 2>&1
python3 tools/studies/prof_summary.py $OUT/trace --steps 20 > $OUT/bench_trace_summary.txt 2>&1
cp $OUT/trace/run_kernel_stats.csv $OUT/bench_kernel_stats.csv 2>/dev/null
rm -rf $OUT/trace $OUT/pmc_fetch $OUT/pmc_write
