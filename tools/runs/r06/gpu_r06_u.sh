#!/usr/bin/env bash
# Round 6, closing check U (2/2), after the last library change: the bench's kernel trace (+
# --stats) and its FETCH_SIZE and WRITE_SIZE PMC passes (each its own run), summarised as in
# round 5 (tools/studies/prof_summary.py), and the compute_encodings timeline.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
B="python3 bench.py --no-secondary --no-cpu-baseline --no-dropin --enc-reps 1 --plan-reps 1"
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 20
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- $B --steps 2 --warmup 1
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- $B --steps 2 --warmup 1
python3 tools/studies/prof_summary.py $OUT/trace $OUT/pmc_fetch $OUT/pmc_write --steps 20 > $OUT/bench_pmc_summary.txt 2>&1
cp $OUT/trace/run_kernel_stats.csv $OUT/bench_kernel_stats.csv 2>/dev/null
rm -rf $OUT/trace $OUT/pmc_fetch $OUT/pmc_write
run enc_trace 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/enc_trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline --no-dropin
python3 tools/studies/enc_timeline.py $OUT/enc_trace > $OUT/enc_timeline.txt 2>&1
rm -rf $OUT/enc_trace
# the AdaRound backward's instruction counts at the final tree (its own --pmc run)
run ada_pmc 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/ada_pmc_final -o run -- python3 tools/studies/ada_bwd_tune.py --scales 1 --reps 1 --tag pmc_final
