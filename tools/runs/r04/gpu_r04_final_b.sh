#!/usr/bin/env bash
# Round 4 closing check B: HBM traffic of the bench (PMC passes), the kernel rooflines, the AdaRound
# backward's VALU count, the 16-bit learned-grid kernels' trace.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run prof_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
run prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
run prof_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
python3 tools/studies/prof_summary.py $OUT/prof_trace $OUT/prof_fetch $OUT/prof_write --steps 5 > $OUT/prof_summary.txt 2>&1
rm -rf $OUT/prof_trace $OUT/prof_fetch $OUT/prof_write
run roofline 600 python -u benchmarks/kernel_roofline.py
run ada_pmc_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/ada_pmc -o run -- python3 tools/studies/ada_bwd_tune.py --reps 1
rm -f $OUT/ada_pmc/run_kernel_trace.csv
run lg16_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_trace -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_trace r04 > $OUT/lg16_trace_summary.txt 2>&1
rm -f $OUT/lg16_trace/run_kernel_trace.csv
