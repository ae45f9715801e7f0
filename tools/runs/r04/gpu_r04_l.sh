#!/usr/bin/env bash
# Round 4, session l: why the MFMA channel-major kernels run 5-10x their latency estimate --
# random vs sequential batch rows, and SQ wave-cycle counters per kernel.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run pw_rand 300 python -u tools/studies/pw_cm_bench.py --reps 100
run pw_seq 300 python -u tools/studies/pw_cm_bench.py --reps 100 --seq
run pw_pmc 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $OUT/pw_pmc -o run -- python3 tools/studies/pw_cm_bench.py --reps 5 --shapes 0,1 --forms mfma
run pw_pmc2 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD --kernel-trace --output-format csv -d $OUT/pw_pmc2 -o run -- python3 tools/studies/pw_cm_bench.py --reps 5 --shapes 0,1 --forms mfma
rm -f $OUT/pw_pmc/run_kernel_trace.csv $OUT/pw_pmc2/run_kernel_trace.csv
