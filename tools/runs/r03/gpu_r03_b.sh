#!/usr/bin/env bash
# Round 3: column-swizzled LDS histogram + parallel skip in the min/max walk.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run stats_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "histogram or hist or minmax or stats or config or calibration or entropy or boundary"
run vit_512_32 300 python -u benchmarks/vit_calibration.py --images 128 --oracle-check 0
run vit_1024_32 300 env AIMET_TUNE_HIST_BLOCK=1024 python -u benchmarks/vit_calibration.py --images 128 --oracle-check 0
run vit_512_16 300 env AIMET_TUNE_HIST_COLS=16 python -u benchmarks/vit_calibration.py --images 128 --oracle-check 0
run vit_256_16 300 env AIMET_TUNE_HIST_COLS=16 AIMET_TUNE_HIST_BLOCK=256 python -u benchmarks/vit_calibration.py --images 128 --oracle-check 0
run vit_1024_16 300 env AIMET_TUNE_HIST_COLS=16 AIMET_TUNE_HIST_BLOCK=1024 python -u benchmarks/vit_calibration.py --images 128 --oracle-check 0
run hist_split 300 python -u tools/studies/vit_hist_split.py
run bench 600 python -u bench.py --no-cpu-baseline
run bench_1024 600 env AIMET_TUNE_HIST_BLOCK=1024 python -u bench.py --no-cpu-baseline
run vit_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vit_trace -o run -- python3 benchmarks/vit_calibration.py --images 96 --oracle-check 0
run vit_pmc_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/vit_pmc_sq -o run -- python3 benchmarks/vit_calibration.py --images 64 --oracle-check 0
