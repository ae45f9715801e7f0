#!/usr/bin/env bash
# Round 3: histogram chunk-size sweep + PMC of the [512][16] LDS histogram on ViT-L/16.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests/test_adaround_wrapper.py -x -q --timeout 300 --timeout-method thread
for e in 65536 131072 262144 524288; do
  run vit_e$e 300 env AIMET_TUNE_HIST_ELEMS=$e python -u benchmarks/vit_calibration.py --images 160 --oracle-check 0
done
run vit_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vit_trace -o run -- python3 benchmarks/vit_calibration.py --images 96 --oracle-check 0
run vit_pmc_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/vit_pmc_sq -o run -- python3 benchmarks/vit_calibration.py --images 64 --oracle-check 0
run vit_pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/vit_pmc_fetch -o run -- python3 benchmarks/vit_calibration.py --images 64 --oracle-check 0
