#!/usr/bin/env bash
# Round-3 first check: smoke, bench line, ViT calibration trace + PMC.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python -u bench.py
run vit 600 python -u benchmarks/vit_calibration.py --images 96 --oracle-check 0
run vit_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/vit_trace -o run -- python3 benchmarks/vit_calibration.py --images 96 --oracle-check 0
run vit_pmc_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/vit_pmc_sq -o run -- python3 benchmarks/vit_calibration.py --images 64 --oracle-check 0
run vit_pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/vit_pmc_fetch -o run -- python3 benchmarks/vit_calibration.py --images 64 --oracle-check 0
