#!/usr/bin/env bash
# Round 3: histogram launch-shape sweep (block x LDS columns) + AdaRound caller-surface tests.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run ada_tests 600 python -u -m pytest tests/test_adaround_wrapper.py -x -q --timeout 300 --timeout-method thread
for bc in 1024x16 1024x8 512x16 512x8 256x8 256x16; do
  b=${bc%x*}; c=${bc#*x}
  run vit_$bc 300 env AIMET_TUNE_HIST_BLOCK=$b AIMET_TUNE_HIST_COLS=$c python -u benchmarks/vit_calibration.py --images 128 --oracle-check 0
  run bench_$bc 300 env AIMET_TUNE_HIST_BLOCK=$b AIMET_TUNE_HIST_COLS=$c python -u bench.py --no-cpu-baseline --steps 20
  run kr_$bc 300 env AIMET_TUNE_HIST_SHAPE=$bc python -u benchmarks/kernel_roofline.py --no-cpu --reps 10
done
run hist_split 300 python -u tools/studies/vit_hist_split.py
run stats_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "histogram or hist or minmax or stats or config or calibration or entropy or boundary"
