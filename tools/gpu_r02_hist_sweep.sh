#!/usr/bin/env bash
# compute_encodings wall-clock vs the histogram pass's elements per workgroup (A/B/A order)
source "$(dirname "$0")/gpu_lib.sh"
for e in 131072 65536 262144 131072 32768 524288 131072; do
  AIMET_TUNE_HIST_ELEMS=$e run hist_$e 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
  echo "HIST_ELEMS=$e $(tail -1 "$OUT/hist_$e.log" | python -c 'import json,sys; c=json.loads(sys.stdin.read())["config"]; print(c["compute_encodings_s"], c["compute_encodings_fresh_quantizers_s"], c["compute_encodings_roofline"]["frac"])')"
done
echo ALLDONE
