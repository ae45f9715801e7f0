#!/usr/bin/env bash
# Round 4, session s: learned-grid per-tensor backward with the fold in the kernel at smaller grids
# (fewer arrivals per ticket counter) vs its own launch; the default (fold launch, tile order).
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
for cap in 512 1024; do
  AIMET_LG_FOLD_IN_KERNEL=1 AIMET_TUNE_LG_BWD="2:$cap" run lg16_cap$cap 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_cap$cap -o run -- python3 benchmarks/lg16_roofline.py --reps 40
  python tools/studies/lg16_trace_summary.py $OUT/lg16_cap$cap cap$cap > $OUT/lg16_cap${cap}_summary.txt 2>&1
  rm -f $OUT/lg16_cap$cap/run_kernel_trace.csv
done
AIMET_TUNE_LG_BWD="2:1024" run lg16_launch1024 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_launch1024 -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_launch1024 launch1024 > $OUT/lg16_launch1024_summary.txt 2>&1
rm -f $OUT/lg16_launch1024/run_kernel_trace.csv
run lg16_default 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lg16_default -o run -- python3 benchmarks/lg16_roofline.py --reps 40
python tools/studies/lg16_trace_summary.py $OUT/lg16_default default > $OUT/lg16_default_summary.txt 2>&1
rm -f $OUT/lg16_default/run_kernel_trace.csv
run t_lg 900 python -u -m pytest tests/test_gpu_parity.py tests/test_llama_quantsim_gpu.py -v --timeout 300 --timeout-method thread -k "learned_grid or lg_ or llama"
bash tools/runs/r04/gpu_r04_r.sh
