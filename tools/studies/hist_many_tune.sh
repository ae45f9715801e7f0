for cfg in "256 131072" "256 262144" "512 131072" "512 262144" "512 524288" "1024 262144" "1024 524288" "1024 1048576"; do
  set -- $cfg
  AIMET_TUNE_HIST_BLOCK=$1 AIMET_TUNE_HIST_ELEMS=$2 timeout -k 10 120 python tools/studies/hist_many_tune.py >> gpurun_out/tune.txt 2>/dev/null || exit 1
done
