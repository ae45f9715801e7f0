#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run t_reset 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_distributed_gpu.py -k "reset or shard or distributed or exchange"
export AIMET_BENCH_BACKEND=gloo
run bench_gpus2 600 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline
unset AIMET_BENCH_BACKEND
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
run bench 600 python bench.py
echo ALLDONE
