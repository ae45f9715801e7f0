#!/usr/bin/env bash
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests
run sched 500 python tools/enc_schedule_tune.py
echo ALLDONE
