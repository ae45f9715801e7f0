#!/usr/bin/env bash
# Shared helper for GPU sessions: `run NAME TIMEOUT CMD...` logs to gpurun_out/NAME.log, stops the
# whole script at the first step that faults / aborts / times out (exit >= 124 or a signal);
# ordinary failures (exit 1, 2) are recorded and the next step still runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "${BASH_SOURCE[0]}")/..}"
OUT=$PWD/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
