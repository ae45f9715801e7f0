#!/usr/bin/env bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel-trace + PMC passes.
# Stops at the first step that faults / aborts / times out (exit >= 124 or signal); ordinary
# test failures (exit 1) are recorded and the next step still runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-smoke,pytest,bench,prof,pmc}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
case ",$STEPS," in *,smoke,*) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()";; esac
case ",$STEPS," in *,pytest,*) run pytest_gpu 1200 python -m pytest tests -q -m gpu -p no:cacheprovider;; esac
case ",$STEPS," in *,bench,*) run bench 600 python bench.py ${BENCH_ARGS:-};; esac
export TMPDIR=/tmp
case ",$STEPS," in *,prof,*)
  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline;; esac
case ",$STEPS," in *,pmc,*)
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline;; esac
echo ALLDONE
