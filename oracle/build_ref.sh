#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY. Compiles the reference DlQuantization CPU sources *in place*
# (read-only, from /root/reference) plus oracle/ref_shim.cpp into oracle/_ref/libdlq_ref.so.
# Flags follow the reference build (CMakeLists.txt:148-156: -O3, x86-64 baseline, no FMA).
# ParserModule.cpp (needs pugixml, absent) and the *ForPython.cpp files (pybind) are left out;
# none of them is on the QDQ/analyzer path. Outputs go only to oracle/_ref/ (git-ignored).
set -euo pipefail
REF=${AIMET_REFERENCE:-/root/reference}
DLQ=$REF/ModelOptimizations/DlQuantization
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/_ref
if [ ! -d "$DLQ/src" ]; then
  echo "reference not present at $DLQ; skipping oracle/_ref build" >&2
  exit 0
fi
mkdir -p "$OUT/obj"
SRCS=(EntropyEncodingAnalyzer MseEncodingAnalyzer PercentileEncodingAnalyzer QuantizerFactory
      TensorQuantizationSim TensorQuantizer TfEncodingAnalyzer TfEnhancedEncodingAnalyzer
      math_functions quantization_utils trim_functions GraphQuantizer MainQuantizationClass
      TfQuantizer TfEnhancedQuantizer)
CXXFLAGS="-std=c++17 -O3 -fPIC -ffp-contract=off -I$DLQ/include -I$DLQ/src"
pids=()
for s in "${SRCS[@]}"; do
  o=$OUT/obj/$s.o
  if [ ! -f "$o" ] || [ "$DLQ/src/$s.cpp" -nt "$o" ]; then
    g++ $CXXFLAGS -c "$DLQ/src/$s.cpp" -o "$o" &
    pids+=($!)
  fi
done
for p in "${pids[@]}"; do wait "$p"; done
g++ $CXXFLAGS -c "$HERE/ref_shim.cpp" -o "$OUT/obj/ref_shim.o"
g++ -shared -o "$OUT/libdlq_ref.so" "$OUT"/obj/*.o -lpthread
echo "built $OUT/libdlq_ref.so"
