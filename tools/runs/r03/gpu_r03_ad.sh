#!/usr/bin/env bash
# Round 3: the 16-bit forward dispatch launches once per call (it launched the default shape a
# second time); lg tests, the lg16 roofline by HIP events, the Llama step and its kernel trace.
source "$(dirname "${BASH_SOURCE[0]}")/../../gpu_lib.sh"
run lg_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "learned or lg or range_learning or qat"
run lg16 300 python -u benchmarks/lg16_roofline.py
run llama 600 python -u benchmarks/llama_qat.py --steps 5 --warmup 2
run llama_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/llama_trace3 -o run -- python3 benchmarks/llama_qat.py --steps 3 --warmup 1
