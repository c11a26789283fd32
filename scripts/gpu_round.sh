#!/bin/bash
# One GPU call: the -m gpu suite (or a subset) then the default bench line, each step under
# its own time limit; the first failure ends the call.
set -o pipefail
OUT=${OUT:-gpurun_out/r03}
mkdir -p "$OUT"
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
  tail -2 "$OUT/bench.log"
fi
