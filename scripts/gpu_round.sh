#!/bin/bash
# One GPU call: the -m gpu suite (or a subset) then bench lines, each step under its own time
# limit; the first failure ends the call.
#   OUT=dir TESTS="files" K="-k expr" BENCH="args" BENCH_AB="ENV=val" WL="strings hop" scripts/gpu_round.sh
# WL: further workloads, one bench line each (--steps 5 --warmup 2, no CPU baseline, no h2d leg)
set -o pipefail
OUT=${OUT:-gpurun_out/r03}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
      > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
  tail -c 400 "$OUT/bench.log"
  if [ -n "$BENCH_AB" ]; then
    timeout -k 10 300 env $BENCH_AB python -u bench.py $BENCH --h2d-records 0 --no-cpu-baseline > "$OUT/bench_ab.log" 2>&1 || { tail -20 "$OUT/bench_ab.log"; exit 1; }
    tail -c 400 "$OUT/bench_ab.log"
  fi
fi
for w in $WL; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --h2d-records 0 \
      > "$OUT/wl_$w.log" 2>&1 || { tail -20 "$OUT/wl_$w.log"; exit 1; }
  tail -c 300 "$OUT/wl_$w.log"
done
