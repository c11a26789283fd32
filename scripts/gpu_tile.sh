# Tile staging check (GPU box): its own tests, TUMBLE parity, then the whole suite and the bench.
# Usage: bash scripts/gpu_tile.sh TAG [SUITE=1] [BENCH=1]
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "tile or golden or tumble or two_phase" \
    > $O/tile_tests.log 2>&1 || { echo "tile tests failed"; tail -40 $O/tile_tests.log; exit 1; }
tail -2 $O/tile_tests.log
if [ "${3:-1}" = 1 ]; then
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --h2d-records 0 > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
python - $O/bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value %.3g  ms/step %.2f  job %.3f  rows %d" % (d["value"], d["ms_per_step"], d["job_roofline"]["frac"], d["rows_fired"]))
for k, v in sorted(d["kernels_warmup"].items(), key=lambda kv: -kv[1]["total_ms"]):
    print("  %-18s %4d launches  %.3f ms avg  %.2f ms total" % (k, v["launches"], v["avg_ms"], v["total_ms"]))
PY
fi
if [ "${2:-1}" = 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
fi
