# Tile passes with slice tables (HOP / CUMULATE flush + fire from tiles): parity, then A/B bench.
# Usage: bash scripts/gpu_tstate.sh TAG [TESTS=1] [BENCH=1]
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
if [ "${2:-1}" = 1 ]; then
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_configs.py -k "hop or cumulate or tile or two_phase or sliding" \
    > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
fi
if [ "${3:-1}" = 1 ]; then
summ() {
python - $1 <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ks = sorted(d["kernels_warmup"].items(), key=lambda kv: -kv[1]["total_ms"])
print("  %.4g rec/s  %.2f ms/step  job %.3f | " % (d["value"], d["ms_per_step"], d["job_roofline"]["frac"]) +
      "  ".join("%s %.3f x%d" % (k, v["avg_ms"], v["launches"]) for k, v in ks[:6]))
PY
}
for W in hop cumulate tumble; do
  for T in 1 0; do
    echo "== $W FG_TILE_STATE=$T"
    FG_TILE_STATE=$T timeout -k 10 300 python bench.py --workload $W --steps 4 --warmup 1 --no-cpu-baseline --h2d-records 0 \
        > $O/${W}_$T.log 2>&1 || { tail -5 $O/${W}_$T.log; exit 1; }
    summ $O/${W}_$T.log
  done
done
fi
