# A/B of an engine knob on the GPU box: parity subset, then the default bench with the knob
# off and on (alternating, twice each). Usage: bash scripts/ab_bench.sh VAR "pytest -k expr"
set -o pipefail
VAR=${1:-FG_SPECULATE}
K=${2:-"stream_parity or lane_conflict or snapshot or regions or outlier or config"}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for v in 0 1 0 1; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-records 0 --steps 5 > gpurun_out/ab_$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ab_$v.log; exit 1; }
  python - "$VAR=$v" gpurun_out/ab_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[1], "ms/step %.3f" % d["ms_per_step"], " ".join("%s=%.4f" % (n, v["avg_ms"]) for n, v in k.items()))
PY
done
